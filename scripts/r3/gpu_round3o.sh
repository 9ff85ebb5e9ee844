# MSK tangent kernel: plain vs non-temporal J_g stores, alternating builds on one box; MSK parity tests on the nt build.

set -o pipefail
out=gpurun_out/r3o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_ntj.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_ntj.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
cat $out/ab.jsonl
CFX_LIB=cocofest_amd/variants/libcfx_ntj.so timeout -k 10 400 python -u -m pytest tests/test_msk_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $out/pytest_ntj.log 2>&1
rc=$?
tail -3 $out/pytest_ntj.log
exit $rc
