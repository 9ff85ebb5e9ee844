# MSK tangent kernel block width A/B: 32 instances per block (one block per CU) vs 16 (two blocks per CU), alternating
# builds on one box; then the MSK parity tests on the 16-wide build.
set -o pipefail
out=gpurun_out/r3n
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_tw16.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_tw16.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
cat $out/ab.jsonl
CFX_LIB=cocofest_amd/variants/libcfx_tw16.so timeout -k 10 400 python -u -m pytest tests/test_msk_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $out/pytest_tw16.log 2>&1
rc=$?
tail -3 $out/pytest_tw16.log
exit $rc
