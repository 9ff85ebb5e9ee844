# MSK value kernel with its RK stage loop rolled (libcfx.so) vs unrolled (variants/libcfx_base.so), alternating
# msk_probe at the bench's batch; then the MSK / interior-point / launch-shape GPU tests on the rolled build.
set -o pipefail
out=gpurun_out/r3aa
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_base.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_base.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
cat $out/ab.jsonl
timeout -k 10 600 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests/test_msk_gpu.py tests/test_ipm_native.py tests/test_launch_shapes.py tests/test_reference_solution.py > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -4 $out/pytest.log; exit $rc
