# MSK: deferred tangent J stores + -freciprocal-math (libcfx.so) vs -freciprocal-math alone vs the previous build (alternating msk_probe at the bench's batch), then the MSK,
# interior-point, launch-shape and reference-solution GPU tests on the new build.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3s
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_recip.so cocofest_amd/variants/libcfx_prev.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_recip.so cocofest_amd/variants/libcfx_prev.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
cat $out/ab.jsonl
timeout -k 10 900 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests/test_msk_gpu.py tests/test_ipm_native.py tests/test_launch_shapes.py tests/test_reference_solution.py tests/test_constant_jac.py > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; exit $rc
