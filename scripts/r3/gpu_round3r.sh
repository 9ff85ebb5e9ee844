# MSK sincos / fast-reciprocal build vs the previous one (alternating, msk_probe at the bench's batch), the MSK and
# interior-point GPU tests on the new build (the Schur sums back on fused multiply-subtract), then the new build's MSK
# kernel trace + SQ counters.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3r
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_oldmsk.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_oldmsk.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
cat $out/ab.jsonl
timeout -k 10 900 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests/test_msk_gpu.py tests/test_ipm_native.py tests/test_launch_shapes.py tests/test_reference_solution.py > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r3/gpu_msk_prof.sh r3r/prof
