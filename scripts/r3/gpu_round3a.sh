# round 3: the fixed GPU tests, the L-BFGS test with its printout, the MSK profile and a default bench run.
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py tests/test_launch_shapes.py::test_bench_shape_cfg5_msk tests/test_reference_solution.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3a/pytest_fixed.log 2>&1 || { echo "fixed tests failed"; }
timeout -k 10 300 python -u -m pytest tests/test_ipm_native.py -k limited_memory -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r3a/pytest_lbfgs.log 2>&1 || { echo "lbfgs test failed"; exit 1; }
bash scripts/r3/gpu_msk_prof.sh r3a/msk || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err || { echo "bench failed"; exit 1; }
tail -c 3000 gpurun_out/r3a/bench.json
