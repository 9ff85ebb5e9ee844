# New library (non-temporal stores, shorter interval chunks) vs the previous build: shooting + collocation tests, then
# the default bench line with each library.
set -o pipefail
mkdir -p gpurun_out/nt_ab
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/nt_ab/pytest.log 2>&1 || { tail -20 gpurun_out/nt_ab/pytest.log; exit 1; }
tail -2 gpurun_out/nt_ab/pytest.log
timeout -k 10 400 env CFX_LIB=var_libs/libcfx_old.so python -u bench.py > gpurun_out/nt_ab/bench_old.json 2> gpurun_out/nt_ab/old.err || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/nt_ab/bench_new.json 2> gpurun_out/nt_ab/new.err || exit 1
