# Full GPU test suite, then the NMPC / convergence bench sections.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/suite.log 2>&1; rc=$?
grep -q HSA_STATUS_ERROR gpurun_out/suite.log && { echo "GPU fault"; exit 3; }
tail -3 gpurun_out/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 65536 --cpu-seconds 0 --no-msk > gpurun_out/bench_nmpc.json 2> gpurun_out/bench_nmpc.err
