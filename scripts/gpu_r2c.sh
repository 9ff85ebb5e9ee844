# Round 2 (re-entry): full GPU suite on HEAD, smoke, full default bench line.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cut -c1-1500 gpurun_out/bench.json
