# Round 2: native interior point (cfx_ipm) parity vs BatchedIpm, then the wall-clock probe.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -v --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_ipm.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_ipm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ipm_native_probe.py > gpurun_out/ipm_probe.json 2> gpurun_out/ipm_probe.err; rc=$?
cat gpurun_out/ipm_probe.json; tail -5 gpurun_out/ipm_probe.err; exit $rc
