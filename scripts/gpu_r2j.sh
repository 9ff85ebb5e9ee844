# Round 2: native IPM parity + batch-1 probe + NMPC probe.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_ipm.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_ipm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ipm_b1_probe.py msk > gpurun_out/b1.json 2>/dev/null || exit 1
cut -c1-130 gpurun_out/b1.json
timeout -k 10 300 python -u scripts/nmpc_probe.py > gpurun_out/nmpc_probe.json 2>/dev/null; rc=$?
cut -c1-300 gpurun_out/nmpc_probe.json; exit $rc
