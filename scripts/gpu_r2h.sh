# Round 2: native IPM with nested dissection of the KKT band (small batches): parity + probes.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_ipm.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_ipm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ipm_native_probe.py native > gpurun_out/ipm_probe.json 2> gpurun_out/ipm_probe.err || exit 1
cut -c1-420 gpurun_out/ipm_probe.json
timeout -k 10 300 python -u scripts/nmpc_probe.py > gpurun_out/nmpc_probe.json 2> gpurun_out/nmpc_probe.err; rc=$?
cut -c1-600 gpurun_out/nmpc_probe.json; exit $rc
