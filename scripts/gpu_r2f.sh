# Round 2: write-bandwidth shapes (micro), native IPM tests + probe after the per-node objective kernels.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 120 ./scripts/micro/write_bw > gpurun_out/write_bw.txt 2>&1; cat gpurun_out/write_bw.txt
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py tests/test_gpu_parity.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_ipm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ipm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ipm_native_probe.py native > gpurun_out/ipm_probe.json 2> gpurun_out/ipm_probe.err; rc=$?
cut -c1-300 gpurun_out/ipm_probe.json; exit $rc
