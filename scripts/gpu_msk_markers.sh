# Marker-constraint GPU tests, then the rest of the MSK and native-IPM GPU suites.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s -m gpu --timeout 300 --timeout-method thread tests/test_msk_gpu.py -k "marker" > gpurun_out/msk_markers.log 2>&1; rc=$?
grep -q HSA_STATUS_ERROR gpurun_out/msk_markers.log && { echo "GPU fault"; exit 3; }
tail -15 gpurun_out/msk_markers.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_msk_gpu.py tests/test_ipm_native.py > gpurun_out/msk_rest.log 2>&1; rc=$?
tail -3 gpurun_out/msk_rest.log; exit $rc
