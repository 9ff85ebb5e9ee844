# Round 2: per-workgroup band-LU store sinks: band tests, IPM parity, multi-start probe.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "band" tests/test_ipm_native.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_band.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_band.log; [ $rc -eq 0 ] || exit $rc
for p in auto 0; do if [ $p = auto ]; then unset CFX_BAND_PLACEMENT; else export CFX_BAND_PLACEMENT=$p; fi
  timeout -k 10 120 python scripts/band_place_probe.py 4096 2>/dev/null || exit 1
  timeout -k 10 120 python scripts/band_place_probe.py 1024 2>/dev/null || exit 1
done
unset CFX_BAND_PLACEMENT
timeout -k 10 400 python -u scripts/ipm_native_probe.py native > gpurun_out/ipm_probe.json 2> gpurun_out/ipm_probe.err; rc=$?
cut -c1-200 gpurun_out/ipm_probe.json; exit $rc
