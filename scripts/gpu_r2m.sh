# Blocked band LU: parity tests, wide-band timings, native interior point on the MSK / cfg3 problems.
set -o pipefail
out=gpurun_out/r2m
mkdir -p $out
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "band" > $out/band.log 2>&1; rc=$?; check $out/band.log; tail -3 $out/band.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/band_wide_probe.py > $out/wide.json 2> $out/wide.err; rc=$?; check $out/wide.err; cat $out/wide.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread tests/test_ipm_native.py tests/test_msk_gpu.py -k "ipm or interior or nmpc" > $out/ipm.log 2>&1; rc=$?; check $out/ipm.log; tail -3 $out/ipm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/profile_msk_native.py 1 64 > $out/msk.json 2> $out/msk.err; rc=$?; check $out/msk.err; cat $out/msk.json; exit $rc
