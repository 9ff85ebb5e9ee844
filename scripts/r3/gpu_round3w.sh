# Ipopt's filter reset heuristic in the native interior point and BatchedIpm: the interior-point / MSK GPU tests, then
# the cfg-5 64-start multistart with the heuristic on / off.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3w
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 700 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests/test_ipm_native.py tests/test_msk_gpu.py tests/test_gpu_parity.py tests/test_distributed_gpu.py > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/r3/resto_ipopt_defaults.py --filter-reset > $out/resto_fr.jsonl 2> $out/resto_fr.err; rc=$?
cat $out/resto_fr.jsonl; exit $rc
