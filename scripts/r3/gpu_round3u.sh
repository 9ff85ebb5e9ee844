# Store policy of the write stream: the micro (plain / nt / sc1 / sc1 nt, back-to-back vs one-by-one), the headline
# launch under CFX_STPOL 0 / 1 / 2 alternating, and the launch-shape + constant-J parity tests under CFX_STPOL=1.
set -o pipefail
out=gpurun_out/r3u
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 120 ./scripts/micro/store_policy > $out/store_policy.txt 2>&1 || { echo "micro failed"; tail -3 $out/store_policy.txt; exit 1; }
cat $out/store_policy.txt
timeout -k 10 400 python3 scripts/r3/stpol_ab.py 2 > $out/stpol_ab.jsonl 2> $out/stpol_ab.err || { echo "ab failed"; tail -3 $out/stpol_ab.err; exit 1; }
cat $out/stpol_ab.jsonl
CFX_STPOL=1 timeout -k 10 400 python -u -m pytest -q --tb=short -m gpu --timeout 250 --timeout-method thread tests/test_launch_shapes.py tests/test_constant_jac.py -k "not msk" > $out/pytest_sc1.log 2>&1; rc=$?; check $out/pytest_sc1.log; tail -3 $out/pytest_sc1.log; exit $rc
