# Constant-J_g path: its GPU tests, then the interior point with / without CFX_KEEP_CONSTANT_JAC (alternating), then
# every GPU test, smoke() and the default bench line.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3q
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python -u -m pytest -q --tb=short -m gpu --timeout 200 --timeout-method thread tests/test_constant_jac.py > $out/pytest_keep.log 2>&1; rc=$?; check $out/pytest_keep.log; tail -3 $out/pytest_keep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 scripts/r3/keepj_ab.py 2 > $out/keepj_ab.jsonl 2> $out/keepj_ab.err; rc=$?; cat $out/keepj_ab.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?; check $out/bench.err; tail -c 400 $out/bench.json; exit $rc
