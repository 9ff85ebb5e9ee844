# Round-3 end, part 1: every GPU test, smoke(), the default bench line.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3end
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 700 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?; check $out/bench.err; tail -c 300 $out/bench.json; exit $rc
