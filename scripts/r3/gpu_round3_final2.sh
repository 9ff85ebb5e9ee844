# Round-3 final tree: every GPU test, smoke(), the default bench line; then the filter-reset diagnostics and the cfg-5
# multistart with the heuristic on / off.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3f2
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 600 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_k20.json 2> $out/bench_k20.err; rc=$?; check $out/bench_k20.err; tail -c 200 $out/bench_k20.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/r3/fr_diag.py > $out/fr_diag.jsonl 2> $out/fr_diag.err || { echo "diag failed"; tail -3 $out/fr_diag.err; exit 1; }
cat $out/fr_diag.jsonl
timeout -k 10 300 python3 scripts/r3/resto_ipopt_defaults.py --filter-reset > $out/resto_fr.jsonl 2> $out/resto_fr.err; rc=$?
cat $out/resto_fr.jsonl; exit $rc
