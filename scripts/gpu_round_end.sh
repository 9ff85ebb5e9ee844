# Round-end check: every GPU test, smoke(), the default bench line.  Stops at the first failure or GPU fault.
set -o pipefail
out=gpurun_out/${1:-round_end}
mkdir -p $out
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 1000 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?; check $out/bench.err; tail -c 400 $out/bench.json; [ $rc -eq 0 ] || exit $rc
# the driver's own short form (K = 20, W = 5)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_k20.json 2> $out/bench_k20.err; rc=$?; check $out/bench_k20.err; exit $rc
