# Round-3 end: every GPU test, smoke(), the default bench line and the driver's K = 20 form, then the rocprofv3
# kernel trace of the bench and one PMC pass per HBM counter (headline kernel traffic).  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3final
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 1100 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?; check $out/bench.err; tail -c 300 $out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_k20.json 2> $out/bench_k20.err; rc=$?; check $out/bench_k20.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-solve > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$pass -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-solve > $out/pmc_$pass.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
python3 scripts/summarize_pmc.py $out $out/summary 1527775232
echo done
