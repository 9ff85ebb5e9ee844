# Round-3 end, part 2: the driver's K = 20 bench form, the rocprofv3 kernel trace of the bench command, one PMC pass per
# HBM counter (headline kernel traffic), the kernel trace of the cfg-3 batch-1 native solve.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3end
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_k20.json 2> $out/bench_k20.err; rc=$?; check $out/bench_k20.err; tail -c 200 $out/bench_k20.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-solve > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$pass -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-solve > $out/pmc_$pass.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
python3 scripts/summarize_pmc.py $out $out/summary 1527775232
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg3_b1 -o run -- python3 scripts/profile_cfg3_native.py 10 1 > $out/cfg3_b1.log 2>&1 || { echo "cfg3 b1 trace failed"; exit 1; }
tail -1 $out/cfg3_b1.log
echo done
