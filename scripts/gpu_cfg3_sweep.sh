# cfg-3 launch-shape sweep (instances per lane x intervals per thread) at batch 2^18, then a kernel trace of the default.
set -o pipefail
out=gpurun_out/cfg3_sweep
mkdir -p $out
export TMPDIR=/tmp
for ni in 1 2; do
  for kpt in 0 2 5 10 25; do
    if [ $kpt -eq 0 ]; then unset CFX_KPT; else export CFX_KPT=$kpt; fi
    CFX_NI=$ni timeout -k 10 120 python -u scripts/cfg3_probe.py >> $out/sweep.jsonl 2> $out/err_${ni}_${kpt}.log || exit $?
    tail -1 $out/sweep.jsonl
  done
done
unset CFX_KPT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/cfg3_probe.py > $out/trace.log 2>&1 || exit $?
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$pass -o run -- python3 scripts/cfg3_probe.py > $out/pmc_$pass.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
echo done
