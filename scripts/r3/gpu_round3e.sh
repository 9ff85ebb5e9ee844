set -o pipefail
out=gpurun_out/r3e
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r3/resto_trace.py phase 300 > $out/trace_phase.log 2>&1 || { echo "trace failed"; tail -20 $out/trace_phase.log; exit 1; }
grep -v "^  resto\|^it " $out/trace_phase.log | tail -5
timeout -k 10 300 python -u scripts/r3/resto_probe.py --cfg5-batch 16 --amp 0.1 --max-iter 600 > $out/resto16.jsonl 2> $out/resto16.err
cat $out/resto16.jsonl
