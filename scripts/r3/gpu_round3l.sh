set -o pipefail
out=gpurun_out/r3l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r3/resto_probe.py --cfg5-batch 64 --amp 0.1 --max-iter 1000 --modes phase > $out/resto.jsonl 2> $out/resto.err || exit 1
cat $out/resto.jsonl
idx=$(python3 -c "import json;d=json.loads(open('$out/resto.jsonl').readline());print(' '.join(map(str,d['failed'][:2])))")
echo "tracing $idx"
timeout -k 10 600 python -u scripts/r3/resto_trace_cfg5.py $idx > $out/trace.log 2>&1
rc=$?
grep "====" $out/trace.log
exit $rc
