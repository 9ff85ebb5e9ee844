# Round 5: kernel breakdown of the reaching task's iteration with the chain layout; warm start and reference-start
# solves of the fatigue objective.  usage: bash scripts/gpu_r5b.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o chain -- python3 scripts/chain_probe.py --layouts chain --iters 6 > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 300 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start stored --max-iter 400 --wall 200 --out $out/warm.jsonl > $out/warm.log 2>&1 || { echo "warm failed"; exit 1; }
timeout -k 10 500 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 3000 --wall 420 --out $out/ref.jsonl > $out/ref.log 2>&1 || { echo "ref failed"; exit 1; }
