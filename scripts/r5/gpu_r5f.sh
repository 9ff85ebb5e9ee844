# Round 5: per-pulse bounds on the pulse's first interval only: warm start, fatigue and force from the reference start
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start stored --max-iter 2000 --wall 150 --out $out/runs.jsonl > $out/warm_fatigue.log 2>&1 || { echo "warm failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 260 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 5000 --wall 240 --out $out/runs.jsonl > $out/ref_force.log 2>&1 || { echo "force failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 5000 --wall 150 --out $out/runs.jsonl > $out/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives force --start stored --max-iter 2000 --wall 150 --out $out/runs.jsonl > $out/warm_force.log 2>&1 || { echo "warm force failed"; exit 1; }
