# Round 5: Ipopt's constant bound-multiplier initialisation on the reaching task; per-pulse bound placement.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
CFX_IPM_TRACE=1 timeout -k 10 260 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --bound-mult-init constant --max-iter 6000 --wall 240 --out $out/runs.jsonl > $out/ref_force_const.log 2>&1 || { echo "force failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --bound-mult-init constant --max-iter 5000 --wall 150 --out $out/runs.jsonl > $out/ref_fatigue_const.log 2>&1 || { echo "fatigue failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue,force --start stored --pulse-bounds first --max-iter 2000 --wall 80 --out $out/runs.jsonl > $out/warm_first.log 2>&1 || { echo "warm failed"; exit 1; }
