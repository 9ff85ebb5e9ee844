# Round 5: the force objective under Ipopt's defaults (soft restoration, filter resets, constant z init)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
CFX_IPM_TRACE=1 timeout -k 10 320 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --ipopt-defaults --max-iter 8000 --wall 300 --out $out/runs.jsonl > $out/ref_force_ipopt.log 2>&1 || { echo "force failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --ipopt-defaults --max-iter 5000 --wall 150 --out $out/runs.jsonl > $out/ref_fatigue_ipopt.log 2>&1 || { echo "fatigue failed"; exit 1; }
