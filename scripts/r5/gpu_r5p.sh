#!/bin/bash
# Round 5: the reaching task's solves from the reference start after the faster stage-chain factorisation.
set -o pipefail
out=gpurun_out/r5p
mkdir -p $out
timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 5000 --wall 150 --out $out/runs.jsonl > $out/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
timeout -k 10 330 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 15000 --wall 300 --out $out/runs.jsonl > $out/ref_force.log 2>&1 || { echo "force failed"; exit 1; }
