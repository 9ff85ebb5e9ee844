#!/bin/bash
# Round 5: default bench (reaching section included) and the force objective from the reference start.
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
T="timeout -k 10"
$T 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
CFX_IPM_TRACE=1 $T 330 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 30000 --wall 300 --out $O/runs.jsonl > $O/ref_force.log 2>&1 || { echo "force failed"; exit 1; }
