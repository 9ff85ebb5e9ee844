#!/bin/bash
# Round 5: the force objective from the reference start under three more option sets (Ipopt's scaling with and
# without the inertia test; one bound per pulse parameter with the inertia test).
set -o pipefail
O=gpurun_out/r5ii
mkdir -p $O
T="timeout -k 10"
R="python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 30000 --wall 280 --out $O/runs.jsonl"
CFX_IPM_TRACE=1 $T 330 $R --range-scaling 0 --inertia-test 1 > $O/rs0_inertia.log 2>&1 || { echo "run 1 failed"; exit 1; }
CFX_IPM_TRACE=1 $T 330 $R --range-scaling 0 > $O/rs0.log 2>&1 || { echo "run 2 failed"; exit 1; }
CFX_IPM_TRACE=1 $T 330 $R --pulse-bounds first --inertia-test 1 > $O/first_inertia.log 2>&1 || { echo "run 3 failed"; exit 1; }
