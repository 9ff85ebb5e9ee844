#!/bin/bash
# Round 5 end: cfg 5 multistart — consecutive p, n resets allowed in a restoration phase (CFX_RS_RR_MAX) before it fails.
set -o pipefail
O=gpurun_out/r5z3
mkdir -p $O
T="timeout -k 10"
for R in 1 3 10 100; do
  CFX_RS_RR_MAX=$R $T 300 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --max-iter 3000 --jsonl $O/ms.jsonl --label rr$R > $O/ms_rr$R.log 2>&1 || { echo "rr$R failed"; exit 1; }
done
