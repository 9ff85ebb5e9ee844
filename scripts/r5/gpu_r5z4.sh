#!/bin/bash
# Round 5 end: cfg 5 multistart with Ipopt's max_resto_iter default (3,000,000) instead of 200.
set -o pipefail
O=gpurun_out/r5z4
mkdir -p $O
T="timeout -k 10"
CFX_RS_RR_MAX=1000000 $T 300 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --max-iter 3000 --opt max_resto_iter=3000000 --jsonl $O/ms.jsonl --label resto_iter_ipopt_rrinf > $O/ms_c.log 2>&1 || { echo "b failed"; exit 1; }
