#!/bin/bash
# Round 5 end: cfg 5 multistart at Ipopt's default max_iter (3000), with and without the restart extension.
set -o pipefail
O=gpurun_out/r5z2
mkdir -p $O
T="timeout -k 10"
$T 300 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --max-iter 3000 --jsonl $O/ms.jsonl --label default_3000 > $O/ms_default.log 2>&1 || { echo "default failed"; exit 1; }
$T 300 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --max-iter 3000 --restart --jsonl $O/ms.jsonl --label restart_3000 > $O/ms_restart.log 2>&1 || { echo "restart failed"; exit 1; }
