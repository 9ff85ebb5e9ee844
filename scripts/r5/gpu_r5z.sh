#!/bin/bash
# Round 5 end: cfg 5 multistart (512 starts, +-10 %) with the round's solver changes — Ipopt's defaults, and the
# restart extension.
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
T="timeout -k 10"
$T 200 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --jsonl $O/ms.jsonl --label default > $O/ms_default.log 2>&1 || { echo "default failed"; exit 1; }
$T 200 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --restart --jsonl $O/ms.jsonl --label restart > $O/ms_restart.log 2>&1 || { echo "restart failed"; exit 1; }
$T 200 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --restart --soft 0.9999 --jsonl $O/ms.jsonl --label restart_soft > $O/ms_restart_soft.log 2>&1 || { echo "restart soft failed"; exit 1; }
