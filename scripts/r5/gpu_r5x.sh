#!/bin/bash
# Round 5: batch-1 latency by KKT layout after the stage-chain speed-ups, and a kernel trace of cfg 3 at batch 1.
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 400 python -u scripts/b1_layout_probe.py --reps 5 > $O/b1_layouts.jsonl 2> $O/b1.err || { echo "b1 failed"; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats -d $O/cfg3 -o run -- python3 -u scripts/profile_cfg3_native.py > $O/cfg3.log 2>&1 || { echo "cfg3 trace failed"; exit 1; }
