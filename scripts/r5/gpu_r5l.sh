#!/bin/bash
# Round 5: per-kernel times of the MSK g + J_g step (cfg 5, B = 65,536) with the stage coefficients split by
# derivative direction and with one thread per stage, after the scratch-memory fixes.
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
CFX_MSK_STAGE=split $T 300 rocprofv3 --kernel-trace --stats -d $O/split -o run -- python -u scripts/msk_probe.py --batch 65536 > $O/split.jsonl 2> $O/split.err &&
$T 300 rocprofv3 --kernel-trace --stats -d $O/par -o run -- python -u scripts/msk_probe.py --batch 65536 > $O/par.jsonl 2> $O/par.err &&
CFX_MSK_STAGE=split $T 240 python -u scripts/msk_probe.py --batch 65536 > $O/split_plain.jsonl 2>> $O/split.err &&
$T 240 python -u scripts/msk_probe.py --batch 65536 > $O/par_plain.jsonl 2>> $O/par.err &&
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msk or Msk or reaching" > $O/tests.log 2>&1
