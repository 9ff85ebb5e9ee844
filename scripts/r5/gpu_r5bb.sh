#!/bin/bash
# Round 5: msk_point with a branch per frame (inline-asm markers against branch merging) — MSK tests and g + J_g timing.
set -o pipefail
O=gpurun_out/r5bb
mkdir -p $O
T="timeout -k 10"
$T 240 python -u scripts/msk_probe.py --batch 4096 65536 > $O/probe.jsonl 2> $O/probe.err || { echo "probe failed"; exit 1; }
$T 240 python -u scripts/msk_probe.py --batch 65536 > $O/probe2.jsonl 2>> $O/probe.err || { echo "probe2 failed"; exit 1; }
$T 700 python -u -m pytest tests/test_msk_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; exit 1; }
