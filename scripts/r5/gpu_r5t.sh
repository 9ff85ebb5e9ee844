#!/bin/bash
# Round 5: the MSK Hessian pair kernel in three groups — MSK / reaching tests, cfg 5 Hessian timing, reaching solve.
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
T="timeout -k 10"
$T 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msk or Msk or reaching or chain" > $O/tests.log 2>&1 || { echo "tests failed"; exit 1; }
$T 240 python -u scripts/msk_probe.py --batch 4096 > $O/probe.jsonl 2> $O/probe.err || { echo "probe failed"; exit 1; }
$T 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 5000 --wall 150 --out $O/runs.jsonl > $O/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
