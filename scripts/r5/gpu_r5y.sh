#!/bin/bash
# Round 5: short chains at small batches — full GPU suite and the batch-1 layout probe with the automatic choice.
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 400 python -u scripts/b1_layout_probe.py --reps 3 > $O/b1_layouts.jsonl 2> $O/b1.err || { echo "b1 failed"; exit 1; }
