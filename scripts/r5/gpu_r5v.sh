#!/bin/bash
# Round 5: Ipopt's Hessian-degeneracy heuristic and the wide curvature sums — full GPU suite (+ the native interior
# point's tests with the wide path forced), then the reaching solves from the reference start.
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
CFX_IPM_WIDE=1 $T 600 python -u -m pytest tests/test_ipm_native.py -x -q --timeout 300 --timeout-method thread > $O/ipm_wide.log 2>&1 || { echo "ipm wide failed"; exit 1; }
$T 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 5000 --wall 150 --out $O/runs.jsonl > $O/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
