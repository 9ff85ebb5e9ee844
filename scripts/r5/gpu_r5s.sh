#!/bin/bash
# Round 5: the split wide barrier-algebra kernels — forced on for the native interior point's tests (CFX_IPM_WIDE=1),
# the chain / reaching tests with the automatic choice, then the reaching solve from the reference start.
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
T="timeout -k 10"
CFX_IPM_WIDE=1 $T 600 python -u -m pytest tests/test_ipm_native.py -x -q --timeout 300 --timeout-method thread > $O/ipm_wide.log 2>&1 || { echo "ipm wide failed"; exit 1; }
$T 600 python -u -m pytest tests/test_chain_kkt.py tests/test_reaching_parity.py -x -q --timeout 300 --timeout-method thread > $O/chain.log 2>&1 || { echo "chain failed"; exit 1; }
$T 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 5000 --wall 150 --out $O/runs.jsonl > $O/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
