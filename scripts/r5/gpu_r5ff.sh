#!/bin/bash
# Round 5: inertia test (Ipopt's inertia correction from the stage chain's pivot-block inertias) — parity tests, then
# the reaching task's two objectives from the reference start with it.
set -o pipefail
O=gpurun_out/r5ff
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_chain_kkt.py -k inertia -x -v --timeout 300 --timeout-method thread > $O/chain_tests.log 2>&1 || { echo "tests failed"; exit 1; }
CFX_IPM_TRACE=1 $T 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 30000 --wall 150 --inertia-test 1 --out $O/runs.jsonl > $O/ref_fatigue.log 2>&1 || { echo "fatigue failed"; exit 1; }
CFX_IPM_TRACE=1 $T 480 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 30000 --wall 420 --inertia-test 1 --out $O/runs.jsonl > $O/ref_force.log 2>&1 || { echo "force failed"; exit 1; }
