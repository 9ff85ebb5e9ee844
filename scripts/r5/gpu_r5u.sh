#!/bin/bash
# Round 5: Hessian projection without run-time register indexing — MSK tests, a kernel trace of 40 reaching iterations.
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 700 python -u -m pytest tests/test_msk_gpu.py tests/test_reaching_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats -d $O/reach -o run -- python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 40 --wall 60 --out $O/reach_runs.jsonl > $O/reach.log 2>&1 || { echo "reach trace failed"; exit 1; }
