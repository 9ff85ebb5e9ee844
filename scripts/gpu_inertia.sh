#!/bin/bash
# inertia routine: the chain / interior-point GPU tests that use it, then the reaching task's kernel trace (Ipopt profile)
set -o pipefail
O=gpurun_out/${1:-inertia}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_chain_kkt.py tests/test_ipm_native.py -x -v --timeout 300 --timeout-method thread -m gpu -k "inertia or btri or chain" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/gpu_reach_prof.sh ${1:-inertia} ipopt || exit 1
