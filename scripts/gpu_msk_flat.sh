#!/bin/bash
# MSK GPU tests, then the reaching solves (kernel-path change in the MSK value recursion at small batches)
set -o pipefail
O=gpurun_out/${1:-msk_flat}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_msk_gpu.py tests/test_reaching_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile ipopt --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_ipopt.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile cfx --bound-relax 1e-8 --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_cfx.txt 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/r.jsonl'):
    r = json.loads(l); print({k: r.get(k) for k in ('profile', 'status', 'iterations', 'solve_wall_s', 's_per_iteration', 'f_end')})
"
