#!/bin/bash
# after an interior-point change: the native IPM GPU tests, then the reaching task (fatigue, reference start) under
# the Ipopt profile and the library profile.  usage: scripts/gpu_oracle_check.sh TAG
set -o pipefail
O=gpurun_out/${1:-oracle_check}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile ipopt --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_ipopt.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile cfx --bound-relax 1e-8 --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_cfx.txt 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/r.jsonl'):
    r = json.loads(l); print({k: r.get(k) for k in ('profile', 'lib', 'status', 'iterations', 'wall_s', 'f')})
"
