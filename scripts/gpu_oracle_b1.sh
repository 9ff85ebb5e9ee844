#!/bin/bash
# one-block oracle with register-cached elements: adaptive-mu tests, then cfg 3 batch-1 wall-clock and kernel trace
set -o pipefail
OUT=gpurun_out/${1:-oracle_b1}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -v --timeout 300 --timeout-method thread -m gpu -k "wide or adaptive or profile" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for p in ipopt cfx; do
  timeout -k 10 120 python -u scripts/ipm_profile_probe.py --profile $p --batch 1 --guess --reps 20 > $OUT/wall_$p.txt 2>&1 || exit 1
  grep profile $OUT/wall_$p.txt
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ipopt -o run -- python3 scripts/ipm_profile_probe.py --profile ipopt --batch 1 --guess --reps 10 > $OUT/trace_ipopt.log 2>&1 || exit 1
