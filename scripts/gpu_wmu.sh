#!/bin/bash
# wide adaptive-mu oracle: the wide/one-block parity tests, the adaptive-mu spec tests, then the reaching iteration trace
set -o pipefail
OUT=gpurun_out/${1:-wmu}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ipm_native.py -x -v --timeout 300 --timeout-method thread -m gpu -k "wide or adaptive or profile" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash scripts/gpu_reach_prof.sh ${1:-wmu} ipopt || exit 1
