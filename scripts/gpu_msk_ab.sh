#!/bin/bash
# MSK g + J_g A/B on one box: the fused stage/tangent kernel (default) against the two-kernel path
# (CFX_MSK_TANGENTS=split), alternating, after the MSK GPU tests.  Usage: scripts/gpu_msk_ab.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-msk}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_msk_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu -k "$K" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
for i in 1 2; do
  timeout -k 10 180 python -u scripts/msk_probe.py --batch 4096 65536 > $OUT/fused_$i.jsonl 2> $OUT/fused_$i.err || exit 1
  CFX_MSK_TANGENTS=split timeout -k 10 180 python -u scripts/msk_probe.py --batch 4096 65536 > $OUT/split_$i.jsonl 2> $OUT/split_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/msk_probe.py --batch 65536 --reps 10 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
grep -h ms_g_jac $OUT/*.jsonl | cut -c1-200
