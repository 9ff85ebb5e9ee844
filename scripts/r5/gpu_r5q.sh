#!/bin/bash
# Round 5: full GPU suite + smoke, default bench (with the reaching section), and a kernel trace of 40 reaching-task
# iterations from the reference start.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/reach -o run -- python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 40 --wall 60 --out $O/reach_runs.jsonl > $O/reach.log 2>&1 || { echo "reach trace failed"; exit 1; }
