#!/bin/bash
# Round 5 end: MSK PMC passes (profiles/msk_pmc.json), the default bench, and a kernel trace of 40 reaching iterations.
set -o pipefail
O=gpurun_out/r5dd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/pmc_sq -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/sq.log 2>&1 || { echo "sq failed"; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/reach -o run -- python3 -u scripts/reaching_warmstart.py --objectives fatigue --start reference --max-iter 40 --wall 60 --out $O/reach_runs.jsonl > $O/reach.log 2>&1 || { echo "reach trace failed"; exit 1; }
