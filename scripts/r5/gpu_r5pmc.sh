#!/bin/bash
# Round 5 end: PMC passes over the cfg 5 g + J_g kernels (FETCH_SIZE, WRITE_SIZE, VALU / FP64 instructions), one
# counter group per run, for profiles/msk_pmc.json (bench.py's msk roofline).
set -o pipefail
O=gpurun_out/r5pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/pmc_sq -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/sq.log 2>&1 || { echo "sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
