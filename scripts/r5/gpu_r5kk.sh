#!/bin/bash
# Round 5: counters of the stage-chain kernels (micro chain_bench, reaching-task shape): wait / active cycles, VALU, LDS.
set -o pipefail
O=gpurun_out/r5kk
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o run -- scripts/micro/bin/chain_bench 1501 > $O/p1.log 2>&1 || { echo "p1 failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CU_CYCLES --output-format csv -d $O/p2 -o run -- scripts/micro/bin/chain_bench 1501 > $O/p2.log 2>&1 || { echo "p2 failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d $O/p3 -o run -- scripts/micro/bin/chain_bench 1501 > $O/p3.log 2>&1 || { echo "p3 failed"; exit 1; }
