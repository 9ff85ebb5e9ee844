#!/bin/bash
# Round 6: the pivot-block kernel (k_chain_elim) before / after the 32-bit key and owner-scaled pivot row — the
# micro-benchmark alternated on one box, VALU counters of both, the chain parity tests.  usage: bash scripts/gpu_chain_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
B=scripts/micro/bin
for r in 1 2; do
  timeout -k 10 60 $B/chain_bench_r5 > $O/micro_r5_$r.txt 2>&1 || exit 1
  timeout -k 10 60 $B/chain_bench > $O/micro_new_$r.txt 2>&1 || exit 1
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $R/$O/pmc_r5 -o run -- $R/$B/chain_bench_r5 > $R/$O/pmc_r5.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $R/$O/pmc_new -o run -- $R/$B/chain_bench > $R/$O/pmc_new.log 2>&1 || exit 1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_chain_kkt.py -x -q --timeout 200 --timeout-method thread > $O/test_chain.log 2>&1
