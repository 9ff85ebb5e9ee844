#!/bin/bash
# Round 5: chain solve kernels, previous (thread per row) against coalesced row sums; kernel durations from rocprofv3.
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 scripts/micro/bin/chain_bench_old 1501 > $O/old.txt 2>&1 &&
timeout -k 10 60 scripts/micro/bin/chain_bench 1501 > $O/new.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/old -o run -- scripts/micro/bin/chain_bench_old 1501 > /dev/null 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/new -o run -- scripts/micro/bin/chain_bench 1501 > /dev/null 2>&1
