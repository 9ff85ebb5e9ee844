#!/bin/bash
# Round 5: chain solves with a wave per row (coalesced, sums into LDS) against a thread per row; chain tests.
set -o pipefail
O=gpurun_out/r5aa
mkdir -p $O
T="timeout -k 10"
$T 60 scripts/micro/bin/chain_bench_rows0 1501 > $O/rows0.txt 2>&1 &&
$T 60 scripts/micro/bin/chain_bench 1501 > $O/rows1.txt 2>&1 &&
$T 600 python -u -m pytest tests/test_chain_kkt.py tests/test_reaching_parity.py -x -q --timeout 300 --timeout-method thread > $O/chain_tests.log 2>&1
