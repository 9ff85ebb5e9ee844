#!/bin/bash
# Round 5: tiled-register Gauss-Jordan of the stage-chain pivot blocks — micro timing and the chain KKT tests.
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
T="timeout -k 10"
$T 120 scripts/micro/bin/chain_bench 1501 > $O/chain_bench.txt 2>&1 &&
$T 600 python -u -m pytest tests/test_chain_kkt.py -x -q --timeout 300 --timeout-method thread > $O/chain_tests.log 2>&1
