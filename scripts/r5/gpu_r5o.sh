#!/bin/bash
# Round 5: ablations of the Gauss-Jordan pivot block (micro only; the variants compute garbage on purpose).
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
for X in 0 1 2 3 4; do
  timeout -k 10 60 scripts/micro/bin/chain_bench_x$X 1501 > $O/x$X.txt 2>&1 || exit 1
done
