#!/bin/bash
# Round 5: MSK g-only evaluations through the value kernel (k_msk_values without stage stores) vs the Dual<0>
# interval kernel (CFX_MSK_G=dual) — timings at batch 1 / 64 / 65,536 (cfg 5) and batch 1 (reaching), then the MSK
# and reference-solution tests.
set -o pipefail
O=gpurun_out/r5jj
mkdir -p $O
T="timeout -k 10"
$T 300 python -u scripts/msk_probe.py --batch 1 64 65536 --reps 20 > $O/cfg5_values.jsonl 2> $O/p1.err || { echo "p1 failed"; exit 1; }
CFX_MSK_G=dual $T 300 python -u scripts/msk_probe.py --batch 1 64 65536 --reps 20 > $O/cfg5_dual.jsonl 2> $O/p2.err || { echo "p2 failed"; exit 1; }
$T 300 python -u scripts/msk_probe.py --reaching --batch 1 --reps 10 > $O/reach_values.jsonl 2> $O/p3.err || { echo "p3 failed"; exit 1; }
CFX_MSK_G=dual $T 300 python -u scripts/msk_probe.py --reaching --batch 1 --reps 10 > $O/reach_dual.jsonl 2> $O/p4.err || { echo "p4 failed"; exit 1; }
$T 900 python -u -m pytest tests/test_msk_gpu.py tests/test_reference_solution.py tests/test_launch_shapes.py -x -q --timeout 300 --timeout-method thread > $O/msk_tests.log 2>&1 || { echo "tests failed"; exit 1; }
