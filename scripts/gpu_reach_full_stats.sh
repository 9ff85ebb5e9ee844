#!/bin/bash
# kernel statistics of the whole reaching solve (fatigue, reference start) under a profile; the per-dispatch trace stays
# on the box (/tmp), only the summary comes back.  usage: scripts/gpu_reach_full_stats.sh TAG PROFILE
set -o pipefail
O=gpurun_out/${1:-reach_full}
PROF=${2:-ipopt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp_$PROF -o run -- python3 scripts/reaching_warmstart.py --objectives fatigue --start reference --profile $PROF --max-iter 3000 --wall 200 --out $O/r_$PROF.jsonl > $O/log_$PROF.txt 2>&1 || { tail -5 $O/log_$PROF.txt; exit 1; }
cp $(find /tmp/rp_$PROF -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$PROF.csv
