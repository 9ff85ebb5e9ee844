#!/bin/bash
# cfg 3 batch-1 solve from the reference's guess under both solver profiles: wall-clock, then a rocprofv3 kernel trace
set -o pipefail
OUT=gpurun_out/${1:-b1_prof}
mkdir -p $OUT
export TMPDIR=/tmp
for p in ipopt cfx; do
  timeout -k 10 120 python -u scripts/ipm_profile_probe.py --profile $p --batch 1 --guess --reps 10 > $OUT/wall_$p.txt 2>&1 || exit 1
  cat $OUT/wall_$p.txt
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$p -o run -- python3 scripts/ipm_profile_probe.py --profile $p --batch 1 --guess --reps 10 > $OUT/trace_$p.log 2>&1 || exit 1
done
