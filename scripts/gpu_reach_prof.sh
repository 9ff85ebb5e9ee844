#!/bin/bash
# kernel trace of the reaching task's first 60 iterations (fatigue, reference start) under a solver profile
set -o pipefail
OUT=gpurun_out/${1:-reach_prof}
PROF=${2:-ipopt}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$PROF -o run -- python3 scripts/reaching_warmstart.py --objectives fatigue --start reference --profile $PROF --max-iter 60 > $OUT/trace_$PROF.log 2>&1 || { tail -5 $OUT/trace_$PROF.log; exit 1; }
tail -2 $OUT/trace_$PROF.log
