#!/bin/bash
# Round 6: the reaching-task fatigue solve from the reference start with round 5's chain kernel (a variant build,
# CFX_LIB) and round 6's blocked one, alternated on one box, under the Ipopt profile and the library profile with
# bound_relax_factor 1e-8 (bench.py's two reaching lines).  usage: bash scripts/gpu_reach_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for lib in variants/libcfx_r5chain.so libcfx.so; do
  for prof in ipopt script; do
    CFX_LIB=$GRAFT_REPO_ROOT/cocofest_amd/$lib timeout -k 10 130 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile $prof --max-iter 3000 --wall 110 --out $O/ab.jsonl > $O/${prof}_$(basename $lib .so).txt 2>&1 || exit 1
  done
done
