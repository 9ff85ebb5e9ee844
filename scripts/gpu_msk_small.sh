#!/bin/bash
# fused vs two-kernel MSK g + J_g across batch sizes, and the cfg-5 batch-1 solve
set -o pipefail
OUT=gpurun_out/${1:-msk_small}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 180 python -u scripts/msk_probe.py --batch 1 64 512 2048 8192 16384 > $OUT/fused_$i.jsonl 2> $OUT/fused_$i.err || exit 1
  CFX_MSK_TANGENTS=split timeout -k 10 180 python -u scripts/msk_probe.py --batch 1 64 512 2048 8192 16384 > $OUT/split_$i.jsonl 2> $OUT/split_$i.err || exit 1
done
timeout -k 10 300 python -u scripts/msk_solve_ab.py --reps 3 > $OUT/solve.jsonl 2> $OUT/solve.err || exit 1
python3 - $OUT <<'PY'
import json, sys, glob, collections
out = sys.argv[1]
d = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/*_?.jsonl")):
    mode = f.split("/")[-1].split("_")[0]
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l); d[(r["batch"], mode)].append(round(r["ms_g_jac"], 4))
for k in sorted(d): print(k, d[k])
print(open(out + "/solve.jsonl").read())
PY
