#!/bin/bash
# Round 5: MSK stage coefficients split by derivative direction — A/B timing against the one-thread-per-stage kernel
# and the 1-wave build, bit comparison of g / J_g, then the MSK GPU tests.
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
T="timeout -k 10"
CFX_MSK_STAGE=split $T 240 python -u scripts/msk_probe.py --batch 4096 65536 --dump $O/split.npz > $O/probe_split.jsonl 2> $O/probe_split.err &&
CFX_MSK_STAGE=par $T 240 python -u scripts/msk_probe.py --batch 4096 65536 --dump $O/par.npz > $O/probe_par.jsonl 2> $O/probe_par.err &&
CFX_LIB=/root/repo/build_w1/libcfx_w1.so $T 240 python -u scripts/msk_probe.py --batch 4096 65536 > $O/probe_w1.jsonl 2> $O/probe_w1.err &&
$T 240 python -u scripts/msk_probe.py --batch 65536 > $O/probe_split2.jsonl 2>> $O/probe_split.err &&
python - > $O/ab.txt <<'PY'
import numpy as np
a=np.load("gpurun_out/r5k/split.npz"); b=np.load("gpurun_out/r5k/par.npz")
for k in "gj":
    d=np.abs(a[k]-b[k]); print(k, "max abs diff", d.max(), "identical", np.array_equal(a[k], b[k]), "max", np.abs(b[k]).max())
PY
cat $O/ab.txt && $T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msk or Msk" > $O/tests.log 2>&1
