#!/bin/bash
# cfg-5 512-start multistart (+-10 %) under the Ipopt profile with every start's status, then CFX_IPM_TRACE runs of
# the first failing starts moved to instance 0.  usage: scripts/gpu_resto_trace.sh TAG
set -o pipefail
O=gpurun_out/${1:-resto_trace}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --profile ipopt --dump $O/b512.npz > $O/b512.jsonl 2> $O/b512.err || exit 1
cat $O/b512.jsonl
python3 - $O > $O/fails.txt <<'PY'
import sys, numpy as np
d = np.load(sys.argv[1] + "/b512.npz")
st = d["status"]
print(" ".join(str(i) for i in np.flatnonzero(st == -2)[:4]))
PY
echo "failing (Restoration_Failed) starts: $(cat $O/fails.txt)"
for i in $(cat $O/fails.txt); do
  CFX_IPM_TRACE=1 timeout -k 10 240 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --profile ipopt --first $i --dump $O/first$i.npz > $O/first$i.jsonl 2> $O/trace$i.txt || exit 1
  python3 -c "import numpy as np; d = np.load('$O/first$i.npz'); print($i, 'status of instance 0:', d['status'][0], 'iterations', d['iterations'][0])"
done
