#!/bin/bash
# cfg-5 512-start multistart (+-10 %) under the Ipopt profile with Ipopt's mu_max option set (the adaptive update's cap
# on the barrier parameter; default: mu_max_fact 1000 x the initial average complementarity)
set -o pipefail
O=gpurun_out/${1:-resto_mumax}
mkdir -p $O
export PYTHONUNBUFFERED=1
for mm in 100 1 0.1; do
  timeout -k 10 240 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --profile ipopt --opt mu_max=$mm --label mu_max=$mm --jsonl $O/b512.jsonl > /dev/null 2> $O/b512_$mm.err || exit 1
done
timeout -k 10 300 python -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --profile ipopt --max-iter 3000 --label max_iter=3000 --jsonl $O/b512.jsonl > /dev/null 2> $O/b512_it3000.err || exit 1
python3 -c "
import json
for l in open('$O/b512.jsonl'):
    r = json.loads(l); print(r['label'], r['converged'], r['status'], r['wall_s'], r['f_converged_min'], r['f_converged_max'])
"
