# Round 5: chain + wide-instance kernels: tests, kernel breakdown, warm-start variants, force objective from the
# reference start.  usage: bash scripts/gpu_r5c.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_chain_kkt.py -x -q --timeout 200 --timeout-method thread > $out/chain_tests.log 2>&1 || { echo "chain tests failed"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o chain -- python3 scripts/chain_probe.py --layouts chain --iters 6 > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
for mu in 1e-9 1e-6 1e-4; do
  CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start stored --mu-init $mu --max-iter 1000 --wall 150 --out $out/warm.jsonl > $out/warm_$mu.log 2>&1 || { echo "warm $mu failed"; exit 1; }
done
timeout -k 10 560 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 5000 --wall 500 --out $out/ref.jsonl > $out/ref_force.log 2>&1 || { echo "ref failed"; exit 1; }
