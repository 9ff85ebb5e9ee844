# Round 5: branch-free Gauss-Jordan; the force objective's curvature-test threshold.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 60 scripts/micro/bin/chain_bench 1501 > $out/chain_bench.txt 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_chain_kkt.py -x -q --timeout 200 --timeout-method thread > $out/chain_tests.log 2>&1 || { echo "chain tests failed"; exit 1; }
for cm in 1e-8 0 -1e-6; do
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --curv-min=$cm --max-iter 4000 --wall 150 --out $out/force.jsonl > $out/force_$cm.log 2>&1 || { echo "force $cm failed"; exit 1; }
done
