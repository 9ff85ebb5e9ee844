# Round 5: chain micro-benchmark; warm start without range scaling (Ipopt's convention); traced force solve.
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 60 scripts/micro/bin/chain_bench 1501 > $out/chain_bench.txt 2>&1 || { echo "bench failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start stored --range-scaling 0 --max-iter 1000 --wall 150 --out $out/warm.jsonl > $out/warm_norange.log 2>&1 || { echo "warm failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives fatigue --start stored --multipliers none --mu-init 1e-9 --range-scaling 0 --max-iter 1000 --wall 150 --out $out/warm.jsonl > $out/cold_norange.log 2>&1 || { echo "cold failed"; exit 1; }
CFX_IPM_TRACE=1 timeout -k 10 200 python3 -u scripts/reaching_warmstart.py --objectives force --start reference --max-iter 1500 --wall 100 --out $out/ref.jsonl > $out/ref_force_trace.log 2>&1 || { echo "ref failed"; exit 1; }
