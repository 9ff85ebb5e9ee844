# Round 5: pattern ceilings (cfg3, msk), batch-1 layouts, named collocation kernels in a trace
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 scripts/micro/bin/shape_bw 262144 100 > $out/shape_bw.jsonl 2>&1 || { echo "shape failed"; exit 1; }
timeout -k 10 120 scripts/micro/bin/colloc_bw 262144 200 > $out/colloc_bw.jsonl 2>&1 || { echo "colloc failed"; exit 1; }
timeout -k 10 300 python3 -u scripts/b1_layout_probe.py --reps 5 --out $out/b1_layouts.jsonl > $out/b1.log 2>&1 || { echo "b1 failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-reaching > $out/bench_trace.log 2>&1 || { echo "bench trace failed"; exit 1; }
