set -o pipefail
out=gpurun_out/r5end_trace
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-solve > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
