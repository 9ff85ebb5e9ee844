# Native interior point on config 5: wall-clock, then a rocprofv3 kernel trace.  usage: bash scripts/gpu_msk_native.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/profile_msk_native.py 1 64 > $out/wall.json 2> $out/wall.err || { tail -20 $out/wall.err; exit 1; }
cat $out/wall.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/profile_msk_native.py 1 > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
f=$(find $out/trace -name "*kernel_stats.csv" | head -1)
cp $f $out/kernel_stats.csv
cut -d, -f1-8 $f | head -25
