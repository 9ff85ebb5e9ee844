# kernel durations of the band LU placements on the wide KKT shapes (rocprofv3 kernel trace)
set -o pipefail
out=gpurun_out/band_trace
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/band_wide_probe.py > $out/log 2>&1 || { tail -20 $out/log; exit 1; }
f=$(find $out/trace -name "*kernel_stats.csv" | head -1)
cp $f $out/kernel_stats.csv
cut -d, -f1-4 $f | head -20
