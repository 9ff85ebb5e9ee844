# rocprofv3 kernel trace of the MSK probe.  usage: bash scripts/gpu_prof_msk.sh <tag>
set -o pipefail
tag=$1
cd /root/repo
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/msk_probe.py --batch 65536 > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
f=$(find $out/trace -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 $f | head -20
