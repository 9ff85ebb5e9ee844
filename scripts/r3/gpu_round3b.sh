# round 3: stage-kernel occupancy A/B (default vs amdgpu_waves_per_eu(2, 2) build), kernel traces of both, and the
# interval-sharded GPU tests.
set -o pipefail
out=gpurun_out/r3b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/msk_probe.py --batch 65536 --reps 30 --libs cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_w2.so cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_w2.so > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -5 $out/ab.err; exit 1; }
CFX_LIB=cocofest_amd/variants/libcfx_w2.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_w2 -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 5 > $out/trace_w2.log 2>&1 || { echo "trace w2 failed"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_dist.log 2>&1 || echo "dist tests failed"
cat $out/ab.jsonl
find $out/trace_w2 -name "*kernel_stats.csv" -exec head -6 {} \;
tail -3 $out/pytest_dist.log
