# round 3: bench line after the fused callbacks + restoration phase, and kernel traces of the cfg-3 native solves
# (batch 1 and 4,096) for the per-iteration breakdown.
set -o pipefail
out=gpurun_out/r3i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
tail -c 600 $out/bench.json
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg3_b1 -o run -- python3 scripts/profile_cfg3_native.py 10 1 > $out/cfg3_b1.log 2>&1 || { echo "cfg3 b1 trace failed"; exit 1; }
tail -1 $out/cfg3_b1.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg3_b4096 -o run -- python3 scripts/profile_cfg3_native.py 3 4096 > $out/cfg3_b4096.log 2>&1 || { echo "cfg3 b4096 trace failed"; exit 1; }
tail -1 $out/cfg3_b4096.log
