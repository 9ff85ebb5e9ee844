# A/B of the XCD-aware block order of the shooting launch (CFX_XCD=0|1), alternating on one box, then the FETCH_SIZE
# pass of the new default.  Each run: the headline section only (no CPU sample, solve, MSK or NMPC sections).
set -o pipefail
out=gpurun_out/xcd_ab
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for x in 0 1; do
    CFX_XCD=$x timeout -k 10 240 python -u bench.py --steps 400 --warmup 20 --cpu-seconds 0 --no-solve --no-msk --nmpc-horizons 0 > $out/x${x}_r${rep}.json 2> $out/x${x}_r${rep}.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['roofline']['kernel_ms'], d['ms_per_step'])" $out/x${x}_r${rep}.json
  done
done
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$pass -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-solve --no-msk --nmpc-horizons 0 > $out/pmc_$pass.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
echo done
