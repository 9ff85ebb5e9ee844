# Launch-shape sweep of the headline kernel after the fused Euler step: instances per lane (CFX_NI) x intervals per
# thread (CFX_KPT), headline section only, two passes over the grid on one box.
set -o pipefail
out=gpurun_out/ni_kpt
mkdir -p $out
for rep in 1 2; do
  for ni in 1 2 4; do
    for kpt in 2 4 5 10; do
      CFX_NI=$ni CFX_KPT=$kpt timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --cpu-seconds 0 --no-solve --no-msk --nmpc-horizons 0 > $out/ni${ni}_k${kpt}_r${rep}.json 2> $out/ni${ni}_k${kpt}_r${rep}.err || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'])" $out/ni${ni}_k${kpt}_r${rep}.json "ni=$ni kpt=$kpt rep=$rep" | tee -a $out/sweep.txt
    done
  done
done
