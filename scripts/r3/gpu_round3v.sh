# Restoration robustness against Ipopt's defaults (bound_relax_factor 1e-8, max_iter 3000): cfg-5 64-start multistart.
set -o pipefail
out=gpurun_out/r3v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 scripts/r3/resto_ipopt_defaults.py > $out/resto_defaults.jsonl 2> $out/resto_defaults.err; rc=$?
cat $out/resto_defaults.jsonl; tail -3 $out/resto_defaults.err; exit $rc
