# Filter reset heuristic: the fatigue-family diagnostics (both solvers, on / off), then the cfg-5 64-start multistart.
set -o pipefail
out=gpurun_out/r3x
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/r3/fr_diag.py > $out/fr_diag.jsonl 2> $out/fr_diag.err || { echo "diag failed"; tail -3 $out/fr_diag.err; exit 1; }
cat $out/fr_diag.jsonl
timeout -k 10 700 python3 scripts/r3/resto_ipopt_defaults.py --filter-reset > $out/resto_fr.jsonl 2> $out/resto_fr.err; rc=$?
cat $out/resto_fr.jsonl; exit $rc
