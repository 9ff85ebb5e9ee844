# Collocation grid-order A/B (instance blocks fast vs intervals fast), alternating on one box, then the collocation
# GPU parity tests under the intervals-fast order.
set -o pipefail
out=gpurun_out/colloc_ab
mkdir -p $out
for rep in 1 2 3; do
  for x in 0 1; do
    CFX_COLLOC_IFAST=$x timeout -k 10 120 python -u scripts/colloc_probe.py >> $out/ab.jsonl 2>> $out/ab.err || exit $?
  done
done
cat $out/ab.jsonl
CFX_COLLOC_IFAST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "colloc" > $out/pytest.log 2>&1; rc=$?; tail -2 $out/pytest.log; exit $rc
