# In-kernel counter publish at batch 1: native IPM GPU tests, then an A/B of the batch-1 solve wall-clock.
set -o pipefail
out=gpurun_out/ipm_pub
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ipm_native.py > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  CFX_IPM_PUB=launch timeout -k 10 200 python -u scripts/ipm_pub_probe.py >> $out/ab.jsonl 2>> $out/ab.err || exit $?
  timeout -k 10 200 python -u scripts/ipm_pub_probe.py >> $out/ab.jsonl 2>> $out/ab.err || exit $?
done
cat $out/ab.jsonl
