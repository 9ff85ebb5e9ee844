# round 3: the restoration phase — native IPM tests, then the cfg-5 multistart and cfg-3 random starts, phase vs step.
set -o pipefail
out=gpurun_out/r3d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ipm_native.py -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_ipm.log 2>&1
rc=$?
tail -15 $out/pytest_ipm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u scripts/r3/resto_probe.py --cfg5-batch 64 --amp 0.1 --cfg3-batch 256 > $out/resto.jsonl 2> $out/resto.err
rc=$?
cat $out/resto.jsonl
tail -5 $out/resto.err
exit $rc
