# round 3: the restoration phase (zero multipliers + fresh filter after it, per-instance budget): native vs BatchedIpm
# parity tests, then cfg-5 multistart (64 starts, max_iter 1000) and cfg-3 random starts, phase vs step.
set -o pipefail
out=gpurun_out/r3g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ipm_native.py tests/test_gpu_parity.py -k "ipm or interior" -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_ipm.log 2>&1
rc=$?
tail -8 $out/pytest_ipm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u scripts/r3/resto_probe.py --cfg5-batch 64 --amp 0.1 --max-iter 1000 --cfg3-batch 256 > $out/resto.jsonl 2> $out/resto.err
rc=$?
cat $out/resto.jsonl
tail -3 $out/resto.err
exit $rc
