set -o pipefail
out=gpurun_out/r3h
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_msk_gpu.py -k "restoration_phase or cfg5_interior" -m gpu -v -s --timeout 280 --timeout-method thread > $out/pytest_resto.log 2>&1
rc=$?
grep -E "^phase|^step|PASS|FAIL|iterations" $out/pytest_resto.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u scripts/r3/resto_probe.py --cfg5-batch 64 --amp 0.1 --max-iter 1000 --modes phase --rir 0.5,0.1,0.01 > $out/resto.jsonl 2> $out/resto.err
rc=$?
cat $out/resto.jsonl
exit $rc
