# round 3: grouped register band LU — parity tests (every band test), then the placement probe.
set -o pipefail
out=gpurun_out/r3k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "band" -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_band.log 2>&1
rc=$?
tail -25 $out/pytest_band.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/r3/band_group_probe.py > $out/probe.jsonl 2> $out/probe.err
rc=$?
cat $out/probe.jsonl
tail -3 $out/probe.err
exit $rc
