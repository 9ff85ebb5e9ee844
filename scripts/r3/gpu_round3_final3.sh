# Round-3 last tree: every GPU test, smoke(), the driver's bench form (K = 20, W = 5).  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3f3
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 600 python -u -m pytest -q --tb=short -m gpu --timeout 300 --timeout-method thread tests > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; check $out/smoke.log; tail -2 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_k20.json 2> $out/bench_k20.err; rc=$?; check $out/bench_k20.err
python3 -c "import json; d=json.loads(open('$out/bench_k20.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k: v for k, v in d['nmpc'].items() if 'ms' in k})"
exit $rc
