# Round 2: shooting-kernel waitcnt restructure -- parity, cold/steady probe, short bench line.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/cold_probe.py > gpurun_out/cold_probe.json 2> gpurun_out/cold_probe.err && cat gpurun_out/cold_probe.json &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 2 --no-solve --nmpc-horizons 0 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err && cut -c1-1200 gpurun_out/bench_short.json
