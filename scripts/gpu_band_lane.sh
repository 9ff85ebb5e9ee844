# Lane-placement band LU: parity tests, then the cfg-3 4096-start solve (lane placement from 1024 instances).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "band_lu" > gpurun_out/band_lane.log 2>&1; rc=$?
grep -q HSA_STATUS_ERROR gpurun_out/band_lane.log && { echo "GPU fault"; exit 3; }
grep -E "PASS|FAIL|Error|error" gpurun_out/band_lane.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --batch 65536 --cpu-seconds 0 --no-msk --nmpc-horizons 0 > gpurun_out/bench_lane.json 2> gpurun_out/bench_lane.err
