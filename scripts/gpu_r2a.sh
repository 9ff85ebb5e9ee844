# Round 2, first GPU call: full GPU suite, cold-start probe of the headline launch, layout micro.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python scripts/cold_probe.py > gpurun_out/cold_probe.json 2> gpurun_out/cold_probe.err && cat gpurun_out/cold_probe.json &&
timeout -k 10 60 ./scripts/micro/layout_bw > gpurun_out/layout_bw.txt 2>&1 && cat gpurun_out/layout_bw.txt
