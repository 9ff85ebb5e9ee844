set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 8 > gpurun_out/bench.log 2>&1 && tail -2 gpurun_out/bench.log
