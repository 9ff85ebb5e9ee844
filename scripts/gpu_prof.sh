# usage: bash scripts/gpu_prof.sh <tag> [bench args]
set -o pipefail
tag=$1; shift
cd /root/repo
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/$tag/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/$tag/pytest_gpu.log; tail -3 gpurun_out/$tag/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py "$@" > gpurun_out/$tag/bench.log 2>&1 && tail -1 gpurun_out/$tag/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 "$@" > gpurun_out/$tag/rocprof.log 2>&1; echo "rocprof rc=$?"
find gpurun_out/$tag/prof -name "*stats.csv" | head -3
