# Run a subset of the GPU tests.  usage: bash scripts/gpu_tests.sh <pytest args...>
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_sub.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_sub.log
exit $rc
