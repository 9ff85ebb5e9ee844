# z-axis canonical MSK frames: every MSK GPU test (incl. joints about x / y against the oracle), then the cfg-5 kernel
# trace and SQ counters (scripts/gpu_pmc_msk_sq.sh).
set -o pipefail
out=gpurun_out/msk_axes
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_msk_gpu.py > $out/pytest.log 2>&1; rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_msk_sq.sh ${1:-msk_axes_sq}
