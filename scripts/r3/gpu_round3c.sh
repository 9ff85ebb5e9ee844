# round 3: the whole GPU suite after the fused g + J_g + Hessian launch (cfx_eval_all_h) and its use in the native
# interior point.
set -o pipefail
out=gpurun_out/r3c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
tail -25 $out/pytest_gpu.log
exit $rc
