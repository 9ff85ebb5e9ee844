# Shooting kernel at 8 waves per SIMD (amdgpu_waves_per_eu(8): 63 VGPRs instead of 78, occupancy 6 -> 8) vs the default
# build, alternating; then the launch-shape parity tests on the 8-wave build.
set -o pipefail
out=gpurun_out/r3y
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 500 python3 scripts/r3/lib_ab.py cocofest_amd/libcfx.so cocofest_amd/variants/libcfx_wpe8.so 3 > $out/ab.jsonl 2> $out/ab.err || { echo "ab failed"; tail -3 $out/ab.err; exit 1; }
cat $out/ab.jsonl
CFX_LIB=cocofest_amd/variants/libcfx_wpe8.so timeout -k 10 400 python -u -m pytest -q --tb=short -m gpu --timeout 250 --timeout-method thread tests/test_launch_shapes.py -k "not msk" > $out/pytest_wpe8.log 2>&1; rc=$?; check $out/pytest_wpe8.log; tail -3 $out/pytest_wpe8.log; exit $rc
