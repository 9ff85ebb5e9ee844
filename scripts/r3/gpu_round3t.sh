# Schur complement LU in registers vs LDS: the bitwise test, batch-1 solve wall-clock alternating (cfg 3, cfg 2), and a
# kernel trace of the cfg-2 batch-1 solve.  Stops at the first failure.
set -o pipefail
out=gpurun_out/r3t
mkdir -p $out
export TMPDIR=/tmp
check() { if grep -q "HSA_STATUS_ERROR" $1; then echo "GPU fault in $1"; exit 3; fi; }
timeout -k 10 300 python -u -m pytest -q --tb=short -m gpu --timeout 250 --timeout-method thread tests/test_ipm_native.py -k "schur or nmpc or cfg3" > $out/pytest.log 2>&1; rc=$?; check $out/pytest.log; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    for p in cfg3 cfg2; do
      CFX_IPM_SCHUR_REG=$v timeout -k 10 120 python3 scripts/r3/profile_native_b1.py $p 15 > $out/b1_${p}_reg${v}_$i.json 2>> $out/b1.err || { echo "b1 failed"; tail -3 $out/b1.err; exit 1; }
      echo "reg=$v $(cut -c1-160 $out/b1_${p}_reg${v}_$i.json)"
    done
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg2_b1 -o run -- python3 scripts/r3/profile_native_b1.py cfg2 10 > $out/cfg2_b1.log 2>&1 || { echo "cfg2 trace failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg3_b1 -o run -- python3 scripts/r3/profile_native_b1.py cfg3 10 > $out/cfg3_b1.log 2>&1 || { echo "cfg3 trace failed"; exit 1; }
echo done
