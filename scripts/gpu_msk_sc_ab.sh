# (The CFX_MSK_SC_BLOCKS switch and the grid-stride kernel were removed after this measurement, profiles/round2/msk_sc_ab/.)
# Grid-stride prefetching k_msk_stagecoef_par: A/B of blocks (512 = ~40 items per thread, 10240 = one item per thread),
# alternating kernel traces of the MSK probe, then the MSK GPU tests.
set -o pipefail
out=gpurun_out/msk_sc_ab
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for nb in 512 10240 256 1024; do
    CFX_MSK_SC_BLOCKS=$nb timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t_${nb}_${rep} -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/t_${nb}_${rep}.log 2>&1 || exit $?
    python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:40], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1])) if 'stagecoef' in r['Name']]" $out/t_${nb}_${rep}/run_kernel_stats.csv "nb=$nb rep=$rep" | tee -a $out/ab.txt
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_msk_gpu.py > $out/pytest.log 2>&1; rc=$?; tail -2 $out/pytest.log; exit $rc
