# Round 2 profile of the bench command: kernel trace + stats of the default bench, then one --pmc pass per
# counter group on the headline section.  usage: bash scripts/gpu_profile_r2.sh <tag>
set -o pipefail
tag=$1
cd /root/repo
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 1; }
tail -c 600 $out/trace.log
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$n -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-solve --no-msk --nmpc-horizons 0 > $out/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
python3 scripts/summarize_pmc.py $out $out/summary 1526726656
