# Full profile of the bench command: kernel trace + stats, then one --pmc pass per counter group.
# usage: bash scripts/gpu_profile_round.sh <tag>
set -o pipefail
tag=$1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-solve > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$n -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-solve > $out/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
python3 scripts/summarize_pmc.py $out $out/summary 1527775232
