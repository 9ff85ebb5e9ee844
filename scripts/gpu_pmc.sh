# usage: bash scripts/gpu_pmc.sh <tag>  — kernel probe + PMC passes on the cfg2 bench kernel
set -o pipefail
tag=$1; shift
cd /root/repo
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kprobe.py > gpurun_out/$tag/kprobe.log 2>&1; tail -1 gpurun_out/$tag/kprobe.log
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/$tag/pmc_$n -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 > gpurun_out/$tag/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
echo done
