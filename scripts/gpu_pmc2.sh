set -o pipefail
tag=$1; shift
cd /root/repo
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/fp64_rate > gpurun_out/$tag/fp64_rate.txt 2>&1; cat gpurun_out/$tag/fp64_rate.txt
for pass in "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" "SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_LEVEL_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/$tag/pmc_$n -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 > gpurun_out/$tag/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
echo done
