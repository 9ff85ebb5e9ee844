# cfg-5 MSK g + J_g kernels: kernel trace + stats and one SQ counter pass over the MSK probe (batch 65,536), plus the
# bench's msk section alone.  usage: bash scripts/r3/gpu_msk_prof.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/msk_probe.py --batch 65536 --reps 20 > $out/probe.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_sq.log 2>&1 || { echo "pmc failed"; tail -5 $out/pmc_sq.log; exit 1; }
python3 scripts/r3/summarize_msk_pmc.py $out > $out/summary.json
cat $out/summary.json
