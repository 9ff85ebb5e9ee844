#!/bin/bash
# cfg-5 g + J_g counters (B = 65,536): one rocprofv3 --pmc pass per counter group over scripts/msk_probe.py, then
# scripts/summarize_msk_pmc.py -> <out>/msk_pmc.json.  usage: bash scripts/gpu_msk_pmc.sh <tag>
set -o pipefail
out=gpurun_out/${1:-msk_pmc}
mkdir -p $out
export TMPDIR=/tmp
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$n -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $out/pmc_$n.log; exit 1; }
done
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 10 > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 scripts/summarize_msk_pmc.py $out $out/msk_pmc.json
