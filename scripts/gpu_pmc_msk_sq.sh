# VALU utilisation of the cfg-5 MSK g + J_g kernels: one SQ counter pass over the MSK probe (batch 65,536), with the
# kernel trace of the same probe.  usage: bash scripts/gpu_pmc_msk_sq.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_sq.log 2>&1 || { echo "pmc failed"; tail -5 $out/pmc_sq.log; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, statistics, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void cfx::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "msk" in k:
        print(k, {c: round(statistics.mean(v), 1) for c, v in d.items()})
PY
