# PMC passes on the MSK probe (one counter group per rocprofv3 run).  usage: bash scripts/gpu_pmc_msk.sh <tag>
set -o pipefail
tag=$1
cd /root/repo
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$n -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $out/pmc_$n.log; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, statistics, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("<")[0].replace("void cfx::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "msk" in k:
        print(k, {c: round(statistics.mean(v), 1) for c, v in d.items()})
PY
