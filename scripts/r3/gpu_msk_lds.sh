# cfg-5 MSK kernels: issue / wait breakdown and LDS counters (one SQ pass each), batch 65,536.
set -o pipefail
out=gpurun_out/r3m
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d $out/pmc_wait -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_wait.log 2>&1 || { echo "pmc wait failed"; tail -5 $out/pmc_wait.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_lds -o run -- python3 scripts/msk_probe.py --batch 65536 --reps 3 > $out/pmc_lds.log 2>&1 || { echo "pmc lds failed"; tail -5 $out/pmc_lds.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, statistics, json
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r3m/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void cfx::", "")
        if "msk" in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in acc.items()}
json.dump(out, open("gpurun_out/r3m/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
