"""Per-kernel means of the MSK SQ counter pass and kernel trace (scripts/r3/gpu_msk_prof.sh) as one JSON object:
VALU wave-instructions per dispatch, average duration (kernel trace), and the issue rate against the measured FP64
FMA peak (profiles/round1/micro_fp64_rate.txt: 5.18e11 wave-instr/s)."""
import collections
import csv
import glob
import json
import statistics
import sys

FMA_PEAK = 5.18e11
out = sys.argv[1]
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void cfx::", "")
        pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = {}
for f in glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0].replace("void cfx::", "")] = float(r["AverageNs"])
res = {}
for k, d in pmc.items():
    if "msk" not in k:
        continue
    valu = statistics.mean(d["SQ_INSTS_VALU"])
    e = {c: statistics.mean(v) for c, v in d.items()}
    if k in dur:
        e["avg_ns"] = dur[k]
        e["valu_wave_instr_per_s"] = valu / (dur[k] * 1e-9)
        e["frac_of_fp64_fma_issue_peak"] = e["valu_wave_instr_per_s"] / FMA_PEAK
    res[k] = e
print(json.dumps(res, indent=1))
