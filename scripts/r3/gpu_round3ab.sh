# Consistency of the headline kernel's duration: the bench's own HIP-event figure and the rocprofv3 kernel trace of the
# same process (K = 100 timed launches after the settle and W = 10 warmup launches).
set -o pipefail
out=gpurun_out/r3ab
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-solve --no-msk > $out/bench.json 2> $out/trace.err || { echo "trace failed"; tail -3 $out/trace.err; exit 1; }
python3 - <<'PY'
import csv, glob, json
out = "gpurun_out/r3ab"
d = json.loads(open(f"{out}/bench.json").read().strip().splitlines()[-1])
rows = list(csv.DictReader(open(glob.glob(f"{out}/trace/**/*kernel_trace.csv", recursive=True)[0])))
ks = [r for r in rows if "k_shooting<0, 1, 2, 1, 2>" in r["Kernel_Name"]]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ks]
start = [int(r["Start_Timestamp"]) for r in ks]
last = dur[-100:]
span = (int(ks[-1]["End_Timestamp"]) - int(ks[-100]["Start_Timestamp"])) / 1e6 / 100
res = {"bench_kernel_ms_events": d["roofline"]["kernel_ms"], "bench_ms_per_step": d["ms_per_step"],
       "trace_launches": len(ks), "trace_avg_ms_last100": sum(last) / 100, "trace_span_ms_per_launch_last100": span,
       "trace_avg_ms_all": sum(dur) / len(dur)}
print(json.dumps(res))
json.dump(res, open(f"{out}/consistency.json", "w"), indent=1)
PY
