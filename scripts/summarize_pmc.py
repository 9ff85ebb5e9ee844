"""Summarize rocprofv3 outputs of bench.py for the shooting kernel into profiles/<round>/.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes, are in KiB, and on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads
(measured here too: 172 MB reported for 352 MB algorithmic reads), so reads are counted 2 x FETCH_SIZE.
"""

import csv
import json
import pathlib
import statistics
import sys


def per_kernel(path, kernel="k_shooting"):
    vals = {}
    for row in csv.DictReader(open(path)):
        if kernel in row["Kernel_Name"]:
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in vals.items()}


def main(src, dst, algorithmic_bytes):
    src, dst = pathlib.Path(src), pathlib.Path(dst)
    dst.mkdir(parents=True, exist_ok=True)
    out = {}
    for d in sorted(src.glob("pmc_*")):
        f = next(d.rglob("*counter_collection.csv"), None)
        if f:
            out.update(per_kernel(f))
    stats = next(src.rglob("*kernel_stats.csv"), None)
    kern = {}
    if stats:
        # the headline launch: the k_shooting instantiation with the most GPU time (the bench command also runs
        # small k_shooting launches inside its convergence sections)
        best = 0.0
        for row in csv.DictReader(open(stats)):
            if "k_shooting" in row["Name"] and float(row["TotalDurationNs"]) > best:
                best = float(row["TotalDurationNs"])
                kern = {"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                        "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
        (dst / "kernel_stats.csv").write_text(stats.read_text())
    summary = {"kernel": kern, "counters_mean_per_dispatch": out}
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        read_b = 2 * out["FETCH_SIZE"] * 1024
        write_b = out["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = read_b + write_b
        summary["hbm_read_bytes_per_launch"] = read_b
        summary["hbm_write_bytes_per_launch"] = write_b
        summary["algorithmic_bytes_per_launch"] = algorithmic_bytes
        if kern:
            summary["hbm_GBps_at_avg_duration"] = (read_b + write_b) / kern["avg_ns"]
    (dst / "pmc_summary.json").write_text(json.dumps(summary, indent=1))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]))
