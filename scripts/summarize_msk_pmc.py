"""Summarize rocprofv3 --pmc passes over scripts/msk_probe.py --batch 65536 (cfg 5 g + J_g: k_msk_values and the
fused k_msk_stage_tangents, or k_msk_stagecoef_par + k_msk_tangents_lds under CFX_MSK_TANGENTS=split) into
profiles/msk_pmc.json, the file bench.py's `msk.roofline` reads.

Per kernel and dispatch (averaged over the dispatches of the batch's g + J_g calls): HBM bytes from FETCH_SIZE and
WRITE_SIZE (separate passes, KiB; FETCH_SIZE doubled on gfx950 as MI355X_MICROARCH.md prescribes), all VALU
wave-instructions (SQ_INSTS_VALU) and the FP64 ones (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64).  Usage:
python scripts/summarize_msk_pmc.py gpurun_out/<dir> [profiles/msk_pmc.json]"""
import csv
import json
import pathlib
import sqlite3
import statistics
import sys

KERNELS = {"k_msk_values": "values", "k_msk_stagecoef_par": "stagecoef", "k_msk_tangents_lds": "tangents",
           "k_msk_stage_tangents": "fused"}
F64 = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"]


def rows(src):
    """(kernel name, dispatch id, counter, value) from rocprofv3's CSV output or its rocpd SQLite database
    (`counters_collection` view; one row per dispatch and counter, summed over the instances of a counter)."""
    for f in pathlib.Path(src).rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            yield row["Kernel_Name"], (str(f), row.get("Dispatch_Id")), row["Counter_Name"], float(row["Counter_Value"])
    for f in pathlib.Path(src).rglob("*.db"):
        con = sqlite3.connect(str(f))
        q = "select kernel_name, dispatch_id, counter_name, sum(value) from counters_collection " \
            "group by dispatch_id, counter_name"
        for name, disp, ctr, val in con.execute(q):
            yield name, (str(f), disp), ctr, float(val)
        con.close()


def collect(src, filt=None):
    vals = {}  # (kernel key, counter) -> [per-dispatch values]
    names = {}
    for name, _, ctr, val in rows(src):
        if filt and filt not in str(_[0]):
            continue
        key = next((k for k in KERNELS if k in name), None)
        if key is None:
            continue
        names[key] = name.split("(")[0]
        vals.setdefault((key, ctr), []).append(val)
    return {k: statistics.mean(v) for k, v in vals.items()}, names


def main(src, dst="profiles/msk_pmc.json"):
    m, names = collect(src, filt="pmc_")
    kernels, step = {}, {"hbm": 0.0, "valu": 0.0, "f64": 0.0}
    for key in KERNELS:
        if key not in names:  # not launched in this run
            continue
        fetch, write = m.get((key, "FETCH_SIZE")), m.get((key, "WRITE_SIZE"))
        hbm = None if fetch is None or write is None else (2 * fetch + write) * 1024.0
        f64 = {c.split("_")[3].lower(): m.get((key, c)) for c in F64}
        f64_sum = sum(v for v in f64.values() if v is not None) if any(v is not None for v in f64.values()) else None
        kernels[names.get(key, key)] = {"hbm_bytes": hbm, "fetch_bytes": None if fetch is None else 2 * fetch * 1024.0,
                                        "write_bytes": None if write is None else write * 1024.0,
                                        "valu_wave_instr": m.get((key, "SQ_INSTS_VALU")),
                                        "f64_wave_instr": f64_sum, "f64_by_kind": f64}
        for k, v in (("hbm", hbm), ("valu", m.get((key, "SQ_INSTS_VALU"))), ("f64", f64_sum)):
            step[k] = None if (v is None or step[k] is None) else step[k] + v
    out = {"source": f"rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ_INSTS_VALU + the four F64 counters) over "
                     f"scripts/msk_probe.py --batch 65536 --reps 3 ({src}); per dispatch of the g + J_g step's kernels",
           "batch": 65536, "hbm_bytes_per_step": step["hbm"], "valu_wave_instr_per_step": step["valu"],
           "f64_wave_instr_per_step": step["f64"], "kernels": kernels}
    pathlib.Path(dst).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
