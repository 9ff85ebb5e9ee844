"""Shooting-kernel shape sweep for the bench workload (cfg 2, B = 2^20, 64-instance tiles): instances per lane
(CFX_NI) x intervals per thread (CFX_KPT), interleaved rounds in one process."""
import json
import os
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ocp = bench.build_problem()
    B = 1 << 20
    handles = {}
    for ifast in (0, 1):
        for ni in (1, 2):
            for kpt in (1, 2, 5, 20):
                os.environ["CFX_NI"], os.environ["CFX_KPT"], os.environ["CFX_IFAST"] = str(ni), str(kpt), str(ifast)
                handles[(ni, kpt, ifast)] = ocp.nlp(batch=B, layout="tiled64")
    for k in ("CFX_NI", "CFX_KPT", "CFX_IFAST"):
        os.environ.pop(k)
    h0 = handles[(2, 20, 0)]
    v = bench.to_tiled(bench.synthetic_soa(ocp, B, 1, "cuda:0"))
    g = torch.empty((B // 64, h0.ng, 64), dtype=torch.float64, device="cuda")
    j = torch.empty((B // 64, h0.nnz_jac, 64), dtype=torch.float64, device="cuda")
    for _ in range(300):  # settle
        h0.eval_all(v, g=g, jac=j)
    torch.cuda.synchronize()
    res = {k: [] for k in handles}
    for _ in range(5):
        for k, h in handles.items():
            for _ in range(3):
                h.eval_all(v, g=g, jac=j)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(40):
                h.eval_all(v, g=g, jac=j)
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 40)
    nb = 8 * (h0.nv + h0.ng + h0.nnz_jac) * B
    out = {f"ni{k[0]}_kpt{k[1]}_if{k[2]}": {"median_ms": sorted(x)[2], "min_ms": min(x), "TBps": nb / (sorted(x)[2] * 1e-3) / 1e12}
           for k, x in res.items()}
    for k, r in sorted(out.items(), key=lambda kv: kv[1]["median_ms"]):
        print(f"{k:14s} {r['median_ms']:.4f} ms  {r['TBps']:.2f} TB/s", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
