"""Kernel probe: time the cfg2 shooting kernel variants in one process (interleaved rounds) so A/B
differences are not cross-process noise.  Usage: python scripts/kprobe.py [--batch B] [--rounds R]"""

import argparse
import json
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--n-shooting", type=int, default=20)
    a = ap.parse_args()
    import os

    ocp = bench.build_problem()
    B = a.batch
    handles = {}
    for ni in (1, 2, 4):
        os.environ["CFX_NI"] = str(ni)
        handles[ni] = ocp.nlp(batch=B, layout="soa")
        handles[f"t{ni}"] = ocp.nlp(batch=B, layout="tiled64")
    os.environ.pop("CFX_NI")
    h = handles[1]
    v = bench.synthetic_soa(ocp, B, 1, "cuda:0")
    g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
    j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
    vt = v.T.reshape(B // 64, 64, -1).transpose(1, 2).contiguous()
    gt = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
    jt = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
    variants = {}
    for ni, hh in handles.items():
        if isinstance(ni, str):
            variants[f"g+J tiled ni={ni[1:]}"] = (hh, dict(v=vt, g=gt, jac=jt))
            continue
        variants[f"g+J ni={ni}"] = (hh, dict(v=v, g=g, jac=j))
        variants[f"g ni={ni}"] = (hh, dict(v=v, g=g))
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, (h, kw) in variants.items():
            for _ in range(3):
                h.eval_all(**kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                h.eval_all(**kw)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.reps)
    out = {k: {"median_ms": sorted(x)[len(x) // 2], "min_ms": min(x)} for k, x in res.items()}
    out["bytes_per_instance_gJ"] = 8 * (h.nv + h.ng + h.nnz_jac)
    out["batch"] = B
    print(json.dumps(out))


if __name__ == "__main__":
    main()
