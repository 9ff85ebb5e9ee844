"""Sustained-rate probe: the bench's back-to-back loop (warmup, then K launches) for SoA NI=1 and tiled NI=2,
alternating, several rounds — distinguishes layout effects from clock/thermal state."""

import json
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ocp = bench.build_problem()
    B = 1 << 20
    hs = ocp.nlp(batch=B, layout="soa")
    ht = ocp.nlp(batch=B, layout="tiled64")
    v = bench.synthetic_soa(ocp, B, 1, "cuda:0")
    vt = bench.to_tiled(v)
    g = torch.empty((hs.ng, B), dtype=torch.float64, device="cuda")
    j = torch.empty((hs.nnz_jac, B), dtype=torch.float64, device="cuda")
    gt = torch.empty((B // 64, hs.ng, 64), dtype=torch.float64, device="cuda")
    jt = torch.empty((B // 64, hs.nnz_jac, 64), dtype=torch.float64, device="cuda")
    runs = {"soa": (hs, v, g, j), "tiled": (ht, vt, gt, jt)}
    out = {k: [] for k in runs}
    for _ in range(4):
        for name, (h, vv, gg, jj) in runs.items():
            for _ in range(20):
                h.eval_all(vv, g=gg, jac=jj)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                h.eval_all(vv, g=gg, jac=jj)
            e1.record()
            torch.cuda.synchronize()
            out[name].append(round(e0.elapsed_time(e1) / 200, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
