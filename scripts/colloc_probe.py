"""Collocation g + J_g launch time (bench.collocation_section: cfg 2 by Legendre degree 4, B = 2^18, 64-instance
tiles) at the launch shapes in --shapes (CFX_KPT:CFX_NI:CFX_IFAST triples, '-' = the handle's default) and layouts;
each shape runs in a child process (cfx_create reads the overrides), alternating --rounds times.  One JSON line per run.

Usage (lists separated by ',' or '+'): python scripts/colloc_probe.py [--shapes -:-:-,1:1:0,...] [--layouts tiled64,soa] [--stores nt,plain]
                                      [--rounds 2] [--steps 200]
With --pmc-only: the default shape once on the first of --layouts, 20 launches (the process rocprofv3 --pmc wraps)."""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="-:-:-")
ap.add_argument("--layouts", default="tiled64")
ap.add_argument("--stores", default="nt", help="output store policies: nt (default) and/or plain (CFX_COLLOC_STORE)")
ap.add_argument("--rounds", type=int, default=1)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--child", default=None)
ap.add_argument("--pmc-only", action="store_true")
args = ap.parse_args()


def child(layout, steps):
    import torch

    import bench

    ocp = bench.build_collocation()
    B = bench.COLLOCATION_BATCH
    dev = "cuda:0"
    h = ocp.nlp(batch=B, layout=layout, device=0)
    v = bench.collocation_synthetic(ocp, B, dev)
    if layout == "soa":
        v = v.transpose(1, 2).reshape(B, h.nv).T.contiguous()  # tiles -> SoA (nv, B)
        mk = lambda n: torch.empty((n, B), dtype=torch.float64, device=dev)  # noqa: E731
    else:
        mk = lambda n: torch.empty((B // 64, n, 64), dtype=torch.float64, device=dev)  # noqa: E731
    g, j = mk(h.ng), mk(h.nnz_jac)
    for _ in range(5):
        h.eval_all(v, g=g, jac=j)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        h.eval_all(v, g=g, jac=j)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = 8 * (h.nv + h.ng + h.nnz_jac) * B
    out = {"layout": layout, "shape": h.launch_shape(), "ms": ms, "GBps": nbytes / (ms * 1e-3) / 1e9,
           "frac": nbytes / (ms * 1e-3) / 8e12}
    h.close()
    return out


if args.child:
    print(json.dumps(child(args.child, args.steps)), flush=True)
    sys.exit(0)
if args.pmc_only:  # the bench's layout (SoA), 20 launches
    print(json.dumps(child(re.split(r"[,+]", args.layouts)[0], 20)), flush=True)
    sys.exit(0)
for rnd in range(args.rounds):
    for shape in re.split(r"[,+]", args.shapes):
        kpt, ni, ifast = shape.split(":")
        env = dict(os.environ)
        for k, val in (("CFX_KPT", kpt), ("CFX_NI", ni), ("CFX_IFAST", ifast)):
            env.pop(k, None)
            if val != "-":
                env[k] = val
        for layout, store in [(la, st) for la in re.split(r"[,+]", args.layouts) for st in re.split(r"[,+]", args.stores)]:
            env.pop("CFX_COLLOC_STORE", None)
            if store != "nt":
                env["CFX_COLLOC_STORE"] = store
            r = subprocess.run([sys.executable, __file__, "--child", layout, "--steps", str(args.steps)], env=env,
                               capture_output=True, text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps({"error": r.stderr[-400:]})
            rec = json.loads(line)
            rec.update(round=rnd, request=shape, store=store)
            print(json.dumps(rec), flush=True)
