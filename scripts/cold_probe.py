"""Cold-start probe of the headline launch: per-launch HIP-event times of the first launches of a fresh process
(cfg 2, B = 2^20, tiled64, NI = 2), then the bench's K = 20 / W = 5 loop and a K = 200 loop, to separate
clock / power ramp-up from the kernel's steady-state time."""

import json
import pathlib
import sys
import time

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def loop(h, v, g, j, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        h.eval_all(v, g=g, jac=j)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    ocp = bench.build_problem()
    B = 1 << 20
    h = ocp.nlp(batch=B, layout="tiled64")
    v = bench.to_tiled(bench.synthetic_soa(ocp, B, 1234, "cuda:0"))
    g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
    j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(61)]
    ev[0].record()
    for i in range(60):
        h.eval_all(v, g=g, jac=j)
        ev[i + 1].record()
    torch.cuda.synchronize()
    first = [round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(60)]
    out = {"first_60_launches_ms": first}
    time.sleep(2.0)  # idle: let clocks drop again
    loop(h, v, g, j, 5)
    out["after_idle_w5_k20"] = round(loop(h, v, g, j, 20), 4)
    out["then_k200"] = round(loop(h, v, g, j, 200), 4)
    out["then_k20"] = round(loop(h, v, g, j, 20), 4)
    time.sleep(2.0)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 0.25:
        loop(h, v, g, j, 20)
        n += 20
    out["settle_launches"] = n
    loop(h, v, g, j, 5)
    out["after_settle_w5_k20"] = round(loop(h, v, g, j, 20), 4)
    print(json.dumps(out))
    h.close()


if __name__ == "__main__":
    main()
