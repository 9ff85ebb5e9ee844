"""Can libcfx launches (via ctypes, on torch's current stream) be captured in a HIP graph by torch.cuda.graph?"""

import pathlib
import sys
import time

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from scripts.probe_hessian import cfg3  # noqa: E402


def main():
    from cocofest_amd import _cfx

    ocp = cfg3()
    B = 4
    h = ocp.nlp(batch=B, layout="aos")
    v = torch.tensor(ocp.initial_guess_vector(), device="cuda").repeat(B, 1) + 0.1
    g = torch.empty((B, h.ng), dtype=torch.float64, device="cuda")
    j = torch.empty((B, h.nnz_jac), dtype=torch.float64, device="cuda")
    f = torch.empty((B,), dtype=torch.float64, device="cuda")
    gr = torch.empty((B, h.nv), dtype=torch.float64, device="cuda")
    lam = torch.randn((B, h.ng), dtype=torch.float64, device="cuda")
    of = torch.ones((B,), dtype=torch.float64, device="cuda")
    H = torch.empty((B, h.nnz_hess), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):  # warm-up on the capture stream (allocations, lazy init)
            h.eval_all(v, g=g, jac=j, f=f, grad=gr)
            h.eval_h(v, of, lam, H)
            out = (g * 2).sum() + j.abs().sum() + H.sum()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = (g.clone(), j.clone(), H.clone(), out.clone())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        h.eval_all(v, g=g, jac=j, f=f, grad=gr)
        h.eval_h(v, of, lam, H)
        out = (g * 2).sum() + j.abs().sum() + H.sum()
    g.zero_(), j.zero_(), H.zero_()
    graph.replay()
    torch.cuda.synchronize()
    ok = all(torch.equal(a, b) for a, b in zip((g, j, H, out), ref))
    print("graph replay identical:", ok)
    v.add_(0.01)
    graph.replay()
    torch.cuda.synchronize()
    print("responds to input change:", not torch.equal(g, ref[0]))
    t0 = time.perf_counter()
    for _ in range(100):
        graph.replay()
    torch.cuda.synchronize()
    print("replay us", (time.perf_counter() - t0) * 1e4)
    t0 = time.perf_counter()
    for _ in range(100):
        h.eval_all(v, g=g, jac=j, f=f, grad=gr)
        h.eval_h(v, of, lam, H)
        out = (g * 2).sum() + j.abs().sum() + H.sum()
    torch.cuda.synchronize()
    print("eager us", (time.perf_counter() - t0) * 1e4)


if __name__ == "__main__":
    main()
