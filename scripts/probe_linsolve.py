"""Probe torch.linalg.solve on the GPU for KKT-sized systems (batch 1 vs >1, default vs magma backend)."""
import sys
import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 502
for lib in ("default", "magma"):
    if lib != "default":
        torch.backends.cuda.preferred_linalg_library(lib)
    for B in (1, 2, 4, 256):
        K = torch.randn(B, n, n, dtype=torch.float64, device="cuda") + n * torch.eye(n, dtype=torch.float64, device="cuda")
        r = torch.randn(B, n, 1, dtype=torch.float64, device="cuda")
        try:
            x = torch.linalg.solve(K, r)
            torch.cuda.synchronize()
            print(lib, B, "ok", float((K @ x - r).abs().max()), flush=True)
        except RuntimeError as e:
            print(lib, B, "FAIL", str(e).splitlines()[0], flush=True)
