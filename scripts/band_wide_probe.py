"""Band LU placements on the wide KKT bands of the MSK interior point (kl = ku = 42): factor (+ one solve) time per
call for the register kernel (3) and the LDS-resident / windowed kernels (1 / 0), via CFX_BAND_PLACEMENT."""
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    from cocofest_amd import _cfx
    from scripts.band_probe import system

    for (B, n, kl, ku) in [(3, 106, 42, 42), (1, 298, 42, 42), (64, 298, 42, 42), (1, 500, 6, 6)]:
        rng = np.random.default_rng(0)
        ab0 = torch.tensor(system(rng, B, n, kl, ku), device="cuda")
        x0 = torch.tensor(rng.standard_normal((B, 1, n)), device="cuda")
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        row = {"B": B, "n": n, "kl": kl}
        ref = None
        for pl in ("3", "1", "0"):
            os.environ["CFX_BAND_PLACEMENT"] = pl
            ts = []
            for _ in range(8):
                ab, x = ab0.clone(), x0.clone()
                torch.cuda.synchronize()
                t = time.perf_counter()
                _cfx.band_lu(ab, ipiv, info, kl, ku)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
                _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
            row["p" + pl + "_us"] = round(1e6 * float(np.median(ts[2:])), 1)
            if ref is None:
                ref = x.clone()
            row["p" + pl + "_diff"] = float((x - ref).abs().max())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
