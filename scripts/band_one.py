"""One band factor + solve of a given shape and placement, for counter collection.
argv: B n kl ku placement [reps]"""

import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    from cocofest_amd import _cfx
    from scripts.band_probe import system

    B, n, kl, ku = (int(v) for v in sys.argv[1:5])
    os.environ["CFX_BAND_PLACEMENT"] = sys.argv[5]
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    rng = np.random.default_rng(0)
    ab0 = torch.tensor(system(rng, B, n, kl, ku), device="cuda")
    x0 = torch.tensor(rng.standard_normal((B, 1, n)), device="cuda")
    ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
    info = torch.empty((B,), dtype=torch.int32, device="cuda")
    for _ in range(reps):
        ab, x = ab0.clone(), x0.clone()
        _cfx.band_lu(ab, ipiv, info, kl, ku)
        _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
    torch.cuda.synchronize()
    print("ok", float(x.abs().max()))


if __name__ == "__main__":
    main()
