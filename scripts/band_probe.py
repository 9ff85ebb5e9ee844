"""Band LU placements side by side on the GPU: time per factor / solve call and agreement of the factors,
for the KKT band shapes of the solver's configurations.  argv: optional 'B,n,kl,ku' tuples."""

import json
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SHAPES = [(1, 500, 6, 6), (1, 1100, 15, 15), (1, 2100, 18, 18), (1, 5100, 45, 45), (1, 410, 101, 101),
          (1, 250, 61, 61), (256, 500, 6, 6), (4096, 500, 6, 6), (1024, 1100, 15, 15)]


def system(rng, B, n, kl, ku):
    ldab = 2 * kl + ku + 1
    ab = np.zeros((B, n, ldab))
    ab[:, :, kl:] = rng.standard_normal((B, n, kl + ku + 1))
    ab[:, :, kl + ku] += 4.0  # a stronger diagonal, some pivoting still
    return ab


def run(shape, placements=("1", "0", "3"), reps=5):
    import torch

    from cocofest_amd import _cfx

    B, n, kl, ku = shape
    rng = np.random.default_rng(0)
    ab0 = torch.tensor(system(rng, B, n, kl, ku), device="cuda")
    rhs0 = torch.tensor(rng.standard_normal((B, 1, n)), device="cuda")
    out, ref = {}, None
    for pl in placements:
        os.environ["CFX_BAND_PLACEMENT"] = pl
        ab = ab0.clone()
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = rhs0.clone()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf, ts = [], []
        for _ in range(reps):
            ab.copy_(ab0)
            x.copy_(rhs0)
            ev[0].record()
            _cfx.band_lu(ab, ipiv, info, kl, ku)
            ev[1].record()
            _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
            ev[2].record()
            torch.cuda.synchronize()
            tf.append(ev[0].elapsed_time(ev[1]))
            ts.append(ev[1].elapsed_time(ev[2]))
        res = (ab[:, :, kl:].cpu().numpy(), ipiv.cpu().numpy(), x.cpu().numpy())
        err = None
        if ref is None:
            ref = res
        else:
            err = {"piv_equal": bool((res[1] == ref[1]).all()),
                   "ab_maxdiff": float(np.max(np.abs(res[0] - ref[0]))),
                   "x_maxrel": float(np.max(np.abs(res[2] - ref[2])) / max(1.0, np.abs(ref[2]).max()))}
        out[pl] = {"factor_ms": round(float(np.median(tf)), 4), "solve_ms": round(float(np.median(ts)), 4), "vs_first": err}
    os.environ.pop("CFX_BAND_PLACEMENT", None)
    return out


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or SHAPES
    res = {}
    for s in shapes:
        res[str(s)] = run(s)
        print(s, res[str(s)], flush=True, file=sys.stderr)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
