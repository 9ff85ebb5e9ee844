"""Single wide bands, batch 1: the panel placement (CFX_BAND_PLACEMENT=5: blocked factorisation, streamed solves)
against the global placement (=2) it replaces — factor (no right-hand side) and solve times per call (HIP events
around each call, median of --reps), and the largest difference between the two placements' solutions.  The
first shape is the KKT band of the 1,500-interval reaching task (scripts/reaching_warmstart.py: n = 119,640,
kl = ku = 108); the global placement is timed there only with --global-big (≈ 1.5 s per factorisation).

Usage (GPU): python scripts/band_panel_probe.py [--reps 5] [--global-big] [--out FILE]"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--global-big", action="store_true")
ap.add_argument("--out", default=None)
args = ap.parse_args()


def band(rng, n, kl, ku):
    """LAPACK band storage (1, n, 2 kl + ku + 1) of a random, diagonally weighted band matrix (fill rows NaN)."""
    import numpy as np

    ldab = 2 * kl + ku + 1
    ab = np.full((1, n, ldab), np.nan)
    ab[0, :, kl:] = rng.standard_normal((n, kl + ku + 1))
    ab[0, :, kl + ku] += 4.0 * (kl + ku)  # the diagonal: pivots mostly on it, as in the interior point's KKT
    for j in range(min(n, ku)):  # above the matrix
        ab[0, j, kl: kl + ku - j] = 0.0
    for j in range(max(0, n - kl), n):  # below it
        ab[0, j, kl + ku + (n - j):] = 0.0
    return ab


def main():
    import numpy as np
    import torch

    from cocofest_amd import _cfx

    rows = []
    for n, kl, ku in [(119640, 108, 108), (20000, 108, 108), (5100, 45, 45), (20000, 200, 200), (50000, 20, 20)]:
        rng = np.random.default_rng(n + kl)
        ab0 = torch.tensor(band(rng, n, kl, ku), device="cuda")
        x0 = torch.tensor(rng.standard_normal((1, 1, n)), device="cuda")
        ipiv = torch.empty((1, n), dtype=torch.int32, device="cuda")
        info = torch.empty((1,), dtype=torch.int32, device="cuda")
        row = {"n": n, "kl": kl, "ku": ku}
        sols = {}
        for pl in ("5", "2"):
            if pl == "2" and n > 50000 and not args.global_big:
                continue
            os.environ["CFX_BAND_PLACEMENT"] = pl
            tf, ts = [], []
            reps = args.reps if pl == "5" or n <= 20000 else 1
            for _ in range(reps):
                ab, x = ab0.clone(), x0.clone()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                torch.cuda.synchronize()
                e[0].record()
                _cfx.band_lu(ab, ipiv, info, kl, ku)
                e[1].record()
                _cfx.band_lu_solve(ab, ipiv, kl, ku, x)
                e[2].record()
                torch.cuda.synchronize()
                tf.append(e[0].elapsed_time(e[1]))
                ts.append(e[1].elapsed_time(e[2]))
            row[f"p{pl}_factor_ms"] = round(float(np.median(tf)), 3)
            row[f"p{pl}_solve_ms"] = round(float(np.median(ts)), 3)
            row[f"p{pl}_info"] = int(info.item())
            sols[pl] = (ab.clone(), x.clone())
        if "2" in sols:
            row["factor_max_diff"] = float((sols["5"][0][:, :, kl:] - sols["2"][0][:, :, kl:]).abs().max())
            row["solution_max_diff"] = float((sols["5"][1] - sols["2"][1]).abs().max())
            row["factor_speedup"] = round(row["p2_factor_ms"] / row["p5_factor_ms"], 1)
            row["solve_speedup"] = round(row["p2_solve_ms"] / row["p5_solve_ms"], 1)
        ldab = 2 * kl + ku + 1
        row["band_MB"] = round(n * ldab * 8 / 1e6, 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del ab0
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "a") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
