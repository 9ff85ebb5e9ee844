"""Batch-1 solves only (cfg 3, cfg 2, cfg 5 RK4 x 5), native solver: for kernel traces of the latency-bound path."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))

import bench  # noqa: E402
from ipm_native_probe import cfg3, run  # noqa: E402

if __name__ == "__main__":
    run("cfg3", cfg3(), 1, which=("native",))
    run("cfg2", bench.build_problem(), 1, which=("native",))
    if len(sys.argv) > 1 and sys.argv[1] == "msk":
        run("cfg5_rk4x5", bench.msk_build(5), 1, max_iter=1000, which=("native",))
