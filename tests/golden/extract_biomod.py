"""Extract the reference's arm26 musculoskeletal models into data fixtures.

Reads ``/root/reference/examples/msk_models/*.bioMod`` AS TEXT with the oracle's bioMod parser
(``oracle.fes_msk.parse_biomod``) and writes the parsed numbers — segment transforms, dofs, masses, centres of
mass, inertias, q ranges, gravity, muscle paths and characteristics — to ``biomod_<name>.json``.  The bioMod
files are model data the reference's own MSK tests load (tests/shard2/test_fes_dynamics.py:20-21); only the
parsed numbers travel (the reference is not present on the GPU box).  Run once in the build container.
"""

import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import fes_msk  # noqa: E402

SRC = pathlib.Path("/root/reference/examples/msk_models")
MODELS = ("arm26_biceps_triceps", "arm26", "arm26_biceps", "arm26_biceps_1dof")


def main():
    for name in MODELS:
        bm = fes_msk.parse_biomod((SRC / f"{name}.bioMod").read_text())
        bm.pop("groups", None)
        out = pathlib.Path(__file__).with_name(f"biomod_{name}.json")
        out.write_text(json.dumps(bm, indent=1) + "\n")
        print(out.name, len(bm["segments"]), "segments", len(bm["muscles"]), "muscles")


if __name__ == "__main__":
    main()
