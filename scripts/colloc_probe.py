"""Collocation g + J_g launch time (bench.collocation_section) for the grid order in the environment
(CFX_COLLOC_IFAST, a tuning switch measured in profiles/round2/colloc_ab/ and then removed: the probe now times the
shipped order either way); prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

r = bench.collocation_section(0, steps=200)
print(json.dumps({"CFX_COLLOC_IFAST": os.environ.get("CFX_COLLOC_IFAST"), "ms": r["ms_per_launch"],
                  "GBps": r["achieved_GBps"]}), flush=True)
