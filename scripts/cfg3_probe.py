"""cfg-3 g + J_g launch time (bench.cfg3_section, no CPU sample) for the launch-shape overrides in the environment
(CFX_NI, CFX_KPT, CFX_IFAST); prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
r = bench.cfg3_section(0, 0.0, steps=100, B=B)
print(json.dumps({k: os.environ.get(k) for k in ("CFX_NI", "CFX_KPT", "CFX_IFAST")} |
                 {"B": B, "ms": r["ms_per_launch"], "GBps": r["achieved_GBps"]}), flush=True)
