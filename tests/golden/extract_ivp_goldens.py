"""Extract the IVP golden vectors of the reference's own test suite into a data fixture.

Reads ``/root/reference/tests/shard1/test_ivp.py`` AS TEXT (no import, nothing executed), pulls every
``np.array([...])`` literal passed to ``assert_almost_equal`` in file order, and writes them, labelled
with the case they belong to, to ``ivp_goldens.json``.  Only the numbers travel; run once in the build
container (the reference is not present on the GPU box).
"""

import ast
import json
import pathlib

SRC = pathlib.Path("/root/reference/tests/shard1/test_ivp.py")
OUT = pathlib.Path(__file__).with_name("ivp_goldens.json")

# Order of the array literals in test_ivp.py (lines 28-44, 65-89, 107-124, 141-169).
LABELS = [
    ("ding2003_with_fatigue", "single", None, "test_ivp.py:28-35"),
    ("ding2003", "single", None, "test_ivp.py:37-44"),
    ("ding2007_with_fatigue", "single", None, "test_ivp.py:65-76"),
    ("ding2007", "single", None, "test_ivp.py:78-89"),
    ("hmed2018_with_fatigue", "single", None, "test_ivp.py:107-114"),
    ("hmed2018", "single", None, "test_ivp.py:116-124"),
    ("ding2003_with_fatigue", "single", None, "test_ivp.py:141-148"),
    ("ding2003_with_fatigue", "doublet", [150, 180], "test_ivp.py:150-158"),
    ("ding2003_with_fatigue", "triplet", [350, 380], "test_ivp.py:160-169"),
]


def main():
    tree = ast.parse(SRC.read_text())
    arrays = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "array" and node.args:
            if isinstance(node.args[0], ast.List) and len(node.args[0].elts) >= 30:
                arrays.append((node.lineno, [ast.literal_eval(e) for e in node.args[0].elts]))
    arrays.sort()
    assert len(arrays) == len(LABELS), len(arrays)
    cases = []
    for (lineno, values), (model, mode, sl, cite) in zip(arrays, LABELS):
        cases.append(dict(model=model, pulse_mode=mode, slice=sl, source=f"{cite} (line {lineno})",
                          stim_time=[0, 0.1, 0.2], final_time=0.3, sum_stim_truncation=3,
                          ode_solver="RK4", n_integration_steps=10,
                          pulse_width=[0.0003, 0.0004, 0.0005] if model.startswith("ding2007") else None,
                          pulse_intensity=[50, 60, 70] if model.startswith("hmed2018") else None,
                          F=values))
    OUT.write_text(json.dumps({"source": str(SRC), "cases": cases}, indent=1))
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
