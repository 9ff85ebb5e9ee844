"""Extract the reference's stored musculoskeletal OCP solution into a numeric fixture.

Source: ``/root/reference/examples/dynamics/reaching_task/result_file/pulse_duration_minimize_muscle_{fatigue,force}.pkl``,
written by the reference's reaching-task example (examples/dynamics/reaching_task/
reaching_task_pulse_duration_optimization.py:80-118; an older revision of it, whose pulse durations were OCP
parameters): a bioptim + Ipopt + biorbd solution of arm26 with six Ding2007-with-fatigue muscles.

The file is never unpickled.  ``pickletools.genops`` only disassembles the opcode stream (it constructs no object and
resolves no global); this script accepts exactly the opcode pattern of a protocol-4 dict of numpy float64 arrays —
``numpy.core.multiarray._reconstruct(numpy.ndarray, (0,), b'b')`` followed by a BUILD state
``(1, shape, dtype('f8'), False, raw_bytes)`` — and reads each array's raw little-endian bytes with numpy.frombuffer.
Any other global, or any other dtype, aborts.  Run once in the build container; only the numbers are committed
(``reaching_pulse_duration_<objective>.npz``), the reference does not travel.
"""

from __future__ import annotations

import pathlib
import pickletools

import numpy as np

SRC = pathlib.Path("/root/reference/examples/dynamics/reaching_task/result_file")
OUT = pathlib.Path(__file__).parent
ALLOWED_GLOBALS = {("numpy.core.multiarray", "_reconstruct"), ("numpy", "ndarray"), ("numpy", "dtype"),
                   ("numpy.core.multiarray", "scalar")}


def extract(path: pathlib.Path) -> dict:
    data = path.read_bytes()
    ops = list(pickletools.genops(data))
    strings = []  # recent unicode strings (keys / module names)
    ints = []  # ints since the last array payload (shape components)
    arrays, scalars = {}, {}
    key_stack = []  # dict keys, most recent last
    qual = None  # the last global's name
    memo = []  # memoised strings (None for anything else), so that a BINGET of a module name is seen as a string
    last = None
    for op, arg, _ in ops:
        name = op.name
        if name == "MEMOIZE":
            memo.append(last if isinstance(last, str) else None)
        elif name in ("BINGET", "LONG_BINGET") and isinstance(memo[arg], str):
            strings.append(memo[arg])
        last = arg if name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE") else (last if name == "MEMOIZE" else None)
        if name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE"):
            strings.append(arg)
            if arg not in {"numpy.core.multiarray", "_reconstruct", "numpy", "ndarray", "dtype", "scalar", "f8", "<",
                           "|"}:
                key_stack.append(arg)
                ints = []
        elif name == "STACK_GLOBAL":
            mod, qual = strings[-2], strings[-1]
            if (mod, qual) not in ALLOWED_GLOBALS:
                raise ValueError(f"{path.name}: global {mod}.{qual} is not a numpy array constructor")
        elif name in ("GLOBAL", "INST", "OBJ", "NEWOBJ", "NEWOBJ_EX", "EXT1", "EXT2", "EXT4", "PERSID", "BINPERSID"):
            raise ValueError(f"{path.name}: opcode {name} outside the numpy-array pattern")
        elif name in ("BININT1", "BININT2", "BININT", "LONG1"):
            ints.append(int(arg))
        elif name in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8") and qual == "scalar":
            scalars.setdefault(key_stack[-1], []).append(float(np.frombuffer(arg, dtype="<f8")[0]))
        elif name in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8") and len(arg) > 1:
            key = key_stack[-1]
            n = len(arg) // 8
            # shape: the ints after the key, past the reconstruct prologue (0,) and the state's version 1 (the first
            # array also carries its dtype's state ints after the shape): the shortest prefix holding n doubles
            dims, prod = [], 1
            for d in ints[2:]:
                if d <= 0 or prod == n:
                    break
                dims.append(d)
                prod *= d
            if prod != n:
                raise ValueError(f"{path.name}: {key}: shape {dims} does not hold {n} doubles")
            arrays[key] = np.frombuffer(arg, dtype="<f8").reshape(dims).copy()
            ints = []
        elif name == "BINFLOAT":
            scalars[key_stack[-1]] = float(arg)
    return {"arrays": arrays, "scalars": scalars, "strings": [s for s in strings if "/" in s]}


def main():
    for objective in ("fatigue", "force"):
        src = SRC / f"pulse_duration_minimize_muscle_{objective}.pkl"
        out = extract(src)
        a = out["arrays"]
        np.savez_compressed(OUT / f"reaching_pulse_duration_{objective}.npz",
                            **{k.replace("/", "_"): v for k, v in a.items()},
                            time_to_optimize=np.array(out["scalars"].get("time_to_optimize", np.nan)))
        print(src.name, {k: v.shape for k, v in a.items()}, out["scalars"], out["strings"])


if __name__ == "__main__":
    main()
