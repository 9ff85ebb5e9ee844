"""Generate formula-level golden vectors from the reference's own code (build container only).

The reference (Ipuch/cocofest) is pure Python whose numerics sit on CasADi/bioptim, which are not
installed (ordinary ModuleNotFoundError, not a permission denial).  Its
formula-level functions (ODE right-hand sides, stimulation table, n_shooting, minimal intensity,
Fourier fit) only use ``casadi.exp/tanh/vertcat`` on numbers, so they run unchanged on numeric
inputs when ``casadi`` resolves to a small numpy-backed module and ``bioptim`` to inert placeholder
classes.  Both are generated into a temporary directory by this script (nothing of them is kept), the
``cocofest`` package ``__init__`` is bypassed (it forces a TkAgg matplotlib backend), and the model
modules are imported from ``/root/reference``.

Only the resulting numbers are committed (``ref_formulas.json``); the reference never travels to the
GPU box.  Transcription (bioptim) and Ipopt are NOT covered by this oracle.
"""

import ast
import importlib
import json
import pathlib
import sys
import tempfile
import types

import numpy as np

REF = pathlib.Path("/root/reference")
OUT = pathlib.Path(__file__).with_name("ref_formulas.json")

CASADI_SHIM = '''
import numpy as _np
exp = _np.exp; tanh = _np.tanh; log = _np.log; sqrt = _np.sqrt; cos = _np.cos; sin = _np.sin
def vertcat(*a):
    return _np.concatenate([_np.atleast_1d(_np.asarray(x, dtype=float)).ravel() for x in a])
def horzcat(*a):
    return _np.column_stack(a)
def sum1(x):
    return _np.sum(x, axis=0)
class _Sym:
    sym = None
    def __init__(self, *a, **k): pass
MX = SX = DM = Function = _Sym
'''

BIOPTIM_SHIM = '''
class _Meta(type):
    def __getattr__(cls, name):
        return _Meta(name, (_Inert,), {})
    def __or__(cls, other):
        return cls
    def __ror__(cls, other):
        return cls
class _Inert(metaclass=_Meta):
    def __init__(self, *a, **k): pass
    def __call__(self, *a, **k): return _Inert()
    def __getattr__(self, name): return _Inert()
def __getattr__(name):
    return _Meta(name, (_Inert,), {})
'''


def _install_shims():
    tmp = pathlib.Path(tempfile.mkdtemp(prefix="cfx_golden_"))
    (tmp / "casadi.py").write_text(CASADI_SHIM)
    (tmp / "bioptim.py").write_text(BIOPTIM_SHIM)
    (tmp / "biorbd.py").write_text("")
    (tmp / "pyorerun.py").write_text("")
    sys.path.insert(0, str(tmp))
    pkg = types.ModuleType("cocofest")
    pkg.__path__ = [str(REF / "cocofest")]
    sys.modules["cocofest"] = pkg


def _mod(name):
    return importlib.import_module(f"cocofest.{name}")


MODEL_CLASSES = {
    "ding2003": ("models.ding2003", "DingModelFrequency"),
    "ding2003_with_fatigue": ("models.ding2003_with_fatigue", "DingModelFrequencyWithFatigue"),
    "ding2007": ("models.ding2007", "DingModelPulseWidthFrequency"),
    "ding2007_with_fatigue": ("models.ding2007_with_fatigue", "DingModelPulseWidthFrequencyWithFatigue"),
    "hmed2018": ("models.hmed2018", "DingModelPulseIntensityFrequency"),
    "hmed2018_with_fatigue": ("models.hmed2018_with_fatigue", "DingModelPulseIntensityFrequencyWithFatigue"),
}


def _make(name, **kw):
    mod, cls = MODEL_CLASSES[name]
    return getattr(_mod(mod), cls)(**kw)


def rhs_cases(rng):
    cases = []
    for name in MODEL_CLASSES:
        T = 10
        model = _make(name, sum_stim_truncation=T)
        fatigue = name.endswith("with_fatigue")
        for _ in range(8):
            n_real = int(rng.integers(1, T + 1))
            real = np.sort(rng.uniform(0.0, 0.9, n_real))
            row = np.concatenate([np.full(T - n_real, -10000000.0), real])
            t = float(real[-1] + rng.uniform(0.0, 0.05))
            x = [float(rng.uniform(0, 1.5)), float(rng.uniform(0, 300))]
            kw = dict(cn=x[0], f=x[1], t=t, t_stim_prev=row.copy())
            if fatigue:
                a0 = model.a_scale if name.startswith("ding2007") else model.a_rest
                x += [float(a0 * rng.uniform(0.5, 1.0)), float(rng.uniform(0.04, 0.1)), float(rng.uniform(0.1, 0.3))]
                kw.update(a=x[2], tau1=x[3], km=x[4])
            u = []
            if name.startswith("ding2007"):
                u = [float(rng.uniform(model.pd0, 6e-4))]
                kw["pulse_width"] = u[0]
            if name.startswith("hmed2018"):
                u = [float(v) for v in rng.uniform(17.1, 130.0, T)]
                kw["pulse_intensity"] = list(u)
            dx = np.asarray(model.system_dynamics(**kw), dtype=float).ravel()
            cases.append(dict(model=name, t=t, row=row.tolist(), x=x, u=u, dxdt=dx.tolist()))
    return cases


def table_cases():
    fes_ocp = _mod("optimization.fes_ocp")
    cfgs = [
        ("ding2003", [0, 0.1, 0.2], 0.3, 3, None),
        ("ding2003", [round(0.1 * i, 1) for i in range(10)], 1.0, 20, None),
        ("ding2003_with_fatigue", [round(0.1 * i, 1) for i in range(10)], 1.0, 20, None),
        ("ding2007", [float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)], 1.0, 10, None),
        ("ding2007_with_fatigue", [float(v) for v in np.linspace(0, 0.2, 11)[:-1]], 0.2, 10,
         {"time": [-0.15, -0.10, -0.05], "pulse_width": [0.0005, 0.0005, 0.0005]}),
        ("hmed2018", [round(0.1 * i, 1) for i in range(10)], 1.0, 10, None),
        ("hmed2018_with_fatigue", [float(v) for v in np.linspace(0, 1, 34)[:-1]], 1.0, 20, None),
    ]
    out = []
    for name, stim, tf, T, prev in cfgs:
        model = _make(name, stim_time=list(stim), sum_stim_truncation=T,
                      previous_stim=json.loads(json.dumps(prev)) if prev else None)
        n = fes_ocp.OcpFes.prepare_n_shooting(model.stim_time, tf)
        table, stim_idx = model.get_numerical_data_time_series(n, tf)
        rows = np.transpose(table["stim_time"], (2, 1, 0))[:, 0, :]
        out.append(dict(model=name, stim_time=list(stim), final_time=tf, truncation=T,
                        previous_stim=(prev or {}).get("time"), n_shooting=n, rows=rows.tolist(),
                        stim_idx_at_node=[list(map(int, s)) for s in stim_idx]))
    return out


def misc_cases():
    hmed = _make("hmed2018")
    fourier = _mod("fourier_approx").FourierSeries()
    src = (REF / "tests/shard1/test_ocp_build.py").read_text()
    tree = ast.parse(src)
    arrays = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Name):
            nm = node.targets[0].id
            if nm in ("force", "time") and isinstance(node.value, ast.Call):
                arrays[nm] = np.array(ast.literal_eval(node.value.args[0]), dtype=float)
    force, time = arrays["force"], arrays["time"]
    init_force = force - force[0]
    ab = fourier.compute_real_fourier_coeffs(time, init_force, 50)
    targets = {}
    for n in (10, 20, 100):
        targets[str(n)] = fourier.fit_func_by_fourier_series_with_real_coeffs(np.linspace(0, 1, n + 1), ab).tolist()
    d03 = _make("ding2003_with_fatigue")
    return dict(
        min_pulse_intensity=float(hmed.min_pulse_intensity()),
        force_tracking=dict(source="tests/shard1/test_ocp_build.py:12-220 (force - force[0], time)",
                            time=time.tolist(), force=init_force.tolist(), targets=targets),
        kat=dict(
            exp_time=float(d03.exp_time_fun(t=0.1, t_stim_i=0.09)),
            ri=float(d03.ri_fun(r0=1.05, time_between_stim=0.1)),
            cn_sum=float(d03.cn_sum_fun(r0=1.05, t=0.11, t_stim_prev=np.array([0, 0.1]), lambda_i=[1, 1])),
            f_dot=float(d03.f_dot_fun(cn=5, f=100, a=3009, tau1=0.050957, km=0.103)),
            a_dot=float(d03.a_dot_fun(a=5, f=100)),
            lambda_30=float(hmed.lambda_i_calculation(pulse_intensity=30)),
            a_calc=float(_make("ding2007").a_calculation(a_scale=4920, pulse_width=0.0002)),
        ),
    )


def main():
    _install_shims()
    rng = np.random.default_rng(20250224)
    data = dict(
        generator="tests/golden/make_golden.py (reference formula code executed with a numpy casadi shim)",
        reference="/root/reference @ 2025-02-24",
        rhs=rhs_cases(rng),
        tables=table_cases(),
        misc=misc_cases(),
    )
    OUT.write_text(json.dumps(data))
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes): {len(data['rhs'])} rhs cases, {len(data['tables'])} tables")


if __name__ == "__main__":
    main()
