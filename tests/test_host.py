"""Host-side logic of the product (no GPU needed): library load + exported symbols, stimulation tables,
problem layout, bounds, objectives, validation messages of the reference API."""

import re

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases
from tests.conftest import ROOT


def _declared_symbols():
    text = (ROOT / "include" / "cfx.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(cfx_\w+)\s*\(", text, re.M)))


def test_library_loads_and_exports_every_declared_symbol():
    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    declared = _declared_symbols()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_cfx.SIGNATURES)
    assert lib.cfx_abi_version() == _cfx.ABI_VERSION


def test_create_without_device_fails_loudly():
    from cocofest_amd import CfxError
    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    if lib.cfx_device_count() > 0:
        pytest.skip("a HIP device is visible")
    ocp = cases.product_ocp(**cases.cfg2())
    with pytest.raises(CfxError) as exc:
        ocp.nlp(batch=4)
    assert exc.value.code == _cfx.ENODEV


@pytest.mark.parametrize("field, value, code, msg", [
    ("abi_version", 99, "EINVAL", "ABI version mismatch"),
    ("model", 6, "EINVAL", "unknown model"),
    ("model", -1, "EINVAL", "unknown model"),
    ("scheme", 3, "EUNSUPPORTED", "scheme must be"),
    ("n_steps", 0, "EINVAL", "must be positive"),
    ("n_shooting", 0, "EINVAL", "must be positive"),
    ("batch", 0, "EINVAL", "must be positive"),
    ("final_time", 0.0, "EINVAL", "must be positive"),
    ("truncation", 0, "EUNSUPPORTED", "truncation must be in [1, 32]"),
    ("truncation", 33, "EUNSUPPORTED", "truncation must be in [1, 32]"),
    ("layout", 7, "EINVAL", "unknown layout"),
    ("stim_rows", None, "EINVAL", "stim_rows is NULL"),
    ("n_params", 2, "EINVAL", "intensity parameters need a Hmed2018 model"),
    ("n_objectives", -1, "EINVAL", "n_objectives < 0, or objectives is NULL"),
    ("n_objectives", 2, "EINVAL", "n_objectives < 0, or objectives is NULL"),  # objectives left NULL
    ("n_shooting", 65536, "EUNSUPPORTED", "n_shooting must be <= 65535"),
])
def test_create_rejects_bad_problem_before_touching_the_device(field, value, code, msg):
    """cfx_create validates the problem before any HIP call (cfx_api.hip:411-434), so every rejection is
    reachable without a GPU; the message is reported through cfx_last_error(NULL)."""
    import ctypes as C

    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    rows = np.zeros(3)
    pb = _cfx.Problem()
    pb.abi_version, pb.model, pb.scheme, pb.n_steps = _cfx.ABI_VERSION, 0, 1, 1
    pb.n_shooting, pb.truncation, pb.layout, pb.batch, pb.final_time = 2, 1, _cfx.LAYOUT_SOA, 1, 1.0
    pb.stim_rows = rows.ctypes.data_as(C.POINTER(C.c_double))
    setattr(pb, field, value)
    h = C.c_void_p()
    assert lib.cfx_create(C.byref(pb), C.byref(h)) == getattr(_cfx, code)
    assert not h.value
    assert msg in lib.cfx_last_error(None).decode()


def test_tiled_layout_and_collocation_limits_are_rejected():
    import ctypes as C

    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    rows = np.zeros(3)

    def create(**kw):
        pb = _cfx.Problem()
        pb.abi_version, pb.model, pb.scheme, pb.n_steps = _cfx.ABI_VERSION, 0, 1, 1
        pb.n_shooting, pb.truncation, pb.layout, pb.batch, pb.final_time = 2, 1, _cfx.LAYOUT_SOA, 64, 1.0
        pb.stim_rows = rows.ctypes.data_as(C.POINTER(C.c_double))
        for k, v in kw.items():
            setattr(pb, k, v)
        return lib.cfx_create(C.byref(pb), C.byref(C.c_void_p())), lib.cfx_last_error(None).decode()

    rc, msg = create(layout=_cfx.LAYOUT_TILED64, batch=65)
    assert rc == _cfx.EUNSUPPORTED and "batch % 64 == 0" in msg
    # collocation on 64-instance tiles passes validation (round 4); without a GPU it stops at the device check
    rc, msg = create(layout=_cfx.LAYOUT_TILED64, scheme=16, n_steps=4)  # CFX_COLLOCATION_LEGENDRE
    assert rc == _cfx.ENODEV and "no HIP device" in msg
    rc, msg = create(scheme=17, n_steps=10)  # CFX_COLLOCATION_RADAU, degree above 9
    assert rc == _cfx.EUNSUPPORTED and "degree" in msg
    # NULL arguments: no handle and no problem are plain EINVAL, not a crash
    assert lib.cfx_create(None, C.byref(C.c_void_p())) == _cfx.EINVAL
    assert lib.cfx_get_sizes(None, C.byref(_cfx.Sizes())) == _cfx.EINVAL
    assert lib.cfx_get_launch_shape(None, C.byref(_cfx.LaunchShape())) == _cfx.EINVAL
    assert lib.cfx_set_stream(None, None) == _cfx.EINVAL
    assert lib.cfx_band_lu_solve(4, 1, 1, 1, None, None, 0, None, None) == _cfx.EINVAL
    assert "nrhs" in lib.cfx_last_error(None).decode()


@pytest.mark.parametrize("field, value, code, msg", [
    ("abi_version", 99, "EINVAL", "ABI version mismatch"),
    ("scheme", 16, "EUNSUPPORTED", "scheme must be CFX_RK1, CFX_RK2 or CFX_RK4"),
    ("n_shooting", 0, "EINVAL", "must be positive"),
    ("final_time", -1.0, "EINVAL", "must be positive"),
    ("truncation", 65, "EINVAL", "truncation must be in [1, 64]"),
    ("layout", 2, "EUNSUPPORTED", "layout must be CFX_LAYOUT_AOS or CFX_LAYOUT_SOA"),
    ("n_shooting", 70000, "EUNSUPPORTED", "n_shooting must be <= 65535"),
    ("n_objectives", -3, "EINVAL", "n_objectives < 0, or objectives is NULL"),
    ("n_objectives", 1, "EINVAL", "n_objectives < 0, or objectives is NULL"),
    (None, None, "EINVAL", "NULL array"),  # a valid header whose geometry arrays are missing
])
def test_msk_create_rejects_bad_problem_before_touching_the_device(field, value, code, msg):
    """cfx_msk_create's header checks (cfx_api.hip:915-928) run before any HIP call."""
    import ctypes as C

    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    pb = _cfx.MskProblem()
    pb.abi_version, pb.scheme, pb.n_steps, pb.n_shooting = _cfx.ABI_VERSION, 4, 1, 2
    pb.truncation, pb.layout, pb.batch, pb.final_time = 10, _cfx.LAYOUT_SOA, 1, 1.0
    if field is not None:
        setattr(pb, field, value)
    h = C.c_void_p()
    assert lib.cfx_msk_create(C.byref(pb), C.byref(h)) == getattr(_cfx, code)
    assert not h.value
    assert msg in lib.cfx_last_error(None).decode()
    assert lib.cfx_msk_create(None, C.byref(h)) == _cfx.EINVAL


def _bare_handle(batch=4, device=0, layout=None):
    """A Handle whose sizes are set by hand (no cfx_create, so no GPU): exercises the Python-side buffer checks
    that run before any libcfx call."""
    from cocofest_amd import _cfx

    h = _cfx.Handle.__new__(_cfx.Handle)
    h.lib, h.h = None, None
    h.batch, h.device, h.layout = batch, device, _cfx.LAYOUT_SOA if layout is None else layout
    h.nv, h.ng, h.nnz_jac, h.nnz_hess, h.nx, h.nu, h.n_shooting, h.n_steps = 6, 4, 10, 9, 2, 0, 2, 1
    return h


def test_buffer_checks_reject_bad_host_arrays():
    """Every host buffer is checked against its slot before the call: libcfx reads / writes exactly batch * len
    doubles, so a wrong dtype, stride or size would be an out-of-bounds host access (_cfx.py)."""
    from cocofest_amd import CfxError

    h = _bare_handle()
    v = np.zeros((4, 6))
    cases_bad = [
        dict(v=np.zeros((4, 5))),                                    # short input
        dict(v=v, g=np.zeros((4, 4), dtype=np.float32)),             # float32 output
        dict(v=v, g=np.zeros((4, 8))[:, ::2]),                       # non-contiguous output
        dict(v=v, g=np.zeros((4, 3))),                               # short output
        dict(v=v, jac=np.zeros((4, 11))),                            # long output
        dict(v=v, f=np.zeros(3)),                                    # f is one value per instance
        dict(v=v, grad=[0.0] * 24),                                  # outputs must be numpy arrays
    ]
    for kw in cases_bad:
        with pytest.raises(CfxError) as exc:
            h.eval_all(**kw)
        assert exc.value.code == -1, kw
    with pytest.raises(CfxError):
        h.eval_h(v, np.ones(4), np.zeros((4, 5)), np.zeros((4, 9)))  # lambda of the wrong size
    with pytest.raises(CfxError):
        h.integrate(x0=np.zeros((4, 3)), traj=np.zeros((4, 6)))      # x0 of the wrong size
    # well-formed inputs are converted (non-contiguous float32 view -> contiguous float64 copy) and accepted
    (vv, g), fl = h._buffers(("v", np.zeros((4, 12), dtype=np.float32)[:, ::2], 6, False),
                             ("g", np.zeros((4, 4)), 4, True))
    assert fl == 0 and vv.dtype == np.float64 and vv.flags.c_contiguous and g.shape == (4, 4)


def test_buffer_checks_reject_bad_tensors():
    """A CPU tensor must never be sent as a device pointer (GPU fault), and device tensors must match the handle's
    device and the slot's size."""
    import torch

    from cocofest_amd import CfxError

    h = _bare_handle()
    with pytest.raises(CfxError) as exc:
        h.eval_all(torch.zeros((4, 6), dtype=torch.float64))
    assert "CPU tensor" in str(exc.value)
    with pytest.raises(CfxError) as exc:
        h.eval_all(torch.zeros((4, 6), dtype=torch.float64), g=np.zeros((4, 4)))
    assert "CPU tensor" in str(exc.value)


def test_objective_target_length_is_checked():
    from cocofest_amd import CfxError
    from cocofest_amd import _cfx

    keep = []
    ok = _cfx._objective_array([dict(kind=0, var_kind=0, var_index=1, node_first=0, node_last=2, weight=1.0,
                                     target=np.zeros(3))], keep, 2)
    assert ok[0].weight == 1.0
    with pytest.raises(CfxError) as exc:
        _cfx._objective_array([dict(kind=0, var_kind=0, var_index=1, node_first=0, node_last=2, weight=1.0,
                                    target=np.zeros(2))], keep, 2)
    assert "expected n_shooting + 1 = 3" in str(exc.value)


def test_missing_library_is_an_error(tmp_path):
    from cocofest_amd import CfxError
    from cocofest_amd import _cfx

    with pytest.raises(CfxError):
        _cfx.load_library(tmp_path / "nope.so")


def test_prepare_n_shooting_matches_reference(ref_formulas):
    from cocofest_amd import OcpFes

    for tb in ref_formulas["tables"]:
        assert OcpFes.prepare_n_shooting(tb["stim_time"], tb["final_time"]) == tb["n_shooting"]
    assert OcpFes.prepare_n_shooting(cases.cfg3()["stims"], 1.0) == 100


def test_stim_table_matches_reference_and_oracle(ref_formulas):
    from cocofest_amd import ModelMaker

    for tb in ref_formulas["tables"]:
        prev = {"time": list(tb["previous_stim"])} if tb["previous_stim"] else None
        if prev and tb["model"].startswith("hmed"):
            prev["pulse_intensity"] = [50] * len(prev["time"])
        model = ModelMaker.create_model(tb["model"], stim_time=list(tb["stim_time"]),
                                        sum_stim_truncation=tb["truncation"], previous_stim=prev)
        table, idx = model.get_numerical_data_time_series(tb["n_shooting"], tb["final_time"])
        rows = table["stim_time"][:, 0, :].T
        assert table["stim_time"].shape == (tb["truncation"], 1, tb["n_shooting"] + 1)
        oracle = O.stim_table(tb["stim_time"], tb["n_shooting"], tb["final_time"], tb["truncation"],
                              previous_stim=tb["previous_stim"])
        np.testing.assert_array_equal(rows, oracle.rows)
        assert idx == oracle.stim_idx_at_node
        if tb["final_time"] != 0.3:  # float-lookup discrepancy case
            np.testing.assert_array_equal(rows, np.array(tb["rows"]))
            assert idx == tb["stim_idx_at_node"]


@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_model_constants_match_oracle(name):
    from cocofest_amd import ModelMaker

    model = ModelMaker.create_model(name, sum_stim_truncation=10)
    c = O.model_constants(name)
    got = model.cfx_constants()
    for k, v in c.items():
        assert got[k] == pytest.approx(v, rel=1e-15), k
    assert model.nb_state == O.n_states(name)
    np.testing.assert_array_equal(model.standard_rest_values()[:, 0], O.rest_values(name, c))


def test_unknown_model_type():
    from cocofest_amd import ModelMaker

    with pytest.raises(ValueError, match="Unknown model type: foo"):
        ModelMaker.create_model("foo")


def test_ocp_layout_bounds_and_objectives():
    from cocofest_amd import _cfx

    t = np.linspace(0, 1, 40)
    force = 80 * np.sin(np.pi * t) ** 2
    for name in O.MODEL_NAMES:
        ocp = cases.product_ocp(name, cases.TEN_PULSES, 1.0, 5, scheme="RK1", m=4,
                                objective={"force_tracking": [t, force], "end_node_tracking": 40})
        pb = cases.oracle_problem(name, cases.TEN_PULSES, 1.0, 5, scheme="RK1", m=4,
                                  objective={"force_tracking": [t, force], "end_node_tracking": 40})
        assert ocp.nv == pb.nv
        lo, hi = O.state_bounds(name, pb.c)
        np.testing.assert_array_equal(ocp.x_bounds[0][:, 0], lo[:, 0])
        np.testing.assert_array_equal(ocp.x_bounds[1][:, 5], hi[:, 1])
        np.testing.assert_array_equal(ocp.x_bounds[1][:, -1], hi[:, 2])
        lb, ub = ocp.bounds_vector()
        assert lb.shape == ub.shape == (ocp.nv,) and np.all(lb <= ub)
        tr = ocp.objectives[0]
        assert tr["kind"] == _cfx.OBJ_LAGRANGE and tr["weight"] == 100.0
        np.testing.assert_allclose(tr["target"], pb.objectives[0].target, rtol=1e-13, atol=1e-12)
        assert ocp.objectives[1]["kind"] == _cfx.OBJ_MAYER and ocp.objectives[1]["node_first"] == pb.n_shooting


def test_hmed_sliding_window_indices_match_oracle():
    ocp = cases.product_ocp("hmed2018", cases.TEN_PULSES, 1.0, 4)
    pb = cases.oracle_problem("hmed2018", cases.TEN_PULSES, 1.0, 4)
    np.testing.assert_array_equal(ocp.last_stim_idx, pb.last_stim_idx)
    assert ocp.n_params == pb.n_params == 10
    assert ocp.intensity_floor == pytest.approx(17.02854931878943, rel=1e-15)


def test_pack_unpack_roundtrip():
    ocp = cases.product_ocp("ding2007_with_fatigue", cases.TEN_PULSES, 1.0, 5)
    v = np.arange(ocp.nv, dtype=float)
    states, controls, params = ocp.unpack(v)
    x = np.concatenate([states[k] for k in ocp.model.name_dof])
    np.testing.assert_array_equal(ocp.pack(x, controls["last_pulse_width"]), v)


def test_ocp_sanity_messages():
    from cocofest_amd import ModelMaker, OcpFes

    model = ModelMaker.create_model("ding2003", stim_time=[0, 0.1])
    with pytest.raises(TypeError, match="force_tracking must be list type"):
        OcpFes.prepare_ocp(model=model, final_time=0.2, objective={"force_tracking": 3})
    with pytest.raises(TypeError, match="end_node_tracking must be int or float type"):
        OcpFes.prepare_ocp(model=model, final_time=0.2, objective={"end_node_tracking": "a"})
    with pytest.raises(TypeError, match="ode_solver must be a OdeSolver type"):
        OcpFes.prepare_ocp(model=model, final_time=0.2, ode_solver=None)
    with pytest.raises(TypeError, match="use_sx must be a bool type"):
        OcpFes.prepare_ocp(model=model, final_time=0.2, use_sx=None)
    with pytest.raises(TypeError, match="n_thread must be a int type"):
        OcpFes.prepare_ocp(model=model, final_time=0.2, n_threads=None)
    with pytest.raises(TypeError, match="it must be a FesModel type"):
        OcpFes._sanity_check(model=3, n_shooting=2, final_time=1.0, objective={})


def test_ivp_validation_messages_match_reference():
    """The input errors of tests/shard1/test_ivp.py:186-332 that the current reference code raises."""
    import re as _re

    from cocofest_amd import IvpFes, ModelMaker

    d03 = ModelMaker.create_model("ding2003", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    d07 = ModelMaker.create_model("ding2007", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    h18 = ModelMaker.create_model("hmed2018", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    with pytest.raises(ValueError, match=_re.escape("The number of stimulation needs to be integer within the final "
                                                    "time t, set round down to True or set final_time * frequency "
                                                    "to make the result an integer.")):
        IvpFes.from_frequency_and_final_time({"model": d03, "frequency": 30, "round_down": False},
                                             {"final_time": 1.25})
    with pytest.raises(ValueError, match="Pulse mode not yet implemented"):
        IvpFes({"model": d03, "stim_time": [0, 0.1, 0.2], "pulse_mode": "Quadruplet"}, {"final_time": 0.3})
    with pytest.raises(ValueError, match=_re.escape("pulse width must be greater than minimum pulse width")):
        IvpFes({"model": d07, "pulse_width": 0.00001}, {"final_time": 0.3})
    with pytest.raises(ValueError, match=_re.escape("pulse width must be greater than minimum pulse width")):
        IvpFes({"model": d07, "pulse_width": [0.001, 0.0001, 0.003]}, {"final_time": 0.3})
    with pytest.raises(TypeError, match="pulse_width must be int, float or list type"):
        IvpFes({"model": d07, "pulse_width": True}, {"final_time": 0.3})
    with pytest.raises(ValueError, match=_re.escape("Pulse intensity must be greater than minimum pulse intensity")):
        IvpFes({"model": h18, "pulse_intensity": 0.1}, {"final_time": 0.3})
    with pytest.raises(ValueError, match=_re.escape("Pulse intensity must be greater than minimum pulse intensity")):
        IvpFes({"model": h18, "pulse_intensity": [20, 30, 0.1]}, {"final_time": 0.3})
    with pytest.raises(TypeError, match="pulse_intensity must be int, float or list type"):
        IvpFes({"model": h18, "pulse_intensity": True}, {"final_time": 0.3})
    with pytest.raises(ValueError, match="ode_solver must be a OdeSolver type"):
        IvpFes({"model": d03}, {"final_time": 0.3, "ode_solver": None})
    with pytest.raises(ValueError, match="n_thread must be a int type"):
        IvpFes({"model": d03}, {"final_time": 0.3, "n_threads": None})


def test_ivp_host_setup_matches_oracle():
    """IvpFes host preparation (n_shooting, pulse modes, table, controls) equals the oracle's."""
    from cocofest_amd import IvpFes, ModelMaker

    h18 = ModelMaker.create_model("hmed2018", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    ivp = IvpFes({"model": h18, "pulse_intensity": [50, 60, 70]}, {"final_time": 0.3})
    tab = O.stim_table([0, 0.1, 0.2], 3, 0.3, 3)
    np.testing.assert_array_equal(ivp.stim_rows, tab.rows)
    np.testing.assert_array_equal(ivp.controls.T, O.ivp_controls("hmed2018", tab, 3, 3, None, [50, 60, 70]))
    d03 = ModelMaker.create_model("ding2003_with_fatigue", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    ivp = IvpFes({"model": d03, "pulse_mode": "doublet"}, {"final_time": 0.3})
    assert ivp.n_shooting == 60 and d03.stim_time == [0, 0.005, 0.1, 0.105, 0.2, 0.205]
    d07 = ModelMaker.create_model("ding2007", stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
    ivp = IvpFes({"model": d07, "pulse_width": [0.0003, 0.0004, 0.0005]}, {"final_time": 0.3})
    np.testing.assert_array_equal(ivp.controls[0], [0.0003, 0.0004, 0.0005])


def test_ipm_abi_null_and_default_options():
    """cfx_ipm_*: NULL arguments are rejected without touching a device; the default options are Ipopt's (and
    those of solver.IpmOptions, the algorithm's executable specification)."""
    import ctypes as C

    from cocofest_amd import _cfx
    from cocofest_amd.solver import _NATIVE_OPTIONS, IpmOptions

    lib = _cfx.load_library()
    opt = _cfx.IpmOptions()
    lib.cfx_ipm_default_options(C.byref(opt))
    ref = IpmOptions()
    for k in _NATIVE_OPTIONS:
        assert getattr(opt, k) == getattr(ref, k), k
    lib.cfx_ipm_default_options(None)  # tolerated
    s = C.c_void_p()
    lb = np.zeros(4)
    assert lib.cfx_ipm_create(None, lb.ctypes.data, lb.ctypes.data, 0, C.byref(opt), C.byref(s)) == _cfx.EINVAL
    assert lib.cfx_ipm_solve(None, None, None, None, None, None, None, None, None, 0) == _cfx.EINVAL
    st = _cfx.IpmStats()
    assert lib.cfx_ipm_get_stats(None, C.byref(st)) == _cfx.EINVAL
    assert lib.cfx_ipm_get_status(None, None) == _cfx.EINVAL
    assert lib.cfx_ipm_n_fixed(None) == -1
    assert lib.cfx_ipm_last_error(None) == b""
    lib.cfx_ipm_destroy(None)


def test_ipm_option_structs_match_the_header():
    """The ctypes mirrors of cfx_ipm_options / cfx_ipm_stats list the header's fields in order."""
    from cocofest_amd import _cfx

    text = (ROOT / "include" / "cfx.h").read_text()
    for struct, cls in (("cfx_ipm_options", _cfx.IpmOptions), ("cfx_ipm_stats", _cfx.IpmStats)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), text, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names += [n.strip() for n in decl.split(None, 1)[1].split(",")]
        assert names == [f for f, _ in cls._fields_], struct


def test_ctypes_mirrors_match_the_c_header_layout(tmp_path):
    """Every ctypes structure of _cfx.py has the size and field offsets gcc gives the include/cfx.h struct of the
    same name (a drifted field would shift every later argument across the C ABI)."""
    import ctypes
    import pathlib
    import shutil
    import subprocess

    from cocofest_amd import _cfx

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    pairs = [(_cfx.Constants, "cfx_constants"), (_cfx.Objective, "cfx_objective"), (_cfx.Problem, "cfx_problem"),
             (_cfx.Sizes, "cfx_sizes"), (_cfx.MskMuscle, "cfx_msk_muscle"), (_cfx.MskMarkerPair, "cfx_msk_marker_pair"),
             (_cfx.MskProblem, "cfx_msk_problem"), (_cfx.IpmOptions, "cfx_ipm_options"), (_cfx.IpmStats, "cfx_ipm_stats"),
             (_cfx.LaunchShape, "cfx_launch_shape")]
    lines, want = [], []
    for cls, cname in pairs:
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        want.append(ctypes.sizeof(cls))
        for name, _ in cls._fields_:
            lines.append(f'printf("%zu\\n", offsetof({cname}, {name}));')
            want.append(getattr(cls, name).offset)
    src = tmp_path / "layout.c"
    inc = pathlib.Path(__file__).resolve().parents[1] / "include"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "cfx.h"\nint main(void) {\n' + "\n".join(lines)
                   + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", str(inc), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == want


def test_ivp_n_shooting_extension():
    """IvpFes(ivp_parameters={"n_shooting": N}) overrides the LCM node count (BASELINE configs[0] asks for 20 nodes
    for 10 pulses); doublets keep the given count; invalid counts are refused."""
    from cocofest_amd import IvpFes, ModelMaker

    stims = [round(0.1 * i, 1) for i in range(10)]
    m = ModelMaker.create_model("ding2003_with_fatigue", stim_time=list(stims), sum_stim_truncation=10)
    assert IvpFes({"model": m}, {"final_time": 1.0}).n_shooting == 10
    ivp = IvpFes({"model": m}, {"final_time": 1.0, "n_shooting": 20})
    assert ivp.n_shooting == 20 and ivp.stim_rows.shape == (21, 10)
    # node 1 (t = 0.05) sees only the first pulse, node 2 (t = 0.1) the first two
    assert np.sum(ivp.stim_rows[1] > -1e6) == 1 and np.sum(ivp.stim_rows[2] > -1e6) == 2
    m2 = ModelMaker.create_model("ding2003", stim_time=[0.0, 0.1], sum_stim_truncation=6)
    assert IvpFes({"model": m2, "pulse_mode": "doublet"}, {"final_time": 0.2, "n_shooting": 8}).n_shooting == 8
    for bad in (0, -3, 2.5, True):
        with pytest.raises(ValueError):
            IvpFes({"model": m}, {"final_time": 1.0, "n_shooting": bad})
