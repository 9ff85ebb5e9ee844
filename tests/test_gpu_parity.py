"""Parity of the gfx950 kernels (through the libcfx C ABI) with the oracle and the reference goldens.

Tolerances: FP64 everywhere.  IVP trajectories vs the reference's 8-decimal golden literals: 6e-9
absolute.  Callback values vs the oracle (same inputs, complex-step derivatives): relative 1e-11 on
g / J / f / grad (RK recursions of <= 40 stages; the kernels use reciprocal-multiply where the oracle
divides, a few ulp per stage).
"""

import json
import pathlib

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases
from tests.conftest import golden_stims

pytestmark = pytest.mark.gpu

RTOL = 1e-11


def _close(actual, desired, rtol=RTOL, what="", scale=None):
    """max |actual - desired| / scale <= rtol; scale defaults to |desired| floored at 1e-6 of its row max."""
    desired = np.asarray(desired)
    floor = np.max(np.abs(desired), axis=-1, keepdims=True) * 1e-6 + 1e-300
    scale = np.maximum(np.abs(desired) if scale is None else scale, floor)
    err = np.max(np.abs(actual - desired) / scale) if desired.size else 0.0
    assert err <= rtol, f"{what}: max scaled error {err:.3e} > {rtol:.1e}"


def _close_g(pb, v, actual, desired, rtol=RTOL, what=""):
    """g is a difference (Phi(x_k, u_k) - x_{k+1}, u_k - window): scale each row by |g| + |x_{k+1}| (resp. |u_k|),
    i.e. compare Phi itself to relative rtol."""
    X, U, _ = pb.unpack(v)
    parts = []
    for k in range(pb.n_shooting):
        parts.append(np.abs(X[:, k + 1, :]))
        if pb.n_slide:
            parts.append(np.abs(U[:, k, :]))
    ref = np.concatenate(parts, axis=1)
    _close(actual, desired, rtol=rtol, what=what, scale=np.abs(np.asarray(desired)) + ref)


@pytest.fixture(scope="module", autouse=True)
def _require_gpu():
    from cocofest_amd import _cfx

    lib = _cfx.load_library()  # raises if libcfx.so is missing: no silent fallback
    if lib.cfx_device_count() < 1:
        pytest.fail("no HIP device visible to libcfx")


def test_ivp_goldens_on_gpu(ivp_goldens):
    """The 9 reference golden trajectories (tests/shard1/test_ivp.py) through IvpFes -> cfx_integrate."""
    from cocofest_amd import IvpFes, ModelMaker, OdeSolver

    shared = {}
    for case in ivp_goldens:
        name = case["model"]
        if case["pulse_mode"] == "single" or name not in shared:
            shared[name] = ModelMaker.create_model(name, stim_time=[0, 0.1, 0.2], sum_stim_truncation=3)
        model = shared[name]  # the pulse-mode cases reuse (and mutate) one model, as the reference's test does
        fes = {"model": model, "pulse_mode": case["pulse_mode"]}
        if case["pulse_width"]:
            fes["pulse_width"] = case["pulse_width"]
        if case["pulse_intensity"]:
            fes["pulse_intensity"] = case["pulse_intensity"]
        ivp = IvpFes(fes, {"final_time": 0.3, "ode_solver": OdeSolver.RK4(n_integration_steps=10)})
        result = ivp.integrate(return_time=False)
        f = result["F"][0]
        if case["slice"]:
            f = f[case["slice"][0]: case["slice"][1]]
        np.testing.assert_allclose(f, case["F"], rtol=0, atol=6e-9, err_msg=case["source"])
        # and against the oracle on every state and sample
        c = O.model_constants(name)
        stims = golden_stims(case["pulse_mode"], case["stim_time"])
        n = O.prepare_n_shooting(stims, 0.3)
        tab = O.stim_table(stims, n, 0.3, 3)
        u = O.ivp_controls(name, tab, n, 3, case["pulse_width"], case["pulse_intensity"])
        ref = O.ivp_integrate(name, c, tab.rows, u, 0.3, "RK4", 10)
        got = np.stack([result[k][0] for k in model.name_dof])
        _close(got, ref, what=f"ivp {name} {case['pulse_mode']}")


STIMS = [0.0, 0.05, 0.1, 0.15]


@pytest.mark.parametrize("scheme", ["RK1", "RK2", "RK4"])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_shooting_g_and_jacobian_vs_oracle(name, scheme):
    T = 3
    ocp = cases.product_ocp(name, STIMS, 0.2, T, scheme=scheme, m=3)
    pb = cases.oracle_problem(name, STIMS, 0.2, T, scheme=scheme, m=3)
    assert ocp.nv == pb.nv and ocp.n_shooting == pb.n_shooting
    B = 7
    v = cases.random_decision(pb, B, seed=11)
    h = ocp.nlp(batch=B, layout="aos")
    assert (h.nv, h.ng) == (pb.nv, pb.ng)
    rows, cols = h.jac_structure()
    orows, ocols = O.jac_structure(pb)
    np.testing.assert_array_equal(rows, orows)
    np.testing.assert_array_equal(cols, ocols)
    g = h.eval_g(v)
    jac = h.eval_jac_g(v)
    _close_g(pb, v, g, O.eval_g(pb, v), what=f"g {name} {scheme}")
    _close(jac, O.eval_jac_g(pb, v), what=f"J {name} {scheme}")
    # fused call gives the same values: g bit for bit; J runs a separately compiled loop body (with / without the
    # g rows), whose FMA contraction may differ by an ulp
    g2, j2 = np.empty_like(g), np.empty_like(jac)
    h.eval_all(v, g=g2, jac=j2)
    np.testing.assert_array_equal(g2, g)
    np.testing.assert_allclose(j2, jac, rtol=1e-14, atol=1e-300)


@pytest.mark.parametrize("T", [1, 5, 10, 17, 32])
def test_hmed_truncation_buckets(T):
    stims = [round(0.02 * i, 2) for i in range(12)]
    for name in ("hmed2018", "hmed2018_with_fatigue"):
        ocp = cases.product_ocp(name, stims, 0.24, T, scheme="RK2", m=2)
        pb = cases.oracle_problem(name, stims, 0.24, T, scheme="RK2", m=2)
        v = cases.random_decision(pb, 3, seed=T)
        h = ocp.nlp(batch=3)
        _close_g(pb, v, h.eval_g(v), O.eval_g(pb, v), what=f"g {name} T={T}")
        _close(h.eval_jac_g(v), O.eval_jac_g(pb, v), what=f"J {name} T={T}")


def test_objective_value_and_gradient():
    t = np.linspace(0, 1, 40)
    force = 80 * np.sin(np.pi * t) ** 2
    obj = {"force_tracking": [t, force], "end_node_tracking": 40}
    for name in ("ding2003", "ding2007_with_fatigue"):
        ocp = cases.product_ocp(name, cases.TEN_PULSES, 1.0, 5, scheme="RK1", m=4, objective=obj)
        pb = cases.oracle_problem(name, cases.TEN_PULSES, 1.0, 5, scheme="RK1", m=4, objective=obj)
        v = cases.random_decision(pb, 4, seed=3)
        h = ocp.nlp(batch=4)
        _close(h.eval_f(v), O.eval_f(pb, v), what=f"f {name}")
        _close(h.eval_grad_f(v), O.eval_grad_f(pb, v), what=f"grad {name}")


def test_layouts_and_device_pointers_are_bitwise_identical():
    import torch

    cfg = cases.cfg2()
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    B = 300  # not a multiple of the 256-thread block
    v = cases.random_decision(pb, B, seed=5)
    ha = ocp.nlp(batch=B, layout="aos")
    hs = ocp.nlp(batch=B, layout="soa")
    ga, ja = ha.eval_g(v), ha.eval_jac_g(v)
    vs = np.ascontiguousarray(v.T)
    gs, js = hs.eval_g(vs), hs.eval_jac_g(vs)
    np.testing.assert_array_equal(gs.T, ga)
    np.testing.assert_array_equal(js.T, ja)
    # torch device buffers, SoA, in place on the current stream
    dv = torch.from_numpy(vs).cuda()
    dg = torch.empty((hs.ng, B), dtype=torch.float64, device="cuda")
    dj = torch.empty((hs.nnz_jac, B), dtype=torch.float64, device="cuda")
    hs.eval_all(dv, g=dg, jac=dj)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dg.cpu().numpy(), gs)
    np.testing.assert_array_equal(dj.cpu().numpy(), js)
    # device AoS
    dva = torch.from_numpy(v).cuda()
    dga = torch.empty((B, ha.ng), dtype=torch.float64, device="cuda")
    ha.eval_all(dva, g=dga)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dga.cpu().numpy(), ga)
    _close_g(pb, v, ga, O.eval_g(pb, v), what="cfg2 g")


@pytest.mark.parametrize("scheme", ["RK1", "RK2"])
@pytest.mark.parametrize("name", ["ding2003", "ding2007", "ding2007_with_fatigue", "hmed2018"])
def test_tiled_layout_is_bitwise_identical(name, scheme):
    """CFX_LAYOUT_TILED64 (64-instance tiles, two instances per lane) gives the same g, J_g, f, grad f bits as SoA
    (one per lane), and matches the oracle; Hmed's sliding rows and the objective kernels included; RK1 of the
    two-state Ding families runs the fused Euler step; so does the Hessian (bitwise), and the fused g + J_g + Hessian
    launch to rounding; a batch the tiles do not divide fails loudly."""
    import torch

    from cocofest_amd import _cfx

    # m = 8: h / tau_c = 0.625, inside the regime where the oracle comparison is meaningful (DESIGN.md section 4;
    # at h = tau_c the RK2 stage calcium amplifies rounding to ~1e-10 in any implementation)
    cfg = dict(name=name, stims=[0.0, 0.1, 0.2, 0.3], final_time=0.4, truncation=4, scheme=scheme, m=8,
               objective={"end_node_tracking": 40.0}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    B = 320
    v = cases.random_decision(pb, B, seed=9)
    hs, ht = ocp.nlp(batch=B, layout="soa"), ocp.nlp(batch=B, layout="tiled64")

    def run(h, vin, shape):
        g = torch.empty(shape(h.ng), dtype=torch.float64, device="cuda")
        j = torch.empty(shape(h.nnz_jac), dtype=torch.float64, device="cuda")
        f = torch.empty((B,), dtype=torch.float64, device="cuda")
        gr = torch.empty(shape(h.nv), dtype=torch.float64, device="cuda")
        h.eval_all(vin, g=g, jac=j, f=f, grad=gr)
        torch.cuda.synchronize()
        return g.cpu().numpy(), j.cpu().numpy(), f.cpu().numpy(), gr.cpu().numpy()

    soa = run(hs, torch.tensor(np.ascontiguousarray(v.T), device="cuda"), lambda n: (n, B))
    vt = np.ascontiguousarray(v.reshape(B // 64, 64, -1).transpose(0, 2, 1))
    til = run(ht, torch.tensor(vt, device="cuda"), lambda n: (B // 64, n, 64))
    untile = lambda a: a.transpose(0, 2, 1).reshape(B, -1).T  # noqa: E731
    np.testing.assert_array_equal(untile(til[0]), soa[0])
    np.testing.assert_array_equal(untile(til[1]), soa[1])
    np.testing.assert_array_equal(til[2], soa[2])
    np.testing.assert_array_equal(untile(til[3]), soa[3])
    _close_g(pb, v, untile(til[0]).T, O.eval_g(pb, v), what=f"tiled g {name} {scheme}")
    _close(untile(til[1]).T, O.eval_jac_g(pb, v), what=f"tiled J {name} {scheme}")
    # the Lagrangian Hessian (and the fused g + J_g + H launch) on tiles: the same bits as SoA
    rng = np.random.default_rng(3)
    lam, of = rng.standard_normal((B, hs.ng)), rng.uniform(0.5, 2.0, B)
    ofd = torch.tensor(of, device="cuda")
    hh_s = hs.eval_h(torch.tensor(np.ascontiguousarray(v.T), device="cuda"), ofd,
                     torch.tensor(np.ascontiguousarray(lam.T), device="cuda"),
                     torch.empty((hs.nnz_hess, B), dtype=torch.float64, device="cuda"))
    lt = torch.tensor(np.ascontiguousarray(lam.reshape(B // 64, 64, -1).transpose(0, 2, 1)), device="cuda")
    hh_t = ht.eval_h(torch.tensor(vt, device="cuda"), ofd, lt,
                     torch.empty((B // 64, ht.nnz_hess, 64), dtype=torch.float64, device="cuda"))
    np.testing.assert_array_equal(untile(hh_t.cpu().numpy()), hh_s.cpu().numpy())
    fg, fj, fh = ht.eval_all_h(torch.tensor(vt, device="cuda"), ofd, lt)
    for got, want in ((fg, soa[0]), (fj, soa[1]), (fh, hh_s.cpu().numpy())):
        assert np.abs(untile(got.cpu().numpy()) - want).max() <= 1e-13 * (np.abs(want).max() + 1.0)
    with pytest.raises(_cfx.CfxError):
        ocp.nlp(batch=100, layout="tiled64")
    hs.close()
    ht.close()


def test_full_size_properties_cfg2():
    """BASELINE config 2 at bench size: batch invariance (instance b gives the same bits alone and inside a
    2^17 batch) and feasibility of the forward RK1 x 10 integration (the 0-DOF optimum): g == 0."""
    import torch

    cfg = cases.cfg2()
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    B = 1 << 17
    v = cases.random_decision(pb, B, seed=9)
    hs = ocp.nlp(batch=B, layout="soa")
    dv = torch.from_numpy(np.ascontiguousarray(v.T)).cuda()
    dg = torch.empty((hs.ng, B), dtype=torch.float64, device="cuda")
    dj = torch.empty((hs.nnz_jac, B), dtype=torch.float64, device="cuda")
    hs.eval_all(dv, g=dg, jac=dj)
    torch.cuda.synchronize()
    pick = np.array([0, 1, 63, 64, 255, 256, 4097, B - 1])
    h1 = ocp.nlp(batch=len(pick), layout="aos")
    np.testing.assert_array_equal(h1.eval_g(v[pick]), dg[:, pick].cpu().numpy().T)
    np.testing.assert_array_equal(h1.eval_jac_g(v[pick]), dj[:, pick].cpu().numpy().T)
    _close_g(pb, v[pick], dg[:, pick].cpu().numpy().T, O.eval_g(pb, v[pick]), what="cfg2 big-batch g")
    # forward-integrated trajectory is feasible
    from cocofest_amd import IvpFes, ModelMaker, OdeSolver

    model = ModelMaker.create_model("ding2003", stim_time=cases.TEN_PULSES, sum_stim_truncation=20)
    ivp = IvpFes({"model": model}, {"final_time": 1.0, "ode_solver": OdeSolver.RK1(n_integration_steps=10)})
    res = ivp.integrate(return_time=False)
    nodes = np.stack([res["Cn"][0][::10], res["F"][0][::10]])  # N = 10 (the reference's LCM rule)
    ocp10 = cases.product_ocp(**cases.cfg2(n_shooting=None))
    g = ocp10.nlp(batch=1).eval_g(ocp10.pack(nodes)[None, :])
    assert np.max(np.abs(g)) < 1e-9


def test_edge_sizes():
    # N = 1, batch 1, truncation 1
    for name in ("ding2003_with_fatigue", "ding2007", "hmed2018"):
        ocp = cases.product_ocp(name, [0.0], 0.1, 1, scheme="RK4", m=1)
        pb = cases.oracle_problem(name, [0.0], 0.1, 1, scheme="RK4", m=1)
        assert pb.n_shooting == 1
        v = cases.random_decision(pb, 1, seed=2)
        h = ocp.nlp(batch=1)
        _close_g(pb, v, h.eval_g(v), O.eval_g(pb, v), what=f"edge g {name}")
        _close(h.eval_jac_g(v), O.eval_jac_g(pb, v), what=f"edge J {name}")


def test_errors_are_loud():
    from cocofest_amd import CfxError
    from cocofest_amd import _cfx

    ocp = cases.product_ocp(**cases.cfg2())
    with pytest.raises(CfxError):
        _cfx.Handle(model_id=9, constants={}, scheme=1, n_steps=1, n_shooting=2, truncation=1, final_time=1.0,
                    stim_rows=np.zeros(3), batch=1)
    with pytest.raises(CfxError):
        _cfx.Handle(model_id=0, constants={}, scheme=3, n_steps=1, n_shooting=2, truncation=1, final_time=1.0,
                    stim_rows=np.zeros(3), batch=1)
    h = ocp.nlp(batch=2)
    with pytest.raises(CfxError):
        h.eval_h(np.zeros((2, h.nv)), None, np.zeros((2, h.ng)))


@pytest.mark.parametrize("name", ["ding2003", "ding2003_with_fatigue", "ding2007", "ding2007_with_fatigue"])
def test_instances_per_lane_variants_are_identical(name, monkeypatch):
    """NI adjacent instances per lane (16-byte accesses) must give the same bits as NI = 1, including a batch
    that is not a multiple of the 256-thread block and a misaligned (offset) device buffer."""
    import torch

    # RK4 with h * (1/tauc) = 1: coarser steps drive the RK4 stage calcium negative on random inputs and the
    # discretisation itself becomes ill-conditioned (1e-10-level rounding amplification in any implementation)
    ocp = cases.product_ocp(name, cases.TEN_PULSES, 1.0, 5, scheme="RK4", m=5)
    pb = cases.oracle_problem(name, cases.TEN_PULSES, 1.0, 5, scheme="RK4", m=5)
    B = 1028  # % 4 == 0, not a multiple of 256
    v = cases.random_decision(pb, B, seed=21)
    dv = torch.from_numpy(np.ascontiguousarray(v.T)).cuda()
    out = {}
    for ni in ("1", "2", "4"):
        monkeypatch.setenv("CFX_NI", ni)
        h = ocp.nlp(batch=B, layout="soa")
        g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
        j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
        h.eval_all(dv, g=g, jac=j)
        torch.cuda.synchronize()
        out[ni] = (g.cpu().numpy(), j.cpu().numpy())
        h.close()
    for ni in ("2", "4"):  # interleaving changes FMA contraction: equal to a few ulp, not bitwise
        np.testing.assert_allclose(out[ni][0], out["1"][0], rtol=1e-14, atol=1e-13)
        np.testing.assert_allclose(out[ni][1], out["1"][1], rtol=1e-14, atol=1e-13)
    # 50 RK4 stages per interval: a little more rounding accumulation than the short cases above
    _close_g(pb, v, out["1"][0].T, O.eval_g(pb, v), rtol=1e-10, what=f"g {name}")
    _close(out["1"][1].T, O.eval_jac_g(pb, v), rtol=1e-10, what=f"J {name}")
    # an 8-byte-offset output buffer forces the scalar path, same result
    monkeypatch.setenv("CFX_NI", "2")
    h = ocp.nlp(batch=B, layout="soa")
    big = torch.empty((h.ng * B + 1,), dtype=torch.float64, device="cuda")
    g_off = big[1:].view(h.ng, B)
    h.eval_all(dv, g=g_off)
    torch.cuda.synchronize()
    np.testing.assert_allclose(g_off.cpu().numpy(), out["1"][0], rtol=1e-14, atol=1e-13)


@pytest.mark.parametrize("scheme", ["RK1", "RK2", "RK4"])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_lagrangian_hessian_vs_oracle(name, scheme):
    """cfx_eval_h vs central differences of complex-step gradients (Richardson, ~1e-10 accurate)."""
    t = np.linspace(0, 1, 30)
    obj = {"force_tracking": [t, 60 * np.sin(np.pi * t) ** 2], "end_node_tracking": 50}
    stims = [0.0, 0.02, 0.04, 0.06]
    ocp = cases.product_ocp(name, stims, 0.08, 3, scheme=scheme, m=2, objective=obj)
    pb = cases.oracle_problem(name, stims, 0.08, 3, scheme=scheme, m=2, objective=obj)
    B = 3
    v = cases.random_decision(pb, B, seed=4)
    rng = np.random.default_rng(5)
    lam = rng.normal(size=(B, pb.ng))
    of = rng.uniform(0.5, 2.0, B)
    h = ocp.nlp(batch=B)
    r, c = h.hess_structure()
    orr, occ = O.hess_structure(pb)
    np.testing.assert_array_equal(r, orr)
    np.testing.assert_array_equal(c, occ)
    got = h.eval_h(v, of, lam)
    ref = O.hessian_values(pb, v, of, lam)
    scale = np.maximum(np.abs(ref), 1e-4 * np.max(np.abs(ref), axis=1, keepdims=True))
    err = np.max(np.abs(got - ref) / scale)
    assert err < 1e-7, f"H {name} {scheme}: {err:.3e}"


@pytest.mark.parametrize("scheme", ["RK1", "RK2", "RK4"])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_fused_g_jacobian_hessian(name, scheme):
    """cfx_eval_all_h — g, J_g, f, grad f and the Lagrangian Hessian from ONE shooting launch on second-order jets
    (Hmed's sliding rows and the objective kernels beside it) — against the separate callbacks: f and grad f bit for
    bit (the same kernels), g, J_g and the Hessian to rounding, 1e-13 of the largest entry (the jets' value and
    first-order parts are the shooting kernel's recursion in another evaluation order; the Hessian instantiation that
    also stores g and J_g is scheduled differently, a few ulp on Hmed), and g / J_g against the oracle."""
    t = np.linspace(0, 1, 30)
    obj = {"force_tracking": [t, 60 * np.sin(np.pi * t) ** 2], "end_node_tracking": 50}
    stims = [0.0, 0.02, 0.04, 0.06]
    ocp = cases.product_ocp(name, stims, 0.08, 3, scheme=scheme, m=2, objective=obj)
    pb = cases.oracle_problem(name, stims, 0.08, 3, scheme=scheme, m=2, objective=obj)
    B = 5
    v = cases.random_decision(pb, B, seed=4)
    rng = np.random.default_rng(5)
    lam, of = rng.normal(size=(B, pb.ng)), rng.uniform(0.5, 2.0, B)
    h = ocp.nlp(batch=B)
    g, jac, grad = (np.empty((B, n)) for n in (h.ng, h.nnz_jac, h.nv))
    f = np.empty(B)
    h.eval_all(v, g=g, jac=jac, f=f, grad=grad)
    hs = h.eval_h(v, of, lam)
    fg, fj, ff, fgr = np.empty_like(g), np.empty_like(jac), np.empty_like(f), np.empty_like(grad)
    _, _, fh = h.eval_all_h(v, of, lam, g=fg, jac=fj, f=ff, grad=fgr)
    h.close()
    np.testing.assert_array_equal(ff, f)
    np.testing.assert_array_equal(fgr, grad)
    for got, want in ((fg, g), (fj, jac), (fh, hs)):
        assert np.abs(got - want).max() <= 1e-13 * (np.abs(want).max() + 1.0)
    _close_g(pb, v, fg, O.eval_g(pb, v), what=f"fused g {name} {scheme}")
    _close(fj, O.eval_jac_g(pb, v), what=f"fused J {name} {scheme}")


def test_fused_callbacks_on_collocation_run_both_passes():
    """cfx_eval_all_h on a collocation handle (one launch since round 4: task 0 of each interval runs the g + J_g body
    beside its Hessian block): the separate callbacks' bits."""
    ocp = cases.product_collocation_ocp("ding2007", COL_STIMS, 0.5, 4, degree=3, method="legendre",
                                        objective={"end_node_tracking": 40.0}, n_shooting=5)
    from tests.oracle_handle import oracle_problem_from_ocp

    pb = oracle_problem_from_ocp(ocp)
    B = 4
    v = cases.random_collocation_decision(pb, B, seed=11)
    rng = np.random.default_rng(3)
    lam, of = rng.standard_normal((B, pb.ng)), rng.uniform(0.5, 2.0, B)
    h = ocp.nlp(batch=B, layout="aos")
    g, jac, hs = h.eval_g(v), h.eval_jac_g(v), h.eval_h(v, of, lam)
    fg, fj, fh = h.eval_all_h(v, of, lam)
    h.close()
    for a, b in ((fg, g), (fj, jac), (fh, hs)):
        np.testing.assert_array_equal(a, b)


def test_interior_point_on_gpu_matches_forward_integration():
    """cfg 2 (0 DOF) solved by the batched interior point over libcfx: every start converges to the RK1 x 10
    forward integration (the reference's optimum for this config)."""
    from cocofest_amd.solver import BatchedIpm, IpmOptions

    cfg = cases.cfg2()
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    B = 64
    rng = np.random.default_rng(3)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1)) + rng.uniform(0, 20, (B, pb.nv))
    ipm = BatchedIpm(ocp, batch=B, options=IpmOptions(tol=1e-8))
    res = ipm.solve(v0)
    ipm.close()
    assert res.converged.all(), res.kkt_error
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), 1.0, "RK1", 10)
    X, _, _ = pb.unpack(res.v)
    np.testing.assert_allclose(X, np.broadcast_to(traj[:, ::10].T, X.shape), rtol=1e-7, atol=1e-8)


def test_interior_point_pulse_width_force_tracking():
    """cfg 3 shape (Ding2007 pulse width, force tracking, N = 100): converges to a feasible KKT point that
    respects the bounds, for a small multi-start batch."""
    from cocofest_amd.solver import BatchedIpm

    ft = json.loads((pathlib.Path(__file__).parent / "golden" / "ref_formulas.json").read_text())
    ft = ft["misc"]["force_tracking"]
    cfg = dict(cases.cfg3(), objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]})
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    ipm = BatchedIpm(ocp, batch=4)
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (4, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (4, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                          lb[free], ub[free])
    res = ipm.solve(v0)
    ipm.close()
    assert res.converged.all(), (res.kkt_error, res.iterations)
    assert np.max(np.abs(O.eval_g(pb, res.v))) < 1e-5
    assert np.all(res.v >= lb - 1e-8) and np.all(res.v <= ub + 1e-8)


def _band_system(rng, B, n, kl, ku, zero_diag=False):
    """Random banded matrices (B, n, n), their LAPACK band storage (B, n, 2kl+ku+1) and right-hand sides."""
    A = np.zeros((B, n, n))
    for d in range(-kl, ku + 1):
        idx = np.arange(max(0, -d), min(n, n - d))
        A[:, idx, idx + d] = rng.standard_normal((B, idx.size))
    if zero_diag:
        A[:, np.arange(n), np.arange(n)] = 0.0  # KKT-like: forces row interchanges
    ldab = 2 * kl + ku + 1
    ab = np.full((B, n, ldab), np.nan)  # fill-in rows must be ignored (zeroed by the factorisation)
    for j in range(n):
        for i in range(max(0, j - ku), min(n, j + kl + 1)):
            ab[:, j, kl + ku + i - j] = A[:, i, j]
    ab[:, :, kl:] = np.nan_to_num(ab[:, :, kl:])
    return A, ab


@pytest.mark.parametrize("n,kl,ku,zero_diag", [(1, 0, 0, False), (7, 3, 1, False), (80, 5, 5, True),
                                               (500, 6, 6, True), (300, 40, 40, False), (64, 63, 63, False),
                                               (200, 70, 2, False)])
def test_band_lu_matches_dense_solve(n, kl, ku, zero_diag):
    """cfx_band_lu / cfx_band_lu_solve vs numpy's dense LU on random band matrices: LDS-resident bands and the
    global-memory variant (300 x 161 band > 160 KiB), bandwidths beyond one wave (kl = 70), zero diagonals."""
    import torch

    from cocofest_amd import _cfx

    rng = np.random.default_rng(n + kl)
    B = 130  # >= 128: the windowed kernels where the band fits their LDS budget
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag)
    rhs = rng.standard_normal((B, 2, n))
    ref = np.linalg.solve(A, rhs.transpose(0, 2, 1)).transpose(0, 2, 1)
    abt = torch.tensor(ab, device="cuda")
    ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
    info = torch.empty((B,), dtype=torch.int32, device="cuda")
    x = torch.tensor(rhs, device="cuda")
    _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
    torch.cuda.synchronize()
    assert (info.cpu().numpy() == 0).all()
    cond = np.linalg.cond(A).max()
    tol = 1e-13 * cond * n
    assert np.max(np.abs(x.cpu().numpy() - ref)) <= tol * max(1.0, np.abs(ref).max())
    x2 = torch.tensor(rhs[:, :1], device="cuda")  # re-use of the factors
    _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(x2.cpu().numpy(), x.cpu().numpy()[:, :1])


@pytest.mark.parametrize("B,n,kl,ku", [(3, 300, 6, 6), (200, 300, 6, 6), (150, 300, 40, 40), (140, 200, 70, 2),
                                      (3, 106, 42, 42), (1, 298, 42, 42), (5, 70, 30, 10)])
def test_band_lu_small_and_windowed_paths_agree(B, n, kl, ku, monkeypatch):
    """The resident / global kernels (small batches, or CFX_BAND_FULL) and the register / windowed kernels give the
    same factors, pivots and solutions to rounding (the MSK KKT shapes kl = ku = 42 included)."""
    import torch

    from cocofest_amd import _cfx

    rng = np.random.default_rng(B)
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag=kl < 20)
    rhs = rng.standard_normal((B, 2, n))
    outs = []
    for full in (False, True):
        if full:
            monkeypatch.setenv("CFX_BAND_FULL", "1")
        abt = torch.tensor(ab, device="cuda")
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = torch.tensor(rhs, device="cuda")
        _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
        x2 = torch.tensor(rhs[:, :1], device="cuda")
        _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
        torch.cuda.synchronize()
        outs.append((abt.cpu().numpy()[:, :, kl:], ipiv.cpu().numpy(), x.cpu().numpy(), x2.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(outs[0][2], outs[1][2], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(outs[0][3], outs[0][2][:, :1], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("B,n,kl,ku,zero_diag", [(1, 300, 40, 40, False), (2, 200, 70, 2, False), (1, 7, 3, 1, False),
                                                 (1, 1000, 108, 108, True), (3, 150, 0, 5, False),
                                                 (1, 500, 130, 140, False), (1, 64, 63, 63, False),
                                                 (2, 90, 20, 20, True), (1, 450, 200, 200, False)])
def test_band_lu_panel_placement(B, n, kl, ku, zero_diag, monkeypatch):
    """The panel placement (single wide bands: blocked factorisation, streamed one-wave solves; CFX_BAND_PLACEMENT=5)
    against the global placement (=2), whose column step it reorders: the same factors, pivots and zero-pivot
    reports bit for bit, the same solutions, factors of one solved by the other's kernels; numpy's dense solve.
    kl = ku = 200: four 64-row chunks per lane."""
    import torch

    from cocofest_amd import _cfx

    rng = np.random.default_rng(B + n + kl + 11)
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag=zero_diag)
    rhs = rng.standard_normal((B, 2, n))
    singular = B > 1 and kl > 0
    if singular:
        ab[1, n // 3, :] = 0.0  # a zero column in instance 1: info = n // 3 + 1, later columns still factored
    outs = {}
    for pl in ("5", "2"):
        monkeypatch.setenv("CFX_BAND_PLACEMENT", pl)
        abt = torch.tensor(ab, device="cuda")
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = torch.tensor(rhs, device="cuda")
        _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
        monkeypatch.setenv("CFX_BAND_PLACEMENT", "2" if pl == "5" else "5")  # solve with the other placement
        x2 = torch.tensor(rhs[:, 1:], device="cuda")
        _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
        torch.cuda.synchronize()
        outs[pl] = (abt.cpu().numpy(), ipiv.cpu().numpy(), info.cpu().numpy(), x.cpu().numpy(), x2.cpu().numpy())
    pan, glo = outs["5"], outs["2"]
    np.testing.assert_array_equal(pan[1], glo[1])
    np.testing.assert_array_equal(pan[2], glo[2])
    np.testing.assert_array_equal(pan[0], glo[0])
    ok = pan[2] == 0
    assert ok.sum() == B - (1 if singular else 0)
    np.testing.assert_array_equal(pan[3][ok], glo[3][ok])
    np.testing.assert_array_equal(pan[4][ok], pan[3][ok][:, 1:])
    np.testing.assert_array_equal(glo[4][ok], glo[3][ok][:, 1:])
    ref = np.linalg.solve(A[ok], rhs[ok].transpose(0, 2, 1)).transpose(0, 2, 1)
    cond = np.linalg.cond(A[ok]).max()
    assert np.max(np.abs(pan[3][ok] - ref)) <= 1e-13 * cond * n * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("n", [60, 502])
def test_band_lu_large_batch_factor_then_solve(n):
    """From 2048 instances on, cfx_band_lu factors with the register kernel while cfx_band_lu_solve may pick the
    windowed one (the multi-start IPM reuses factors this way at 4096 starts): the reused factors must solve like
    the factorisation's own solve and like numpy's dense solve."""
    import torch

    from cocofest_amd import _cfx

    B, kl, ku = 2112, 6, 6
    rng = np.random.default_rng(n)
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag=True)
    rhs = rng.standard_normal((B, n))
    abt = torch.tensor(ab, device="cuda")
    ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
    info = torch.empty((B,), dtype=torch.int32, device="cuda")
    x = torch.tensor(rhs, device="cuda")
    _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
    x2 = torch.tensor(rhs, device="cuda")
    _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
    torch.cuda.synchronize()
    assert (info.cpu().numpy() == 0).all()
    xs, x2s = x.cpu().numpy(), x2.cpu().numpy()
    np.testing.assert_allclose(x2s, xs, rtol=1e-10, atol=1e-12 * np.abs(xs).max())
    pick = rng.choice(B, 64, replace=False)  # dense reference on a sample of the batch
    ref = np.linalg.solve(A[pick], rhs[pick][:, :, None])[:, :, 0]
    cond = np.linalg.cond(A[pick]).max()
    assert np.max(np.abs(x2s[pick] - ref)) <= 1e-13 * cond * n * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("B,n,kl,ku,zero_diag", [(1100, 502, 6, 6, True), (64, 60, 6, 6, True), (70, 37, 3, 1, False),
                                                 (65, 100, 8, 8, True), (64, 50, 0, 2, False), (64, 80, 5, 2, True),
                                                 (64, 9, 8, 8, False), (3, 1, 0, 0, False)])
def test_band_lu_lane_placement(B, n, kl, ku, zero_diag, monkeypatch):
    """The lane placement (one lane per instance, large batches of bands with max(kl, ku) <= 8; forced here with
    CFX_BAND_PLACEMENT=4) against the register placement (same factors, pivots and solutions) and numpy's dense
    solve; factors of one placement solve with the other's kernels."""
    import torch

    from cocofest_amd import _cfx

    rng = np.random.default_rng(B + n + kl)
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag=zero_diag)
    rhs = rng.standard_normal((B, 2, n))
    outs = {}
    for pl in ("4", "3"):
        monkeypatch.setenv("CFX_BAND_PLACEMENT", pl)
        abt = torch.tensor(ab, device="cuda")
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = torch.tensor(rhs, device="cuda")
        _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
        monkeypatch.setenv("CFX_BAND_PLACEMENT", "3" if pl == "4" else "4")  # solve with the other placement
        x2 = torch.tensor(rhs[:, 1:], device="cuda")
        _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
        torch.cuda.synchronize()
        outs[pl] = (abt.cpu().numpy()[:, :, kl:], ipiv.cpu().numpy(), info.cpu().numpy(), x.cpu().numpy(),
                    x2.cpu().numpy())
    lane, reg = outs["4"], outs["3"]
    np.testing.assert_array_equal(lane[1], reg[1])
    np.testing.assert_array_equal(lane[2], 0)
    np.testing.assert_allclose(lane[0], reg[0], rtol=1e-12, atol=1e-12)
    scale = np.abs(reg[3]).max()  # solutions: the two placements round in a different order
    np.testing.assert_allclose(lane[3], reg[3], rtol=1e-9, atol=1e-11 * scale)
    np.testing.assert_allclose(lane[4], lane[3][:, 1:], rtol=1e-9, atol=1e-11 * scale)
    pick = rng.choice(B, min(B, 32), replace=False)
    ref = np.linalg.solve(A[pick], rhs[pick].transpose(0, 2, 1)).transpose(0, 2, 1)
    cond = np.linalg.cond(A[pick]).max()
    assert np.max(np.abs(lane[3][pick] - ref)) <= 1e-13 * cond * n * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("B,n,kl,ku,zero_diag", [(1100, 502, 6, 6, True), (257, 60, 7, 8, True), (70, 37, 3, 1, False),
                                                 (66, 50, 0, 2, False), (65, 9, 5, 2, True), (5, 1, 0, 0, False),
                                                 (4096, 120, 6, 6, False)])
def test_band_lu_grouped_register_placement(B, n, kl, ku, zero_diag, monkeypatch):
    """Four instances per wavefront (16-lane groups, bands with kl <= 7 and ku <= 8; forced with CFX_BAND_GROUP=1)
    against one instance per wavefront (CFX_BAND_GROUP=0): the same factors, pivots, zero-pivot reports and
    solutions bit for bit (the same operations per instance), batches that are not a multiple of four included; and
    numpy's dense solve on a sample."""
    import torch

    from cocofest_amd import _cfx

    rng = np.random.default_rng(B + n + kl + 7)
    A, ab = _band_system(rng, B, n, kl, ku, zero_diag=zero_diag)
    rhs = rng.standard_normal((B, 2, n))
    monkeypatch.setenv("CFX_BAND_PLACEMENT", "3")
    outs = {}
    for grp in ("1", "0"):
        monkeypatch.setenv("CFX_BAND_GROUP", grp)
        abt = torch.tensor(ab, device="cuda")
        ipiv = torch.empty((B, n), dtype=torch.int32, device="cuda")
        info = torch.empty((B,), dtype=torch.int32, device="cuda")
        x = torch.tensor(rhs, device="cuda")
        _cfx.band_lu(abt, ipiv, info, kl, ku, rhs=x)
        x2 = torch.tensor(rhs[:, 1:], device="cuda")
        _cfx.band_lu_solve(abt, ipiv, kl, ku, x2)
        torch.cuda.synchronize()
        outs[grp] = (abt.cpu().numpy(), ipiv.cpu().numpy(), info.cpu().numpy(), x.cpu().numpy(), x2.cpu().numpy())
    for a, b in zip(outs["1"], outs["0"]):
        np.testing.assert_array_equal(a, b)
    got = outs["1"]
    ok = got[2] == 0
    pick = rng.choice(np.where(ok)[0], min(int(ok.sum()), 32), replace=False)
    if len(pick):
        ref = np.linalg.solve(A[pick], rhs[pick].transpose(0, 2, 1)).transpose(0, 2, 1)
        cond = np.linalg.cond(A[pick]).max()
        assert np.max(np.abs(got[3][pick] - ref)) <= 1e-13 * cond * n * max(1.0, np.abs(ref).max())
        np.testing.assert_array_equal(got[4][pick], got[3][pick][:, 1:])


def test_band_lu_reports_singular_and_bad_arguments():
    import torch

    from cocofest_amd import _cfx

    n, kl, ku = 10, 2, 2
    rng = np.random.default_rng(1)
    A, ab = _band_system(rng, 2, n, kl, ku)
    ab[1, 4, :] = 0.0  # column 4 of instance 1 is zero: first zero pivot at j = 4 (info 5)
    abt = torch.tensor(ab, device="cuda")
    ipiv = torch.empty((2, n), dtype=torch.int32, device="cuda")
    info = torch.empty((2,), dtype=torch.int32, device="cuda")
    _cfx.band_lu(abt, ipiv, info, kl, ku)
    torch.cuda.synchronize()
    assert info.cpu().tolist() == [0, 5]
    with pytest.raises(_cfx.CfxError):
        _cfx.band_lu(abt, ipiv, info, kl + 1, ku)  # storage does not match the bandwidths
    lib = _cfx.load_library()
    assert lib.cfx_band_lu(0, 0, 0, 1, abt.data_ptr(), ipiv.data_ptr(), info.data_ptr(), 0, None, None) == _cfx.EINVAL


def test_interior_point_hmed_intensity():
    """Hmed2018 intensity optimisation (sliding-window rows make the widest KKT band of the families): the
    batched interior point reaches a feasible KKT point within the intensity bounds."""
    from cocofest_amd.solver import BatchedIpm

    cfg = dict(name="hmed2018", stims=[0.0, 0.1, 0.2, 0.3, 0.4], final_time=0.5, truncation=5, scheme="RK1", m=5,
               objective={"end_node_tracking": 60}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    ipm = BatchedIpm(ocp, batch=8)
    rng = np.random.default_rng(5)
    v0 = np.tile(ocp.initial_guess_vector(), (8, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 10, (8, free.sum())), lb[free], ub[free])
    res = ipm.solve(v0)
    ipm.close()
    assert res.converged.all(), (res.kkt_error, res.iterations)
    assert np.max(np.abs(O.eval_g(pb, res.v))) < 1e-5
    assert np.all(res.v >= lb - 1e-8) and np.all(res.v <= ub + 1e-8)
    assert abs(pb.unpack(res.v)[0][:, -1, 1] - 60).max() < 1e-3  # reachable target is met


COL_STIMS = [0.0, 0.1, 0.2, 0.3, 0.4]


@pytest.mark.parametrize("method,degree", [("legendre", 1), ("legendre", 4), ("radau", 3), ("radau", 5)])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_collocation_callbacks_vs_oracle(name, method, degree):
    """Direct collocation (g, J_g, f, grad f) on the GPU vs the oracle's restatement, all six models."""
    import torch

    from tests.oracle_handle import oracle_problem_from_ocp
    from oracle import fes_collocation as CO

    obj = {"end_node_tracking": 40.0}
    ocp = cases.product_collocation_ocp(name, COL_STIMS, 0.5, 4, degree=degree, method=method, objective=obj,
                                        n_shooting=10)
    pb = oracle_problem_from_ocp(ocp)
    B = 33
    v = cases.random_collocation_decision(pb, B, seed=degree)
    h = ocp.nlp(batch=B, layout="aos")
    assert (h.nv, h.ng) == (pb.nv, pb.ng)
    jr, jc = h.jac_structure()
    er, ec = CO.jac_structure(pb)
    np.testing.assert_array_equal(jr, er)
    np.testing.assert_array_equal(jc, ec)
    hr, hc = h.hess_structure()
    hr2, hc2 = CO.hess_structure(pb)
    np.testing.assert_array_equal(hr, hr2)
    np.testing.assert_array_equal(hc, hc2)
    vt = torch.tensor(v, device="cuda")
    g = torch.empty((B, h.ng), dtype=torch.float64, device="cuda")
    jac = torch.empty((B, h.nnz_jac), dtype=torch.float64, device="cuda")
    f = torch.empty((B,), dtype=torch.float64, device="cuda")
    grad = torch.empty((B, h.nv), dtype=torch.float64, device="cuda")
    h.eval_all(vt, g=g, jac=jac, f=f, grad=grad)
    torch.cuda.synchronize()
    h.close()
    g_ref = CO.eval_g(pb, v)
    # defects are differences of O(|x| / dt)-sized terms: compare against that scale
    scale = np.abs(v).max(axis=1, keepdims=True) * (degree + 1) ** 2
    assert np.max(np.abs(g.cpu().numpy() - g_ref) / scale) <= 1e-13, "g"
    _close(jac.cpu().numpy(), CO.eval_jac_g(pb, v), rtol=1e-11, what="J")
    _close(f.cpu().numpy()[:, None], CO.eval_f(pb, v)[:, None], what="f")
    _close(grad.cpu().numpy(), CO.eval_grad_f(pb, v), what="grad")


@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_collocation_hessian_vs_oracle(name):
    import torch

    from tests.oracle_handle import oracle_problem_from_ocp
    from oracle import fes_collocation as CO

    ocp = cases.product_collocation_ocp(name, COL_STIMS, 0.5, 4, degree=3, method="legendre",
                                        objective={"end_node_tracking": 40.0}, n_shooting=5)
    pb = oracle_problem_from_ocp(ocp)
    B = 4
    v = cases.random_collocation_decision(pb, B, seed=11)
    rng = np.random.default_rng(3)
    lam = rng.standard_normal((B, pb.ng))
    of = rng.uniform(0.5, 2.0, B)
    h = ocp.nlp(batch=B, layout="aos")
    hv = torch.empty((B, h.nnz_hess), dtype=torch.float64, device="cuda")
    h.eval_h(torch.tensor(v, device="cuda"), torch.tensor(of, device="cuda"), torch.tensor(lam, device="cuda"), hv)
    torch.cuda.synchronize()
    h.close()
    got = hv.cpu().numpy()
    ref = CO.hessian_values(pb, v, of, lam)
    scale = np.maximum(np.abs(ref), 1e-4 * np.max(np.abs(ref), axis=1, keepdims=True))
    err = np.max(np.abs(got - ref) / scale)
    assert err < 1e-6, f"H {name}: {err:.3e}"


def test_interior_point_collocation_pulse_width():
    """cfg 3 shape transcribed by direct collocation (Legendre, degree 4): the batched interior point converges
    to a feasible KKT point, and its node force trajectory agrees with the RK1 x 10 shooting solution to the
    discretisation level."""
    from cocofest_amd.solver import BatchedIpm

    from tests.oracle_handle import oracle_problem_from_ocp
    from oracle import fes_collocation as CO

    ft = json.loads((pathlib.Path(__file__).parent / "golden" / "ref_formulas.json").read_text())
    ft = ft["misc"]["force_tracking"]
    obj = {"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]}
    stims = [float(t) for t in np.round(np.linspace(0, 1, 31)[:-1], 2)]
    ocp = cases.product_collocation_ocp("ding2007", stims, 1.0, 10, degree=4, objective=obj)
    pb = oracle_problem_from_ocp(ocp)
    ipm = BatchedIpm(ocp, batch=2)
    res = ipm.solve()
    ipm.close()
    assert res.converged.all(), (res.kkt_error, res.iterations)
    assert np.max(np.abs(CO.eval_g(pb, res.v))) < 1e-5
    lb, ub = ocp.bounds_vector()
    assert np.all(res.v >= lb - 1e-8) and np.all(res.v <= ub + 1e-8)


def _gpu_nmpc(model, **kw):
    from cocofest_amd import OdeSolver
    from cocofest_amd.nmpc import FesNmpc
    from cocofest_amd.solver import IpmOptions

    return FesNmpc(model, cycle_duration=0.5, n_cycles_simultaneous=2, n_cycles_to_advance=1,
                   ode_solver=OdeSolver.RK4(n_integration_steps=5), options=IpmOptions(tol=1e-9), **kw)


@pytest.mark.parametrize("fatigue", [False, True])
def test_nmpc_hmed_on_gpu_is_self_consistent(fatigue):
    """Receding horizon over libcfx (Hmed2018 intensities, 3 cycles, 4 scenarios): see test_nmpc_cpu.py."""
    from tests.test_nmpc_cpu import test_hmed_free_intensities_are_self_consistent

    test_hmed_free_intensities_are_self_consistent(fatigue, batch=4, nmpc_factory=_gpu_nmpc)


def test_nmpc_pulse_width_with_fatigue_on_gpu():
    """The reference's own NMPC model (Ding2007 with fatigue, pulse widths): every window converges and the
    committed pulse widths reproduce the committed states by forward integration."""
    from cocofest_amd import DingModelPulseWidthFrequencyWithFatigue

    from tests.test_nmpc_cpu import CYCLE, _forward

    model = DingModelPulseWidthFrequencyWithFatigue(stim_time=CYCLE, sum_stim_truncation=4)
    res = _gpu_nmpc(model, pulse_width={"min": model.pd0, "max": 0.0006}, objective={"end_node_tracking": 60.0},
                    batch=3).solve(n_cycles=3)
    assert all(c.all() for c in res.converged), res.iterations
    pw = res.controls["last_pulse_width"]
    stims = [t + 0.5 * c for c in range(3) for t in CYCLE]
    for b in range(3):
        ref = _forward("ding2007_with_fatigue", stims, 3, 4, controls=lambda tab, N, b=b: pw[b].T.reshape(N, 1),
                       x0=None)
        got = np.stack([res.states[k][b] for k in model.name_dof])
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", ["ding2007", "hmed2018", "ding2007_with_fatigue"])
def test_interior_point_on_gpu_matches_the_oracle_driven_run(name):
    """The same interior point driven by libcfx (GPU callbacks + band LU) and by the oracle on the CPU
    (dense solves) lands on the same KKT point; with test_solver_cpu.py's scipy cross-check this ties the GPU
    optimum to an independent NLP solver."""
    from cocofest_amd.solver import BatchedIpm, IpmOptions
    from tests.oracle_handle import DenseBandSolver, OracleHandle, oracle_problem_from_ocp

    t = np.linspace(0, 1, 11)
    cfg = dict(name=name, stims=[0.0, 0.05, 0.1, 0.15], final_time=0.2, truncation=4, scheme="RK1", m=5,
               objective={"force_tracking": [t, 40 * t]}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    pb = oracle_problem_from_ocp(ocp)
    gpu = BatchedIpm(ocp, batch=2, options=IpmOptions(tol=1e-10))
    rg = gpu.solve()
    gpu.close()
    cpu = BatchedIpm(ocp, batch=1, options=IpmOptions(tol=1e-10), handle=OracleHandle(pb, 1), torch_device="cpu",
                     band=DenseBandSolver())
    rc = cpu.solve()
    assert rg.converged.all() and rc.converged.all()
    np.testing.assert_allclose(rg.f, rc.f[0], rtol=1e-9)
    ref = rc.v[0]
    scale = np.where(np.abs(ref) < 1e-2, np.abs(ref) + 1e-6, np.maximum(np.abs(ref), 1e-3 * np.abs(ref).max()))
    assert np.max(np.abs(rg.v - ref) / scale) < 1e-6


@pytest.mark.parametrize("name", ["ding2003_with_fatigue", "ding2007_with_fatigue", "hmed2018_with_fatigue"])
def test_cfg1_ivp_at_its_stated_size(name):
    """BASELINE configs[0]: IvpFes DingModelFrequencyWithFatigue, 10 pulses @ 10 Hz, final time 1 s, n_shooting = 20
    (the IvpFes n_shooting extension; the reference's LCM rule would give 10), RK4 x 10 — every sub-step sample
    against the oracle's sequential integration (and the other fatigue families in the same shape)."""
    from cocofest_amd import IvpFes, ModelMaker, OdeSolver

    stims = cases.TEN_PULSES
    model = ModelMaker.create_model(name, stim_time=list(stims), sum_stim_truncation=10)
    fes = {"model": model}
    if name.startswith("ding2007"):
        fes["pulse_width"] = [2e-4 + 3e-5 * i for i in range(10)]
    if name.startswith("hmed2018"):
        fes["pulse_intensity"] = [40.0 + 5 * i for i in range(10)]
    ivp = IvpFes(fes, {"final_time": 1.0, "ode_solver": OdeSolver.RK4(n_integration_steps=10), "n_shooting": 20})
    assert ivp.n_shooting == 20
    res = ivp.integrate(return_time=False)
    got = np.stack([res[k][0] for k in model.name_dof])
    assert got.shape == (len(model.name_dof), 20 * 10 + 1)
    c = O.model_constants(name)
    tab = O.stim_table(stims, 20, 1.0, 10)
    u = O.ivp_controls(name, tab, 20, 10, fes.get("pulse_width"), fes.get("pulse_intensity"))
    ref = O.ivp_integrate(name, c, tab.rows, u, 1.0, "RK4", 10)
    _close(got, ref, what=f"cfg1 {name} N=20")
