"""Direct collocation on the GPU at every launch shape, and the fused g + J_g + Hessian launch (round 4).

The collocation g + J_g kernel (cfx_colloc.h k_colloc) runs `intervals_per_thread` consecutive intervals per thread
(the start state x^0 of interval k + 1 carried from interval k's continuity row), orders its grid intervals-fast, and
moves one or two adjacent instances per lane, on SoA or 64-instance tiles (CFX_LAYOUT_TILED64); cfx_eval_all_h writes
g, J_g and the Lagrangian Hessian from ONE launch (k_colloc_hess<GJ>: task 0 of each interval runs the g + J_g body
beside its Hessian block).  Every shape is forced through cfx_create's overrides (CFX_KPT, CFX_IFAST, CFX_NI) and
compared bit for bit with the trivial shape (one interval per thread, one instance per lane, SoA), which is compared
with the oracle's restatement (oracle/fes_collocation.py; relative 1e-11 as tests/test_gpu_parity.py).  bioptim's own
collocation output is not available: parity with it is unpinned.
Reference: cocofest/optimization/fes_ocp.py:334-338 (OdeSolver.COLLOCATION accepted by OcpFes)."""

import numpy as np
import pytest

from tests import cases
from tests.test_gpu_parity import COL_STIMS, _close
from tests.test_launch_shapes import ENV, _run, _tile, _untile

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _clean_env(monkeypatch):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    from cocofest_amd import _cfx

    if _cfx.load_library().cfx_device_count() < 1:
        pytest.fail("no HIP device visible to libcfx")


def _col(name, degree, method, n_shooting=10):
    from tests.oracle_handle import oracle_problem_from_ocp

    obj = {"end_node_tracking": 40.0} if name != "ding2003" else {"end_node_tracking": 40.0}
    ocp = cases.product_collocation_ocp(name, COL_STIMS, 0.5, 4, degree=degree, method=method, objective=obj,
                                        n_shooting=n_shooting)
    return ocp, oracle_problem_from_ocp(ocp)


KPTS = [1, 2, 4, 5, 10]


def _close_col_g(v, g, g_ref, degree, what):
    """Defects are differences of O(|x| / dt)-sized terms: compare against that scale (as test_gpu_parity.py)."""
    scale = np.abs(v).max(axis=1, keepdims=True) * (degree + 1) ** 2
    assert np.max(np.abs(g - g_ref) / scale) <= 1e-13, what


@pytest.mark.parametrize("degree,method", [(3, "legendre"), (4, "legendre"), (2, "radau"), (6, "legendre")])
@pytest.mark.parametrize("name", ["ding2003", "ding2003_with_fatigue", "ding2007", "ding2007_with_fatigue",
                                  "hmed2018", "hmed2018_with_fatigue"])
def test_collocation_launch_shapes_are_bitwise_identical(name, degree, method, monkeypatch):
    from oracle import fes_collocation as CO

    ocp, pb = _col(name, degree, method)
    assert pb.n_shooting == 10
    B = 1152  # 18 tiles; partial last instance blocks at one and two instances per lane
    v = cases.random_collocation_decision(pb, B, seed=degree)
    (g_ref, j_ref), shape = _run(ocp, v, "soa", monkeypatch, {"CFX_KPT": 1, "CFX_IFAST": 0, "CFX_NI": 1})
    assert (shape["intervals_per_thread"], shape["intervals_fast"], shape["instances_per_lane"]) == (1, 0, 1)
    pick = np.array([0, 1, 63, 64, 255, 256, 511, 512, 700, 1023, 1024, B - 2, B - 1])
    _close_col_g(v[pick], g_ref[pick], CO.eval_g(pb, v[pick]), degree, f"colloc g {name} {degree}")
    _close(j_ref[pick], CO.eval_jac_g(pb, v[pick]), what=f"colloc J {name} {degree}")
    pairs = not name.startswith("hmed") and degree <= 5  # two instances per lane: Ding families, degrees 1..5
    seen = set()
    for layout in ("soa", "tiled64"):
        for ni in (1, 2):
            for kpt in KPTS:
                for ifast in (0, 1):
                    env = {"CFX_KPT": kpt, "CFX_IFAST": ifast, "CFX_NI": ni}
                    (g, j), shape = _run(ocp, v, layout, monkeypatch, env)
                    want_ni = ni if pairs else 1
                    assert (shape["intervals_per_thread"], shape["intervals_fast"], shape["instances_per_lane"]) == \
                        (kpt, ifast, want_ni), (env, shape)
                    np.testing.assert_array_equal(g, g_ref, err_msg=f"g {layout} {env}")
                    np.testing.assert_array_equal(j, j_ref, err_msg=f"J {layout} {env}")
                    (g0, _), _ = _run(ocp, v, layout, monkeypatch, env, g_only=True)
                    np.testing.assert_array_equal(g0, g_ref, err_msg=f"g-only {layout} {env}")
                    seen.add((layout, want_ni, kpt, ifast))
    assert len(seen) == 2 * (2 if pairs else 1) * len(KPTS) * 2


def _fused(ocp, v, lam, of, layout):
    """(g, J, H) of eval_all + eval_h and of the fused eval_all_h, instance-major, through device buffers."""
    import torch

    B = v.shape[0]
    h = ocp.nlp(batch=B, layout=layout)
    if layout == "tiled64":
        conv, back = (lambda a: torch.tensor(_tile(a), device="cuda")), (lambda t: _untile(t.cpu().numpy()))
        mk = lambda n: torch.empty((B // 64, n, 64), dtype=torch.float64, device="cuda")  # noqa: E731
        dof = torch.tensor(_tile(of[:, None]), device="cuda")
    else:
        conv, back = (lambda a: torch.tensor(np.ascontiguousarray(a.T), device="cuda")), (lambda t: t.cpu().numpy().T)
        mk = lambda n: torch.empty((n, B), dtype=torch.float64, device="cuda")  # noqa: E731
        dof = torch.tensor(of, device="cuda")
    dv, dl = conv(v), conv(lam)
    g, j, hh = mk(h.ng), mk(h.nnz_jac), mk(h.nnz_hess)
    h.eval_all(dv, g=g, jac=j)
    h.eval_h(dv, dof, dl, hh)
    fg, fj, fh = mk(h.ng), mk(h.nnz_jac), mk(h.nnz_hess)
    h.eval_all_h(dv, dof, dl, g=fg, jac=fj, hess=fh)
    torch.cuda.synchronize()
    out = [back(t) for t in (g, j, hh, fg, fj, fh)]
    h.close()
    return out


@pytest.mark.parametrize("name", ["ding2003", "ding2003_with_fatigue", "ding2007", "ding2007_with_fatigue",
                                  "hmed2018", "hmed2018_with_fatigue"])
def test_collocation_fused_launch_matches_the_separate_callbacks(name):
    """cfx_eval_all_h on collocation handles is one launch whose g and J_g are eval_all's bits and whose Hessian is
    eval_h's bits, on SoA and on 64-instance tiles (the tiled Hessian equal to the SoA one), and within the oracle's
    tolerance."""
    from oracle import fes_collocation as CO

    ocp, pb = _col(name, 4, "legendre", n_shooting=5)
    B = 128
    v = cases.random_collocation_decision(pb, B, seed=5)
    rng = np.random.default_rng(9)
    lam, of = rng.standard_normal((B, pb.ng)), rng.uniform(0.5, 2.0, B)
    res = {lay: _fused(ocp, v, lam, of, lay) for lay in ("soa", "tiled64")}
    for lay, (g, j, hh, fg, fj, fh) in res.items():
        np.testing.assert_array_equal(fg, g, err_msg=f"{lay} g")
        np.testing.assert_array_equal(fj, j, err_msg=f"{lay} J")
        np.testing.assert_array_equal(fh, hh, err_msg=f"{lay} H")
    for a, b in zip(res["soa"], res["tiled64"]):
        np.testing.assert_array_equal(a, b)
    g, j, hh = res["soa"][:3]
    pick = np.array([0, 1, 63, 64, 100, B - 1])
    _close_col_g(v[pick], g[pick], CO.eval_g(pb, v[pick]), 4, f"fused colloc g {name}")
    _close(j[pick], CO.eval_jac_g(pb, v[pick]), what=f"fused colloc J {name}")


def test_bench_shape_collocation():
    """bench.py's collocation launches: cfg 2 by direct collocation (Legendre degree 4), B = 2^18, SoA (the roofline
    line) and 64-instance tiles (timed beside it), the handle's default shape, on the bench's synthetic batch: sampled
    instances bit for bit against a small AoS handle (trivial shape) and against the oracle."""
    import torch

    import bench
    from oracle import fes_collocation as CO
    from tests.oracle_handle import oracle_problem_from_ocp
    from tests.test_launch_shapes import _picks

    ocp = bench.build_collocation()
    pb = oracle_problem_from_ocp(ocp)
    B = bench.COLLOCATION_BATCH
    vt = bench.collocation_synthetic(ocp, B, device="cuda:0")
    pick = _picks(B, n_random=24)
    t, e = pick // 64, pick % 64
    vp = vt[t, :, e].cpu().numpy()
    small = ocp.nlp(batch=len(pick), layout="aos")
    g_ref, j_ref = small.eval_g(vp), small.eval_jac_g(vp)
    small.close()
    _close_col_g(vp, g_ref, CO.eval_g(pb, vp), 4, "bench colloc g")
    _close(j_ref, CO.eval_jac_g(pb, vp), what="bench colloc J")
    for layout in ("tiled64", "soa"):
        h = ocp.nlp(batch=B, layout=layout)
        shape = h.launch_shape()
        assert shape["instances_per_lane"] == 2, (layout, shape)
        if layout == "tiled64":
            g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
            j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
            h.eval_all(vt, g=g, jac=j)
            torch.cuda.synchronize()
            gp, jp = g[t, :, e].cpu().numpy(), j[t, :, e].cpu().numpy()
        else:
            v = vt.transpose(1, 2).reshape(B, h.nv).T.contiguous()
            g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
            j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
            h.eval_all(v, g=g, jac=j)
            torch.cuda.synchronize()
            idx = torch.as_tensor(pick, device="cuda")
            gp, jp = g[:, idx].T.cpu().numpy(), j[:, idx].T.cpu().numpy()
            del v
        h.close()
        del g, j
        np.testing.assert_array_equal(gp, g_ref)
        np.testing.assert_array_equal(jp, j_ref)


@pytest.mark.parametrize("name,degree", [("ding2003", 4), ("ding2007_with_fatigue", 3), ("hmed2018", 2)])
def test_collocation_keep_constant(name, degree):
    """The constant collocation J_g values (cfx_jac_constant_mask): the basis coefficients C[i][j] off the point's own
    state, the whole calcium row (its right-hand side (cs - cn) / tau_c is linear in cn), the continuity values D[i]
    and the -1 — 48 of 56 per interval for Ding2003 at degree 4.  With CFX_KEEP_CONSTANT_JAC the g + J_g launch (two
    instances per lane where it applies) and the fused g + J_g + Hessian launch leave them in place and write every
    other value bit for bit (tests/test_constant_jac.py's check); the mask's values equal the oracle's."""
    import torch

    from oracle import fes_collocation as CO
    from tests.test_constant_jac import _keep_check

    ocp, pb = _col(name, degree, "legendre")
    B = 256
    h = ocp.nlp(batch=B, layout="soa")
    mask = h.jac_constant_mask()
    N = pb.n_shooting
    if name == "ding2003":
        assert (h.nnz_jac // N, int(mask.sum()) // N) == (56, 48)
    v1, v2 = (cases.random_collocation_decision(pb, B, seed=s) for s in (5, 6))
    d1, d2 = (torch.tensor(np.ascontiguousarray(v.T), device="cuda") for v in (v1, v2))

    def full(j, v=d2):
        j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda") if j is None else j
        h.eval_all(v, jac=j)
        return j

    def keep(j):
        h.eval_all(d2, jac=j, keep_constant_jac=True)

    a = _keep_check(h, full, keep, mask)
    b = full(None, d1).cpu().numpy()
    np.testing.assert_array_equal(a[mask], b[mask])  # constant over instances and points
    np.testing.assert_array_equal(a[mask], np.broadcast_to(a[mask][:, :1], a[mask].shape))
    _close(a[:, :3].T, CO.eval_jac_g(pb, v2[:3]), what=f"colloc J {name} {degree}")
    of = torch.linspace(0.5, 1.5, B, dtype=torch.float64, device="cuda")
    lam = torch.randn((h.ng, B), dtype=torch.float64, device="cuda")

    def full_h(j):
        _, j, _ = h.eval_all_h(d2, of, lam, jac=j)
        return j

    def keep_h(j):
        h.eval_all_h(d2, of, lam, jac=j, keep_constant_jac=True)

    _keep_check(h, full_h, keep_h, mask)
    h.close()
