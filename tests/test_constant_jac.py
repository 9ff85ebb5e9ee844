"""Constant J_g values (cfx_jac_constant_mask) and CFX_KEEP_CONSTANT_JAC.

The -1 on x_{k+1} of every continuity row, and for the Ding families the calcium row's only entry dCn+/dCn0 (the
calcium state is affine in its start value, so its tangent is the host slope cna[m S]), depend on neither the instance
nor the point.  cfx_jac_constant_mask lists them; with CFX_KEEP_CONSTANT_JAC the g + J_g launches skip their stores and
the output buffer keeps the values of an earlier full evaluation.  Checked here:

* the mask's entries are constant over instances and points and equal -1 / cna (the oracle's Jacobian agrees: the
  continuity parity tests compare every J_g value), and it covers exactly 60 of cfg 2's 100 values per instance;
* a keep-constant evaluation writes every other value bit for bit as the full evaluation does and leaves the masked
  positions untouched (poisoned with NaN beforehand), on device buffers in SoA, 64-instance tiles (the headline
  launch at B = 2^20) and AoS, through the fused g + J_g + Hessian launch, and for a musculoskeletal handle;
* on host buffers the handle's own staging buffer carries the constants: the first keep-constant call evaluates in
  full, later ones reproduce the full evaluation.

Reference semantics: the continuity rows Phi(x_k, u_k) - x_{k+1} (cocofest/models/
ding2003.py:153-198 for the calcium ODE that makes dCn+/dCn0 point-independent).
"""

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases

pytestmark = pytest.mark.gpu

FAMILIES = ["ding2003", "ding2003_with_fatigue", "ding2007", "ding2007_with_fatigue", "hmed2018",
            "hmed2018_with_fatigue"]
STIMS = [0.0, 0.05, 0.1, 0.15, 0.2, 0.25, 0.3, 0.35, 0.4, 0.45]


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible to torch")
    return torch


def _problem(name, scheme):
    cfg = dict(name=name, stims=STIMS, final_time=0.5, truncation=4, scheme=scheme, m=5, objective=None,
               n_shooting=None)
    return cases.product_ocp(**cfg), cases.oracle_problem(**cfg)


def _keep_check(h, full_fn, keep_fn, mask_rows):
    """full_fn(jac) / keep_fn(jac) evaluate into a device J buffer; mask_rows: boolean index of the constant rows in
    that buffer's first axis-view (elements).  The keep-constant call must leave poisoned masked slots alone and
    write every other slot as the full call does."""
    torch = _torch()
    j_full = full_fn(None)
    j_keep = torch.full_like(j_full, float("nan"))
    keep_fn(j_keep)
    torch.cuda.synchronize()
    a, b = j_full.cpu().numpy(), j_keep.cpu().numpy()
    assert np.isnan(b[mask_rows]).all(), "keep-constant evaluation wrote a constant value"
    np.testing.assert_array_equal(b[~mask_rows], a[~mask_rows])
    # and over a buffer that holds the constants: the full result, bit for bit
    m = torch.as_tensor(mask_rows, device=j_full.device)
    j_keep[m] = j_full[m]
    keep_fn(j_keep)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(j_keep.cpu().numpy(), a)
    return a


@pytest.mark.parametrize("scheme", ["RK1", "RK4"])
@pytest.mark.parametrize("name", FAMILIES)
def test_mask_values_are_constant_and_keep_skips_only_them(name, scheme):
    torch = _torch()
    ocp, pb = _problem(name, scheme)
    B = 640
    h = ocp.nlp(batch=B, layout="soa")
    mask = h.jac_constant_mask()
    jr, jc = h.jac_structure()
    N, nx, nz = pb.n_shooting, pb.nx, pb.nx + pb.nu
    # -1 on x_{k+1} always; the calcium row's dCn+/dCn0 for the Ding families
    neg = (jc == (jr // (h.ng // N) + 1) * nz + jr % (h.ng // N)) & (jr % (h.ng // N) < nx)
    cal = (jr % (h.ng // N) == 0) & (jc == (jr // (h.ng // N)) * nz)
    want = neg | (cal if not name.startswith("hmed") else False)
    np.testing.assert_array_equal(mask, want)
    v1, v2 = cases.random_decision(pb, B, seed=5), cases.random_decision(pb, B, seed=6)
    d1 = torch.tensor(np.ascontiguousarray(v1.T), device="cuda")
    d2 = torch.tensor(np.ascontiguousarray(v2.T), device="cuda")
    mk = lambda: torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")  # noqa: E731

    def full(j, v=d2):
        j = mk() if j is None else j
        h.eval_all(v, jac=j)
        return j

    def keep(j):
        h.eval_all(d2, jac=j, keep_constant_jac=True)

    a = _keep_check(h, full, keep, mask)
    b = full(None, d1).cpu().numpy()
    # constant over instances and points
    np.testing.assert_array_equal(a[mask], b[mask])
    np.testing.assert_array_equal(a[mask], np.broadcast_to(a[mask][:, :1], a[mask].shape))
    assert np.all(a[neg] == -1.0)
    # and what the oracle says for a sample
    pick = [0, 333, B - 1]
    ref = O.eval_jac_g(pb, v2[pick])
    np.testing.assert_allclose(a[mask][:, pick].T, ref[:, mask], rtol=1e-11, atol=0)
    h.close()


def test_cfg2_headline_shape_keep_constant():
    """bench.py's headline launch (cfg 2, B = 2^20, 64-instance tiles, 4 intervals per thread, 2 instances per lane)
    with CFX_KEEP_CONSTANT_JAC: 60 of the 100 values per instance are constant and left in place."""
    torch = _torch()
    import bench

    ocp = bench.build_problem()
    B = 1 << 20
    v = bench.to_tiled(bench.synthetic_soa(ocp, B, seed=1234, device="cuda:0"))
    h = ocp.nlp(batch=B, layout="tiled64")
    mask = h.jac_constant_mask()
    assert (h.nnz_jac, int(mask.sum())) == (100 * ocp.n_shooting // 20, 60 * ocp.n_shooting // 20)
    mk = lambda: torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")  # noqa: E731

    def full(j):
        j = mk() if j is None else j
        h.eval_all(v, jac=j)
        return j

    def keep(j):
        h.eval_all(v, jac=j, keep_constant_jac=True)

    torch.cuda.synchronize()
    j_full = full(None)
    j_keep = torch.full_like(j_full, float("nan"))
    keep(j_keep)
    torch.cuda.synchronize()
    m = torch.as_tensor(mask, device="cuda")
    assert bool(torch.isnan(j_keep[:, m, :]).all())
    assert bool(torch.equal(j_keep[:, ~m, :], j_full[:, ~m, :]))
    j_keep[:, m, :] = j_full[:, m, :]
    keep(j_keep)
    torch.cuda.synchronize()
    assert bool(torch.equal(j_keep, j_full))
    h.close()


@pytest.mark.parametrize("name", ["ding2003", "ding2007_with_fatigue", "hmed2018"])
def test_fused_g_jacobian_hessian_keep_constant(name):
    torch = _torch()
    ocp, pb = _problem(name, "RK4")
    B = 128
    h = ocp.nlp(batch=B, layout="soa")
    mask = h.jac_constant_mask()
    v = torch.tensor(np.ascontiguousarray(cases.random_decision(pb, B, seed=9).T), device="cuda")
    of = torch.linspace(0.5, 1.5, B, dtype=torch.float64, device="cuda")
    lam = torch.randn((h.ng, B), dtype=torch.float64, device="cuda")

    def full(j):
        _, j, _ = h.eval_all_h(v, of, lam, jac=j)
        return j

    def keep(j):
        h.eval_all_h(v, of, lam, jac=j, keep_constant_jac=True)

    _keep_check(h, full, keep, mask)
    h.close()


def test_aos_device_and_host_staging_keep_constant():
    """AoS outputs go through the handle's staging buffer: the first keep-constant call fills it in full, the later
    ones skip the constants there and still return every value."""
    torch = _torch()
    ocp, pb = _problem("ding2003_with_fatigue", "RK2")
    B = 200
    v = cases.random_decision(pb, B, seed=3)
    h = ocp.nlp(batch=B, layout="aos")
    ref = h.eval_jac_g(v)
    for _ in range(2):  # host path: staging buffer
        np.testing.assert_array_equal(h.eval_jac_g(v, keep_constant_jac=True), ref)
    jd = torch.full((B, h.nnz_jac), float("nan"), dtype=torch.float64, device="cuda")
    h.eval_all(torch.tensor(v, device="cuda"), jac=jd, keep_constant_jac=True)  # AoS device: staged as well
    torch.cuda.synchronize()
    np.testing.assert_array_equal(jd.cpu().numpy(), ref)
    h.close()


def test_msk_keep_constant():
    """cfg 5 (arm26, Ding2007 with fatigue): the -1 entries are the constant ones; the three-launch g + J_g path skips
    them under the flag."""
    torch = _torch()
    from tests import msk_cases as MC

    cfg = MC.cfg5()
    ocp = MC.product_ocp(**cfg)
    pb = MC.oracle_problem(**cfg)
    B = 96
    h = ocp.nlp(batch=B, layout="soa")
    mask = h.jac_constant_mask()
    assert int(mask.sum()) == pb.n_shooting * pb.nx
    V = MC.random_decision(pb, B, seed=4)
    dv = torch.tensor(np.ascontiguousarray(V.T), device="cuda")

    def full(j):
        j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda") if j is None else j
        h.eval_all(dv, jac=j)
        return j

    def keep(j):
        h.eval_all(dv, jac=j, keep_constant_jac=True)

    a = _keep_check(h, full, keep, mask)
    assert np.all(a[mask] == -1.0)
    h.close()

