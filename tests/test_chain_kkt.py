"""The stage-chain KKT layout: block cyclic reduction of the block-tridiagonal KKT matrix (csrc/cfx_chain.hip,
cfx_btri_factor / cfx_btri_solve) and its use by the native interior point for single large OCPs (cfx_ipm's chain
grouping, CFX_IPM_KKT=chain|band).

* cfx_btri_* against numpy's dense solve on random block-tridiagonal systems whose diagonal blocks need row
  interchanges (node sizes 16..96, node counts that are not powers of two, several right-hand sides, batches);
* a singular pivot block is reported in info;
* the interior point with the chain layout lands on the band layout's KKT point (same convergence, decision vectors
  within 1e-6 of their range) on cfg 3, cfg 5 (MSK, RK4 x 5), collocation and Hmed with intensity parameters (the
  parameters go to the dense border), and on the 1,500-interval reaching task its first iterates equal the panel
  band factorisation's."""

import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu


def _system(B, M, sp, seed, pivoting=True):
    rng = np.random.default_rng(seed)
    D = rng.normal(size=(B, M, sp, sp)) + 2.0 * np.sqrt(sp) * np.eye(sp)
    if pivoting:  # rows permuted: the largest entry of each column is off the diagonal
        for b in range(B):
            for k in range(M):
                D[b, k] = D[b, k][rng.permutation(sp)]
    L = 0.3 * rng.normal(size=(B, M, sp, sp))
    U = 0.3 * rng.normal(size=(B, M, sp, sp))
    L[:, 0] = 0.0
    U[:, M - 1] = 0.0
    return D, L, U


def _dense(D, L, U, b):
    M, sp = D.shape[1], D.shape[2]
    A = np.zeros((M * sp, M * sp))
    for k in range(M):
        s = slice(k * sp, (k + 1) * sp)
        A[s, s] = D[b, k]
        if k > 0:
            A[s, (k - 1) * sp: k * sp] = L[b, k]
        if k < M - 1:
            A[s, (k + 1) * sp: (k + 2) * sp] = U[b, k]
    return A


def _btri(D, L, U, rhs):
    import torch

    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    B, M, sp = D.shape[:3]
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")  # noqa: E731
    dD, dL, dU, dr = t(D), t(L), t(U), t(rhs)
    work = torch.zeros(2 * B * M * sp * sp, dtype=torch.float64, device="cuda")
    scratch = torch.zeros_like(dr)
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert lib.cfx_btri_factor(B, M, sp, dD.data_ptr(), dL.data_ptr(), dU.data_ptr(), work.data_ptr(),
                               info.data_ptr(), st) == 0, lib.cfx_last_error(None)
    assert lib.cfx_btri_solve(B, M, sp, dD.data_ptr(), dL.data_ptr(), dU.data_ptr(), work.data_ptr(), rhs.shape[1],
                              dr.data_ptr(), scratch.data_ptr(), st) == 0, lib.cfx_last_error(None)
    torch.cuda.synchronize()
    return dr.cpu().numpy(), info.cpu().numpy()


@pytest.mark.parametrize("sp,M,B", [(16, 1, 1), (16, 2, 2), (16, 37, 3), (32, 64, 1), (48, 16, 2), (80, 33, 1),
                                    (96, 5, 2), (112, 9, 1), (128, 6, 1)])
def test_btri_matches_dense_solve(sp, M, B):
    D, L, U = _system(B, M, sp, seed=sp + M)
    rng = np.random.default_rng(1)
    nrhs = 3
    rhs = rng.normal(size=(B, nrhs, M * sp))
    x, info = _btri(D, L, U, rhs)
    assert np.all(info == 0)
    for b in range(B):
        A = _dense(D, L, U, b)
        ref = np.linalg.solve(A, rhs[b].T).T
        err = np.abs(x[b] - ref).max() / np.abs(ref).max()
        res = np.abs(x[b] @ A.T - rhs[b]).max() / (np.abs(A).max() * np.abs(x[b]).max())
        assert err < 1e-11 and res < 1e-14, (b, err, res)


def test_btri_wide_levels_at_sp96():
    """sp = 96 with M = 520 nodes: level 0 has 260 survivors, so its Schur updates take the variant with the right
    operand in L2 (k_chain_upd<96, false>, 74,496 B of LDS: above the 64 KiB default, raised like the staged variant's —
    ADVICE round 5); the solution is checked by its block residual (the dense matrix would be 20 GB)."""
    sp, M, B = 96, 520, 1
    D, L, U = _system(B, M, sp, seed=9)
    rng = np.random.default_rng(2)
    rhs = rng.normal(size=(B, 1, M * sp))
    x, info = _btri(D, L, U, rhs)
    assert np.all(info == 0)
    X = x[0, 0].reshape(M, sp)
    R = np.einsum("kij,kj->ki", D[0], X)
    R[1:] += np.einsum("kij,kj->ki", L[0, 1:], X[:-1])
    R[:-1] += np.einsum("kij,kj->ki", U[0, :-1], X[1:])
    res = np.abs(R.reshape(-1) - rhs[0, 0]).max() / (np.abs(D).max() * np.abs(X).max())
    assert res < 1e-14, res


def test_btri_reports_a_non_finite_pivot_block():
    """A pivot block of NaN has no finite pivot candidate in any column: reported singular at its first column, and the
    pivot search keeps its row indices in range (the empty search used to decode row 127)."""
    D, L, U = _system(2, 8, 16, seed=4)
    D[1, 5] = np.nan
    _, info = _btri(D, L, U, np.ones((2, 1, 8 * 16)))
    assert info[0] == 0 and info[1] == 5 * 16 + 1, info


def test_btri_reports_a_singular_pivot_block():
    D, L, U = _system(1, 8, 16, seed=3)
    D[0, 5] = 0.0  # node 5 is eliminated at level 0: its block has no pivot at all
    _, info = _btri(D, L, U, np.ones((1, 1, 8 * 16)))
    assert info[0] == 5 * 16 + 1, info


def _sym_system(B, M, sp, seed):
    """Symmetric indefinite block-tridiagonal systems shaped like the interior point's KKT nodes: each diagonal block
    [[H, J^T], [J, -1e-3 I]] with H symmetric indefinite and J of full row rank, couplings L_k = U_{k-1}^T."""
    rng = np.random.default_rng(seed)
    nr = sp // 3
    D = np.zeros((B, M, sp, sp))
    for b in range(B):
        for k in range(M):
            H = rng.normal(size=(sp - nr, sp - nr))
            H = H + H.T + rng.uniform(-2, 6) * np.eye(sp - nr)
            J = rng.normal(size=(nr, sp - nr))
            D[b, k, : sp - nr, : sp - nr] = H
            D[b, k, sp - nr:, : sp - nr] = J
            D[b, k, : sp - nr, sp - nr:] = J.T
            D[b, k, sp - nr:, sp - nr:] = -1e-3 * np.eye(nr)
    U = 0.5 * rng.normal(size=(B, M, sp, sp))
    U[:, M - 1] = 0.0
    L = np.zeros_like(U)
    L[:, 1:] = np.transpose(U[:, :-1], (0, 1, 3, 2))
    return D, L, U


@pytest.mark.parametrize("sp,M,B", [(16, 37, 2), (48, 16, 2), (80, 33, 1), (128, 6, 1)])
def test_btri_inertia_counts_negative_eigenvalues(sp, M, B):
    """cfx_btri_inertia after cfx_btri_factor: the number of negative eigenvalues of the symmetric system (Bunch-Kaufman
    LDL^T of every pivot block's inverse, summed over the reduction's levels) equals numpy's eigvalsh count."""
    import torch

    from cocofest_amd import _cfx

    lib = _cfx.load_library()
    D, L, U = _sym_system(B, M, sp, seed=sp + 7 * M)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")  # noqa: E731
    dD, dL, dU = t(D), t(L), t(U)
    work = torch.zeros(2 * B * M * sp * sp, dtype=torch.float64, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    neg = torch.full((B,), -7, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert lib.cfx_btri_factor(B, M, sp, dD.data_ptr(), dL.data_ptr(), dU.data_ptr(), work.data_ptr(),
                               info.data_ptr(), st) == 0, lib.cfx_last_error(None)
    assert lib.cfx_btri_inertia(B, M, sp, dD.data_ptr(), neg.data_ptr(), st) == 0, lib.cfx_last_error(None)
    torch.cuda.synchronize()
    assert np.all(info.cpu().numpy() == 0)
    got = neg.cpu().numpy()
    for b in range(B):
        A = _dense(D, L, U, b)
        ev = np.linalg.eigvalsh(A)
        assert np.abs(ev).min() > 1e-8 * np.abs(ev).max()  # well away from singular: the count is unambiguous
        assert got[b] == int((ev < 0).sum()), (b, got[b], int((ev < 0).sum()))


def _solve(ocp, B, v0, kkt, monkeypatch, **opt):
    from cocofest_amd.solver import IpmOptions, NativeIpm

    monkeypatch.setenv("CFX_IPM_KKT", kkt)
    ipm = NativeIpm(ocp, batch=B, options=IpmOptions(**{"tol": 1e-8, "max_iter": 500, **opt}))
    st = dict(ipm.ipm.stats())
    r = ipm.solve(v0)
    ipm.close()
    return r, st


def _compare(ocp, ra, rb, vtol=1e-6, it_slack=3):
    assert ra.converged.all() and rb.converged.all(), (ra.status, rb.status)
    assert np.all(np.abs(ra.iterations - rb.iterations) <= it_slack), (ra.iterations, rb.iterations)
    np.testing.assert_allclose(ra.f, rb.f, rtol=1e-8, atol=1e-10)
    lb, ub = ocp.bounds_vector()
    span = np.where(np.isfinite(ub - lb), ub - lb, np.maximum(np.abs(rb.v).max(0), 1.0))
    assert np.max(np.abs(ra.v - rb.v) / np.maximum(span, 1e-12)) < vtol


def _starts(ocp, B, seed):
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    if B > 1:
        rng = np.random.default_rng(seed)
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10.0),
                              lb[free], ub[free])
    return v0


@pytest.mark.parametrize("B", [1, 4])
def test_chain_layout_matches_band_cfg3(B, monkeypatch):
    import json
    import pathlib

    ft = json.loads((pathlib.Path(__file__).parent / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    ocp = cases.product_ocp(**dict(cases.cfg3(), objective={"force_tracking": [np.array(ft["time"]),
                                                                                 np.array(ft["force"])]}))
    v0 = _starts(ocp, B, 0)
    rc, sc = _solve(ocp, B, v0, "chain", monkeypatch)
    rb, sb = _solve(ocp, B, v0, "band", monkeypatch)
    # node = (Cn, F, pulse width) of one shooting node + its two continuity rows: 5 unknowns in 16-wide blocks
    assert sc["kkt_chain_nodes"] == 101 and sc["kkt_chain_sp"] == 16 and sb["kkt_chain_nodes"] == 0, sc
    _compare(ocp, rc, rb)


def test_chain_layout_matches_band_msk_cfg5(monkeypatch):
    from tests import msk_cases as MC

    ocp = MC.product_ocp(**MC.cfg5(m=5))
    v0 = _starts(ocp, 1, 0)
    rc, sc = _solve(ocp, 1, v0, "chain", monkeypatch, tol=1e-6, max_iter=1000)
    rb, _ = _solve(ocp, 1, v0, "band", monkeypatch, tol=1e-6, max_iter=1000)
    assert sc["kkt_chain_nodes"] == 11, sc
    # cfg 5's end-game crawl is sensitive to rounding: the same optimum, iterations may differ
    assert rc.converged.all() and rb.converged.all()
    np.testing.assert_allclose(rc.f, rb.f, rtol=1e-6)
    np.testing.assert_allclose(rc.f, 0.7520497, rtol=1e-5)


def test_chain_layout_matches_band_collocation(monkeypatch):
    stims = [float(t) for t in np.round(np.linspace(0, 1, 31)[:-1], 2)]
    t = np.linspace(0, 1, 21)
    ocp = cases.product_collocation_ocp("ding2007", stims, 1.0, 10, degree=4,
                                        objective={"force_tracking": [t, 60 * t]})
    v0 = _starts(ocp, 2, 4)
    rc, sc = _solve(ocp, 2, v0, "chain", monkeypatch, tol=1e-6)
    rb, _ = _solve(ocp, 2, v0, "band", monkeypatch, tol=1e-6)
    assert sc["kkt_chain_nodes"] > 0, sc
    _compare(ocp, rc, rb)


def test_chain_layout_with_parameter_border_hmed(monkeypatch):
    cfg = dict(name="hmed2018", stims=[0.0, 0.1, 0.2, 0.3, 0.4], final_time=0.5, truncation=5, scheme="RK1", m=5,
               objective={"end_node_tracking": 60}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    rng = np.random.default_rng(5)
    v0 = np.tile(ocp.initial_guess_vector(), (4, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 10, (4, free.sum())), lb[free], ub[free])
    rc, sc = _solve(ocp, 4, v0, "chain", monkeypatch)
    rb, _ = _solve(ocp, 4, v0, "band", monkeypatch)
    assert sc["kkt_chain_nodes"] > 0 and sc["kkt_border"] >= 5, sc
    # degenerate intensity valley (test_ipm_native.py): same f, intensities within 1e-4 of their range
    _compare(ocp, rc, rb, vtol=1e-4)


def test_chain_layout_reaching_task_first_iterates(monkeypatch):
    """The 1,500-interval reaching task (stored revision's conventions, from the stored fatigue optimum): chain layout
    by default (M = 1,501 nodes of 80 unknowns + a border of the marker and end rows); its first iterates equal the
    panel band factorisation's to 1e-9 of each variable's range."""
    from tests import test_reference_solution as R

    ocp = R.legacy_product("fatigue")
    X, U = R.trajectory(R.load("fatigue"))
    nz = ocp.nx + ocp.nu
    v0 = R.decision_vector(X, U[: len(R.MUSCLES)], nz)[None]
    out = {}
    for kkt in ("auto", "band"):
        r, st = _solve(ocp, 1, v0, kkt, monkeypatch, tol=1e-6, max_iter=3, bound_relax_factor=1e-8)
        out[kkt] = (r, st)
    (rc, sc), (rb, sb) = out["auto"], out["band"]
    print("chain", sc["kkt_chain_nodes"], sc["kkt_chain_sp"], sc["kkt_border"], "band", sb["kkt_kl"], sb["kkt_n"])
    assert sc["kkt_chain_nodes"] == R.N + 1 and sc["kkt_chain_sp"] == 80 and sc["kkt_border"] <= 32, sc
    assert sb["kkt_chain_nodes"] == 0
    lb, ub = ocp.bounds_vector()
    span = np.where(np.isfinite(ub - lb) & (ub > lb), ub - lb, np.maximum(1.0, np.abs(v0[0])))
    assert np.max(np.abs(rc.v - rb.v) / span) < 1e-9
    np.testing.assert_array_equal(rc.iterations, rb.iterations)


def test_inertia_test_reaches_the_curvature_tests_optimum(monkeypatch):
    """inertia_test=True (Ipopt's inertia correction from the chain's pivot-block inertias and the border's Schur
    complement) lands on the curvature test's KKT point: cfg 3 (batch 4, no border) and Hmed with its intensity
    parameters in the border (batch 4)."""
    import json
    import pathlib

    ft = json.loads((pathlib.Path(__file__).parent / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    ocp = cases.product_ocp(**dict(cases.cfg3(), objective={"force_tracking": [np.array(ft["time"]),
                                                                                 np.array(ft["force"])]}))
    v0 = _starts(ocp, 4, 0)
    ri, _ = _solve(ocp, 4, v0, "chain", monkeypatch, inertia_test=True)
    rc, _ = _solve(ocp, 4, v0, "chain", monkeypatch)
    _compare(ocp, ri, rc, it_slack=10)
    cfg = dict(name="hmed2018", stims=[0.0, 0.1, 0.2, 0.3, 0.4], final_time=0.5, truncation=5, scheme="RK1", m=5,
               objective={"end_node_tracking": 60}, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    rng = np.random.default_rng(5)
    v0 = np.tile(ocp.initial_guess_vector(), (4, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 10, (4, free.sum())), lb[free], ub[free])
    ri, si = _solve(ocp, 4, v0, "chain", monkeypatch, inertia_test=True)
    rc, _ = _solve(ocp, 4, v0, "chain", monkeypatch)
    assert si["kkt_border"] >= 5, si
    # the intensity valley is flat (test_ipm_native.py): a different regularisation path ends elsewhere on it, at the
    # same f (measured: intensities 1.4 % of their range apart)
    assert ri.converged.all() and rc.converged.all(), (ri.status, rc.status)
    np.testing.assert_allclose(ri.f, rc.f, rtol=1e-8, atol=1e-10)
