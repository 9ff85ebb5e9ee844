"""The oracle itself, pinned against the reference's golden vectors and formula fixtures (CPU only)."""

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests.conftest import golden_stims


def test_oracle_reproduces_reference_ivp_goldens(ivp_goldens):
    """All 9 force trajectories of tests/shard1/test_ivp.py (8-decimal literals -> 5e-9 rounding)."""
    for case in ivp_goldens:
        name = case["model"]
        c = O.model_constants(name)
        stims = golden_stims(case["pulse_mode"], case["stim_time"])
        n = O.prepare_n_shooting(stims, case["final_time"])
        tab = O.stim_table(stims, n, case["final_time"], case["sum_stim_truncation"])
        u = O.ivp_controls(name, tab, n, case["sum_stim_truncation"], case["pulse_width"], case["pulse_intensity"])
        traj = O.ivp_integrate(name, c, tab.rows, u, case["final_time"], "RK4", 10)
        f = traj[1]
        if case["slice"]:
            f = f[case["slice"][0]: case["slice"][1]]
        np.testing.assert_allclose(f, case["F"], rtol=0, atol=6e-9, err_msg=case["source"])


def test_float_lookup_reproduces_documented_discrepancy(ivp_goldens):
    """The literal float lookup of ding2003.py:411 misses the 0.1/0.2 s pulses at T=0.3, N=3."""
    case = ivp_goldens[1]
    c = O.model_constants(case["model"])
    tab = O.stim_table([0, 0.1, 0.2], 3, 0.3, 3, lookup="float")
    traj = O.ivp_integrate(case["model"], c, tab.rows, np.zeros((3, 0)), 0.3)
    assert np.max(np.abs(traj[1] - case["F"])) > 10.0


def test_oracle_rhs_matches_reference_formulas(ref_formulas):
    for cs in ref_formulas["rhs"]:
        c = O.model_constants(cs["model"])
        u = np.array(cs["u"]) if cs["u"] else None
        dx = O.rhs(cs["model"], c, cs["t"], np.array(cs["x"]), u, np.array(cs["row"]))
        np.testing.assert_allclose(dx, cs["dxdt"], rtol=1e-14, atol=1e-300)


def test_oracle_tables_match_reference(ref_formulas):
    for tb in ref_formulas["tables"]:
        n = O.prepare_n_shooting(tb["stim_time"], tb["final_time"])
        assert n == tb["n_shooting"]
        tab = O.stim_table(tb["stim_time"], n, tb["final_time"], tb["truncation"], previous_stim=tb["previous_stim"])
        if tb["final_time"] == 0.3:  # the float-lookup case: the reference table itself differs (see above)
            continue
        np.testing.assert_array_equal(tab.rows, np.array(tb["rows"]))
        assert tab.stim_idx_at_node == tb["stim_idx_at_node"]


def test_oracle_misc_matches_reference(ref_formulas):
    m = ref_formulas["misc"]
    assert O.min_pulse_intensity(O.model_constants("hmed2018")) == pytest.approx(m["min_pulse_intensity"], rel=1e-15)
    ft = m["force_tracking"]
    for n, tgt in ft["targets"].items():
        np.testing.assert_allclose(O.fourier_target(np.array(ft["time"]), np.array(ft["force"]), int(n)), tgt,
                                   rtol=1e-13, atol=1e-12)
    kat = m["kat"]
    c = O.model_constants("ding2003_with_fatigue")
    assert O.cn_sum(c | {"km_rest": 0.01}, 0.11, np.array([0.0, 0.1])) == pytest.approx(kat["cn_sum"], rel=1e-14)
    assert O.lambda_i(O.model_constants("hmed2018"), 30.0) == pytest.approx(kat["lambda_30"], rel=1e-14)
    assert O.a_calculation(O.model_constants("ding2007"), 4920, 0.0002) == pytest.approx(kat["a_calc"], rel=1e-14)


def _small_problem(name, scheme="RK4", m=3, n=4, T=3, seed=0, params=False):
    c = O.model_constants(name)
    stims = [0.0, 0.05, 0.1, 0.15]
    tab = O.stim_table(stims, n, 0.2, T)
    pb = O.Problem(name=name, c=c, n_shooting=n, final_time=0.2, truncation=T, rows=tab.rows, scheme=scheme,
                   n_steps=m)
    if params:
        pb.n_params = len(stims)
        pb.last_stim_idx = [s[-1] for s in tab.stim_idx_at_node[:n]]
        pb.intensity_floor = O.min_pulse_intensity(c)
    r = np.random.default_rng(seed)
    v = _random_v(pb, r, 3)
    return pb, v


def _random_v(pb, r, B):
    X = np.empty((B, pb.n_shooting + 1, pb.nx))
    X[..., 0] = r.uniform(0, 1.0, X.shape[:2])
    X[..., 1] = r.uniform(0, 200, X.shape[:2])
    if pb.nx == 5:
        a0 = pb.c.get("a_scale", pb.c["a_rest"]) if pb.name.startswith("ding2007") else pb.c["a_rest"]
        X[..., 2] = a0 * r.uniform(0.8, 1.0, X.shape[:2])
        X[..., 3] = r.uniform(0.05, 0.07, X.shape[:2])
        X[..., 4] = r.uniform(0.1, 0.2, X.shape[:2])
    U = np.empty((B, pb.n_shooting, pb.nu))
    if pb.nu == 1:
        U[...] = r.uniform(2e-4, 6e-4, U.shape)
    elif pb.nu:
        U[...] = r.uniform(20, 120, U.shape)
    P = r.uniform(20, 120, (B, pb.n_params))
    body = np.concatenate([X[:, :-1, :], U], axis=2).reshape(B, -1)
    return np.concatenate([body, X[:, -1, :], P], axis=1)


@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_oracle_complex_step_jacobian_agrees_with_finite_differences(name):
    pb, v = _small_problem(name)
    J = O.continuity_blocks(pb, v)
    nz = pb.nx + pb.nu
    for j in range(nz):
        offs = [(pb.x_off(k) + j) if j < pb.nx else (pb.u_off(k) + j - pb.nx) for k in range(pb.n_shooting)]
        step = 1e-6 * np.maximum(1.0, np.abs(v[:, offs]))
        vp, vm = v.copy(), v.copy()
        vp[:, offs] += step
        vm[:, offs] -= step
        X, U, _ = pb.unpack(vp)
        gp = O._phi_all(pb, X, U)
        X, U, _ = pb.unpack(vm)
        gm = O._phi_all(pb, X, U)
        fd = (gp - gm) / (2 * step[:, :, None])
        np.testing.assert_allclose(J[:, :, :, j], fd, rtol=2e-5, atol=1e-6 * np.max(np.abs(fd)) + 1e-7)


def test_oracle_sliding_window_and_structure():
    pb, v = _small_problem("hmed2018", params=True)
    g = O.eval_g(pb, v)
    assert g.shape == (3, pb.ng)
    rows, cols = O.jac_structure(pb)
    vals = O.eval_jac_g(pb, v)
    assert vals.shape == (3, rows.size)
    # dense reconstruction: J @ dv == directional derivative of g (g is exact-linear in the sliding rows)
    dv = np.random.default_rng(1).normal(size=pb.nv) * 1e-7
    lin = np.zeros((3, pb.ng))
    for i, (r, c) in enumerate(zip(rows, cols)):
        lin[:, r] += vals[:, i] * dv[c]
    fd = O.eval_g(pb, v + dv) - g
    np.testing.assert_allclose(lin, fd, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("scheme", ["RK1", "RK4"])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_c_port_matches_numpy_oracle(name, scheme):
    from oracle import c_oracle

    pb, v = _small_problem(name, scheme=scheme, params=name.startswith("hmed"))
    g, jac = c_oracle.shooting(pb, v, threads=2)
    np.testing.assert_allclose(g, O.eval_g(pb, v), rtol=1e-12, atol=1e-10)
    np.testing.assert_allclose(jac, O.eval_jac_g(pb, v), rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("scheme", ["RK1", "RK2", "RK4"])
@pytest.mark.parametrize("name", O.MODEL_NAMES)
def test_structural_pattern_covers_every_nonzero(name, scheme):
    for m in (1, 2, 3):
        pb, v = _small_problem(name, scheme=scheme, m=m)
        blocks = O.continuity_blocks(pb, v)
        pattern = O.structural_pattern(pb)
        for r in range(pb.nx):
            outside = [c for c in range(pb.nx + pb.nu) if c not in pattern[r]]
            assert np.all(blocks[:, :, r, outside] == 0.0), (r, outside)
        if not name.startswith("hmed"):  # Hmed placeholder entries are structural but numerically zero
            for r in range(pb.nx):
                inside = sorted(pattern[r])
                assert np.all(np.any(blocks[:, :, r, inside] != 0.0, axis=(0, 1)))


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_same_formulation_cpu_baseline_matches_the_oracle(cfg):
    """oracle/c/fes_affine.c — bench.py's same-formulation CPU leg (affine calcium tables, fused Euler step, 64-instance
    tiles) — gives the oracle's g and J_g (complex step) to 1e-12 on BASELINE configs[1] and [2]."""
    from oracle import c_affine
    from tests import cases

    pb = cases.oracle_problem(**getattr(cases, cfg)())
    B = 128
    v = cases.random_decision(pb, B, seed=4)
    vt = np.ascontiguousarray(v.reshape(B // 64, 64, -1).transpose(0, 2, 1))
    g, j = c_affine.Evaluator(pb)(vt, threads=2)
    g = g.transpose(0, 2, 1).reshape(B, -1)
    j = j.transpose(0, 2, 1).reshape(B, -1)
    X, _, _ = pb.unpack(v)
    ref_g, ref_j = O.eval_g(pb, v), O.eval_jac_g(pb, v)
    assert np.max(np.abs(g - ref_g) / (np.abs(ref_g) + np.abs(X[:, 1:, :].reshape(B, -1)))) < 1e-12
    assert np.max(np.abs(j - ref_j) / (np.abs(ref_j) + 1e-300)) < 1e-12
