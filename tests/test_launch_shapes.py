"""Parity at the launch shapes the benchmark times.

The g + J_g kernels pick their launch shape from the batch size (cfx_get_launch_shape): the shooting kernel carries
x_{k+1} in registers through `intervals_per_thread` consecutive intervals, orders the grid intervals-fast, and moves
1 / 2 / 4 adjacent instances per lane; the musculoskeletal tangent kernel runs `msk_intervals_per_block` intervals per
block with the next sub-step's stage coefficients streamed into a second LDS buffer by direct-to-LDS loads.  Small
test batches get the trivial shape (1 interval per thread / block), so every shape is forced here through the
environment overrides cfx_create reads (CFX_KPT, CFX_IFAST, CFX_NI, CFX_MSK_KPB) and checked

* bit for bit against the trivial shape on the same instances (the arithmetic of an interval does not depend on
  which thread runs it), and
* against the oracle (relative 1e-11 for the Ding / Hmed models, as tests/test_gpu_parity.py; 1e-10 / 1e-9 for the
  musculoskeletal g / J_g, as tests/test_msk_gpu.py),

then the exact benchmark shapes (bench.py: cfg 2 at B = 2^20 in 64-instance tiles, cfg 3 at B = 2^18, cfg 5 at
B = 65,536) are run as timed and a sample of their instances is checked the same way.
Reference semantics: cocofest/models/ding2003.py:153-198 (RHS), continuity rows per SURVEY.md section 8 a15.
"""

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases
from tests.test_gpu_parity import _close, _close_g

pytestmark = pytest.mark.gpu

ENV = ("CFX_KPT", "CFX_IFAST", "CFX_NI", "CFX_MSK_KPB")


@pytest.fixture(autouse=True)
def _clean_env(monkeypatch):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    from cocofest_amd import _cfx

    if _cfx.load_library().cfx_device_count() < 1:
        pytest.fail("no HIP device visible to libcfx")


def _tile(a):
    """(B, n) instance-major -> CFX_LAYOUT_TILED64 (B / 64, n, 64)."""
    B, n = a.shape
    return np.ascontiguousarray(a.reshape(B // 64, 64, n).transpose(0, 2, 1))


def _untile(a):
    nt, n, _ = a.shape
    return a.transpose(0, 2, 1).reshape(nt * 64, n)


def _run(ocp, v, layout, monkeypatch, env, g_only=False):
    """Evaluate (g, J_g) — or g alone — of the instances v (B, nv) through device buffers in `layout`, with the
    launch-shape overrides `env`; returns instance-major host arrays and the handle's launch shape."""
    import torch

    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    for k, val in env.items():
        monkeypatch.setenv(k, str(val))
    B = v.shape[0]
    h = ocp.nlp(batch=B, layout=layout)
    shape = h.launch_shape()
    if layout == "tiled64":
        dv = torch.tensor(_tile(v), device="cuda")
        mk = lambda n: torch.empty((B // 64, n, 64), dtype=torch.float64, device="cuda")  # noqa: E731
        back = lambda t: _untile(t.cpu().numpy())  # noqa: E731
    else:
        dv = torch.tensor(np.ascontiguousarray(v.T), device="cuda")
        mk = lambda n: torch.empty((n, B), dtype=torch.float64, device="cuda")  # noqa: E731
        back = lambda t: t.cpu().numpy().T  # noqa: E731
    g = mk(h.ng)
    j = None if g_only else mk(h.nnz_jac)
    h.eval_all(dv, g=g, jac=j)
    torch.cuda.synchronize()
    out = (back(g), None if g_only else back(j))
    h.close()
    for k in env:
        monkeypatch.delenv(k, raising=False)
    return out, shape


# Ding families: 10 intervals so that 2 / 4 / 5 intervals per thread leave full and ragged chunks; h / tau_c <= 1
SHAPE_STIMS = [round(0.05 * i, 2) for i in range(10)]
LAYOUTS = [("soa", 1), ("soa", 4), ("tiled64", 2)]
KPTS = [1, 2, 4, 5, 10]


@pytest.mark.parametrize("scheme", ["RK1", "RK2", "RK4"])
@pytest.mark.parametrize("name", ["ding2003", "ding2003_with_fatigue", "ding2007", "ding2007_with_fatigue",
                                  "hmed2018", "hmed2018_with_fatigue"])
def test_shooting_launch_shapes_are_bitwise_identical(name, scheme, monkeypatch):
    cfg = dict(name=name, stims=SHAPE_STIMS, final_time=0.5, truncation=4, scheme=scheme, m=5,
               objective=None, n_shooting=None)
    ocp = cases.product_ocp(**cfg)
    pb = cases.oracle_problem(**cfg)
    assert pb.n_shooting == 10
    B = 1152  # 18 tiles; 4.5 / 2.25 / 1.125 instance blocks at 1 / 2 / 4 instances per lane: partial last blocks
    v = cases.random_decision(pb, B, seed=21)
    hmed = name.startswith("hmed")
    (g_ref, j_ref), shape = _run(ocp, v, "soa", monkeypatch, {"CFX_KPT": 1, "CFX_IFAST": 0, "CFX_NI": 1})
    assert (shape["intervals_per_thread"], shape["intervals_fast"], shape["instances_per_lane"]) == (1, 0, 1)
    # the trivial shape against the oracle on a sample spanning lanes, waves, blocks and the last instance
    pick = np.array([0, 1, 63, 64, 255, 256, 511, 512, 700, 1023, 1024, B - 2, B - 1])
    _close_g(pb, v[pick], g_ref[pick], O.eval_g(pb, v[pick]), what=f"g {name} {scheme}")
    _close(j_ref[pick], O.eval_jac_g(pb, v[pick]), what=f"J {name} {scheme}")
    seen = set()
    # Hmed carries its Jacobian directions in chunks, one instance per lane (CFX_NI does not apply)
    for layout, ni in ([("soa", 1), ("tiled64", 1)] if hmed else LAYOUTS):
        for kpt in KPTS:
            for ifast in (0, 1):
                env = {"CFX_KPT": kpt, "CFX_IFAST": ifast, "CFX_NI": ni}
                (g, j), shape = _run(ocp, v, layout, monkeypatch, env)
                want_ni = 1 if hmed else ni
                assert (shape["intervals_per_thread"], shape["intervals_fast"], shape["instances_per_lane"]) == \
                    (kpt, ifast, want_ni), (env, shape)
                np.testing.assert_array_equal(g, g_ref, err_msg=f"g {layout} {env}")
                np.testing.assert_array_equal(j, j_ref, err_msg=f"J {layout} {env}")
                # the g-only pass (no Jacobian directions; its own instances-per-lane choice)
                (g0, _), shape0 = _run(ocp, v, layout, monkeypatch, env, g_only=True)
                assert shape0["instances_per_lane_g"] == want_ni
                np.testing.assert_array_equal(g0, g_ref, err_msg=f"g-only {layout} {env}")
                seen.add((layout, want_ni, kpt, ifast))
    assert len(seen) == (2 if hmed else 3) * len(KPTS) * 2


def _bench_shape_check(ocp, pb, v_dev_tiled, B, pick, expect, what):
    """Run the benchmark's launch (default shape for this batch) on a device-resident tiled batch, then compare the
    picked instances bit for bit with a small AoS handle (trivial shape) and with the oracle."""
    import torch

    h = ocp.nlp(batch=B, layout="tiled64")
    shape = h.launch_shape()
    for k, val in expect.items():
        assert shape[k] == val, (what, shape)
    g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device="cuda")
    j = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device="cuda")
    h.eval_all(v_dev_tiled, g=g, jac=j)
    torch.cuda.synchronize()
    t, e = pick // 64, pick % 64
    gp = g[t, :, e].cpu().numpy()
    jp = j[t, :, e].cpu().numpy()
    vp = v_dev_tiled[t, :, e].cpu().numpy()
    h.close()
    del g, j
    small = ocp.nlp(batch=len(pick), layout="aos")
    assert small.launch_shape()["intervals_per_thread"] == 1
    np.testing.assert_array_equal(gp, small.eval_g(vp), err_msg=f"{what} g vs trivial shape")
    np.testing.assert_array_equal(jp, small.eval_jac_g(vp), err_msg=f"{what} J vs trivial shape")
    small.close()
    _close_g(pb, vp, gp, O.eval_g(pb, vp), what=f"{what} g vs oracle")
    _close(jp, O.eval_jac_g(pb, vp), what=f"{what} J vs oracle")


def _picks(B, n_random=48, seed=0):
    edges = [0, 1, 2, 63, 64, 65, 127, 511, 512, 513, 1023, 1024, 131071, 131072, B // 2, B - 513, B - 512,
             B - 65, B - 64, B - 2, B - 1]
    rnd = np.random.default_rng(seed).integers(0, B, n_random)
    return np.unique(np.concatenate([np.array([e for e in edges if 0 <= e < B]), rnd]))


def test_bench_shape_cfg2_headline():
    """bench.py's headline launch: cfg 2 (BASELINE configs[1]), B = 2^20, CFX_LAYOUT_TILED64, the synthetic batch of
    bench.synthetic_soa — 4 intervals per thread, intervals-fast grid, 2 instances per lane."""
    import bench

    ocp = bench.build_problem()
    pb = cases.oracle_problem(**cases.cfg2())
    B = 1 << 20
    v = bench.to_tiled(bench.synthetic_soa(ocp, B, seed=1234, device="cuda:0"))
    _bench_shape_check(ocp, pb, v, B, _picks(B), {"intervals_per_thread": 4, "intervals_fast": 1,
                                                  "instances_per_lane": 2}, "cfg2 B=2^20")


def test_bench_shape_cfg3_callbacks():
    """bench.py's cfg3_callbacks launch: cfg 3 (BASELINE configs[2], Ding2007 pulse width, N = 100), B = 2^18 tiled —
    5 intervals per thread, intervals-fast grid, 2 instances per lane."""
    import torch

    import bench

    ocp = bench.build_cfg3()
    cfg = cases.cfg3()
    pb = cases.oracle_problem(**cfg)
    assert ocp.n_shooting == pb.n_shooting == 100
    B = 1 << 18
    va = bench.cfg3_synthetic(ocp, B, seed=0)
    v = bench.to_tiled(torch.from_numpy(np.ascontiguousarray(va.T)).cuda())
    _bench_shape_check(ocp, pb, v, B, _picks(B, n_random=24), {"intervals_per_thread": 5, "intervals_fast": 1,
                                                               "instances_per_lane": 2}, "cfg3 B=2^18")


# ---- musculoskeletal tangent kernel (k_msk_tangents_lds) -----------------------------------------------------------
def _msk_run(ocp, V, monkeypatch, kpb):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    if kpb is not None:
        monkeypatch.setenv("CFX_MSK_KPB", str(kpb))
    B = V.shape[0]
    h = ocp.nlp(batch=B, layout="aos")
    shape = h.launch_shape()
    g, j = np.empty((B, h.ng)), np.empty((B, h.nnz_jac))
    h.eval_all(V, g=g, jac=j)
    h.close()
    monkeypatch.delenv("CFX_MSK_KPB", raising=False)
    return g, j, shape


def _msk_oracle_check(pb, V, g, jac, jr, jc, what, intervals=None):
    from oracle import fes_msk as M
    from tests.test_msk_gpu import _dense_blocks, _ngk

    ngk = _ngk(pb)
    for b in range(V.shape[0]):
        ref_g = M.eval_g(pb, V[b])
        nxt = np.concatenate([np.concatenate([V[b][(k + 1) * pb.nz:(k + 1) * pb.nz + pb.nx], np.full(ngk - pb.nx, 130.0)])
                              for k in range(pb.n_shooting)])
        assert np.max(np.abs(g[b] - ref_g) / (np.abs(ref_g) + np.abs(nxt) + 1e-12)) < 1e-10, (what, b)
        for k in intervals or range(pb.n_shooting):
            ref = M.continuity_jacobian(pb, V[b], k)
            D, neg = _dense_blocks(pb, jr, jc, jac[b], k)
            np.testing.assert_array_equal(neg, -np.eye(pb.nx))
            scale = np.abs(ref) + 1e-9 * np.max(np.abs(ref), axis=1, keepdims=True)
            assert np.max(np.abs(D - ref) / scale) < 1e-9, (what, b, k)


MSK_SHAPES = {
    "cfg5_d07f_rk4": dict(),
    "d07_rk1_residual": dict(model="ding2007", scheme="RK1", m=5, residual=True, fatigue=False),
    "hmed_f_rk4_residual": dict(model="hmed2018_with_fatigue", residual=True, m=5),  # h / tau_c = 1
    "arm26_6muscles_d03_rk1": dict(biomod="arm26", model="ding2003", fatigue=False, scheme="RK1", m=3,
                                   muscles=("BIClong", "BICshort", "BRA", "TRIlong", "TRIlat", "TRImed")),
}


@pytest.mark.parametrize("B", [96, 95])  # even: direct-to-LDS double buffer; odd: staged through registers
@pytest.mark.parametrize("case", list(MSK_SHAPES))
def test_msk_intervals_per_block_are_bitwise_identical(case, B, monkeypatch):
    from tests import msk_cases as MC

    cfg = MC.cfg5(**MSK_SHAPES[case])
    ocp = MC.product_ocp(**cfg)
    pb = MC.oracle_problem(**cfg)
    N = pb.n_shooting
    V = MC.random_decision(pb, B, seed=17)
    g1, j1, s1 = _msk_run(ocp, V, monkeypatch, 1)
    assert s1["msk_intervals_per_block"] == 1
    for kpb in (2, 3, 5, N):
        g, j, s = _msk_run(ocp, V, monkeypatch, kpb)
        assert s["msk_intervals_per_block"] == kpb
        np.testing.assert_array_equal(g, g1, err_msg=f"{case} g kpb={kpb}")
        np.testing.assert_array_equal(j, j1, err_msg=f"{case} J kpb={kpb}")
    h = ocp.nlp(batch=1, layout="aos")
    jr, jc = h.jac_structure()
    h.close()
    pick = [0, 31, 32, B - 1]  # first / last lane of a 32-instance block, the next block, the last instance
    _msk_oracle_check(pb, V[pick[:2]], g1[pick[:2]], j1[pick[:2]], jr, jc, case, intervals=(0, N // 2, N - 1))
    _msk_oracle_check(pb, V[pick[2:]], g1[pick[2:]], j1[pick[2:]], jr, jc, case, intervals=(1, N - 2))


def test_msk_six_muscles_large_batch_multi_interval_blocks(monkeypatch):
    """The round-2 memory-aperture fault was seen in the 6-muscle instantiation at batch 300.
    The surviving kernels that shared its code (msk_frames, the via-point segment loops, the [N][Q][NC][B] scratch
    at a batch that is not a multiple of the block) at B = 300 and at a batch whose default shape runs several
    intervals per tangent block; every instance against the B = 2 run, a sample against the oracle."""
    from tests import msk_cases as MC

    cfg = MC.cfg5(**MSK_SHAPES["arm26_6muscles_d03_rk1"])
    ocp = MC.product_ocp(**cfg)
    pb = MC.oracle_problem(**cfg)
    N = pb.n_shooting
    Bl = 1 << 15  # 1,024 tangent blocks x 10 intervals / 4,096: 2 intervals per block by default
    V = MC.random_decision(pb, Bl, seed=23)
    g_big, j_big, s = _msk_run(ocp, V, monkeypatch, None)
    assert s["msk_intervals_per_block"] == 2
    g300, j300, _ = _msk_run(ocp, V[:300], monkeypatch, N)
    g300d, j300d, s300 = _msk_run(ocp, V[:300], monkeypatch, None)
    assert s300["msk_intervals_per_block"] == 1
    np.testing.assert_array_equal(g300, g300d)
    np.testing.assert_array_equal(j300, j300d)
    np.testing.assert_array_equal(g_big[:300], g300d)
    np.testing.assert_array_equal(j_big[:300], j300d)
    pick = np.array([0, 299, 4097, Bl - 1])
    g2, j2, _ = _msk_run(ocp, V[pick], monkeypatch, None)
    np.testing.assert_array_equal(g_big[pick], g2)
    np.testing.assert_array_equal(j_big[pick], j2)
    h = ocp.nlp(batch=1, layout="aos")
    jr, jc = h.jac_structure()
    h.close()
    _msk_oracle_check(pb, V[pick[[0, 3]]], g_big[pick[[0, 3]]], j_big[pick[[0, 3]]], jr, jc, "6 muscles",
                      intervals=(0, N - 1))
    # the stage-wise Hessian at the large-batch projection path agrees with the small-batch path on those instances
    lam = np.random.default_rng(3).normal(size=(300, pb.ng))
    of = np.linspace(0.2, 1.5, 300)
    hl = ocp.nlp(batch=300, layout="aos")
    H300 = hl.eval_h(V[:300].copy(), of, lam)
    hl.close()
    hs = ocp.nlp(batch=2, layout="aos")
    H2 = hs.eval_h(V[[0, 299]].copy(), of[[0, 299]].copy(), lam[[0, 299]].copy())
    hs.close()
    scale = np.abs(H2) + 1e-9 * np.abs(H2).max()
    assert np.max(np.abs(H300[[0, 299]] - H2) / scale) < 1e-12


def test_bench_shape_cfg5_msk():
    """bench.py's msk launch: cfg 5 (arm26 biceps / triceps, Ding2007 with fatigue, RK4 x 1), B = 65,536 SoA, the
    synthetic batch of bench.msk_throughput — 5 intervals per tangent block; a sample of instances bit for bit
    against a small batch (1 interval per block) and against the oracle."""
    import torch

    import bench
    from tests import msk_cases as MC

    ocp = bench.msk_build(1)
    pb = MC.oracle_problem(**MC.cfg5())
    assert (ocp.nv, ocp.n_shooting) == (pb.nv, pb.n_shooting)
    B = 1 << 16
    h = ocp.nlp(batch=B, layout="soa")
    assert h.launch_shape()["msk_intervals_per_block"] == 5
    lo, hi = ocp.bounds_vector()
    lo = np.where(np.isfinite(lo), lo, -2.0)
    hi = np.minimum(np.where(np.isfinite(hi), hi, 2.0), lo + 100.0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    r = 0.2 + 0.6 * torch.rand((h.nv, B), generator=gen, dtype=torch.float64, device="cuda")
    v = (torch.as_tensor(lo, device="cuda")[:, None] + torch.as_tensor(hi - lo, device="cuda")[:, None] * r).contiguous()
    g = torch.empty((h.ng, B), dtype=torch.float64, device="cuda")
    j = torch.empty((h.nnz_jac, B), dtype=torch.float64, device="cuda")
    h.eval_all(v, g=g, jac=j)
    torch.cuda.synchronize()
    pick = np.array([0, 31, 32, 4095, 32767, B - 33, B - 1])
    vp = v[:, pick].cpu().numpy().T.copy()
    gp, jp = g[:, pick].cpu().numpy().T, j[:, pick].cpu().numpy().T
    jr, jc = h.jac_structure()
    h.close()
    small = ocp.nlp(batch=len(pick), layout="aos")
    assert small.launch_shape()["msk_intervals_per_block"] == 1
    gs, js = np.empty(gp.shape), np.empty(jp.shape)
    small.eval_all(vp, g=gs, jac=js)
    small.close()
    np.testing.assert_array_equal(gp, gs)
    np.testing.assert_array_equal(jp, js)
    _msk_oracle_check(pb, vp[[0, 6]], gp[[0, 6]], jp[[0, 6]], jr, jc, "cfg5 B=65536", intervals=(0, 4, pb.n_shooting - 1))
