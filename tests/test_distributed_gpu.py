"""The interval-sharded callbacks (cocofest_amd/distributed.py IntervalShardedNlp) over libcfx GPU handles: a
world-2 run on one card (gloo, the ranks share cuda:0 — the driver's 8-GPU node runs the same code over RCCL)
reassembles the single-process libcfx callbacks, and the batched interior point converges on them in lockstep.
SURVEY.md section 8(e); the reference's analogue is CasADi's `map` over intervals with n_threads
(cocofest/optimization/fes_ocp.py:122,189)."""

import json
import os
import pathlib
import socket

import numpy as np
import pytest

from tests import cases
from tests.test_distributed import CFGS, _dense

pytestmark = pytest.mark.gpu
WORLD = 2
_FT = json.loads((pathlib.Path(__file__).parent / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
# BASELINE configs[2] (cfg 3: Ding2007 pulse widths, 30 pulses, N = 100, force tracking) for the interior point
IPM_CFG = dict(cases.cfg3(), objective={"force_tracking": [np.array(_FT["time"]), np.array(_FT["force"])]})


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out_dir):
    import torch
    import torch.distributed as dist

    from cocofest_amd.distributed import IntervalShardedNlp
    from cocofest_amd.solver import BatchedIpm, IpmOptions
    from tests.oracle_handle import oracle_problem_from_ocp

    import datetime

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    # a rank left waiting in a collective fails after 60 s instead of hanging the test
    dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=60))
    try:
        B = 3
        for ci, cfg in enumerate(CFGS):
            ocp = cases.product_ocp(**cfg)
            nlp = IntervalShardedNlp(ocp, batch=B, device=0)  # libcfx handle of this rank's interval slice
            v = cases.random_decision(oracle_problem_from_ocp(ocp), B, seed=7)
            vt = torch.tensor(v, device="cuda")
            g = torch.empty((B, nlp.ng), dtype=torch.float64, device="cuda")
            jac = torch.empty((B, nlp.nnz_jac), dtype=torch.float64, device="cuda")
            f = torch.empty((B,), dtype=torch.float64, device="cuda")
            grad = torch.empty((B, nlp.nv), dtype=torch.float64, device="cuda")
            nlp.eval_all(vt, g=g, jac=jac, f=f, grad=grad)
            rng = np.random.default_rng(ci)
            lam = rng.standard_normal((B, nlp.ng))
            of = rng.uniform(0.5, 2.0, B)
            hv = torch.empty((B, nlp.nnz_hess), dtype=torch.float64, device="cuda")
            nlp.eval_h(vt, torch.tensor(of, device="cuda"), torch.tensor(lam, device="cuda"), hv)
            torch.cuda.synchronize()
            jr, jc = nlp.jac_structure()
            hr, hc = nlp.hess_structure()
            np.savez(os.path.join(out_dir, f"cfg{ci}_r{rank}.npz"), v=v, g=g.cpu().numpy(), f=f.cpu().numpy(),
                     grad=grad.cpu().numpy(), lam=lam, of=of,
                     J=_dense(B, (nlp.ng, nlp.nv), jr, jc, jac.cpu().numpy()),
                     H=_dense(B, (nlp.nv, nlp.nv), hr, hc, hv.cpu().numpy(), sym=True))
            nlp.close()
        ocp = cases.product_ocp(**IPM_CFG)
        nlp = IntervalShardedNlp(ocp, batch=2, device=0)
        ipm = BatchedIpm(ocp, batch=2, options=IpmOptions(tol=1e-6, max_iter=500), handle=nlp, torch_device="cuda")
        v0 = np.tile(ocp.initial_guess_vector(), (2, 1))  # the reference's initial guess, and a perturbed one
        lb, ub = ocp.bounds_vector()
        free = lb != ub
        v0[1, free] = np.clip(v0[1, free] + np.random.default_rng(1).uniform(0, 1, free.sum()) * 0.01 *
                              np.minimum(ub[free] - lb[free], 10.0), lb[free], ub[free])
        res = ipm.solve(v0)
        np.savez(os.path.join(out_dir, f"ipm_r{rank}.npz"), v=res.v, converged=res.converged, f=res.f, v0=v0,
                 iterations=res.iterations, kkt=res.kkt_error)
        ipm.close()
        # libcfx's own interior point on the sharded callbacks (cfx_ipm_create_ext; value slices placed by
        # cfx_gather_sum)
        from cocofest_amd.distributed import ShardedNativeIpm

        nat = ShardedNativeIpm(ocp, batch=2, options=IpmOptions(tol=1e-6, max_iter=500), device=0)
        rn = nat.solve(v0)
        nat.close()
        np.savez(os.path.join(out_dir, f"native_r{rank}.npz"), v=rn.v, converged=rn.converged, f=rn.f,
                 iterations=rn.iterations, status=rn.status)
        # a per-rank wall clock is refused; one rank's failing evaluation fails every rank's solve
        try:
            ShardedNativeIpm(ocp, batch=2, options=IpmOptions(max_wall_time=10.0), device=0)
            wall_refused = False
        except ValueError:
            wall_refused = True
        nat = ShardedNativeIpm(ocp, batch=2, options=IpmOptions(tol=1e-6, max_iter=50), device=0)
        if rank == 1:
            calls = {"n": 0}
            orig = nat.nlp.h.eval_all

            def failing(*a, **k):
                calls["n"] += 1
                if calls["n"] == 3:
                    raise RuntimeError("injected evaluation failure")
                return orig(*a, **k)

            nat.nlp.h.eval_all = failing
        failed, msg = False, ""
        try:
            nat.solve(v0)
        except Exception as e:  # noqa: BLE001
            failed, msg = True, str(e)
        nat.close()
        np.savez(os.path.join(out_dir, f"fail_r{rank}.npz"), wall_refused=wall_refused, failed=failed, msg=msg)
        if rank == 0:  # the same algorithms on one process-local handle of the whole problem
            from cocofest_amd.solver import NativeIpm

            one = BatchedIpm(ocp, batch=2, options=IpmOptions(tol=1e-6, max_iter=500))
            r1 = one.solve(v0)
            one.close()
            np.savez(os.path.join(out_dir, "ipm_single.npz"), v=r1.v, converged=r1.converged, f=r1.f,
                     iterations=r1.iterations)
            one = NativeIpm(ocp, batch=2, options=IpmOptions(tol=1e-6, max_iter=500))
            r1 = one.solve(v0)
            one.close()
            np.savez(os.path.join(out_dir, "native_single.npz"), v=r1.v, converged=r1.converged, f=r1.f,
                     iterations=r1.iterations)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def sharded_gpu_run(tmp_path_factory):
    import torch.multiprocessing as mp

    out = tmp_path_factory.mktemp("dist_gpu")
    mp.spawn(_worker, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    return out


def _single_process(ocp, v, lam, of):
    h = ocp.nlp(batch=v.shape[0], layout="aos")
    g, jac = h.eval_g(v), h.eval_jac_g(v)
    f, grad = h.eval_f(v), h.eval_grad_f(v)
    hv = h.eval_h(v, of, lam)
    jr, jc = h.jac_structure()
    hr, hc = h.hess_structure()
    h.close()
    B = v.shape[0]
    return dict(g=g, f=f, grad=grad, J=_dense(B, (h.ng, h.nv), jr, jc, jac),
                H=_dense(B, (h.nv, h.nv), hr, hc, hv, sym=True))


@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_interval_sharded_libcfx_matches_single_process(sharded_gpu_run, ci):
    r0 = np.load(sharded_gpu_run / f"cfg{ci}_r0.npz")
    r1 = np.load(sharded_gpu_run / f"cfg{ci}_r1.npz")
    for k in ("g", "f", "grad", "J", "H"):  # every rank holds the same full values
        np.testing.assert_array_equal(r0[k], r1[k])
    ref = _single_process(cases.product_ocp(**CFGS[ci]), r0["v"], r0["lam"], r0["of"])
    scale = lambda a: np.abs(a).max() + 1e-300  # noqa: E731
    # the slices' stim times are shifted by k0 dt: rounding-level differences in the calcium tables only
    for k in ("g", "J", "grad", "H"):
        assert np.abs(r0[k] - ref[k]).max() <= 1e-12 * scale(ref[k]), k
    np.testing.assert_allclose(r0["f"], ref["f"], rtol=1e-12)


def test_batched_interior_point_on_interval_sharded_libcfx(sharded_gpu_run):
    """BatchedIpm over the 2-rank interval-sharded libcfx callbacks (cfg 3, 50 intervals per rank, from the
    reference's initial guess and a perturbed start) converges in lockstep on both ranks, to the point — and in the
    iterations — of the same algorithm on one process-local handle of the whole problem."""
    r0 = np.load(sharded_gpu_run / "ipm_r0.npz")
    r1 = np.load(sharded_gpu_run / "ipm_r1.npz")
    one = np.load(sharded_gpu_run / "ipm_single.npz")
    assert one["converged"].all(), one["iterations"]
    assert r0["converged"].all(), (r0["iterations"], r0["kkt"])
    np.testing.assert_array_equal(r0["v"], r1["v"])
    assert np.all(np.abs(r0["iterations"] - one["iterations"]) <= 2), (r0["iterations"], one["iterations"])
    ocp = cases.product_ocp(**IPM_CFG)
    lb, ub = ocp.bounds_vector()
    # fixed variables (lb == ub) have zero span: floor it with the variable's own magnitude
    span = np.where(np.isfinite(ub - lb), ub - lb, 0.0)
    span = np.maximum(span, np.maximum(1e-12, np.abs(one["v"]).max(axis=0)))
    assert np.max(np.abs(r0["v"] - one["v"]) / span) < 1e-6
    np.testing.assert_allclose(r0["f"], one["f"], rtol=1e-7)


def test_native_interior_point_on_interval_sharded_libcfx(sharded_gpu_run):
    """libcfx's own interior point (cfx_ipm through cfx_ipm_create_ext: its callbacks are the 2-rank interval-sharded
    libcfx slices, all-gathered and placed by one cfx_gather_sum launch per output) converges in lockstep on both
    ranks, to the single-process cfx_ipm point (cfg 3, from the reference's initial guess and a perturbed start)."""
    r0 = np.load(sharded_gpu_run / "native_r0.npz")
    r1 = np.load(sharded_gpu_run / "native_r1.npz")
    one = np.load(sharded_gpu_run / "native_single.npz")
    assert one["converged"].all(), one["iterations"]
    assert r0["converged"].all(), (r0["iterations"], r0["status"])
    np.testing.assert_array_equal(r0["v"], r1["v"])
    np.testing.assert_array_equal(r0["iterations"], r1["iterations"])
    assert np.all(np.abs(r0["iterations"] - one["iterations"]) <= 2), (r0["iterations"], one["iterations"])
    ocp = cases.product_ocp(**IPM_CFG)
    lb, ub = ocp.bounds_vector()
    span = np.where(np.isfinite(ub - lb), ub - lb, 0.0)
    span = np.maximum(span, np.maximum(1e-12, np.abs(one["v"]).max(axis=0)))
    assert np.max(np.abs(r0["v"] - one["v"]) / span) < 1e-6
    np.testing.assert_allclose(r0["f"], one["f"], rtol=1e-7)


def test_sharded_native_ipm_fails_on_every_rank_together(sharded_gpu_run):
    """ShardedNativeIpm refuses a finite max_wall_time (each rank would stop on its own clock), and a
    rank whose local evaluation raises makes every rank's solve fail at the same callback — rank 0, whose evaluation
    succeeded, raises too instead of waiting in the next all-gather (the process group's 60 s timeout would fail the
    run otherwise)."""
    for r in range(WORLD):
        d = np.load(sharded_gpu_run / f"fail_r{r}.npz")
        assert bool(d["wall_refused"]) and bool(d["failed"]), (r, str(d["msg"]))
    assert "injected evaluation failure" in str(np.load(sharded_gpu_run / "fail_r1.npz")["msg"])
    assert "another rank" in str(np.load(sharded_gpu_run / "fail_r0.npz")["msg"])
