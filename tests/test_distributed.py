"""Multi-process paths of cocofest_amd/distributed.py on the CPU (gloo, world size 2), with the oracle as the
per-rank evaluator: the interval-sharded callbacks reassemble exactly the single-process callbacks, the
interior point runs on them, and instance sharding round-trips."""

import os
import socket

import numpy as np
import pytest

from oracle import fes_oracle as O
from tests import cases

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dense(B, shape, rows, cols, vals, sym=False):
    M = np.zeros((B,) + shape)
    for b in range(B):
        np.add.at(M[b], (rows, cols), vals[b])
        if sym:
            off = rows != cols
            np.add.at(M[b], (cols[off], rows[off]), vals[b][off])
    return M


CFGS = [
    dict(name="ding2003", stims=[0.0, 0.1, 0.2, 0.3, 0.4], final_time=0.5, truncation=5, scheme="RK1", m=5,
         objective={"end_node_tracking": 40}, n_shooting=None),
    dict(name="ding2007_with_fatigue", stims=[0.0, 0.05, 0.1, 0.15, 0.2, 0.25], final_time=0.3, truncation=4,
         scheme="RK4", m=2, objective={"force_tracking": [np.linspace(0, 1, 11), np.linspace(10, 60, 11)]},
         n_shooting=None),
    dict(name="hmed2018", stims=[0.0, 0.1, 0.2, 0.3, 0.4], final_time=0.5, truncation=3, scheme="RK2", m=5,
         objective={"end_node_tracking": 30}, n_shooting=None),
]


def _worker(rank, port, out_dir):
    import torch
    import torch.distributed as dist

    from cocofest_amd.distributed import IntervalShardedNlp, gather_instances, shard_instances, shard_range
    from tests.oracle_handle import DenseBandSolver, OracleHandle, oracle_problem_from_ocp

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ev = lambda sub, B: OracleHandle(oracle_problem_from_ocp(sub), B)  # noqa: E731
        B = 3
        for ci, cfg in enumerate(CFGS):
            ocp = cases.product_ocp(**cfg)
            nlp = IntervalShardedNlp(ocp, batch=B, evaluator=ev)
            assert nlp.nv == ocp.nv
            full = oracle_problem_from_ocp(ocp)
            v = cases.random_decision(full, B, seed=7)  # same seed on every rank
            vt = torch.tensor(v)
            g = torch.empty((B, nlp.ng), dtype=torch.float64)
            jac = torch.empty((B, nlp.nnz_jac), dtype=torch.float64)
            f = torch.empty((B,), dtype=torch.float64)
            grad = torch.empty((B, nlp.nv), dtype=torch.float64)
            nlp.eval_all(vt, g=g, jac=jac, f=f, grad=grad)
            rng = np.random.default_rng(ci)
            lam = rng.standard_normal((B, nlp.ng))
            of = rng.uniform(0.5, 2.0, B)
            hv = torch.empty((B, nlp.nnz_hess), dtype=torch.float64)
            nlp.eval_h(vt, torch.tensor(of), torch.tensor(lam), hv)
            jr, jc = nlp.jac_structure()
            hr, hc = nlp.hess_structure()
            np.savez(os.path.join(out_dir, f"cfg{ci}_r{rank}.npz"), v=v, g=g.numpy(), f=f.numpy(), grad=grad.numpy(),
                     J=_dense(B, (nlp.ng, nlp.nv), jr, jc, jac.numpy()), lam=lam, of=of,
                     H=_dense(B, (nlp.nv, nlp.nv), hr, hc, hv.numpy(), sym=True))
            nlp.close()

        # the interior point on the interval-sharded callbacks (replicated driver, identical data on each rank)
        from cocofest_amd.solver import BatchedIpm, IpmOptions

        cfg = dict(CFGS[0])
        ocp = cases.product_ocp(**cfg)
        nlp = IntervalShardedNlp(ocp, batch=2, evaluator=ev)
        ipm = BatchedIpm(ocp, batch=2, options=IpmOptions(tol=1e-8), handle=nlp, torch_device="cpu",
                         band=DenseBandSolver())
        v0 = np.tile(ocp.initial_guess_vector(), (2, 1)) + np.random.default_rng(1).uniform(0, 5, (2, ocp.nv))
        res = ipm.solve(v0)
        np.savez(os.path.join(out_dir, f"ipm_r{rank}.npz"), v=res.v, converged=res.converged)

        # instance sharding: blocks of sizes 4 / 3 reassemble in rank order
        rows = torch.arange(7 * 3, dtype=torch.float64).reshape(7, 3)
        mine = shard_instances(rows, rank, WORLD)
        assert mine.shape[0] == shard_range(7, rank, WORLD)[1] - shard_range(7, rank, WORLD)[0]
        back = gather_instances(mine * 1.0)
        assert torch.equal(back, rows)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def sharded_run(tmp_path_factory):
    import torch.multiprocessing as mp

    out = tmp_path_factory.mktemp("dist")
    mp.spawn(_worker, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    return out


@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_interval_sharded_callbacks_match_single_process(sharded_run, ci):
    from tests.oracle_handle import OracleHandle, oracle_problem_from_ocp

    cfg = CFGS[ci]
    ocp = cases.product_ocp(**cfg)
    pb = oracle_problem_from_ocp(ocp)
    r0 = np.load(sharded_run / f"cfg{ci}_r0.npz")
    r1 = np.load(sharded_run / f"cfg{ci}_r1.npz")
    for k in ("g", "f", "grad", "J", "H"):  # every rank holds the same full values
        np.testing.assert_array_equal(r0[k], r1[k])
    v = r0["v"]
    h = OracleHandle(pb, v.shape[0])
    jr, jc = h.jac_structure()
    hr, hc = h.hess_structure()
    J = _dense(v.shape[0], (pb.ng, pb.nv), jr, jc, O.eval_jac_g(pb, v))
    H = _dense(v.shape[0], (pb.nv, pb.nv), hr, hc, O.hessian_values(pb, v, r0["of"], r0["lam"]), sym=True)
    scale = lambda a: np.abs(a).max() + 1e-300  # noqa: E731
    # stim times are shifted by k0 dt in the slices: rounding-level differences only
    assert np.abs(r0["g"] - O.eval_g(pb, v)).max() <= 1e-12 * scale(v)
    assert np.abs(r0["J"] - J).max() <= 1e-11 * scale(J)
    np.testing.assert_allclose(r0["f"], O.eval_f(pb, v), rtol=1e-12)
    assert np.abs(r0["grad"] - O.eval_grad_f(pb, v)).max() <= 1e-12 * scale(r0["grad"])
    assert np.abs(r0["H"] - H).max() <= 1e-6 * scale(H)  # oracle Hessians are finite differences


def test_interior_point_on_interval_sharded_callbacks(sharded_run):
    r0 = np.load(sharded_run / "ipm_r0.npz")
    r1 = np.load(sharded_run / "ipm_r1.npz")
    assert r0["converged"].all()
    np.testing.assert_array_equal(r0["v"], r1["v"])  # the replicated driver stays in lockstep
    pb = cases.oracle_problem(**CFGS[0])
    c = O.model_constants("ding2003")
    traj = O.ivp_integrate("ding2003", c, pb.rows, np.zeros((pb.n_shooting, 0)), pb.final_time, "RK1", 5)
    X, _, _ = pb.unpack(r0["v"])
    np.testing.assert_allclose(X, np.broadcast_to(traj[:, ::5].T, X.shape), rtol=1e-7, atol=1e-8)


def test_shard_range_covers_everything():
    from cocofest_amd.distributed import shard_range

    for total in (1, 7, 20, 100):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
