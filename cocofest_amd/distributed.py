"""Multi-GPU paths: one process per GPU, torch.distributed (RCCL on ROCm, gloo in the
CPU tests).

Two ways the callbacks shard:

* ``shard_instances`` — independent instances (multi-start, parameter sweeps, independent NMPC scenarios):
  rank r owns a contiguous block of the batch and evaluates / solves it with its own libcfx handle.  No
  data-path collective; ``gather_instances`` collects results at the end.

* ``IntervalShardedNlp`` — ONE large OCP split by interval ranges.  Block k of g / J_g / H depends only on
  x_k, u_k, x_{k+1} (a one-node halo) and the parameters, so rank r evaluates intervals [k0, k1) through
  ``FesOcp.interval_slice`` and the exchange step is one all-gather per callback of the value slices (fixed
  sparsity, so every rank knows where each gathered value lands).  Overlapping contributions (the objective
  at shared nodes, parameter gradients, Hessian entries of the halo node) are summed by the index-add that
  places the gathered slices.  Every rank ends with the full callback values, so the host driver can run
  replicated on every rank (or on rank 0 only) on identical data.
"""

from __future__ import annotations

import numpy as np


def shard_range(total: int, rank: int, world: int):
    """Contiguous block [lo, hi) of ``total`` items owned by ``rank`` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of size {world}")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_instances(v0, rank: int, world: int):
    """The block of instance rows (B, nv) this rank owns."""
    lo, hi = shard_range(len(v0), rank, world)
    return v0[lo:hi]


def gather_instances(local, group=None):
    """All-gather per-rank blocks of rows (sizes may differ by one) into the full (B, ...) tensor on every
    rank, in rank order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    pad = max(sizes)
    buf = torch.zeros((pad,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return torch.cat([o[:s] for o, s in zip(out, sizes)], dim=0)


class IntervalShardedNlp:
    """The callbacks of one OCP with its intervals split over the ranks of ``group``.

    ``evaluator(sub_ocp, batch)`` opens the per-rank evaluator of an interval slice; by default a libcfx
    handle (AoS, batch-major) on this rank's GPU.  The interface mirrors ``_cfx.Handle`` for the calls the
    host driver makes (``eval_all``, ``eval_h``, structures), on (B, nv) torch tensors of the FULL problem.
    """

    def __init__(self, ocp, batch: int = 1, group=None, device=None, evaluator=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.ocp, self.B = ocp, batch
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if self.world > ocp.n_shooting:
            raise ValueError(f"{self.world} ranks for {ocp.n_shooting} intervals")
        self.k0, self.k1 = shard_range(ocp.n_shooting, self.rank, self.world)
        self.sub = ocp.interval_slice(self.k0, self.k1)
        if evaluator is None:
            local = torch.cuda.current_device() if device is None else device
            self.h = self.sub.nlp(batch=batch, layout="aos", device=local)
            self.dev = torch.device("cuda", local)
        else:
            self.h = evaluator(self.sub, batch)
            self.dev = torch.device("cpu") if device is None else torch.device(device)
        self.nz = ocp.nzb   # decision block of one interval (shooting or collocation)
        self.ngk = ocp.ngk  # constraint rows of one interval
        self._exchange_structures()

    # ---- global structure and the local -> global maps ------------------------------------------------
    def _exchange_structures(self):
        """Map this slice's structures to global indices and all-gather them (host objects, once)."""
        torch, o = self.torch, self.ocp
        body = (self.k1 - self.k0) * self.nz + o.nx
        cols = np.empty(self.sub.nv, dtype=np.int64)
        cols[:body] = self.k0 * self.nz + np.arange(body)
        cols[body:] = o.nv - o.n_params + np.arange(self.sub.nv - body)
        jr, jc = (np.asarray(a, np.int64) for a in self.h.jac_structure())
        hr, hc = (np.asarray(a, np.int64) for a in self.h.hess_structure())
        g0 = self.k0 * self.ngk
        mine = dict(jr=jr + g0, jc=cols[jc], hr=cols[hr], hc=cols[hc], cols=cols,
                    grows=g0 + np.arange(self.sub.n_shooting * self.ngk))
        parts = [None] * self.world
        self.dist.all_gather_object(parts, mine, group=self.group)
        self._jr = np.concatenate([p["jr"] for p in parts])
        self._jc = np.concatenate([p["jc"] for p in parts])
        hp = np.unique(np.stack([np.concatenate([p["hr"] for p in parts]), np.concatenate([p["hc"] for p in parts])],
                                1), axis=0)
        self._hr, self._hc = hp[:, 0], hp[:, 1]
        hindex = {(int(r), int(c)): i for i, (r, c) in enumerate(zip(self._hr, self._hc))}
        L = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.long, device=self.dev)  # noqa: E731
        offs = np.cumsum([0] + [len(p["jr"]) for p in parts])
        self.map_j = [L(np.arange(offs[i], offs[i + 1])) for i in range(self.world)]
        self.map_g = [L(p["grows"]) for p in parts]
        self.map_v = [L(p["cols"]) for p in parts]
        self.map_h = [L([hindex[(int(r), int(c))] for r, c in zip(p["hr"], p["hc"])]) for p in parts]
        self.cols_local = self.map_v[self.rank]
        self.nv, self.ng = o.nv, o.n_shooting * self.ngk
        self.nnz_jac, self.nnz_hess = len(self._jr), len(self._hr)
        # placement of the all-gathered slices: one fixed gather-sum table per output (libcfx cfx_gather_sum on a GPU)
        self._tables = {}
        if self.dev.type == "cuda":
            from . import _cfx

            self._lib = _cfx.load_library()
            maps = {"g": (self.map_g, self.ng), "jac": (self.map_j, self.nnz_jac), "grad": (self.map_v, self.nv),
                    "hess": (self.map_h, self.nnz_hess)}
            for name, (mp, width) in maps.items():
                self._tables[name] = self._gather_table([m.cpu().numpy() for m in mp], width)
            # selections of this rank's inputs from the full vectors (v columns, lambda rows), and the identity
            g0 = self.k0 * self.ngk
            self._tables["v_local"] = self._select_table(self.cols_local.cpu().numpy())
            self._tables["lam_local"] = self._select_table(np.arange(g0, g0 + self.sub.n_shooting * self.ngk))
            self._tables["one"] = self._select_table(np.zeros(1, dtype=np.int64))

    def _gather_table(self, maps, width):
        """CSR (ptr, idx) over the concatenated gathered buffer [rank r's slice at r * pad]: the sources of every
        destination, in rank order (the index_add_ order)."""
        pad = max(len(m) for m in maps)
        dst = np.concatenate([np.asarray(m, np.int64) for m in maps])
        src = np.concatenate([r * pad + np.arange(len(m)) for r, m in enumerate(maps)])
        order = np.argsort(dst, kind="stable")
        ptr = np.zeros(width + 1, dtype=np.int32)
        np.add.at(ptr, dst + 1, 1)
        ptr = np.cumsum(ptr).astype(np.int32)
        T = self.torch
        return (T.as_tensor(ptr, device=self.dev), T.as_tensor(src[order].astype(np.int32), device=self.dev), pad)

    def _select_table(self, cols):
        T = self.torch
        n = len(cols)
        return (T.as_tensor(np.arange(n + 1, dtype=np.int32), device=self.dev),
                T.as_tensor(np.asarray(cols, dtype=np.int32), device=self.dev), None)

    def _gather_sum(self, table, src_ptr, src_len, dst_ptr, n_dst):
        from . import _cfx

        ptr, idx, _ = table
        rc = self._lib.cfx_gather_sum(self.B, n_dst, ptr.data_ptr(), idx.data_ptr(), src_ptr, src_len, dst_ptr,
                                      self.torch.cuda.current_stream(self.dev).cuda_stream)
        if rc != _cfx.OK:
            raise _cfx.CfxError(rc, self._lib.cfx_last_error(None).decode())

    def jac_structure(self):
        return self._jr.astype(np.int32), self._jc.astype(np.int32)

    def hess_structure(self):
        return self._hr.astype(np.int32), self._hc.astype(np.int32)

    # ---- exchange -------------------------------------------------------------------------------------
    def _allgather(self, local, pad):
        """All-gather every rank's (B, L_r) slice, padded to ``pad``, as one (B, world * pad) tensor on self.dev."""
        torch, dist = self.torch, self.dist
        # gloo moves host memory only: a rank with device tensors stages the exchange through the host (the
        # nccl / RCCL backend gathers the device buffers directly over xGMI)
        cdev = torch.device("cpu") if (self.dev.type == "cuda" and dist.get_backend(self.group) == "gloo") else self.dev
        buf = torch.zeros((self.B, pad), dtype=torch.float64, device=cdev)
        buf[:, : local.shape[1]] = local.to(cdev)
        out = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(out, buf, group=self.group)
        return torch.cat([o.to(self.dev) for o in out], dim=1).contiguous()

    def _allgather_place(self, local, maps, width, name=None, dst=None):
        """All-gather every rank's (B, L_r) slice and sum it into a (B, width) global array: on a GPU with the
        precomputed table ``name`` (one cfx_gather_sum launch, written into ``dst`` — a tensor or a device pointer —
        when given), otherwise by an index-add per rank."""
        torch = self.torch
        pad = max(m.numel() for m in maps)
        cat = self._allgather(local, pad)
        if name in self._tables:
            out = dst if dst is not None else torch.empty((self.B, width), dtype=torch.float64, device=self.dev)
            self._gather_sum(self._tables[name], cat.data_ptr(), cat.shape[1],
                             out if isinstance(out, int) else out.data_ptr(), width)
            return out
        full = torch.zeros((self.B, width), dtype=torch.float64, device=self.dev)
        for r, m in enumerate(maps):
            full.index_add_(1, m, cat[:, r * pad: r * pad + m.numel()])
        return full

    # ---- callbacks (same signatures as _cfx.Handle, AoS (B, ...) tensors) ------------------------------
    def eval_all(self, v, g=None, jac=None, f=None, grad=None):
        torch = self.torch
        vl = v[:, self.cols_local].contiguous()
        sub = self.sub
        gl = torch.empty((self.B, sub.n_shooting * self.ngk), dtype=torch.float64, device=self.dev) \
            if (g is not None or jac is not None) else None
        jl = torch.empty((self.B, self.h.nnz_jac), dtype=torch.float64, device=self.dev) if jac is not None else None
        fl = torch.empty((self.B,), dtype=torch.float64, device=self.dev) if f is not None else None
        dl = torch.empty((self.B, sub.nv), dtype=torch.float64, device=self.dev) if grad is not None else None
        self.h.eval_all(vl, g=gl, jac=jl, f=fl, grad=dl)
        if g is not None:
            g.copy_(self._allgather_place(gl, self.map_g, self.ng, "g"))
        if jac is not None:
            jac.copy_(self._allgather_place(jl, self.map_j, self.nnz_jac, "jac"))
        if f is not None:
            f.copy_(self._reduce_f(fl))
        if grad is not None:
            grad.copy_(self._allgather_place(dl, self.map_v, self.nv, "grad"))

    def _reduce_f(self, fl):
        fs = fl.cpu() if (self.dev.type == "cuda" and self.dist.get_backend(self.group) == "gloo") else fl.clone()
        self.dist.all_reduce(fs, group=self.group)
        return fs.to(self.dev)

    # ---- the same callbacks on raw device pointers (AoS, the full problem), for libcfx's own interior point
    # (cfx_ipm_create_ext, ShardedNativeIpm): inputs selected by the gather table, outputs placed straight into the
    # solver's buffers
    def _agree(self, ok: bool) -> bool:
        """True when every rank's local evaluation succeeded (one MAX all-reduce of a failure flag): the callbacks run
        their collectives only when all ranks reached them, so a rank whose evaluation raised makes every rank's
        callback fail at the same call instead of leaving the others blocked in an all-gather."""
        torch, dist = self.torch, self.dist
        cdev = torch.device("cpu") if (self.dev.type != "cuda" or dist.get_backend(self.group) == "gloo") else self.dev
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        return int(flag.item()) == 0

    def eval_all_ptr(self, v, g, jac, f, grad):
        torch, sub = self.torch, self.sub
        err = None
        try:
            vl = torch.empty((self.B, sub.nv), dtype=torch.float64, device=self.dev)
            self._gather_sum(self._tables["v_local"], v, self.nv, vl.data_ptr(), sub.nv)
            gl = torch.empty((self.B, sub.n_shooting * self.ngk), dtype=torch.float64, device=self.dev) \
                if (g or jac) else None
            jl = torch.empty((self.B, self.h.nnz_jac), dtype=torch.float64, device=self.dev) if jac else None
            fl = torch.empty((self.B,), dtype=torch.float64, device=self.dev) if f else None
            dl = torch.empty((self.B, sub.nv), dtype=torch.float64, device=self.dev) if grad else None
            self.h.eval_all(vl, g=gl, jac=jl, f=fl, grad=dl)
        except Exception as e:  # noqa: BLE001 — every rank learns of it below, then re-raised through the solver
            err = e
        if not self._agree(err is None):
            if err is not None:
                raise err
            raise RuntimeError("interval-sharded eval_all: another rank's evaluation failed")
        if g:
            self._allgather_place(gl, self.map_g, self.ng, "g", dst=g)
        if jac:
            self._allgather_place(jl, self.map_j, self.nnz_jac, "jac", dst=jac)
        if f:
            fs = self._reduce_f(fl).contiguous()
            self._gather_sum(self._tables["one"], fs.data_ptr(), 1, f, 1)
        if grad:
            self._allgather_place(dl, self.map_v, self.nv, "grad", dst=grad)
        return 0

    def eval_h_ptr(self, v, of, lam, hess):
        torch, sub = self.torch, self.sub
        err = None
        try:
            vl = torch.empty((self.B, sub.nv), dtype=torch.float64, device=self.dev)
            self._gather_sum(self._tables["v_local"], v, self.nv, vl.data_ptr(), sub.nv)
            ngl = sub.n_shooting * self.ngk
            laml = torch.empty((self.B, ngl), dtype=torch.float64, device=self.dev)
            self._gather_sum(self._tables["lam_local"], lam, self.ng, laml.data_ptr(), ngl)
            ofl = torch.empty((self.B,), dtype=torch.float64, device=self.dev)
            self._gather_sum(self._tables["one"], of, 1, ofl.data_ptr(), 1)
            hl = torch.empty((self.B, self.h.nnz_hess), dtype=torch.float64, device=self.dev)
            self.h.eval_h(vl, ofl, laml, hl)
        except Exception as e:  # noqa: BLE001
            err = e
        if not self._agree(err is None):
            if err is not None:
                raise err
            raise RuntimeError("interval-sharded eval_h: another rank's evaluation failed")
        self._allgather_place(hl, self.map_h, self.nnz_hess, "hess", dst=hess)
        return 0

    def eval_h(self, v, of, lam, hess):
        torch = self.torch
        vl = v[:, self.cols_local].contiguous()
        g0 = self.k0 * self.ngk
        laml = lam[:, g0: g0 + self.sub.n_shooting * self.ngk].contiguous()
        hl = torch.empty((self.B, self.h.nnz_hess), dtype=torch.float64, device=self.dev)
        self.h.eval_h(vl, of.contiguous(), laml, hl)
        hess.copy_(self._allgather_place(hl, self.map_h, self.nnz_hess, "hess"))
        return hess

    def close(self):
        self.h.close()


class ShardedNativeIpm:
    """libcfx's own interior point (cfx_ipm, csrc/cfx_ipm.hip) over the interval-sharded callbacks of ONE OCP: every
    rank holds the full KKT system (the band assembly and factorisation run replicated on identical data, as the
    callbacks' all-gather leaves every rank the full values) and evaluates only its interval slice — the solver reaches
    its callbacks through cfx_ipm_create_ext, the value slices land in its buffers by one cfx_gather_sum launch each.
    Same ``solve`` / result as solver.NativeIpm.  SURVEY.md section 8(e); the reference's analogue is CasADi's `map`
    over intervals with n_threads (cocofest/optimization/fes_ocp.py:122,189)."""

    def __init__(self, ocp, batch: int = 1, options=None, group=None, device=None):
        import torch

        from . import _cfx
        from .solver import IpmOptions, native_options

        self.torch = torch
        self.ocp, self.B = ocp, batch
        self.opt = options or IpmOptions()
        # max_wall_time reads each rank's own clock at the top of each iteration: ranks could stop at different
        # iterations, and one left inside a callback's collective would wait forever — refused here
        if self.opt.max_wall_time < 1e19:
            raise ValueError("ShardedNativeIpm: max_wall_time must stay unset (each rank would stop on its own clock); "
                             "bound the solve with max_iter")
        self.nlp = IntervalShardedNlp(ocp, batch=batch, group=group, device=device)
        lb, ub = ocp.bounds_vector()
        self.n, self.m = self.nlp.nv, self.nlp.ng
        self.ipm = _cfx.Ipm.external(
            batch, self.nlp.nv, self.nlp.ng, self.nlp.jac_structure(), self.nlp.hess_structure(),
            self.nlp.eval_all_ptr, self.nlp.eval_h_ptr, lb, ub, int(getattr(ocp, "n_params", 0) or 0),
            native_options(self.opt),
            device=self.nlp.dev.index, stream=torch.cuda.current_stream(self.nlp.dev).cuda_stream)

    def solve(self, v0=None, fixed_values=None):
        import time

        from .solver import IpmResult

        t0 = time.perf_counter()
        if v0 is None:
            v0 = np.tile(self.ocp.initial_guess_vector(), (self.B, 1))
        v, y, f, conv, its, kkt = self.ipm.solve(v0, fixed_values)
        st = self.ipm.stats()
        self.last_stats = st
        return IpmResult(v=v, y=y, f=f, converged=conv, iterations=its, kkt_error=kkt,
                         wall_time=time.perf_counter() - t0,
                         n_callbacks={k: int(st[k]) for k in ("eval_all", "eval_h", "eval_g_f", "kkt_factor")},
                         status=self.ipm.status())

    def close(self):
        self.ipm.close()
        self.nlp.close()
