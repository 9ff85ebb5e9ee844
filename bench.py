#!/usr/bin/env python
"""bench.py — NLP callback throughput (constraint + Jacobian evaluations per second) on MI355X.

Workload (BASELINE.json configs[1], SURVEY.md section 8(d) cfg 2): OcpFes DingModelFrequency, 10 pulses at
10 Hz, final time 1 s, n_shooting 20, end-force 100 N objective, bioptim default transcription RK1 x 10
multiple shooting.  One "instance-evaluation" = g (40 continuity rows) + J_g (120 values) of one OCP
instance.  Each GPU evaluates a resident batch of B instances (synthetic decision vectors, seeded) per
step with ONE libcfx call (cfx_eval_all, device pointers, 64-instance tiled layout) = one kernel launch.

Multi-GPU (torchrun): instances are independent, so each rank owns its own batch (weak scaling, no
data-path collective); only the timing max-reduction crosses ranks.

Prints ONE JSON line on rank 0 with the roofline of the shooting kernel (achieved algorithmic HBM GB/s
from HIP events on the launch stream vs 8 TB/s) and the CPU baseline (the plain-C oracle port of the
as-written reference evaluation, OpenMP, timed on a bounded sample on this host).
"""

from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "NLP callback evals/s (constraint+Jac) and wall-clock to Ipopt-equiv convergence"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1 << 20, help="instances per GPU")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed launches before the warmup steps (power-management transient, DESIGN.md)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget (0: skip)")
    ap.add_argument("--no-solve", action="store_true", help="skip the wall-clock-to-convergence section")
    ap.add_argument("--no-msk", action="store_true", help="skip the cfg-5 musculoskeletal section")
    ap.add_argument("--no-multistart", action="store_true", help="skip the cfg-5 512-start restoration-robustness run")
    ap.add_argument("--no-reaching", action="store_true",
                    help="skip the 1,500-interval reaching-task solve (wall-clock to convergence, ~30 s)")
    ap.add_argument("--nmpc-horizons", type=int, default=200, help="cfg-4 NMPC horizons (0: skip)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend; gloo (ranks may share a GPU) rehearses the N > 1 path on one card")
    return ap.parse_args()


def build_problem():
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    model = ModelMaker.create_model("ding2003", stim_time=[round(0.1 * i, 1) for i in range(10)],
                                    sum_stim_truncation=20)
    return OcpFes.prepare_ocp(model=model, final_time=1, objective={"end_node_tracking": 100},
                              ode_solver=OdeSolver.RK1(n_integration_steps=10), n_shooting=20)


def synthetic_soa(ocp, B, seed, device):
    """SoA decision vectors (nv, B): Cn ~ U(0, 1.5), F ~ U(0, 250) at every node."""
    import torch

    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    v = torch.rand((ocp.nv, B), generator=gen, dtype=torch.float64, device=device)
    scale = torch.tensor([1.5, 250.0] * (ocp.nv // 2), dtype=torch.float64, device=device)[:, None]
    return v * scale


def to_tiled(a):
    """(len, B) SoA -> CFX_LAYOUT_TILED64 (B / 64, len, 64): element e of instance b at ((b/64) len + e) 64 + b%64."""
    n, B = a.shape
    return a.T.reshape(B // 64, 64, n).transpose(1, 2).contiguous()


def pmc_traffic():
    """HBM bytes per launch of the shooting kernel from the committed rocprofv3 PMC summary, if any."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get("hbm_bytes_per_launch")
    except Exception:
        return None


def _timed(fn, budget_s, per_call):
    """Calls fn() until budget_s has elapsed (one untimed call first); returns (units per second, units, seconds)."""
    fn()
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += per_call
        el = time.perf_counter() - t0
        if el >= budget_s:
            return done / el, done, el


def casadi_probe():
    """the reference's CPU callback is CasADi's; record whether this host can import it (no install)."""
    try:
        import casadi  # noqa: F401

        return {"importable": True, "version": getattr(casadi, "__version__", "?")}
    except Exception as e:  # noqa: BLE001
        return {"importable": False, "error": f"{type(e).__name__}: {e}"}


FP64_FMA_ISSUE_PEAK = 5.18e11  # wave-instr/s, measured (profiles/round1/micro_fp64_rate.txt: 8 chains, 8192 blocks)


def msk_pmc():
    """HBM bytes and VALU wave-instructions per cfg-5 g + J_g step (k_msk_values + k_msk_stage_tangents at B = 65,536)
    from the committed rocprofv3 passes (profiles/msk_pmc.json, written by scripts/summarize_msk_pmc.py from
    scripts/gpu_msk_pmc.sh), if any."""
    f = ROOT / "profiles" / "msk_pmc.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text())
    except Exception:
        return None


def cpu_baseline(ocp, budget_s, name="ding2003", truncation=20, label="cfg2"):
    """CPU legs on a bounded sample of the same workload, on this host's cores and on one core:

    * as written (``kind: port``, the headline value): the plain-C port of the reference's evaluation as CasADi
      would run its expression graph — 2T-1 exponentials per RK stage, dual-number derivatives (oracle/c/fes_oracle.c);
    * same formulation: the GPU kernel's own algorithm on the CPU — affine calcium tables, the fused Euler step with
      hand-derived tangents, 64-instance tiles, vectorised over the tile (oracle/c/fes_affine.c) — so that the GPU /
      CPU ratio of this leg is hardware only."""
    from oracle import c_affine, c_oracle, fes_oracle as O

    threads = min(16, len(os.sched_getaffinity(0)))
    pb = O.Problem(name=name, c=O.model_constants(name), n_shooting=ocp.n_shooting, final_time=1.0,
                   truncation=truncation, rows=ocp.stim_rows, scheme="RK1", n_steps=ocp.ode_solver.n_integration_steps)
    rng = np.random.default_rng(0)
    chunk = 4096 if name == "ding2003" else 1024
    v = rng.uniform(0.0, 1.0, (chunk, pb.nv))
    per = np.array([1.5, 250.0] + ([5e-4] if pb.nu else []))
    v *= np.tile(per, pb.nv // len(per) + 1)[: pb.nv]
    if pb.nu:
        v[:, 2::3] = np.maximum(v[:, 2::3], pb.c["pd0"])
    legs = {}
    rate, done, el = _timed(lambda: c_oracle.shooting(pb, v, threads=threads), budget_s * 0.5, chunk)
    legs["as_written"] = {"value": rate, "threads": threads, "instances": done, "seconds": el}
    rate, done, el = _timed(lambda: c_oracle.shooting(pb, v[: chunk // 8], threads=1), budget_s * 0.2, chunk // 8)
    legs["as_written_1core"] = {"value": rate, "threads": 1, "instances": done, "seconds": el}
    ev = c_affine.Evaluator(pb)
    Bt = 1 << 15
    vt = np.ascontiguousarray(np.tile(v, (Bt // chunk + 1, 1))[:Bt].reshape(Bt // 64, 64, pb.nv).transpose(0, 2, 1))
    g, jac = np.empty((Bt // 64, ev.ng, 64)), np.empty((Bt // 64, ev.nnz, 64))
    rate, done, el = _timed(lambda: ev(vt, threads=threads, g=g, jac=jac), budget_s * 0.15, Bt)
    legs["same_formulation"] = {"value": rate, "threads": threads, "instances": done, "seconds": el}
    rate, done, el = _timed(lambda: ev(vt, threads=1, g=g, jac=jac), budget_s * 0.15, Bt)
    legs["same_formulation_1core"] = {"value": rate, "threads": 1, "instances": done, "seconds": el}
    a = legs["as_written"]
    return {"value": a["value"], "unit": "instance-evals/s", "cores": threads, "kind": "port",
            "sample": f"{a['instances']} instances of {label} (g + J_g, as-written calcium sum: 2T-1 exp per RK stage), "
                      f"oracle/c/fes_oracle.c, OpenMP {threads} threads, {a['seconds']:.1f} s; the other legs in `legs`",
            "legs": legs, "casadi": casadi_probe()}


def build_cfg3():
    """BASELINE.json configs[2]: Ding2007 pulse width, 30 pulses (round(linspace(0, 1, 31)[:-1], 2)), N = 100,
    truncation 10, force tracking of the reference force curve (Fourier 50), RK1 x 10."""
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = ModelMaker.create_model("ding2007", stim_time=[float(v) for v in np.round(np.linspace(0, 1, 31)[:-1], 2)],
                                    sum_stim_truncation=10)
    return OcpFes.prepare_ocp(model=model, final_time=1, pulse_width={"min": model.pd0, "max": 0.0006},
                              objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                              ode_solver=OdeSolver.RK1(n_integration_steps=10))


def cfg3_synthetic(ocp, B, seed):
    """Instance-major decision vectors (B, nv) of cfg 3: Cn ~ U(0, 1.5), F ~ U(0, 250), pw ~ U(pd0, 6e-4)."""
    rng = np.random.default_rng(seed)
    nz = 3
    per = np.array([1.5, 250.0, 0.0])
    v = rng.uniform(0.0, 1.0, (B, ocp.nv))
    for k in range(ocp.nv):
        e = k % nz
        v[:, k] = v[:, k] * per[e] if e < 2 else ocp.model.pd0 + v[:, k] * (6e-4 - ocp.model.pd0)
    return v


def cfg3_section(device, cpu_seconds, steps=50, B=1 << 18):
    """BASELINE.json configs[2] callback throughput: g + J_g of cfg 3 (the fused Euler step of Ding2007, one pulse
    width per interval) over a device-resident CFX_LAYOUT_TILED64 batch, HIP events on the launch stream; its
    algorithmic HBM rate (read v, write g and J_g values) and the C port on the host cores on a bounded sample."""
    import torch

    ocp = build_cfg3()
    dev = f"cuda:{device}"
    h = ocp.nlp(batch=B, layout="tiled64", device=device)
    va = cfg3_synthetic(ocp, B, seed=0)
    v = to_tiled(torch.from_numpy(np.ascontiguousarray(va.T)).to(dev))
    g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device=dev)
    jac = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device=dev)
    for _ in range(5):
        h.eval_all(v, g=g, jac=jac)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        h.eval_all(v, g=g, jac=jac)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = 8 * (h.nv + h.ng + h.nnz_jac)
    out = {"workload": "cfg3: OcpFes DingModelPulseWidthFrequency, 30 pulses, n_shooting=100, truncation 10, force "
                       "tracking, RK1 x 10; one launch = g + J_g of every instance",
           "batch": B, "nv": h.nv, "ng": h.ng, "nnz_jac": h.nnz_jac, "layout": "CFX_LAYOUT_TILED64",
           "ms_per_launch": ms, "instance_evals_per_s": B / (ms * 1e-3),
           "achieved_GBps": nbytes * B / (ms * 1e-3) / 1e9, "bytes_per_instance": nbytes, "cpu_baseline": None}
    h.close()
    if cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(ocp, cpu_seconds, name="ding2007", truncation=10, label="cfg3")
    return out


def keep_constant_section(h, v, g, jac, steps=50):
    """The headline launch for a caller that keeps J_g's constant values between calls (CFX_KEEP_CONSTANT_JAC, listed
    by cfx_jac_constant_mask: the -1 on x_{k+1} and the calcium row's dCn+/dCn0, 60 of cfg 2's 100 values).  Not the
    headline: Ipopt's TNLP asks for every value on every call.  `jac` holds the constants from the full evaluations."""
    import torch

    n_const = int(h.jac_constant_mask().sum())
    for _ in range(5):
        h.eval_all(v, g=g, jac=jac, keep_constant_jac=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        h.eval_all(v, g=g, jac=jac, keep_constant_jac=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = 8 * (h.nv + h.ng + h.nnz_jac - n_const)
    achieved = nbytes * h.batch / (ms * 1e-3) / 1e9
    return {"batch": h.batch, "constant_values": n_const, "nnz_jac": h.nnz_jac, "ms_per_launch": ms,
            "instance_evals_per_s": h.batch / (ms * 1e-3), "bytes_per_instance": nbytes, "achieved_GBps": achieved,
            "frac_of_hbm_peak": achieved / HBM_PEAK_GBS}


def convergence(device):
    """Second half of the BASELINE metric: wall-clock to an Ipopt-equivalent KKT point (tol 1e-6) of the batched
    interior-point driver over libcfx (cocofest_amd/solver.py), single instance and multi-start batch.  Each case under
    this library's profile (IpmOptions(): monotone mu; the keys without suffix, as in earlier rounds) and under the
    facade's default, the Ipopt / bioptim profile the reference solves with (Solver.IPOPT(): adaptive mu, Ipopt's bound
    push / multipliers / relaxation; keys "..._ipopt_profile")."""
    from cocofest_amd.solver import IpmOptions, NativeIpm

    out = {}
    # cfg 3: Ding2007 pulse width, 30 pulses, N = 100, force tracking (reference force curve), RK1 x 10
    ocp3 = build_cfg3()
    cases = {"cfg3_single": (ocp3, 1), "cfg3_multistart_256": (ocp3, 256), "cfg3_multistart_4096": (ocp3, 4096),
             "cfg2_single": (build_problem(), 1)}
    for name, (ocp, B) in cases.items():
        rng = np.random.default_rng(0)
        v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
        if B > 1:
            lb, ub = ocp.bounds_vector()
            free = lb != ub
            v0[:, free] = np.clip(v0[:, free] + rng.uniform(0, 1, (B, free.sum())) * np.minimum(ub[free] - lb[free], 10),
                                  lb[free], ub[free])
        for suffix, opts in (("", IpmOptions(tol=1e-6, max_iter=300)),
                             ("_ipopt_profile", IpmOptions.ipopt(tol=1e-6, max_iter=300))):
            ipm = NativeIpm(ocp, batch=B, device=device, options=opts)
            ipm.solve(v0[:, :] if B > 1 else None)  # warm-up (kernel loading, allocator)
            ipm.calls = {k: 0 for k in ipm.calls}
            res = ipm.solve(v0 if B > 1 else None)
            ipm.close()
            out[name + suffix] = {"batch": B, "wall_s": res.wall_time, "converged": int(res.converged.sum()),
                                  "iterations_max": int(res.iterations.max()),
                                  "iterations_median": float(np.median(res.iterations)),
                                  "solves_per_s": float(res.converged.sum() / res.wall_time),
                                  "callbacks": res.n_callbacks, "nv": ipm.n, "ng": ipm.m,
                                  "mu_strategy": opts.mu_strategy, "f_median": float(np.median(res.f))}
    return out


COLLOCATION_BATCH = 1 << 18


def build_collocation():
    """cfg 2 transcribed by direct collocation (OdeSolver.COLLOCATION(4, "legendre"), bioptim's default degree; the
    transcription north_star names; the reference accepts it at cocofest/optimization/fes_ocp.py:334-338)."""
    from cocofest_amd import ModelMaker, OcpFes, OdeSolver

    model = ModelMaker.create_model("ding2003", stim_time=[round(0.1 * i, 1) for i in range(10)],
                                    sum_stim_truncation=20)
    return OcpFes.prepare_ocp(model=model, final_time=1, objective={"end_node_tracking": 100},
                              ode_solver=OdeSolver.COLLOCATION(4, "legendre"), n_shooting=20)


def collocation_synthetic(ocp, B, device, seed=7):
    """Tiled (B / 64, nv, 64) decision vectors of the collocation cfg 2: Cn ~ U(0, 1.5), F ~ U(0, 250) at every node
    and collocation point."""
    import torch

    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    v = torch.rand((ocp.nv, B), generator=gen, dtype=torch.float64, device=device)
    v *= torch.tensor([1.5, 250.0] * (ocp.nv // 2), dtype=torch.float64, device=device)[:, None]
    return to_tiled(v)


def collocation_pmc():
    """HBM bytes per launch of the collocation g + J_g kernel from the committed PMC summary, if any."""
    f = ROOT / "profiles" / "pmc_traffic_collocation.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d if d.get("batch") == COLLOCATION_BATCH else None
    except Exception:
        return None


def collocation_pattern_ceiling():
    """The collocation kernel's traffic pattern with no arithmetic (scripts/micro/colloc_bw.hip, committed run):
    ms per launch by variant, or None."""
    f = ROOT / "profiles" / "round4" / "collocation" / "colloc_bw.jsonl"
    try:
        return {d["variant"]: d["ms"] for d in map(json.loads, f.read_text().splitlines()) if d.get("batch") ==
                COLLOCATION_BATCH}
    except Exception:
        return None


def collocation_section(device, steps=50):
    """The same cfg-2 problem transcribed by direct collocation: g + J_g throughput of k_colloc over a device-resident
    SoA batch (the handle's default launch shape: two instances per lane, intervals-fast grid; 64-instance tiles timed
    beside it), its roofline (algorithmic HBM bytes — read v, write g and J_g — over the launch time from HIP events on
    the launch stream) against the pattern's own ceiling (the same traffic with no arithmetic), and the fused g + J_g +
    Hessian launch (cfx_eval_all_h, one kernel) timed the same way."""
    import torch

    ocp = build_collocation()
    B = COLLOCATION_BATCH
    dev = f"cuda:{device}"
    vt = collocation_synthetic(ocp, B, dev)
    ht = ocp.nlp(batch=B, layout="tiled64", device=device)
    gt = torch.empty((B // 64, ht.ng, 64), dtype=torch.float64, device=dev)
    jt = torch.empty((B // 64, ht.nnz_jac, 64), dtype=torch.float64, device=dev)
    h = ocp.nlp(batch=B, layout="soa", device=device)
    v = vt.transpose(1, 2).reshape(B, h.nv).T.contiguous()  # tiles -> SoA (nv, B)
    g = torch.empty((h.ng, B), dtype=torch.float64, device=dev)
    jac = torch.empty((h.nnz_jac, B), dtype=torch.float64, device=dev)

    def timed(fn, n):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    ms_tiled = timed(lambda: ht.eval_all(vt, g=gt, jac=jt), steps)
    ht.close()
    del gt, jt
    ms = timed(lambda: h.eval_all(v, g=g, jac=jac), steps)
    nbytes = 8 * (h.nv + h.ng + h.nnz_jac)
    achieved = nbytes * B / (ms * 1e-3) / 1e9
    # the caller that keeps the constant J_g values (cfx_jac_constant_mask: C off the point's own state, the calcium
    # row, D and -1 — 48 of 56 per interval) in its buffer: CFX_KEEP_CONSTANT_JAC skips their stores
    n_const = int(h.jac_constant_mask().sum())
    ms_keep = timed(lambda: h.eval_all(v, g=g, jac=jac, keep_constant_jac=True), steps)
    nbytes_keep = 8 * (h.nv + h.ng + h.nnz_jac - n_const)
    pmc = collocation_pmc()
    lam = torch.randn((h.ng, B), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(3))
    of = torch.ones((B,), dtype=torch.float64, device=dev)
    hs = torch.empty((h.nnz_hess, B), dtype=torch.float64, device=dev)
    ms_h = timed(lambda: h.eval_all_h(v, of, lam, g=g, jac=jac, hess=hs), max(steps // 5, 5))
    nbytes_h = 8 * (2 * h.nv + 2 * h.ng + h.nnz_jac + h.nnz_hess)  # + read lambda, write the Hessian values
    shape = h.launch_shape()
    h.close()
    ceil = collocation_pattern_ceiling()
    return {"workload": "cfg2 by direct collocation, Legendre degree 4 (nv = 202, ng = 200); one launch = g + J_g of "
                        "every instance", "batch": B, "nv": ocp.nv, "ng": int(ocp.n_shooting * ocp.ngk),
            "nnz_jac": nbytes // 8 - ocp.nv - ocp.n_shooting * ocp.ngk, "layout": "CFX_LAYOUT_SOA",
            "launch_shape": shape, "ms_per_launch": ms, "instance_evals_per_s": B / (ms * 1e-3),
            "achieved_GBps": achieved, "bytes_per_instance": nbytes,
            "tiled64_ms_per_launch": ms_tiled,
            "pattern_ceiling": None if not ceil else {
                "source": "scripts/micro/colloc_bw.hip (profiles/round4/collocation/colloc_bw.jsonl): the same reads "
                          "and stores, no arithmetic", "soa_nt_ms": ceil.get("soa_nt"), "tiled_nt_ms": ceil.get("tiled_nt"),
                "kernel_over_pattern_soa": ceil["soa_nt"] / ms if ceil.get("soa_nt") else None},
            "roofline": {"bound": "hbm", "kernel": "cfx::k_colloc_soa<DING2003, TMAX=1, DEG=4, NI=2> (its own name in traces since round 5)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                         "traffic_source": pmc.get("source") if pmc else None},
            "jac_constants_kept": {"constant_values": n_const, "ms_per_launch": ms_keep,
                                   "bytes_per_instance": nbytes_keep, "instance_evals_per_s": B / (ms_keep * 1e-3),
                                   "achieved_GBps": nbytes_keep * B / (ms_keep * 1e-3) / 1e9},
            "fused_g_jac_hess": {"kernel": "cfx::k_colloc_hess<DING2003, DJ=2, TMAX=1, GJ=true>",
                                 "ms_per_launch": ms_h, "bytes_per_instance": nbytes_h,
                                 "achieved_GBps": nbytes_h * B / (ms_h * 1e-3) / 1e9}}


def nmpc_section(device, n_windows, dist=None, world=1, rank=0, backend="nccl", batch=64):
    """cfg 4 (BASELINE.json configs[3]): Hmed2018 pulse-intensity NMPC, receding 1 s horizons of 10 pulses
    (N = 10, truncation 10, RK1 x 10, the reference force curve tracked in every horizon), ``batch`` independent
    scenarios (random initial states) advancing in lockstep per GPU.  Horizons of one trajectory are sequential;
    scenarios are what shards: every rank runs its own ``batch`` scenarios (weak scaling), timed between
    barriers (max over ranks), and the committed force trajectories of all ranks are all-gathered at the end
    (RCCL over xGMI with the nccl backend) — the only exchange the path has."""
    import torch

    from cocofest_amd import DingModelPulseIntensityFrequency, OdeSolver
    from cocofest_amd.nmpc import FesNmpc

    ft = json.loads((ROOT / "tests" / "golden" / "ref_formulas.json").read_text())["misc"]["force_tracking"]
    model = DingModelPulseIntensityFrequency(stim_time=[round(0.1 * i, 1) for i in range(10)], sum_stim_truncation=10)
    nmpc = FesNmpc(model, cycle_duration=1.0, n_cycles_simultaneous=1, n_cycles_to_advance=1,
                   objective={"force_tracking": [np.array(ft["time"]), np.array(ft["force"])]},
                   pulse_intensity={"max": 130}, ode_solver=OdeSolver.RK1(n_integration_steps=10), batch=batch,
                   device=device)
    rng = np.random.default_rng(rank)
    x0 = np.stack([rng.uniform(0, 0.5, batch), rng.uniform(0, 50, batch)], axis=1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    res = nmpc.solve(n_cycles=n_windows, x0=x0)
    wall = time.perf_counter() - t0
    its = np.stack(res.iterations)
    conv = np.stack(res.converged)
    out = {"workload": "Hmed2018 pulse-intensity NMPC, 1 s horizons x 10 pulses, N = 10, truncation 10, RK1 x 10, "
                       "force tracking per horizon", "horizons": n_windows, "scenarios_per_gpu": batch, "n_gpus": world,
           "scaling": "weak", "parallelism": f"scenarios sharded over {world} GPU(s); committed trajectories "
                                             "all-gathered at the end"}
    conv_frac = float(conv.mean())
    if dist:
        dev = f"cuda:{device}" if backend == "nccl" else "cpu"
        t = torch.tensor([wall, 1.0 - conv_frac], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, conv_frac = float(t[0]), 1.0 - float(t[1])
        F = torch.as_tensor(np.ascontiguousarray(res.states["F"]), dtype=torch.float64, device=dev)
        parts = [torch.empty_like(F) for _ in range(world)]
        dist.all_gather(parts, F)
        out["gathered_force_shape"] = [world] + list(F.shape)
    out.update({"wall_s": wall, "ms_per_horizon": wall / n_windows * 1e3,
                "scenario_horizons_per_s": world * batch * n_windows / wall, "converged_frac": conv_frac,
                "iterations_median": float(np.median(its)), "iterations_max": int(its.max()),
                # the interior point's share of a horizon (NativeIpm.solve wall-clock); the rest is the host's window
                # bookkeeping (warm start shift, history, fixed values)
                "solve_ms_per_horizon": float(np.sum(res.solve_wall)) / n_windows * 1e3})
    return out


def ivp_section(device):
    """IvpFes.integrate on the configuration of the reference's own timings
    (examples/sensitivity/truncation/sensitivity_analysis.py: DingModelFrequencyWithFatigue, 10 single pulses,
    truncation 10, final time 1 s, default RK4 x 10; 106.9 ms per integrate() in the authors' pickle,
    truncation_single.pkl, unknown hardware): per-call latency at batch 1 (host arrays in / out, as
    integrate() is called), and the batched kernel throughput over device-resident initial states."""
    import torch

    from cocofest_amd import DingModelFrequencyWithFatigue, IvpFes

    ivp = IvpFes(fes_parameters={"model": DingModelFrequencyWithFatigue(stim_time=[round(0.1 * i, 1) for i in range(10)],
                                                                        sum_stim_truncation=10)},
                 ivp_parameters={"final_time": 1})
    for _ in range(5):
        ivp.integrate(return_time=False)
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        ivp.integrate(return_time=False)
    ms_b1 = (time.perf_counter() - t0) / reps * 1e3
    ivp.close()
    B = 1 << 16
    h = ivp.handle(batch=B, layout="soa", device=device)
    rest = torch.tensor([0.0, 0.0, 3009.0, 0.050957, 0.103], dtype=torch.float64, device=f"cuda:{device}")
    gen = torch.Generator(device=f"cuda:{device}")
    gen.manual_seed(5)
    x0 = (rest[:, None] * (0.8 + 0.2 * torch.rand((5, B), generator=gen, dtype=torch.float64,
                                                  device=f"cuda:{device}"))).contiguous()
    traj = torch.empty((h.n_shooting * h.n_steps + 1) * h.nx, B, dtype=torch.float64, device=f"cuda:{device}")
    for _ in range(3):
        h.integrate(x0=x0, traj=traj)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        h.integrate(x0=x0, traj=traj)
    e1.record()
    torch.cuda.synchronize()
    ms_batch = e0.elapsed_time(e1) / 10
    h.close()
    return {"config": "IvpFes DingModelFrequencyWithFatigue, 10 pulses @10 Hz, truncation 10, final_time 1 s, "
                      "RK4 x 10 (N = 10, 101 samples per state)",
            "ms_per_integrate_b1": ms_b1, "reference_ms_per_integrate": 106.9,
            "reference_source": "truncation_single.pkl (authors' data, older API, unknown hardware)",
            "batch": B, "ms_per_batched_launch": ms_batch, "integrations_per_s": B / (ms_batch * 1e-3)}


def msk_cpu_baseline(ocp, budget_s):
    """cfg-5 CPU baseline: the plain-C port of the musculoskeletal oracle (oracle/c/fes_msk.c: full segment tree,
    Newton-Euler forward dynamics with unit accelerations, as-written calcium sum, complex-step Jacobian columns),
    all usable host cores, on a bounded sample of the same workload (g + J_g of cfg-5 instances at RK4 x 1)."""
    from oracle import c_msk, fes_msk as M, fes_oracle as O

    threads = min(16, len(os.sched_getaffinity(0)))
    bm = json.loads((ROOT / "tests" / "golden" / "biomod_arm26_biceps_triceps.json").read_text())
    mus = [M.MskMuscle(model="ding2007_with_fatigue", name=n, c=O.model_constants("ding2007_with_fatigue"))
           for n in ("BIClong", "TRIlong")]
    pb = M.MskProblem(bm=bm, muscles=mus, rows=np.asarray(ocp.stim_rows, dtype=np.float64),
                      n_shooting=ocp.n_shooting, final_time=1.0, scheme="RK4", m=1, fv_on=True)
    lo, hi = ocp.bounds_vector()
    lo = np.where(np.isfinite(lo), lo, -2.0)
    hi = np.minimum(np.where(np.isfinite(hi), hi, 2.0), lo + 100.0)
    chunk = 16 * threads
    v = lo + (hi - lo) * (0.2 + 0.6 * np.random.default_rng(11).random((chunk, pb.nv)))
    c_msk.shooting(pb, v[:threads], threads=threads)  # load
    done, t0 = 0, time.perf_counter()
    while True:
        c_msk.shooting(pb, v, threads=threads)
        done += chunk
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": done / el, "unit": "instance-evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} cfg-5 instances (g + J_g, RK4 x 1), oracle/c/fes_msk.c, OpenMP {threads} threads, "
                      f"{el:.1f} s"}


def msk_build(m):
    """BASELINE.json configs[4]: arm26 biceps / triceps + Ding2007 with fatigue, 10 pulses
    @ 10 Hz, 1 s, elbow 5 -> 90 deg, force-length / force-velocity on, qdot(end) = 0 and minimize_muscle_fatigue
    (examples/dynamics/minimize_fatigue/pulse_duration_optimization_minimize_fatigue.py:15-55), RK4 x m."""
    import cocofest_amd as C

    mm = C.FesMskModel(biorbd_path=str(ROOT / "tests" / "golden" / "biomod_arm26_biceps_triceps.json"),
                       muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=10)
                                      for n in ("BIClong", "TRIlong")],
                       stim_time=[round(0.1 * i, 1) for i in range(10)], activate_force_length_relationship=True,
                       activate_force_velocity_relationship=True)
    ol = C.ObjectiveList()
    ol.add(C.ObjectiveFcn.Mayer.MINIMIZE_STATE, key="qdot", index=[0, 1], node=C.Node.END,
           target=np.zeros((2, 1)), weight=100)
    return C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, objective={"custom": ol, "minimize_muscle_fatigue": True},
                                   msk_info={"bound_type": "start_end", "bound_data": [[0, 5], [0, 90]]},
                                   ode_solver=C.OdeSolver.RK4(n_integration_steps=m))


def msk_throughput(local, dist, world, rank, backend, steps=10, B=1 << 16):
    """cfg-5 g + J_g throughput at OcpFesMsk's default transcription (RK4 x 1) over a device-resident SoA batch of
    B instances per GPU (the "multi-muscle batched Jacobian on 1 -> 8 GPUs" of configs[4]): every rank evaluates
    its own instances (no data-path collective), timed between barriers, max over ranks."""
    import torch

    ocp = msk_build(1)
    dev = f"cuda:{local}"
    h = ocp.nlp(batch=B, layout="soa", device=local)
    lo, hi = ocp.bounds_vector()
    lo = np.where(np.isfinite(lo), lo, -2.0)
    hi = np.minimum(np.where(np.isfinite(hi), hi, 2.0), lo + 100.0)  # forces up to 100 N, |qdot| <= 2 rad/s
    gen = torch.Generator(device=dev)
    gen.manual_seed(11 + rank)
    r = 0.2 + 0.6 * torch.rand((h.nv, B), generator=gen, dtype=torch.float64, device=dev)
    v = (torch.as_tensor(lo, device=dev)[:, None] + torch.as_tensor(hi - lo, device=dev)[:, None] * r).contiguous()
    g = torch.empty((h.ng, B), dtype=torch.float64, device=dev)
    jac = torch.empty((h.nnz_jac, B), dtype=torch.float64, device=dev)
    for _ in range(3):
        h.eval_all(v, g=g, jac=jac)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        h.eval_all(v, g=g, jac=jac)
    e1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    nbytes = 8 * (h.nv + h.ng + h.nnz_jac)
    out = {"workload": "cfg5: arm26 biceps/triceps + Ding2007 with fatigue, 10 pulses @ 10 Hz, 1 s, 5 -> 90 deg, "
                       "FL/FV on, RK4 x 1 (OcpFesMsk default); one step = g + J_g of every instance",
           "n_gpus": world, "batch_per_gpu": B, "nv": h.nv, "ng": h.ng, "nnz_jac": h.nnz_jac,
           "ms_per_step": wall_max / steps * 1e3, "kernel_ms_per_step": e0.elapsed_time(e1) / steps,
           "instance_evals_per_s": world * B / (wall_max / steps),
           "algorithmic_GBps": nbytes * world * B / (wall_max / steps) / 1e9, "bytes_per_instance": nbytes,
           "scaling": "weak", "parallelism": f"instances sharded over {world} GPU(s), no data-path collective",
           "kernels": "k_msk_values + k_msk_stagecoef_par + k_msk_tangents_lds (compute-bound: FP64 VALU, see profiles/)"}
    pmc = msk_pmc()
    if pmc and pmc.get("batch") == B:
        # compute-bound: the FP64 instruction issue rate of the step's three kernels (committed SQ_INSTS_VALU_{FMA,
        # MUL,ADD,TRANS}_F64 per step over the step's kernel time measured here) against the measured FP64 FMA issue
        # peak; the all-VALU rate beside it (an upper bound on FP64-pipe use)
        f64 = pmc.get("f64_wave_instr_per_step")
        valu = pmc.get("valu_wave_instr_per_step")
        t = out["kernel_ms_per_step"] * 1e-3
        achieved = (f64 if f64 else valu) / t
        traffic = pmc.get("hbm_bytes_per_step")
        out["roofline"] = {"bound": "fp64_valu", "achieved": achieved, "peak": FP64_FMA_ISSUE_PEAK,
                           "unit": "FP64 wave-instr/s" if f64 else "VALU wave-instr/s",
                           "frac": achieved / FP64_FMA_ISSUE_PEAK,
                           "valu_frac": valu / t / FP64_FMA_ISSUE_PEAK if valu else None,
                           "traffic": traffic, "traffic_over_algorithmic": traffic / (nbytes * B) if traffic else None,
                           "traffic_GBps": traffic / t / 1e9 if traffic else None,
                           "per_kernel": pmc.get("kernels"), "source": pmc.get("source")}
    h.close()
    return out, ocp


def msk_section(device, tp, ocp1, cpu_seconds=0.0, multistart=True):
    """The N = 1 extras of the cfg-5 section: the C port's CPU baseline on a bounded sample of the same workload,
    and the batched interior point's wall-clock to convergence at RK4 x 5 (the default RK4 x 1 is infeasible for
    Ding2007's tau_c)."""
    from cocofest_amd.solver import IpmOptions, NativeIpm

    out = dict(tp)
    out["cpu_baseline"] = msk_cpu_baseline(ocp1, cpu_seconds) if cpu_seconds > 0 else None
    for key, opts in (("convergence_rk4x5", IpmOptions(tol=1e-6, max_iter=1000)),
                      ("convergence_rk4x5_ipopt_profile", IpmOptions.ipopt(tol=1e-6, max_iter=1000))):
        ipm = NativeIpm(msk_build(5), batch=1, device=device, options=opts)
        res = ipm.solve()
        ipm.close()
        out[key] = {"wall_s": res.wall_time, "converged": int(res.converged.sum()), "status": int(res.status[0]),
                    "iterations": int(res.iterations.max()), "f": float(res.f[0])}
    if multistart:
        out["multistart_512"] = msk_multistart(device)
    return out


def msk_multistart(device, B=512, amp=0.1):
    """Restoration robustness: cfg 5 at RK4 x 5 from B starts perturbed by +-amp of each free
    variable's range (capped at 10; seed 0; scripts/msk_multistart_probe.py's starts), max_iter 1000, tol 1e-6, under
    the facade's Ipopt / bioptim profile, the same with Ipopt's mu_max option at 0.1 (= mu_init: the adaptive update never
    raises the barrier above its start), and this library's monotone profile."""
    from cocofest_amd._cfx import IPM_STATUS
    from cocofest_amd.solver import IpmOptions, NativeIpm

    ocp = msk_build(5)
    rng = np.random.default_rng(0)
    v0 = np.tile(ocp.initial_guess_vector(), (B, 1))
    lb, ub = ocp.bounds_vector()
    free = lb != ub
    span = np.minimum(np.where(np.isfinite(ub - lb), ub - lb, 10.0), 10.0)[free]
    v0[:, free] = np.clip(v0[:, free] + amp * rng.uniform(-1, 1, (B, free.sum())) * span, lb[free], ub[free])
    out = {"starts": B, "amplitude": amp, "max_iter": 1000}
    for key, opts in (("ipopt_profile", IpmOptions.ipopt(tol=1e-6, max_iter=1000)),
                      ("ipopt_profile_mu_max_0.1", IpmOptions.ipopt(tol=1e-6, max_iter=1000, mu_max=0.1)),
                      ("library_profile", IpmOptions(tol=1e-6, max_iter=1000))):
        ipm = NativeIpm(ocp, batch=B, device=device, options=opts)
        res = ipm.solve(v0)
        ipm.close()
        conv = res.converged.astype(bool)
        hist = {}
        for st in res.status:
            k = IPM_STATUS.get(int(st), str(int(st)))
            hist[k] = hist.get(k, 0) + 1
        out[key] = {"converged": int(conv.sum()), "rate": float(conv.mean()), "status": hist, "wall_s": res.wall_time,
                    "f_converged": [float(res.f[conv].min()), float(res.f[conv].max())] if conv.any() else None}
    return out


REACHING_MUSCLES = ["BIClong", "BICshort", "TRIlong", "TRIlat", "TRImed", "BRA"]


def build_reaching(objective="fatigue"):
    """The reference's reaching task (examples/dynamics/reaching_task/reaching_task_pulse_duration_optimization.py:
    27-118) as the product states its stored revision (tests/test_reference_solution.py::legacy_product): arm26 with
    six Ding2007-with-fatigue muscles (fibre-type and PCSA proportions, the stored revision's fatigue rates x 10), 60
    pulses at 40 Hz over 1.5 s, N = 1,500, RK4 x 1, the hand on the target at node 1000, per-pulse widths, no residual
    torque.  Data only from tests/golden (the bioMod as parsed JSON)."""
    import cocofest_amd as C

    root = os.path.dirname(os.path.abspath(__file__))
    alpha_a_prop = [0.607, 0.607, 0.465, 0.465, 0.465, 0.457]
    a_scale_prop = [12.7 / 28.3, 12.7 / 28.3, 1.0, 1.0, 1.0, 11.6 / 28.3]
    stims = [float(s) for s in np.round(np.linspace(0, 1.5, 61), 3)[:-1]]
    models = []
    for i, n in enumerate(REACHING_MUSCLES):
        mm = C.DingModelPulseWidthFrequencyWithFatigue(muscle_name=n, sum_stim_truncation=60)
        mm.alpha_a = mm.alpha_a * alpha_a_prop[i] * 10.0
        mm.alpha_tau1 = mm.alpha_tau1 * 10.0
        mm.alpha_km = mm.alpha_km * 10.0
        mm.a_scale = mm.a_scale * a_scale_prop[i]
        models.append(mm)
    model = C.FesMskModel(biorbd_path=os.path.join(root, "tests", "golden", "biomod_arm26.json"), muscles_model=models,
                          stim_time=stims, activate_force_length_relationship=True,
                          activate_force_velocity_relationship=True, activate_residual_torque=False,
                          legacy_calcium=True)
    cl = C.ConstraintList()
    cl.add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker="COM_hand", second_marker="reaching_target", phase=0,
           node=1000, axes=[C.Axis.X, C.Axis.Y])
    return C.OcpFesMsk.prepare_ocp(model=model, final_time=1.5, n_shooting=1500,
                                   pulse_width={"min": C.DingModelPulseWidthFrequency().pd0, "max": 0.0006,
                                                "per_pulse": True},
                                   objective={f"minimize_muscle_{objective}": True},
                                   msk_info={"with_residual_torque": False, "bound_type": "start_end",
                                             "bound_data": [[0, 5], [0, 5]], "custom_constraint": cl},
                                   ode_solver=C.OdeSolver.RK4(n_integration_steps=1), apply_custom_constraint=True)


def reaching_section(device, wall_limit=150.0):
    """Wall-clock to convergence of the one reference OCP with a timed reference solve: the fatigue objective of the
    reaching task from the product's default initial guess (the reference script's own start), Ipopt's termination
    tests at tol 1e-6; the stage-chain KKT layout (block cyclic reduction).  Headline: the reference's own solver
    settings — the script's Solver.IPOPT(_max_iter=10000) through the facade's Ipopt / bioptim profile (adaptive mu,
    bound_relax_factor 1e-8, ...); beside it this library's profile (monotone mu).  And the reference's own
    time_to_optimize (sol.real_time_to_optimize, cocofest/result/pickle.py:32; unknown hardware, an older revision,
    use_sx=False) — a max_iter iterate, not a converged solve (tests/test_reaching_termination.py)."""
    from cocofest_amd import Solver
    from cocofest_amd.solver import IpmOptions, NativeIpm

    root = os.path.dirname(os.path.abspath(__file__))
    ref_t = float(np.load(os.path.join(root, "tests", "golden", "reaching_pulse_duration_fatigue.npz"))["time_to_optimize"])
    ocp = build_reaching("fatigue")
    out = {}
    for key, opts in (("ipopt_profile", Solver.IPOPT(_max_iter=10000, _max_wall_time=wall_limit).options()),
                      ("library_profile", IpmOptions(tol=1e-6, max_iter=5000, bound_relax_factor=1e-8,
                                                     max_wall_time=wall_limit))):
        ipm = NativeIpm(ocp, batch=1, device=device, options=opts)
        res = ipm.solve()
        st = dict(ipm.last_stats)
        ipm.close()
        out[key] = {"wall_s": res.wall_time, "iterations": int(res.iterations[0]), "status": int(res.status[0]),
                    "converged": bool(res.converged[0]), "f": float(res.f[0]), "mu_strategy": opts.mu_strategy,
                    "s_per_iteration": res.wall_time / max(1, int(res.iterations[0])),
                    "reference_over_product": ref_t / res.wall_time}
    head = out["ipopt_profile"]
    return {"objective": "fatigue (minimize_muscle_fatigue)", "start": "product default initial guess",
            "solver": "Solver.IPOPT(_max_iter=10000) (the reference script's call; the facade's Ipopt / bioptim profile)",
            **head, "library_profile": out["library_profile"], "f_stored_reference_iterate": 7.841959196,
            "kkt_layout": {"chain_nodes": int(st["kkt_chain_nodes"]), "node_size": int(st["kkt_chain_sp"]),
                           "border": int(st["kkt_border"]), "kkt_unknowns": int(st["kkt_n"])},
            "reference_time_to_optimize_s": ref_t,
            "note": "reference timing on unknown hardware with an older revision (use_sx=False), ending at its max_iter "
                    "(tests/test_reaching_termination.py); stated as context"}


def main():
    args = parse()
    import torch

    from cocofest_amd import _cfx

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.backend == "gloo":  # rehearsal: ranks share the visible GPUs
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":  # RCCL on ROCm
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    ocp = build_problem()
    B = args.batch
    h = ocp.nlp(batch=B, layout="tiled64", device=local)
    v = to_tiled(synthetic_soa(ocp, B, seed=1234 + rank, device=f"cuda:{local}"))
    g = torch.empty((B // 64, h.ng, 64), dtype=torch.float64, device=f"cuda:{local}")
    jac = torch.empty((B // 64, h.nnz_jac, 64), dtype=torch.float64, device=f"cuda:{local}")

    # Settle: an idle MI355X that starts this load runs the first few launches fast (0.30 ms), then drops to
    # 0.43 ms for ~20 ms of power-management transient before settling near 0.31 ms (profiles/round2/cold_probe.json).
    # A K = 20 loop right behind W = 5 warmup steps would time that transient, not the sustained rate, so the
    # headline launch runs untimed for `--settle` seconds first (then the W warmup steps, then the K timed steps).
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(10):
            h.eval_all(v, g=g, jac=jac)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        h.eval_all(v, g=g, jac=jac)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        h.eval_all(v, g=g, jac=jac)
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel launch per step, on this stream

    t = torch.tensor([wall], dtype=torch.float64, device=f"cuda:{local}" if args.backend == "nccl" else "cpu")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    ms_per_step = wall_max / args.steps * 1e3
    value = world * B / (wall_max / args.steps)

    bytes_per_instance = 8 * (h.nv + h.ng + h.nnz_jac)  # read v, write g and J_g values
    achieved = bytes_per_instance * B / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic()

    kept = keep_constant_section(h, v, g, jac) if (world == 1 and not args.no_solve) else None
    msk_tp, msk_ocp = msk_throughput(local, dist, world, rank, args.backend) if not args.no_msk else (None, None)
    # cfg 4 on every rank (scenarios shard; weak scaling)
    nm = nmpc_section(local, args.nmpc_horizons, dist, world, rank, args.backend) \
        if (not args.no_solve and args.nmpc_horizons) else None

    out = None
    if rank == 0:
        cpu = cpu_baseline(ocp, args.cpu_seconds) if (world == 1 and args.cpu_seconds > 0) else None
        conv = convergence(local) if (world == 1 and not args.no_solve) else None
        ivp = ivp_section(local) if (world == 1 and not args.no_solve) else None
        col = collocation_section(local) if (world == 1 and not args.no_solve) else None
        c3 = cfg3_section(local, args.cpu_seconds / 4) if (world == 1 and not args.no_solve) else None
        reach = reaching_section(local) if (world == 1 and not args.no_solve and not args.no_reaching) else None
        msk = msk_tp
        if msk_tp is not None and world == 1 and not args.no_solve:
            msk = msk_section(local, msk_tp, msk_ocp, cpu_seconds=args.cpu_seconds / 2, multistart=not args.no_multistart)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "instance-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded decision vectors around physiological states)",
            "config": {
                "workload": "cfg2: OcpFes DingModelFrequency n_stim=10 @10Hz, final_time=1s, n_shooting=20, "
                            "end_node_tracking=100N, RK1 x 10 multiple shooting; one step = g + J_g of every instance",
                "batch_per_gpu": B,
                "nv": h.nv, "ng": h.ng, "nnz_jac": h.nnz_jac,
                "layout": "CFX_LAYOUT_TILED64 (64-instance tiles, element-major inside a tile), device-resident",
                "parallelism": f"instances sharded over {world} GPU(s), no data-path collective",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "cfx::k_shooting<DING2003, RK1, D=2, NI=2>",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_instance": bytes_per_instance,
                "kernel_ms": kern_ms,
            },
            "cpu_baseline": cpu,
            "jac_constants_kept": kept,
            "convergence": conv,
            "ivp": ivp,
            "collocation": col,
            "cfg3_callbacks": c3,
            "nmpc": nm,
            "msk": msk,
            "reaching": reach,
        }
    h.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
