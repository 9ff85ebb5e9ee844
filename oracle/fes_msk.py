"""CPU oracle for the musculoskeletal FES path (FesMskModel / OcpFesMsk).

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``cocofest_amd``) imports, links or executes this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it, as the checker.

What it restates (Ipuch/cocofest @ 2025-02-24):
  - ``FesMskModel.muscle_dynamic`` / ``muscles_joint_torque`` (cocofest/models/dynamical_model.py:133-334): every
    muscle's FES ODE (the six Ding / Hmed right-hand sides, ``oracle.fes_oracle.rhs``) scaled by the De Groote
    force-length / force-velocity / passive-force coefficients (cocofest/models/hill_coefficients.py:11-126), the
    joint torque ``-J_L(q)^T F`` from the muscle-tendon length Jacobian, and the rigid-body forward dynamics;
  - the reference's flag quirk: the force-length coefficient is computed only when
    ``activate_force_velocity_relationship`` is set (dynamical_model.py:260-267), and ``OcpFesMsk`` rebuilds the
    model without ``activate_passive_force_relationship`` (fes_ocp_dynamics.py:120-131), so passive force is off
    in every OCP;
  - the OCP layout of ``OcpFesMsk`` (fes_ocp_dynamics.py:33-801): states [muscle blocks (Cn, F[, A, Tau1, Km]) in
    muscle order, q, qdot] (dynamical_model.py:382-404, state_configure.py:294-307), controls [last_pulse_width
    per muscle (Ding2007)] then [tau] with residual torque, bounds and objective terms.

What lives in an absent third-party library and is restated from its published algorithm (biorbd, the C++
rigid-body library behind bioptim's ``BiorbdModel``; no version pinned by the reference, ``environment.yml``):
  - bioMod parsing (the subset the reference's ``examples/msk_models/*.bioMod`` use): a segment's frame is
    parent frame x RT x R(dofs) with RT given as a 4x4 matrix (``RTinMatrix 1``) and the dofs rotations about the
    segment's own axes in the declared order;
  - muscle-tendon length = sum of the straight segments origin -> via points -> insertion in the global frame;
    muscle (fibre) length = (muscle-tendon length - tendon slack length) / cos(pennation angle); length Jacobian
    = sum of u_i^T (J_{P_{i+1}} - J_{P_i}) with u_i the unit segment vectors; muscle velocity = J_L qdot;
  - forward dynamics qddot = M(q)^-1 (tau - C(q, qdot) qdot - G(q)) (RBDL's ABA returns the same quantity): here
    from a recursive Newton-Euler inverse dynamics in world coordinates, M by unit accelerations.  The HIP kernel
    forms M from body Jacobians instead, so the two are independent computations.

Parity status: **parity unpinned** against the reference for the MSK path — biorbd, bioptim, CasADi and Ipopt
are absent here, and the reference's MSK golden costs (tests/shard2/test_fes_dynamics.py:58,139) are written
against a stale API (``is_approximated`` models, pulse widths as parameters).  The oracle is checked for
self-consistency instead (tests/test_msk_oracle.py): energy conservation of the unforced arm under gravity, the
length Jacobian against finite differences of the length, M symmetric positive definite, and the Hill
coefficients against the reference's own closed forms.

Derivatives of the NLP callbacks are complex-step (every function on the path is analytic; the only branch,
the passive-force clip at 0, tests the real part), independent of the kernels' forward-mode dual numbers.
"""

from __future__ import annotations

import ast
import operator
from dataclasses import dataclass, field

import numpy as np

from . import fes_oracle as O

# --------------------------------------------------------------------------------------------------------------
# bioMod subset parser (biorbd file format)
# --------------------------------------------------------------------------------------------------------------

_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv}


def _num(tok: str) -> float:
    """A bioMod number: a literal or a small arithmetic expression in ``pi`` (``-2*pi``)."""

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant) and isinstance(n.value, (int, float)):
            return float(n.value)
        if isinstance(n, ast.Name) and n.id == "pi":
            return float(np.pi)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, (ast.USub, ast.UAdd)):
            v = ev(n.operand)
            return -v if isinstance(n.op, ast.USub) else v
        if isinstance(n, ast.BinOp) and type(n.op) in _BINOPS:
            return _BINOPS[type(n.op)](ev(n.left), ev(n.right))
        raise ValueError(f"bioMod: cannot read number {tok!r}")

    return ev(ast.parse(tok, mode="eval"))


def parse_biomod(text: str) -> dict:
    """Segments (parent, RT, rotation dofs, mass, com, inertia, q ranges), gravity, markers (parent segment,
    position) and muscles (origin, via points, insertion, optimal length, maximal force, tendon slack length,
    pennation angle)."""
    toks = []
    for line in text.splitlines():
        line = line.split("//")[0]
        toks.extend(line.split())
    pos = 0

    def nxt():
        nonlocal pos
        pos += 1
        return toks[pos - 1]

    def nums(n):
        return [_num(nxt()) for _ in range(n)]

    out = {"gravity": [0.0, 0.0, -9.81], "segments": [], "markers": [], "muscles": [], "groups": {}}
    vias = []
    while pos < len(toks):
        t = nxt()
        tl = t.lower()
        if tl == "version":
            nxt()
        elif tl == "gravity":
            out["gravity"] = nums(3)
        elif tl == "segment":
            seg = {"name": nxt(), "parent": None, "RT": np.eye(4).tolist(), "rotations": "", "mass": 0.0,
                   "com": [0.0, 0.0, 0.0], "inertia": np.zeros((3, 3)).tolist(), "rangesQ": []}
            in_matrix = False
            while True:
                k = nxt()
                kl = k.lower()
                if kl == "endsegment":
                    break
                if kl == "parent":
                    seg["parent"] = nxt()
                elif kl == "rtinmatrix":
                    in_matrix = bool(int(_num(nxt())))
                elif kl == "rt":
                    if not in_matrix:
                        raise NotImplementedError("bioMod: RT given as Euler angles (RTinMatrix 0) is not supported")
                    seg["RT"] = np.array(nums(16)).reshape(4, 4).tolist()
                elif kl == "rotations":
                    seg["rotations"] = nxt().lower()
                elif kl == "translations":
                    raise NotImplementedError("bioMod: translational dofs are not supported")
                elif kl == "mass":
                    seg["mass"] = _num(nxt())
                elif kl == "com":
                    seg["com"] = nums(3)
                elif kl == "inertia":
                    seg["inertia"] = np.array(nums(9)).reshape(3, 3).tolist()
                elif kl == "rangesq":
                    seg["rangesQ"] = np.array(nums(2 * len(seg["rotations"]))).reshape(-1, 2).tolist()
                elif kl in ("meshfile",):
                    nxt()
                elif kl in ("meshscale", "meshcolor", "mesh"):
                    nums(3)
                else:
                    raise NotImplementedError(f"bioMod: unsupported segment keyword {k!r}")
            out["segments"].append(seg)
        elif tl == "marker":  # a point fixed in its parent segment (biorbd Marker): parent, position
            mk = {"name": nxt(), "parent": None, "position": [0.0, 0.0, 0.0]}
            while True:
                k = nxt()
                kl = k.lower()
                if kl == "endmarker":
                    break
                if kl == "parent":
                    mk["parent"] = nxt()
                elif kl == "position":
                    mk["position"] = nums(3)
                elif kl in ("technical", "anatomical", "axestoremove"):
                    nxt()
                else:
                    raise NotImplementedError(f"bioMod: unsupported marker keyword {k!r}")
            out["markers"].append(mk)
        elif tl == "musclegroup":
            name = nxt()
            grp = {}
            while True:
                k = nxt()
                if k.lower() == "endmusclegroup":
                    break
                grp[k.lower()] = nxt()
            out["groups"][name] = grp
        elif tl == "muscle":
            mus = {"name": nxt(), "via": []}
            while True:
                k = nxt()
                kl = k.lower()
                if kl == "endmuscle":
                    break
                if kl in ("type", "statetype", "musclegroup"):
                    mus[kl] = nxt()
                elif kl == "originposition":
                    mus["origin"] = nums(3)
                elif kl == "insertionposition":
                    mus["insertion"] = nums(3)
                elif kl in ("optimallength", "maximalforce", "tendonslacklength", "pennationangle", "maxvelocity",
                            "pcsa", "maxexcitation", "maxactivation"):
                    mus[kl] = _num(nxt())
                elif kl == "fatigueparameters":
                    while nxt().lower() != "endfatigueparameters":
                        pass
                else:
                    raise NotImplementedError(f"bioMod: unsupported muscle keyword {k!r}")
            out["muscles"].append(mus)
        elif tl == "viapoint":
            via = {"name": nxt()}
            while True:
                k = nxt()
                kl = k.lower()
                if kl == "endviapoint":
                    break
                if kl in ("parent", "muscle", "musclegroup"):
                    via[kl] = nxt()
                elif kl == "position":
                    via["position"] = nums(3)
                else:
                    raise NotImplementedError(f"bioMod: unsupported via-point keyword {k!r}")
            vias.append(via)
        elif tl in ("wrap", "wrapping", "contact", "imu", "actuator", "externalforce"):
            raise NotImplementedError(f"bioMod: {t!r} blocks are not supported")
        else:
            raise NotImplementedError(f"bioMod: unsupported keyword {t!r}")
    for mus in out["muscles"]:
        grp = out["groups"][mus["musclegroup"]]
        mus["origin_parent"] = grp["originparent"]
        mus["insertion_parent"] = grp["insertionparent"]
        mus["via"] = [{"parent": v["parent"], "position": v["position"]} for v in vias if v["muscle"] == mus["name"]]
    return out


# --------------------------------------------------------------------------------------------------------------
# kinematics over the full segment tree (complex-safe)
# --------------------------------------------------------------------------------------------------------------


def _rot4(axis: str, a):
    c, s = np.cos(a), np.sin(a)
    R = np.eye(4, dtype=np.result_type(a, float))
    i, j = {"x": (1, 2), "y": (2, 0), "z": (0, 1)}[axis]
    R[i, i], R[i, j], R[j, i], R[j, j] = c, -s, s, c
    return R


def nb_q(bm: dict) -> int:
    return sum(len(s["rotations"]) for s in bm["segments"])


def forward_kinematics(bm: dict, q):
    """Global 4x4 frame of every segment, and per dof (global order) its world axis, origin and segment."""
    q = np.asarray(q)
    frames, dofs = {}, []
    dt = np.result_type(q.dtype, float)
    qi = 0
    for seg in bm["segments"]:
        T = frames[seg["parent"]] if seg["parent"] else np.eye(4, dtype=dt)
        T = T @ np.asarray(seg["RT"], dtype=float)
        for ax in seg["rotations"]:
            e = {"x": 0, "y": 1, "z": 2}[ax]
            dofs.append({"axis": T[:3, e].copy(), "origin": T[:3, 3].copy(), "segment": seg["name"]})
            T = T @ _rot4(ax, q[qi])
            qi += 1
        frames[seg["name"]] = T
    return frames, dofs


def _ancestors(bm: dict, name: str) -> set:
    parent = {s["name"]: s["parent"] for s in bm["segments"]}
    out = set()
    while name is not None:
        out.add(name)
        name = parent[name]
    return out


def _point_world(frames, seg, p):
    T = frames[seg]
    return T[:3, :3] @ np.asarray(p, dtype=float) + T[:3, 3]


def _point_jacobian(bm, dofs, seg, P):
    """dP/dq (3 x nq) of a point fixed in segment ``seg``: axis_k x (P - origin_k) for the dofs above it."""
    anc = _ancestors(bm, seg)
    J = np.zeros((3, len(dofs)), dtype=np.result_type(P.dtype, float))
    for k, d in enumerate(dofs):
        if d["segment"] in anc:
            J[:, k] = np.cross(d["axis"], P - d["origin"])
    return J


def marker_position(bm: dict, name: str, q):
    """World position of a bioMod marker (a point fixed in its parent segment) at q (biorbd ``markers(q)``)."""
    for mk in bm.get("markers", []):
        if mk["name"] == name:
            frames, _ = forward_kinematics(bm, q)
            return _point_world(frames, mk["parent"], mk["position"])
    raise ValueError(f"marker {name!r} is not in the bioMod")


def muscle_path(mus: dict):
    return ([(mus["origin_parent"], mus["origin"])] + [(v["parent"], v["position"]) for v in mus["via"]]
            + [(mus["insertion_parent"], mus["insertion"])])


def muscle_tendon_length(bm, mus, q):
    frames, _ = forward_kinematics(bm, q)
    pts = [_point_world(frames, s, p) for s, p in muscle_path(mus)]
    return sum(np.sqrt(np.sum((pts[i + 1] - pts[i]) ** 2)) for i in range(len(pts) - 1))


def muscle_geometry(bm, mus, q, qdot):
    """(muscle-tendon length, length Jacobian dL/dq (nq,), fibre length, muscle-tendon velocity)."""
    frames, dofs = forward_kinematics(bm, q)
    path = muscle_path(mus)
    pts = [_point_world(frames, s, p) for s, p in path]
    jac = [_point_jacobian(bm, dofs, s, P) for (s, _), P in zip(path, pts)]
    L = 0
    JL = 0
    for i in range(len(pts) - 1):
        d = pts[i + 1] - pts[i]
        n = np.sqrt(np.sum(d * d))
        L = L + n
        JL = JL + (d @ (jac[i + 1] - jac[i])) / n
    fibre = (L - mus["tendonslacklength"]) / np.cos(mus["pennationangle"])
    vel = JL @ np.asarray(qdot)
    return L, JL, fibre, vel


# --------------------------------------------------------------------------------------------------------------
# De Groote coefficients (cocofest/models/hill_coefficients.py)
# --------------------------------------------------------------------------------------------------------------


def force_length(norm_length):
    """hill_coefficients.py:11-63."""
    b11, b21, b31, b41 = 0.815, 1.055, 0.162, 0.063
    b12, b22, b32, b42 = 0.433, 0.717, -0.030, 0.200
    b13, b23, b33, b43 = 0.100, 1.000, 0.354, 0.0
    nl = norm_length
    return (b11 * np.exp((-0.5 * ((nl - b21) * (nl - b21))) / ((b31 + b41 * nl) * (b31 + b41 * nl)))
            + b12 * np.exp((-0.5 * ((nl - b22) * (nl - b22))) / ((b32 + b42 * nl) * (b32 + b42 * nl)))
            + b13 * np.exp((-0.5 * ((nl - b23) * (nl - b23))) / ((b33 + b43 * nl) * (b33 + b43 * nl))))


def force_velocity(velocity):
    """hill_coefficients.py:66-96 (maximal shortening speed constant 10)."""
    nv = velocity / 10
    d1, d2, d3, d4 = -0.318, -8.149, -0.374, 0.886
    return d1 * np.log((d2 * nv + d3) + np.sqrt((d2 * nv + d3) * (d2 * nv + d3) + 1)) + d4


def passive_force(norm_length):
    """hill_coefficients.py:99-126 (clipped at 0)."""
    kpe, e0 = 4, 0.6
    fp = (np.exp(kpe * (norm_length - 1) / e0) - 1) / (np.exp(kpe) - 1)
    return fp if np.real(fp) > 0 else 0 * fp


# --------------------------------------------------------------------------------------------------------------
# rigid-body dynamics (recursive Newton-Euler in world coordinates, complex-safe)
# --------------------------------------------------------------------------------------------------------------


def _inverse_dynamics(bm, q, qdot, qddot, gravity=True):
    frames, dofs = forward_kinematics(bm, q)
    nq = len(dofs)
    dt = np.result_type(np.asarray(q).dtype, np.asarray(qdot).dtype, np.asarray(qddot).dtype, float)
    g = np.asarray(bm["gravity"], dtype=float) if gravity else np.zeros(3)
    # dof chain: parent dof of each dof (the previous dof on its segment path) -> motion of each dof's link
    seg_last_dof = {}
    parent_of = {s["name"]: s["parent"] for s in bm["segments"]}
    link_parent = []
    for k, d in enumerate(dofs):
        s = d["segment"]
        p = k - 1 if (k > 0 and dofs[k - 1]["segment"] == s) else None
        if p is None:
            a = parent_of[s]
            while a is not None and a not in seg_last_dof:
                a = parent_of[a]
            p = seg_last_dof.get(a) if a is not None else None
        link_parent.append(p)
        seg_last_dof[s] = k
    w = np.zeros((nq, 3), dtype=dt)
    al = np.zeros((nq, 3), dtype=dt)
    acc = np.zeros((nq, 3), dtype=dt)
    for k, d in enumerate(dofs):
        p = link_parent[k]
        wp, alp, ap = (np.zeros(3, dt), np.zeros(3, dt), -g.astype(dt)) if p is None else (w[p], al[p], acc[p])
        op = np.zeros(3) if p is None else dofs[p]["origin"]
        r = d["origin"] - op
        w[k] = wp + d["axis"] * qdot[k]
        al[k] = alp + d["axis"] * qddot[k] + np.cross(wp, d["axis"] * qdot[k])
        acc[k] = ap + np.cross(alp, r) + np.cross(wp, np.cross(wp, r))
    # bodies: each massive segment moves with the last dof on its path
    tau = np.zeros(nq, dtype=dt)
    for seg in bm["segments"]:
        if seg["mass"] == 0 and not np.any(seg["inertia"]):
            continue
        a = seg["name"]
        while a is not None and a not in seg_last_dof:
            a = parent_of[a]
        if a is None:
            continue  # fixed to the ground
        k = seg_last_dof[a]
        T = frames[seg["name"]]
        R = T[:3, :3]
        c = R @ np.asarray(seg["com"], dtype=float) + T[:3, 3]
        Iw = R @ np.asarray(seg["inertia"], dtype=float) @ R.T
        r = c - dofs[k]["origin"]
        ac = acc[k] + np.cross(al[k], r) + np.cross(w[k], np.cross(w[k], r))
        Fb = seg["mass"] * ac
        Nb = Iw @ al[k] + np.cross(w[k], Iw @ w[k])
        # every dof on the body's path feels the body's wrench about its own origin
        j = k
        while j is not None:
            tau[j] = tau[j] + dofs[j]["axis"] @ (np.cross(c - dofs[j]["origin"], Fb) + Nb)
            j = link_parent[j]
    return tau


def mass_matrix(bm, q):
    nq = nb_q(bm)
    z = np.zeros(nq)
    g0 = _inverse_dynamics(bm, q, z, z, gravity=False)
    return np.stack([_inverse_dynamics(bm, q, z, np.eye(nq)[j], gravity=False) - g0 for j in range(nq)], axis=1)


def forward_dynamics(bm, q, qdot, tau):
    """qddot = M^-1 (tau - h(q, qdot)), h = ID(q, qdot, 0) (Coriolis, centrifugal, gravity)."""
    nq = nb_q(bm)
    h = _inverse_dynamics(bm, q, qdot, np.zeros(nq))
    return np.linalg.solve(mass_matrix(bm, q), tau - h)


def energy(bm, q, qdot):
    """Kinetic + gravitational potential energy (test helper)."""
    frames, _ = forward_kinematics(bm, q)
    M = mass_matrix(bm, q)
    ke = 0.5 * qdot @ M @ qdot
    pe = 0.0
    g = np.asarray(bm["gravity"], dtype=float)
    for seg in bm["segments"]:
        if seg["mass"]:
            T = frames[seg["name"]]
            c = T[:3, :3] @ np.asarray(seg["com"], dtype=float) + T[:3, 3]
            pe = pe - seg["mass"] * g @ c
    return ke + pe


# --------------------------------------------------------------------------------------------------------------
# FesMskModel right-hand side and the OcpFesMsk transcription
# --------------------------------------------------------------------------------------------------------------


@dataclass
class MskMuscle:
    model: str  # oracle model name (fes_oracle.MODEL_NAMES)
    name: str  # bioMod muscle name
    c: dict  # constants


@dataclass
class MskProblem:
    bm: dict
    muscles: list
    rows: np.ndarray  # (N+1, T) stim table shared by every muscle (muscles_dynamics_model[0])
    n_shooting: int
    final_time: float
    scheme: str = "RK4"
    m: int = 1
    fv_on: bool = False  # activate_force_velocity_relationship (also gates force-length, reference quirk)
    fp_on: bool = False
    residual: bool = False
    objectives: list = field(default_factory=list)  # O.Objective-like: kind, var_kind, index, nodes, weight, target
    fatigue_weight: float = 0.0  # minimize_muscle_fatigue Mayer at node N: w * sum_m (a_rest_m / A_m)^2
    # Hmed2018 muscles: T intensity controls each; with n_params > 0 the trailing parameters are the pulses'
    # intensities (muscle m's block at param_offset[m]) tied to the controls by sliding-window rows
    n_params: int = 0
    last_stim_idx: list = None
    param_offset: list = None
    # bioptim ConstraintFcn.SUPERIMPOSE_MARKERS as OcpFesMsk's msk_info["custom_constraint"] passes it
    # (fes_ocp_dynamics.py:424-450): dicts node, first, second (marker names), axes (world axis indices); rows
    # marker(second) - marker(first) at q_node, after every interval's rows
    marker_pairs: list = field(default_factory=list)
    # muscle-model conventions of the revision that wrote the reference's stored reaching-task solutions
    # (fes_oracle.rhs ``legacy``); test infrastructure for tests/test_reference_solution.py
    legacy: bool = False

    @property
    def nq(self):
        return nb_q(self.bm)

    @property
    def nxm(self):
        return sum(O.n_states(m.model) for m in self.muscles)

    @property
    def nx(self):
        return self.nxm + 2 * self.nq

    @property
    def n_pw(self):
        return sum(1 for m in self.muscles if O.control_kind(m.model) == "pulse_width")

    @property
    def T(self):
        return self.rows.shape[1]

    @property
    def n_int(self):
        return sum(self.T for m in self.muscles if O.control_kind(m.model) == "pulse_intensity")

    @property
    def n_slide(self):
        return self.n_int if self.n_params else 0

    @property
    def nu(self):
        return self.n_pw + self.n_int + (self.nq if self.residual else 0)

    @property
    def nz(self):
        return self.nx + self.nu

    @property
    def nv(self):
        return self.n_shooting * self.nz + self.nx + self.n_params

    @property
    def n_marker_rows(self):
        return sum(len(c["axes"]) for c in self.marker_pairs)

    @property
    def ng(self):
        return self.n_shooting * (self.nx + self.n_slide) + self.n_marker_rows

    @property
    def dt(self):
        return self.final_time / self.n_shooting


def _bio_muscle(pb: MskProblem, name: str) -> dict:
    for m in pb.bm["muscles"]:
        if m["name"] == name:
            return m
    raise ValueError(f"muscle {name} not in the bioMod")


def msk_rhs(pb: MskProblem, t, x, u, row):
    """FesMskModel.muscle_dynamic (dynamical_model.py:133-203) for one node: x (nx,), u (nu,), row (T,)."""
    nq = pb.nq
    q = x[pb.nxm: pb.nxm + nq]
    qdot = x[pb.nxm + nq:]
    JL_rows, F, dx = [], [], []
    off, pw = 0, 0
    for mus in pb.muscles:
        nxm = O.n_states(mus.model)
        xm = x[off: off + nxm]
        bio = _bio_muscle(pb, mus.name)
        _, JL, fibre, vel = muscle_geometry(pb.bm, bio, q, qdot)
        nl = fibre / bio["optimallength"]
        fl = force_length(nl) if pb.fv_on else 1.0  # dynamical_model.py:260-267 (gated by the FV flag)
        fv = force_velocity(vel) if pb.fv_on else 1.0  # dynamical_model.py:272-284
        fp = passive_force(nl) if pb.fp_on else 0.0  # dynamical_model.py:289-297
        um = None
        if O.control_kind(mus.model) == "pulse_width":
            um = np.array([u[pw]])
            pw += 1
        elif O.control_kind(mus.model) == "pulse_intensity":  # the muscle's T intensities (dynamical_model.py:253-255)
            um = u[pw: pw + pb.T]
            pw += pb.T
        dxm = O.rhs(mus.model, mus.c, t, xm, um, row, fl=fl, fv=fv, fp=fp, legacy=pb.legacy)
        dx.extend(list(dxm))
        JL_rows.append(JL)
        F.append(xm[1])
        off += nxm
    JLm = np.stack(JL_rows)  # (n_muscles, nq): musclesLengthJacobian rows in muscle order
    tau = -JLm.T @ np.array(F)  # dynamical_model.py:331-332
    if pb.residual:
        tau = tau + u[pb.n_pw + pb.n_int: pb.n_pw + pb.n_int + nq]
    qddot = forward_dynamics(pb.bm, q, qdot, tau)
    return np.concatenate([np.array(dx), qdot, qddot])


def integrate_interval(pb: MskProblem, k, x, u, keep_substeps=False):
    """Phi_m(x_k, u_k): m RK sub-steps over interval k (bioptim convention, oracle.fes_oracle._step)."""
    h = pb.dt / pb.m
    f = lambda t, xx: msk_rhs(pb, t, xx, u, pb.rows[k])  # noqa: E731
    t0 = k * pb.dt
    out = [x]
    for j in range(pb.m):
        x = O._step(pb.scheme, f, t0 + j * h, h, x)
        out.append(x)
    return out if keep_substeps else x


def unpack(pb: MskProblem, v):
    N, nx, nz = pb.n_shooting, pb.nx, pb.nz
    body = v[: N * nz].reshape(N, nz)
    X = np.concatenate([body[:, :nx], v[None, N * nz: N * nz + nx]], axis=0)  # (N+1, nx)
    U = body[:, nx:]
    return X, U


def sliding_rows(pb: MskProblem, v, k):
    """custom_constraints.py:102-119 per Hmed muscle: u_k's T intensities minus the last T parameters up to the
    node's last pulse, left-padded with muscles_dynamics_model[0]'s I_min (custom_constraints.py:107-114 pads every
    muscle's window with the first muscle model's min_pulse_intensity())."""
    X, U = unpack(pb, v)
    P = v[pb.n_shooting * pb.nz + pb.nx:]
    out, off = [], pb.n_pw
    for mi, mus in enumerate(pb.muscles):
        idx = pb.last_stim_idx[k]
        cols = [P[pb.param_offset[mi] + i] for i in range(idx + 1)]
        while len(cols) < pb.T:
            cols.insert(0, O.min_pulse_intensity(pb.muscles[0].c))
        cols = cols[len(cols) - pb.T:]
        out.append(U[k, off: off + pb.T] - np.array(cols))
        off += pb.T
    return np.concatenate(out)


def marker_rows(pb: MskProblem, v):
    """SUPERIMPOSE_MARKERS rows (bioptim penalty ``superimpose_markers``: marker(second) - marker(first), the
    selected axes), in the order of ``pb.marker_pairs``."""
    X, _ = unpack(pb, v)
    out = []
    for c in pb.marker_pairs:
        q = X[c["node"], pb.nxm: pb.nxm + pb.nq]
        d = marker_position(pb.bm, c["second"], q) - marker_position(pb.bm, c["first"], q)
        out.extend(d[a] for a in c["axes"])
    return np.array(out, dtype=np.result_type(v.dtype, float))


def eval_g(pb: MskProblem, v):
    """Per interval: continuity rows Phi(x_k, u_k) - x_{k+1}, then (Hmed with parameters) the sliding rows; then
    the marker rows."""
    X, U = unpack(pb, v)
    parts = []
    for k in range(pb.n_shooting):
        parts.append(integrate_interval(pb, k, X[k], U[k]) - X[k + 1])
        if pb.n_slide:
            parts.append(sliding_rows(pb, v, k))
    if pb.marker_pairs:
        parts.append(marker_rows(pb, v))
    return np.concatenate(parts)


def continuity_jacobian(pb: MskProblem, v, k):
    """Dense d Phi(x_k, u_k) / d(x_k, u_k) (nx x nz) by complex step."""
    X, U = unpack(pb, v)
    z = np.concatenate([X[k], U[k]]).astype(complex)
    h = 1e-30
    J = np.empty((pb.nx, pb.nz))
    for j in range(pb.nz):
        zz = z.copy()
        zz[j] += 1j * h
        J[:, j] = np.imag(integrate_interval(pb, k, zz[: pb.nx], zz[pb.nx:])) / h
    return J


def eval_f(pb: MskProblem, v):
    X, U = unpack(pb, v)
    f = 0.0
    for o in pb.objectives:
        arr = X if o["var_kind"] == 0 else U
        for k in range(o["node_first"], o["node_last"] + 1):
            tgt = o["target"][k] if o.get("target") is not None else o.get("target_value", 0.0)
            w = o["weight"] * (pb.dt if o["kind"] == 0 else 1.0)
            f += w * (arr[k, o["var_index"]] - tgt) ** 2
    if pb.fatigue_weight:
        off = 0
        for mus in pb.muscles:
            if O.n_states(mus.model) == 5:
                f += pb.fatigue_weight * (mus.c["a_rest"] / X[-1, off + 2]) ** 2
            off += O.n_states(mus.model)
    return f


def eval_grad_f(pb: MskProblem, v):
    g = np.empty(pb.nv)
    for j in range(pb.nv):
        vv = v.astype(complex)
        vv[j] += 1e-30j
        g[j] = np.imag(eval_f(pb, vv)) / 1e-30
    return g


def ivp(pb: MskProblem, x0, U):
    """Single shooting over all intervals from x0 with per-interval controls U (N, nu): (N*m+1, nx)."""
    out = [np.asarray(x0, dtype=float)]
    x = out[0]
    for k in range(pb.n_shooting):
        sub = integrate_interval(pb, k, x, U[k], keep_substeps=True)
        out.extend(sub[1:])
        x = sub[-1]
    return np.array(out)
