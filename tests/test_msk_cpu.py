"""CPU tests of the musculoskeletal path: the oracle's self-consistency (it is the checker of the GPU kernels and
is pinned by physics, not by reference outputs), the bioMod fixtures, the product's bioMod reader and chain
reduction, and the OcpFesMsk facade (layout, bounds, objective terms, the reference's validation messages)."""

import json
import pathlib

import numpy as np
import pytest

from oracle import fes_msk as M
from tests import msk_cases as MC

REF_MODELS = pathlib.Path("/root/reference/examples/msk_models")
FIXTURES = ("arm26_biceps_triceps", "arm26", "arm26_biceps", "arm26_biceps_1dof")


def _bm(name="arm26_biceps_triceps"):
    return json.loads(pathlib.Path(MC.biomod_path(name)).read_text())


# ---- oracle self-consistency ----------------------------------------------------------------------------------

def test_oracle_unforced_arm_conserves_energy():
    bm = _bm()
    x = np.array([0.3, 1.0, 0.5, -1.2])
    f = lambda x: np.concatenate([x[2:], M.forward_dynamics(bm, x[:2], x[2:], np.zeros(2))])  # noqa: E731
    e0 = M.energy(bm, x[:2], x[2:])
    h = 2e-4
    for _ in range(1500):
        k1 = f(x)
        k2 = f(x + h / 2 * k1)
        k3 = f(x + h / 2 * k2)
        k4 = f(x + h * k3)
        x = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    assert abs(M.energy(bm, x[:2], x[2:]) - e0) < 1e-9 * (abs(e0) + 1)


def test_oracle_mass_matrix_spd_and_static_gravity_torque():
    bm = _bm()
    q = np.array([0.4, 1.1])
    Mm = M.mass_matrix(bm, q)
    assert np.allclose(Mm, Mm.T, atol=1e-14) and np.all(np.linalg.eigvalsh(Mm) > 0)
    # at rest, the dynamics bias is the gravity torque = -dV/dq (V the potential energy)
    h = M._inverse_dynamics(bm, q, np.zeros(2), np.zeros(2))
    eps = 1e-6
    dV = [(M.energy(bm, q + eps * e, np.zeros(2)) - M.energy(bm, q - eps * e, np.zeros(2))) / (2 * eps)
          for e in np.eye(2)]
    np.testing.assert_allclose(h, dV, rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_length_jacobian_matches_finite_differences(name):
    bm = _bm(name)
    nq = M.nb_q(bm)
    q = np.linspace(0.2, 1.0, nq)
    for mus in bm["muscles"]:
        _, JL, _, vel = M.muscle_geometry(bm, mus, q, np.ones(nq))
        eps = 1e-6
        fd = [(M.muscle_tendon_length(bm, mus, q + eps * e) - M.muscle_tendon_length(bm, mus, q - eps * e)) / (2 * eps)
              for e in np.eye(nq)]
        np.testing.assert_allclose(JL, fd, rtol=1e-7, atol=1e-10)
        assert vel == pytest.approx(np.sum(JL))


def test_oracle_hill_coefficients():
    """Closed forms of hill_coefficients.py: FL peaks near the optimal length, FV(0) = d1 asinh(d3) + d4,
    FP = 0 below the optimal length and (e^kpe(l-1)/e0 - 1)/(e^kpe - 1) above."""
    assert M.force_velocity(0.0) == pytest.approx(-0.318 * np.arcsinh(-0.374) + 0.886, rel=1e-15)
    ls = np.linspace(0.5, 1.5, 1001)
    fl = np.array([M.force_length(v) for v in ls])
    assert 0.95 < ls[fl.argmax()] < 1.1 and 0.9 < fl.max() < 1.05
    assert M.passive_force(0.9) == 0.0
    assert M.passive_force(1.2) == pytest.approx((np.exp(4 * 0.2 / 0.6) - 1) / (np.exp(4) - 1), rel=1e-14)


def test_oracle_muscle_torque_signs():
    """BIClong flexes the elbow (its length shrinks with flexion), TRIlong extends it."""
    bm = _bm()
    q = np.array([0.0, 1.0])
    mus = {m["name"]: m for m in bm["muscles"]}
    assert M.muscle_geometry(bm, mus["BIClong"], q, np.zeros(2))[1][1] < 0
    assert M.muscle_geometry(bm, mus["TRIlong"], q, np.zeros(2))[1][1] > 0


# ---- fixtures and the product's bioMod reader -----------------------------------------------------------------

@pytest.mark.skipif(not REF_MODELS.exists(), reason="reference bioMod files not present")
@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_and_product_parser_match_the_reference_files(name):
    from cocofest_amd.msk import parse_biomod

    text = (REF_MODELS / f"{name}.bioMod").read_text()
    ref = M.parse_biomod(text)
    ref.pop("groups")
    assert json.loads(json.dumps(ref)) == _bm(name)
    assert json.loads(json.dumps(parse_biomod(text))) == _bm(name)


def _chain_frames(chain, q):
    R, o = [], []
    Rp, op = np.eye(3), np.zeros(3)
    for j, ax in enumerate(chain["axis"]):
        A = chain["frame"][j, :9].reshape(3, 3)
        t = chain["frame"][j, 9:]
        o_j = op + Rp @ t
        Rb = Rp @ A
        c, s = np.cos(q[j]), np.sin(q[j])
        Rot = np.eye(3)
        a, b = {0: (1, 2), 1: (2, 0), 2: (0, 1)}[ax]
        Rot[a, a], Rot[a, b], Rot[b, a], Rot[b, b] = c, -s, s, c
        Rp, op = Rb @ Rot, o_j
        R.append(Rp)
        o.append(op)
    return R, o


def _chain_points(chain, mus, q):
    """World path points of a muscle through the reduced chain (numpy, independent of the kernels)."""
    R, o = _chain_frames(chain, q)
    g = chain["muscles"][mus]
    return [p if f < 0 else R[f] @ p + o[f] for f, p in zip(g["point_frame"], g["point_pos"])]


@pytest.mark.parametrize("name", FIXTURES)
def test_chain_reduction_reproduces_tree_kinematics_and_inertia(name):
    from cocofest_amd.msk import reduce_to_chain

    bm = _bm(name)
    ch = reduce_to_chain(bm)
    nq = M.nb_q(bm)
    q = np.linspace(-0.3, 1.2, nq)
    frames, _ = M.forward_kinematics(bm, q)
    for mus in bm["muscles"]:
        pts = [M._point_world(frames, s, p) for s, p in M.muscle_path(mus)]
        np.testing.assert_allclose(_chain_points(ch, mus["name"], q), pts, atol=1e-14)
    # the composite bodies give the tree's mass matrix: M = sum_b m_b Jv^T Jv + Jw^T I_w Jw
    R, o = _chain_frames(ch, q)
    z = [R[j][:, a] for j, a in enumerate(ch["axis"])]
    Mc = np.zeros((nq, nq))
    for j in range(nq):
        c = o[j] + R[j] @ ch["com"][j]
        Iw = R[j] @ ch["inertia"][j].reshape(3, 3) @ R[j].T
        Jv = np.array([np.cross(z[i], c - o[i]) if i <= j else np.zeros(3) for i in range(nq)]).T
        Jw = np.array([z[i] if i <= j else np.zeros(3) for i in range(nq)]).T
        Mc += ch["mass"][j] * Jv.T @ Jv + Jw.T @ Iw @ Jw
    np.testing.assert_allclose(Mc, M.mass_matrix(bm, q), rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", FIXTURES)
def test_chain_reduction_reproduces_tree_marker_positions(name):
    """Markers re-expressed in the frame of the dof they move with land where the full tree puts them."""
    from cocofest_amd.msk import reduce_to_chain

    bm = _bm(name)
    ch = reduce_to_chain(bm)
    assert set(ch["markers"]) == {m["name"] for m in bm["markers"]}
    for q in (np.linspace(-0.3, 1.2, M.nb_q(bm)), np.linspace(0.9, -0.4, M.nb_q(bm))):
        R, o = _chain_frames(ch, q)
        for mk in bm["markers"]:
            g = ch["markers"][mk["name"]]
            got = g["pos"] if g["frame"] < 0 else R[g["frame"]] @ g["pos"] + o[g["frame"]]
            np.testing.assert_allclose(got, M.marker_position(bm, mk["name"], q), atol=1e-14)


REACH = [dict(first="COM_hand", second="target", node="end", axes=(0, 1))]


def test_custom_constraint_is_ignored_as_in_the_reference_unless_applied():
    """The reference drops msk_info["custom_constraint"] (fes_ocp_dynamics.py:107 calls _build_constraints without
    it): by default the OCP has no marker rows (and says so); apply_custom_constraint=True adds them."""
    import cocofest_amd as C

    cfg = MC.cfg5()
    cl = C.ConstraintList()
    cl.add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker="COM_hand", second_marker="target", node=C.Node.END,
           axes=[C.Axis.X, C.Axis.Y], phase=0)
    assert len(cl) == 1 and len(cl[0]) == 1
    base = MC.product_ocp(**cfg)
    mm = base.model
    info = {"bound_type": "start_end", "bound_data": [[0, 5], [0, 90]], "custom_constraint": cl}
    with pytest.warns(UserWarning, match="not applied, as in the reference"):
        ign = C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info=info)
    assert ign.marker_pairs == []
    app = C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info=info, apply_custom_constraint=True)
    assert len(app.marker_pairs) == 1 and app.n_marker_rows == 2
    c = app.marker_pairs[0]
    assert c["node"] == app.n_shooting and c["axes"] == 3 and c["frame"] == [1, -1]
    # the product's pair and the oracle's rows agree at a random point (same layout, chain vs tree kinematics)
    pb = MC.oracle_problem(**cfg, markers=REACH)
    v = MC.random_decision(pb, 1, seed=2)[0]
    X, _ = M.unpack(pb, v)
    q = X[-1, pb.nxm: pb.nxm + pb.nq]
    R, o = _chain_frames(mm.chain, q)
    p1 = R[1] @ np.asarray(c["pos"][0]) + o[1]
    np.testing.assert_allclose((np.asarray(c["pos"][1]) - p1)[:2], M.marker_rows(pb, v), atol=1e-14)
    assert pb.ng == pb.n_shooting * pb.nx + 2


def test_custom_constraint_validation():
    import cocofest_amd as C

    with pytest.raises(NotImplementedError, match="SUPERIMPOSE_MARKERS only"):
        C.ConstraintList().add("track_state", node=1)
    with pytest.raises(NotImplementedError, match="unsupported arguments"):
        C.ConstraintList().add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker="a", second_marker="b", node=1,
                               min_bound=0)
    with pytest.raises(ValueError, match="give the node"):
        C.ConstraintList().add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, first_marker="a", second_marker="b")
    mm = MC.product_ocp(**MC.cfg5()).model
    for kw, err, msg in ((dict(first_marker="COM_hand", second_marker="nowhere", node=3), ValueError, "not in"),
                         (dict(first_marker="COM_hand", second_marker="target", node=11), ValueError, "outside"),
                         (dict(first_marker="target", second_marker="target", node=2), ValueError, "ground")):
        cl = C.ConstraintList()
        cl.add(C.ConstraintFcn.SUPERIMPOSE_MARKERS, **kw)
        with pytest.raises(err, match=msg):
            C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info={"custom_constraint": cl},
                                    apply_custom_constraint=True)


@pytest.mark.parametrize("pair, msg", [
    (dict(node=11, axes=1, frame=[1, -1]), "marker pair node out of"),
    (dict(node=2, axes=0, frame=[1, -1]), "axes must select"),
    (dict(node=2, axes=8, frame=[1, -1]), "axes must select"),
    (dict(node=2, axes=3, frame=[2, -1]), "marker frame out of range"),
    (dict(node=2, axes=3, frame=[-1, -1]), "fixed to the ground"),
])
def test_msk_create_rejects_bad_marker_pairs(pair, msg):
    """cfx_msk_create validates the marker pairs before any HIP call (EINVAL and the reason)."""
    from cocofest_amd import CfxError, _cfx

    ocp = MC.product_ocp(**MC.cfg5())
    ocp.marker_pairs = [dict(pos=[[0.0] * 3, [0.0] * 3], **pair)]
    with pytest.raises(CfxError, match=msg) as e:
        ocp.nlp(batch=1)
    assert e.value.code == _cfx.EINVAL


# ---- OcpFesMsk facade -----------------------------------------------------------------------------------------

def test_ocp_fes_msk_layout_bounds_and_objective():
    ocp = MC.product_ocp(**MC.cfg5())
    pb = MC.oracle_problem(**MC.cfg5())
    assert (ocp.n_shooting, ocp.nx, ocp.nu, ocp.nv) == (10, 14, 2, 174)
    assert ocp.state_names[:5] == ["Cn_BIClong", "F_BIClong", "A_BIClong", "Tau1_BIClong", "Km_BIClong"]
    assert ocp.control_names == ["last_pulse_width_BIClong", "last_pulse_width_TRIlong"]
    lo, hi = ocp.bounds_vector()
    xs_lo, _, _ = ocp.unpack(lo)
    xs_hi, us_hi, _ = ocp.unpack(hi)
    q1 = "q_r_ulna_radius_hand_rotation1_RotZ"
    assert xs_lo[q1][0, 0] == xs_hi[q1][0, 0] == pytest.approx(3.14 / 36)  # 5 deg, the reference's 3.14 / 180
    assert xs_lo[q1][0, -1] == xs_hi[q1][0, -1] == pytest.approx(1.57)
    assert xs_lo[q1][0, 5] == 0.0 and xs_hi[q1][0, 5] == pytest.approx(np.pi)
    assert xs_hi["Cn_BIClong"][0, 3] == 10 and xs_hi["F_TRIlong"][0, 3] == 1000
    assert xs_lo["qdot_r_humerus_rotation1_RotZ"][0, 0] == 0 and xs_hi["qdot_r_humerus_rotation1_RotZ"][0, 0] == 0
    assert np.all(us_hi["last_pulse_width_BIClong"] == 0.0006)
    v = MC.random_decision(pb, 1, seed=2)[0]
    # the terms the product hands to libcfx evaluate to the oracle's objective
    f = 0.0
    X, U = M.unpack(pb, v)
    for t in ocp.objectives:
        z = (X if t["var_kind"] == 0 else U)[t["node_first"]: t["node_last"] + 1, t["var_index"]]
        if t["kind"] == 2:
            f += t["weight"] * np.sum((t["target_value"] / z) ** 2)
        else:
            f += t["weight"] * (0.1 if t["kind"] == 0 else 1.0) * np.sum((z - t["target_value"]) ** 2)
    assert f == pytest.approx(M.eval_f(pb, v), rel=1e-13)


def test_ocp_fes_msk_validation_messages():
    import cocofest_amd as C

    mm = C.FesMskModel(biorbd_path=MC.biomod_path(), stim_time=list(MC.STIMS),
                       muscles_model=[C.DingModelPulseWidthFrequencyWithFatigue(muscle_name="BIClong"),
                                      C.DingModelPulseWidthFrequencyWithFatigue(muscle_name="TRIlong")])
    with pytest.raises(ValueError, match="bound_type should be a string and should be equal to start, end or start_end"):
        C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info={"bound_type": "middle", "bound_data": [0, 5]})
    with pytest.raises(TypeError, match="bound_data should be a list of two list"):
        C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info={"bound_type": "start_end", "bound_data": [0, 5]})
    with pytest.raises(ValueError, match="bound_data should be a list of 2 elements"):
        C.OcpFesMsk.prepare_ocp(model=mm, final_time=1, msk_info={"bound_type": "start_end",
                                                                  "bound_data": [[0, 5, 1], [0, 90, 1]]})
    with pytest.raises(TypeError, match="The given muscles_model must be a list of FesModel"):
        C.FesMskModel(biorbd_path=MC.biomod_path(), muscles_model=C.DingModelFrequency(muscle_name="BIClong"))
    with pytest.raises(ValueError, match="not in"):
        C.FesMskModel(biorbd_path=MC.biomod_path(), muscles_model=[C.DingModelFrequency(muscle_name="DELT1")])
    # the reference validates MSK objectives with OcpFes._sanity_check first (fes_ocp_dynamics.py:50-58), so a
    # per-muscle force_tracking list is rejected exactly as there
    with pytest.raises(TypeError, match="force_tracking argument must be np.ndarray type"):
        C.OcpFesMsk.prepare_ocp(model=mm, final_time=1,
                                objective={"force_tracking": [np.linspace(0, 1, 5), [np.ones(5), np.ones(5)]]})


def test_msk_handle_fails_loudly_without_a_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from cocofest_amd import CfxError

    ocp = MC.product_ocp(**MC.cfg5())
    with pytest.raises(CfxError):
        ocp.nlp(batch=4)


@pytest.mark.parametrize("kw", [MC.cfg5(), MC.cfg5(model="ding2007", scheme="RK1", residual=True, fatigue=False),
                                MC.cfg5(model="ding2003", biomod="arm26",
                                        muscles=("BIClong", "BICshort", "BRA", "TRIlong", "TRIlat", "TRImed"),
                                        fatigue=False)],
                         ids=["cfg5", "d07_rk1_residual", "arm26_6muscles"])
def test_c_port_matches_numpy_oracle(kw):
    """The C port (bench.py's cfg-5 CPU baseline) reproduces the numpy oracle's g and interval Jacobians."""
    from oracle import c_msk

    pb = MC.oracle_problem(**kw)
    v = MC.random_decision(pb, 2, seed=5)
    g, J = c_msk.shooting(pb, v, threads=2)
    for b in range(2):
        gr = M.eval_g(pb, v[b])
        np.testing.assert_allclose(g[b], gr, rtol=1e-12, atol=1e-12 * np.abs(gr).max())
        k = pb.n_shooting - 1
        Jr = M.continuity_jacobian(pb, v[b], k)
        np.testing.assert_allclose(J[b, k], Jr, rtol=1e-11, atol=1e-12 * np.abs(Jr).max())


def test_legacy_calcium_and_per_pulse_flags():
    """Extensions for the stored reaching-task revision: FesMskModel(legacy_calcium=True) sets CFX_MSK_LEGACY_CALCIUM,
    pulse_width["per_pulse"] sets CFX_MSK_PULSE_WIDTH_PER_PULSE on the handle (Ding2007 muscles only)."""
    from cocofest_amd import _cfx
    from tests import msk_cases as MC
    from tests import test_reference_solution as R

    ocp = MC.product_ocp(**MC.cfg5(legacy=True))
    assert ocp.model.cfx_flags() & _cfx.MSK_LEGACY_CALCIUM and not ocp.per_pulse
    assert not MC.product_ocp(**MC.cfg5()).model.cfx_flags() & _cfx.MSK_LEGACY_CALCIUM
    assert R.legacy_product().per_pulse
    with pytest.raises(ValueError, match="per_pulse"):
        import cocofest_amd as C

        mm = C.FesMskModel(biorbd_path=MC.biomod_path("arm26_biceps_triceps"),
                           muscles_model=[C.DingModelFrequencyWithFatigue(muscle_name="BIClong")],
                           stim_time=[0.0, 0.1], activate_force_length_relationship=True,
                           activate_force_velocity_relationship=True)
        C.OcpFesMsk.prepare_ocp(model=mm, final_time=0.2, pulse_width={"per_pulse": True},
                                msk_info={"bound_type": "start", "bound_data": [0, 5]})
