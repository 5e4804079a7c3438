"""PinocchioModel's Jacobians and closed-loop IK (python/pybind_pinocchio.hpp:
47-58, src/pinocchio_model.cpp:335-496), host side (csrc/host/kinjac.cpp):
pinocchio 2.6.21 is not under /root/reference, so these floating-point
results are pinned by geometry -- the WORLD / LOCAL link Jacobians against
finite differences of the oracle's forward kinematics, the single-link local
Jacobian against the full one, the IK solutions against their targets (FK
of the answer) and the joint limits."""
import numpy as np
import pytest

import worlds as Wd

HAND = 8  # user link index of panda_hand (its collision object has an identity origin)


@pytest.fixture(scope="module")
def models():
    from mplib_amd import scenes
    pin = scenes.panda().get_pinocchio_model()
    ow = Wd.oracle_world(2)
    return pin, ow


def _hand_pose(ow, q7):
    _, objT = ow.fk_batch(np.asarray(q7, np.float64).reshape(1, 7))
    T = objT[0, HAND]
    return T[:9].reshape(3, 3), T[9:].copy()


def _full(q7):
    return list(np.asarray(q7, np.float64)) + [0.0, 0.0]


def test_link_jacobian_matches_finite_differences(models):
    """WORLD convention (pinocchio): angular part w with dR R^T = [w]x, linear
    part the velocity of the point at the world origin, v = dp - w x p;
    LOCAL: (R^T dp, R^T w).  Central differences of the oracle's FK, 1e-6."""
    pin, ow = models
    rng = np.random.default_rng(4)
    lim = ow.art.joint_limits()[:7]
    for _ in range(5):
        q = rng.uniform(lim[:, 0], lim[:, 1])
        pin.compute_full_jacobian(_full(q))
        Jw = pin.get_link_jacobian(HAND, False)
        Jl = pin.get_link_jacobian(HAND, True)
        assert Jw.shape == (6, 9)
        R, p = _hand_pose(ow, q)
        h = 1e-6
        for j in range(7):
            dq = np.zeros(7)
            dq[j] = h
            Rp, pp = _hand_pose(ow, q + dq)
            Rm, pm = _hand_pose(ow, q - dq)
            dp = (pp - pm) / (2 * h)
            W = (Rp - Rm) / (2 * h) @ R.T
            w = np.array([W[2, 1] - W[1, 2], W[0, 2] - W[2, 0], W[1, 0] - W[0, 1]]) / 2
            np.testing.assert_allclose(Jw[3:, j], w, atol=1e-7)
            np.testing.assert_allclose(Jw[:3, j], dp - np.cross(w, p), atol=1e-7)
            np.testing.assert_allclose(Jl[:3, j], R.T @ dp, atol=1e-7)
            np.testing.assert_allclose(Jl[3:, j], R.T @ w, atol=1e-7)
        assert not Jw[:, 7:].any()  # the fingers do not move the hand
        np.testing.assert_allclose(pin.compute_single_link_local_jacobian(_full(q), HAND), Jl, atol=1e-12)


def test_ik_clik_reaches_its_targets(models):
    """compute_IK_CLIK from a perturbed start: success, error below eps, and
    the oracle's FK of the answer reaches the target pose; compute_IK_CLIK_JL
    keeps the answer inside the limits it was given."""
    from oracle import model as M
    pin, ow = models
    rng = np.random.default_rng(9)
    lim = ow.art.joint_limits()[:7]
    ok = 0
    for _ in range(6):
        q_goal = rng.uniform(lim[:, 0] * 0.8, lim[:, 1] * 0.8)
        R, p = _hand_pose(ow, q_goal)
        w, x, y, z = M.mat_to_quat(list(R.reshape(-1)))
        pose = list(p) + [w, x, y, z]
        q0 = np.clip(q_goal + rng.normal(scale=0.2, size=7), lim[:, 0], lim[:, 1])
        q, success, err = pin.compute_IK_CLIK(HAND, pose, _full(q0))
        assert q.shape == (9,) and err.shape == (6,)
        if not success:
            continue
        ok += 1
        assert np.linalg.norm(err) < 1e-5
        R2, p2 = _hand_pose(ow, q[:7])
        assert np.linalg.norm(p2 - p) < 1e-5 and np.abs(R2 - R).max() < 1e-5
        lo = list(lim[:, 0]) + [0.0, 0.0]
        hi = list(lim[:, 1]) + [0.04, 0.04]
        qj, sj, _ = pin.compute_IK_CLIK_JL(HAND, pose, _full(q0), lo, hi)
        assert (qj >= np.array(lo) - 1e-12).all() and (qj <= np.array(hi) + 1e-12).all()
        if sj:
            R3, p3 = _hand_pose(ow, qj[:7])
            assert np.linalg.norm(p3 - p) < 1e-5
    assert ok >= 4


def test_ik_mask_freezes_joints(models):
    """mask[j] zeroes joint j's Jacobian column: that joint never moves."""
    from oracle import model as M
    pin, ow = models
    q_goal = np.array([0.3, -0.4, 0.2, -2.0, 0.1, 1.8, 0.5])
    R, p = _hand_pose(ow, q_goal)
    w, x, y, z = M.mat_to_quat(list(R.reshape(-1)))
    q0 = q_goal + np.array([0.0, 0.1, -0.1, 0.1, 0.0, -0.1, 0.1])
    mask = [True] + [False] * 8
    q, _, _ = pin.compute_IK_CLIK(HAND, list(p) + [w, x, y, z], _full(q0), mask, maxIter=50)
    assert q[0] == q0[0]
    with pytest.raises(RuntimeError, match="out of bound"):
        pin.compute_IK_CLIK(99, list(p) + [w, x, y, z], _full(q0))


def test_print_frames(models, capfd):
    pin, _ = models
    pin.print_frames()
    out = capfd.readouterr().out.splitlines()
    assert out[0].startswith("Joint dim ") and any(" panda_hand " in l for l in out if l.startswith("Frame "))


# ------------------------------------------------------------------ KDL
def test_kdl_model_chain_and_tree_ik(models):
    """KDLModel (python/pybind_kdl.hpp): the tree root, the chain solvers NR /
    NR_JL / LMA from a perturbed start reach the FK target (return code 0),
    NR_JL stays inside its limits, and the tree solver meets two endpoints
    at once.  orocos KDL is absent here: its solver semantics are restated
    (kinjac.cpp), the answers are checked against their targets."""
    import os
    from oracle import model as M
    from mplib_amd import pymp, scenes
    _, ow = models
    joints = ["panda_joint%d" % i for i in range(1, 8)] + ["panda_finger_joint1", "panda_finger_joint2"]
    links = ["panda_link%d" % i for i in range(8)] + ["panda_hand", "panda_leftfinger", "panda_rightfinger"]
    kdl = pymp.kdl.KDLModel(os.path.join(scenes.PANDA_DIR, "panda.urdf"), joints, links, False)
    assert kdl.get_tree_root_name() == "panda_link0"
    rng = np.random.default_rng(12)
    lim = ow.art.joint_limits()[:7]
    lo = np.array(list(lim[:, 0]) + [0.0, 0.0])
    hi = np.array(list(lim[:, 1]) + [0.04, 0.04])
    solved = {"nr": 0, "jl": 0, "lma": 0}
    for _ in range(5):
        q_goal = rng.uniform(lim[:, 0] * 0.8, lim[:, 1] * 0.8)
        R, p = _hand_pose(ow, q_goal)
        w, x, y, z = M.mat_to_quat(list(R.reshape(-1)))
        pose = list(p) + [w, x, y, z]
        q0 = np.array(_full(np.clip(q_goal + rng.normal(scale=0.15, size=7), lim[:, 0], lim[:, 1])))
        for name, (q, rc) in (("nr", kdl.chain_IK_NR(HAND, q0, pose)),
                              ("jl", kdl.chain_IK_NR_JL(HAND, q0, pose, lo, hi)),
                              ("lma", kdl.chain_IK_LMA(HAND, q0, pose))):
            assert q.shape == (9,)
            assert (q[7:] == q0[7:]).all()  # joints off the chain keep their values
            if name == "jl":
                assert (q >= lo - 1e-12).all() and (q <= hi + 1e-12).all()
            if rc != 0:
                continue
            solved[name] += 1
            R2, p2 = _hand_pose(ow, q[:7])
            assert np.linalg.norm(p2 - p) < 1e-4 and np.abs(R2 - R).max() < 1e-3, name
    assert min(solved.values()) >= 3, solved
    # two endpoints at once: the hand and link 4 of one configuration
    q_goal = np.array([0.2, -0.3, 0.1, -2.1, 0.2, 1.9, 0.4])
    _, objT = ow.fk_batch(q_goal.reshape(1, 7))
    poses = []
    for k in (4, HAND):
        T = objT[0, k]
        w, x, y, z = M.mat_to_quat(list(T[:9]))
        poses.append(list(T[9:]) + [w, x, y, z])
    q0 = np.array(_full(q_goal + 0.05))
    q, rc = kdl.tree_IK_NR_JL(["panda_link4", "panda_hand"], q0, poses, lo, hi)
    assert rc == 0
    _, objT2 = ow.fk_batch(q[:7].reshape(1, 7))
    for k in (4, HAND):
        assert np.linalg.norm(objT2[0, k, 9:] - objT[0, k, 9:]) < 1e-4
