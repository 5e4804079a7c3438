"""A pair of two OcTrees (fcl::collide(OcTree, OcTree) ->
OcTreeSolver::OcTreeIntersectRecurse [ext FCL 0.7.0]): a point cloud held by
the robot (attachObject takes any FCL geometry, src/planning_world.cpp:174-191)
against a scene point cloud (addPointCloud, :102-110).  Without contacts or
costs FCL reports a collision as soon as two occupied leaves' OBBs overlap --
no box test (oracle/collide_oracle.c octree_octree_intersect, device
mpg_kernels.hip octree_octree_wave).  FCL is not under /root/reference: the
restatement is pinned by geometry (voxel faces touching / 1 mm apart,
rotated) and the device equals the oracle bit for bit.  Contacts and
distances of such a pair are refused (NotImplementedError)."""
import ctypes

import numpy as np
import pytest

import worlds as Wd
from test_oracle import _T, _pair_world

P = ctypes.POINTER(ctypes.c_double)


def _hit(w, ga, Ta, gb, Tb):
    import oracle
    return bool(oracle.lib().orc_collide_pair(ctypes.byref(w._w), ga, np.ascontiguousarray(Ta).ctypes.data_as(P),
                                              gb, np.ascontiguousarray(Tb).ctypes.data_as(P)))


def _plate(n=6, res=0.005):
    """n x n points in the plane z = res / 2, one per voxel of a res grid."""
    g = (np.arange(n) + 0.5) * res
    return np.array([[x, y, res / 2] for x in g for y in g], np.float64)


def test_octree_octree_known_answers():
    """Two voxel plates (5 mm leaves): touching faces collide (OBB overlap,
    obbDisjoint's 1e-6 widening), 1 mm apart do not; the same offset
    vertical, sideways and with the second plate turned 45 degrees; both
    argument orders."""
    from oracle import model as M
    res = 0.005
    a, b = M.OcTreeGeom(_plate(), res), M.OcTreeGeom(_plate(4), res)
    assert len(a.leaves) and len(b.leaves)
    w, (ga, gb) = _pair_world([a, b])
    c45 = (np.cos(np.pi / 8), 0.0, 0.0, np.sin(np.pi / 8))
    cases = [(_T(p=(0.0, 0.0, 0.005)), True), (_T(p=(0.0, 0.0, 0.006)), False),
             (_T(p=(0.0, 0.0, -0.0049)), True), (_T(p=(0.0, 0.0, -0.0061)), False),
             (_T(p=(0.030, 0.0, 0.0)), True), (_T(p=(0.031, 0.0, 0.0)), False),
             (_T(p=(0.0, 0.0, 0.0)), True),
             (_T(q=c45, p=(0.01, 0.01, 0.0049)), True), (_T(q=c45, p=(0.01, 0.01, 0.0061)), False)]
    for k, (Tb, want) in enumerate(cases):
        assert _hit(w, ga, _T(), gb, Tb) == want, k
        assert _hit(w, gb, Tb, ga, _T()) == want, ("swapped", k)


def test_octree_octree_matches_brute_force_sat():
    """Random poses of two small clouds: the oracle's answer equals an
    independent 15-axis separating-axis test over every leaf pair (exact
    boxes; the poses keep clear of grazing contact)."""
    from oracle import model as M
    rng = np.random.default_rng(3)
    res = 0.01
    pa = rng.uniform(0.0, 0.06, (40, 3))
    pb = rng.uniform(0.0, 0.05, (30, 3))
    a, b = M.OcTreeGeom(pa, res), M.OcTreeGeom(pb, res)
    w, (ga, gb) = _pair_world([a, b])

    def boxes(geom, T):
        R, t = T[:9].reshape(3, 3), T[9:]
        L = np.asarray(geom.leaves)
        return (L[:, :3] + L[:, 3:]) / 2 @ R.T + t, (L[:, 3:] - L[:, :3]) / 2, R

    def sat(ca, ea, Ra, cb, eb, Rb):
        axes = [Ra[:, i] for i in range(3)] + [Rb[:, i] for i in range(3)]
        axes += [np.cross(Ra[:, i], Rb[:, j]) for i in range(3) for j in range(3)]
        for ax in axes:
            n = np.linalg.norm(ax)
            if n < 1e-9:
                continue
            ax = ax / n
            ra = np.abs(Ra.T @ ax) @ ea
            rb = np.abs(Rb.T @ ax) @ eb
            s = abs((cb - ca) @ ax) - ra - rb
            if s > 0:
                return s  # separated by s along ax
        return -1.0

    seen = set()
    for _ in range(60):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        Tb = _T(q=tuple(q), p=tuple(rng.uniform(-0.05, 0.08, 3)))
        CA, EA, RA = boxes(a, _T())
        CB, EB, RB = boxes(b, Tb)
        gaps = [sat(CA[i], EA[i], RA, CB[j], EB[j], RB) for i in range(len(CA)) for j in range(len(CB))]
        best = min(gaps, key=lambda g: (g > 0, g))  # any overlap -> -1
        if 0 < best < 1e-6:
            continue  # grazing: obbDisjoint's widening decides
        want = best < 0
        assert _hit(w, ga, _T(), gb, Tb) == want
        seen.add(want)
    assert seen == {True, False}


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_held_cloud_against_scene_cloud_matches_oracle():
    """cfg3 + the blue box's point cloud (5 mm) as a scene object + a held
    point cloud under panda_hand: every flag and pair bit equal to the
    oracle's on both batch paths, the (held cloud, scene cloud) pair
    exercised; contacts and distances of the world raise."""
    import oracle
    from oracle import model as M
    from mplib_amd import pymp, scenes
    from test_gpu_parity import _oracle_T
    res = 0.005
    w, art = scenes.cloud_world("blue", res)
    pts = scenes.box_surface_points(np.random.default_rng(11), (0.06, 0.06, 0.05), 800, (0.0, 0.0, 0.0))
    pose = [0.0, 0.0, 0.16, 1.0, 0.0, 0.0, 0.0]
    touch = ["panda_hand", "panda_leftfinger", "panda_rightfinger"]
    w.attach_object("held_cloud", pymp.fcl.OcTree(pts, res), "panda", 8, pose, touch)
    base = Wd.oracle_cloud_world("blue", res)
    o2 = oracle.OracleWorld(base.art, scene=base.scene,
                            attached=[("held_cloud", 8, M.OcTreeGeom(pts, res), _oracle_T(pose))],
                            allowed=[(t, "held_cloud") for t in touch] + [("panda_link0", "table")])
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == o2.pair_names()
    q = Wd.sample_q(base.art, 6000, 35)
    fo, mo = o2.collide_batch(q, nthreads=8)
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)
    k = o2.pair_names().index(("held_cloud", "scene_pcd"))
    assert ((mo[:, k >> 5] >> (k & 31)) & 1).sum() > 0  # the two clouds do meet
    with pytest.raises(NotImplementedError, match="two OcTrees"):
        w.distance_batch(q[:4])
    with pytest.raises(NotImplementedError):
        w.set_qpos_all(list(q[0]))
        w.collide_full(pymp.fcl.CollisionRequest(enable_contact=True))
