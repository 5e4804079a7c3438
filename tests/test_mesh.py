"""Non-convex meshes: fcl::BVHModel<OBBRSS> (load_mesh_as_BVH,
src/urdf_utils.cpp:136-155; FCLModel with use_convex=False,
src/fcl_model.cpp:224-227; PlanningWorld::attachMesh,
src/planning_world.cpp:212-218; fcl.BVHModel, python/pybind_fcl.hpp:177-219).

CPU: the oracle's triangle tests (FCL Intersect::intersect_Triangle and
sphereTriangleIntersect restated in oracle/collide_oracle.c) on constructed
known answers; the BVH of a convex hull's own surface against the convex
hull itself (they agree except when the other shape is strictly inside the
hull); the host loader against the oracle loader; the BVHModel builder API;
descriptor checks of the C ABI.  GPU: the device's mesh walk against the
oracle on the Panda with convex=False (mesh-mesh self pairs, mesh-box scene
pairs, attached sphere / box / mesh), both batch paths.
FCL is absent here: the triangle tests are pinned by these
constructed cases and the convex-hull property, not by FCL outputs.
"""
import os

import numpy as np
import pytest

import oracle
import worlds as Wd
from mplib_amd import pymp, scenes
from oracle import model as M

T0 = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], dtype=np.float64)


@pytest.mark.parametrize("Q,want", [
    ([[0.2, 0.2, -0.5], [0.2, 0.2, 0.5], [0.3, 0.3, 0.5]], True),    # pierces the interior
    ([[0.6, 0.6, -0.5], [0.6, 0.6, 0.5], [0.9, 0.9, 0.5]], False),   # pierces the plane beyond the hypotenuse
    ([[0, 0, 0.1], [1, 0, 0.1], [0, 1, 0.1]], False),                # parallel, 0.1 above
    ([[0.2, 0.2, 0], [1.2, 0.2, 0], [0.2, 1.2, 0]], True),           # coplanar, overlapping
    ([[1.1, 1.1, 0], [2, 1.1, 0], [1.1, 2, 0]], False),              # coplanar, disjoint
    ([[1, 0, 0], [2, 0, 0], [1, 1, 1]], True),                       # shares a vertex
    ([[0.5, -0.5, 0.0], [0.5, 0.5, 0.0], [0.5, 0.0, 1.0]], True),    # edge on edge (touching)
    ([[0.5, -0.5, 1e-9], [0.5, 0.5, 1e-9], [0.5, 0.0, 1.0]], False),  # lifted clear
])
def test_triangle_triangle_known_answers(Q, want):
    Q = np.array(Q, dtype=np.float64)
    assert oracle.tri_tri(T0, Q) is want
    assert oracle.tri_tri(Q, T0) is want  # symmetric on these cases


@pytest.mark.parametrize("c,r,want", [
    ([0.2, 0.2, 0.09], 0.1, True),    # above the face, within r
    ([0.2, 0.2, 0.11], 0.1, False),   # above the face, out of reach
    ([-0.05, -0.05, 0.0], 0.1, True),  # beside vertex P1 (|d| = 0.0707)
    ([-0.08, -0.08, 0.0], 0.1, False),  # |d| = 0.113
    ([0.55, 0.55, 0.0], 0.1, True),   # 0.0707 past the hypotenuse, in the plane
    ([0.55, 0.55, 0.08], 0.1, False),  # distance to that edge sqrt(0.005 + 0.0064) > 0.1
])
def test_sphere_triangle_known_answers(c, r, want):
    assert oracle.sphere_tri(r, c, T0) is want


def _gi(ob, g):
    return next(i for i, x in enumerate(ob.geoms) if x is g)


def _hull_as_bvh(art, link):
    g = next(o.geom for o in art.objects if o.link == link)
    return g, M.MeshGeom(g.vertices.copy(), [tuple(f) for f in g.faces])


def test_bvh_of_hull_surface_agrees_with_hull():
    """A shape meets the hull's surface triangles iff it meets the hull and
    is not strictly inside it: boxes / spheres / hulls at random poses."""
    art = Wd.panda_articulation()
    hull, bvh = _hull_as_bvh(art, "panda_link3")
    rng = np.random.default_rng(5)
    shapes = [M.BoxGeom((0.05, 0.08, 0.03)), M.SphereGeom(0.04), M.CapsuleGeom(0.02, 0.1), _hull_as_bvh(art, "panda_hand")[0]]
    n_hit = n_in = 0
    for k in range(600):
        sh = shapes[k % len(shapes)]
        w, x, y, z = Wd.random_quat(rng)
        T = (M.quat_to_mat(w, x, y, z), [float(v) for v in rng.uniform(-0.15, 0.15, 3)])
        ob = oracle.OracleWorld(art, scene=[("h", hull, M.IDENT), ("b", bvh, M.IDENT), ("s", sh, T)])
        gh, gb, gs = _gi(ob, hull), _gi(ob, bvh), _gi(ob, sh)
        a = Wd.collide_pair(ob, gs, T, gh, M.IDENT)
        b = Wd.collide_pair(ob, gs, T, gb, M.IDENT)
        c = Wd.collide_pair(ob, gb, M.IDENT, gs, T)  # mesh first: the shape is still o1 of the leaf test
        assert b == c
        if b:
            assert a, k  # touching the surface means touching the hull
            n_hit += 1
        elif a:
            n_in += 1  # inside the hull without reaching its surface
    assert n_hit > 50


def test_mesh_mesh_hull_surfaces():
    """Two hull surfaces as BVH meshes: intersecting triangles imply the
    hulls overlap (MPR), and disjoint hulls never have intersecting
    triangles."""
    art = Wd.panda_articulation()
    h1, b1 = _hull_as_bvh(art, "panda_link5")
    h2, b2 = _hull_as_bvh(art, "panda_hand")
    rng = np.random.default_rng(9)
    both = 0
    for k in range(300):
        w, x, y, z = Wd.random_quat(rng)
        T = (M.quat_to_mat(w, x, y, z), [float(v) for v in rng.uniform(-0.15, 0.15, 3)])
        ob = oracle.OracleWorld(art, scene=[("h1", h1, M.IDENT), ("b1", b1, M.IDENT), ("h2", h2, T), ("b2", b2, T)])
        G = lambda g: _gi(ob, g)  # noqa: E731
        hull_hit = Wd.collide_pair(ob, G(h1), M.IDENT, G(h2), T)
        mesh_hit = Wd.collide_pair(ob, G(b1), M.IDENT, G(b2), T)
        assert mesh_hit == Wd.collide_pair(ob, G(b2), T, G(b1), M.IDENT)
        if mesh_hit:
            assert hull_hit
            both += 1
    assert both > 20


def test_host_loader_matches_oracle_loader():
    d = os.path.join(Wd.panda_dir(), "franka_description", "meshes", "collision")
    for name in ("link0.stl", "link3.stl", "finger.stl"):
        a = M.load_bvh_mesh(os.path.join(d, name), (1.0, 2.0, 0.5))
        b = pymp.fcl.load_mesh_as_BVH(os.path.join(d, name), [1.0, 2.0, 0.5])
        assert np.array_equal(a.vertices, b.get_vertices())
        assert np.array_equal(np.array(a.faces), b.get_faces())
        assert b.num_faces == len(a.faces) and b.num_vertices == len(a.vertices)


def test_bvh_model_builder():
    m = pymp.fcl.BVHModel()
    m.beginModel()
    m.addSubModel(T0, np.array([[0, 1, 2]]))
    m.addSubModel(T0 + 1.0, np.array([[0, 2, 1]]))
    m.endModel()
    assert m.num_vertices == 6 and m.num_faces == 2
    assert m.get_faces().tolist() == [[0, 1, 2], [3, 5, 4]]
    with pytest.raises(ValueError):
        m.addSubModel(T0, np.array([[0, 1, 3]]))


def test_mesh_world_pair_table_and_known_answers():
    """convex=False: the same pair table; the detect_collision.py known
    answers hold on the meshes too."""
    ob = Wd.oracle_world(3, convex=False)
    assert all(isinstance(o.geom, M.MeshGeom) for o in ob.art.objects)
    w, _ = scenes.world(3, convex=False)
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == ob.pair_names()
    f, _ = Wd.oracle_world(2, convex=False).collide_batch(np.array([Wd.KAT_FREE, Wd.KAT_COLLIDING]))
    assert f.tolist() == [0, 1]


def test_capi_mesh_descriptor_checks():
    from mplib_amd.batch import DeviceWorld
    ob = Wd.oracle_world(3, convex=False)
    a = Wd.desc_arrays(ob)
    assert 6 in a["geom_type"] and len(a["mesh_triangle"]) > 0
    bad = dict(a)
    bad["mesh_triangle"] = np.array(a["mesh_triangle"]).copy()
    bad["mesh_triangle"][0] = 10 ** 6
    with pytest.raises(ValueError, match="mesh triangle"):
        DeviceWorld(bad)
    bad = dict(a)
    bad["geom_param"] = list(a["geom_param"])
    g = a["geom_type"].index(6)
    bad["geom_param"][4 * g + 1] = 1e9
    with pytest.raises(ValueError, match="mesh triangle range"):
        DeviceWorld(bad)


# ----------------------------------------------------------------------------
# GPU parity
# ----------------------------------------------------------------------------
def _oracle_T(pose):
    return oracle.pose7_to_se3(pose)


def _mesh_scene(w, art_o):
    """extra scene objects: a link mesh (BVH) and a link hull in the scene"""
    d = os.path.join(Wd.panda_dir(), "franka_description", "meshes", "collision")
    p_mesh = [0.45, 0.25, 0.35, 0.9238795325112867, 0.0, 0.3826834323650898, 0.0]
    p_hull = [0.5, -0.3, 0.45, 0.7071067811865476, 0.0, 0.0, 0.7071067811865476]
    w.add_normal_object("scene_mesh", pymp.fcl.CollisionObject(
        pymp.fcl.load_mesh_as_BVH(os.path.join(d, "link3.stl"), [1, 1, 1]), p_mesh[:3], p_mesh[3:]))
    w.add_normal_object("scene_hull", pymp.fcl.CollisionObject(
        pymp.fcl.load_mesh_as_Convex(os.path.join(d, "link5.stl.convex.stl"), [1, 1, 1]), p_hull[:3], p_hull[3:]))
    return [("scene_mesh", M.load_bvh_mesh(os.path.join(d, "link3.stl")), _oracle_T(p_mesh)),
            ("scene_hull", M.load_convex_mesh(os.path.join(d, "link5.stl.convex.stl")), _oracle_T(p_hull))]


def _bits(M_, P):
    return np.stack([(M_[:, p >> 5] >> (p & 31)) & 1 for p in P], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("convex", [False, True])
def test_mesh_worlds_match_oracle(convex):
    """Panda links as BVH meshes (convex=False) or hulls, the cfg3 boxes, a
    BVH mesh and a hull in the scene, an attached sphere, box and BVH mesh:
    every pair class (mesh-mesh, mesh-box / sphere / convex, sphere
    closed form vs triangles) on both batch paths."""
    d = os.path.join(Wd.panda_dir(), "franka_description", "meshes", "collision")
    w, art = scenes.world(3, convex=convex)
    base = Wd.oracle_world(3, convex=convex)
    extra = _mesh_scene(w, base.art)
    p_orb = [0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0]
    p_blk = [0.0, 0.06, 0.0, 1.0, 0.0, 0.0, 0.0]
    p_fing = [0.0, 0.0, 0.2, 0.7071067811865476, 0.7071067811865476, 0.0, 0.0]
    w.attach_object("orb", pymp.fcl.Sphere(0.05), "panda", 8, p_orb,
                    ["panda_hand", "panda_leftfinger", "panda_rightfinger"])
    w.attach_object("blk", pymp.fcl.Box([0.04, 0.04, 0.1]), "panda", 6, p_blk,
                    ["panda_link5", "panda_link6", "panda_link7"])
    w.attach_object("tool", pymp.fcl.load_mesh_as_BVH(os.path.join(d, "finger.stl"), [2, 2, 2]), "panda", 8, p_fing,
                    ["panda_hand", "orb"])
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + extra,
                            attached=[("orb", 8, M.SphereGeom(0.05), _oracle_T(p_orb)),
                                      ("blk", 6, M.BoxGeom((0.04, 0.04, 0.1)), _oracle_T(p_blk)),
                                      ("tool", 8, M.load_bvh_mesh(os.path.join(d, "finger.stl"), (2, 2, 2)),
                                       _oracle_T(p_fing))],
                            allowed=[("panda_hand", "orb"), ("panda_leftfinger", "orb"), ("panda_rightfinger", "orb"),
                                     ("panda_link5", "blk"), ("panda_link6", "blk"), ("panda_link7", "blk"),
                                     ("panda_hand", "tool"), ("orb", "tool"), ("panda_link0", "table")])
    order = {pn: k for k, pn in enumerate(o2.pair_names())}
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    assert sorted(names) == sorted(o2.pair_names())
    perm = [order[n] for n in names]
    q = Wd.sample_q(base.art, 6000, 31)
    q = np.vstack([q, [Wd.KAT_FREE, Wd.KAT_COLLIDING]])
    fo, mo = o2.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(_bits(m, range(len(perm))), _bits(mo, perm))
    hit = _bits(mo, perm)
    # sphere-triangle, mesh-mesh and link-mesh classes are exercised (oracle counts: 31, 11, 54)
    for pair in [("orb", "scene_mesh"), ("tool", "scene_mesh"), ("panda_link4", "scene_mesh")]:
        assert hit[:, names.index(pair)].sum() > 0, pair
    assert 0 < int(fo.sum()) < len(q)
    assert int(hit.sum()) > 0


@pytest.mark.gpu
def test_mesh_world_unsupported_queries():
    w, _ = scenes.world(2, convex=False)
    w.set_qpos_all(Wd.KAT_COLLIDING)
    assert w.collide() and len(w.collide_full()) > 0
    w.set_qpos_all(Wd.KAT_FREE)
    assert not w.collide() and w.collide_full() == []
    with pytest.raises(NotImplementedError, match="BVH mesh"):
        w.self_distance()
    with pytest.raises(NotImplementedError):
        w.collide(pymp.fcl.CollisionRequest(enable_contact=True))


@pytest.mark.gpu
def test_planner_on_mesh_robot_matches_oracle_checker():
    """RRTConnect on the Panda with BVH mesh links: the device checker
    (latency path, mesh walk) gives the same path as the oracle's mesh
    restatement used as the checker."""
    ob = Wd.oracle_world(3, convex=False)
    w, _ = scenes.world(3, convex=False)
    dev = pymp.ompl.OMPLPlanner(w)
    ref = pymp.ompl.OMPLPlanner(scenes.world(3, convex=False)[0],
                                state_validity_checker=lambda s: ob.collide_batch(s)[0] == 0)
    start = np.array(scenes.PLAN_START)
    goal = np.array(scenes.PLAN_GOALS["near"])
    pymp.set_global_seed(3)
    s1, p1 = dev.plan(start, [goal], range=0.1, time=60.0)
    pymp.set_global_seed(3)
    s2, p2 = ref.plan(start, [goal], range=0.1, time=60.0)
    assert s1 == s2 == "Exact solution"
    assert np.array_equal(p1, p2)
    body = p1[1:] if ob.collide_batch(start[None])[0][0] else p1  # an invalid start is resampled and prefixed
    assert (ob.collide_batch(body)[0] == 0).all()
