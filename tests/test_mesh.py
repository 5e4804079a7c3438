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


def _seg_seg(p1, q1, p2, q2):
    """exact distance of two segments (clamped closest-point parameters)"""
    d1, d2, r = q1 - p1, q2 - p2, p1 - p2
    a, e, f, c, b = d1 @ d1, d2 @ d2, d2 @ r, d1 @ r, d1 @ d2
    den = a * e - b * b
    s = np.clip((b * f - c * e) / den, 0, 1) if den != 0 else 0.0
    t = (b * s + f) / e
    if t < 0:
        t, s = 0.0, np.clip(-c / a, 0, 1)
    elif t > 1:
        t, s = 1.0, np.clip((b - c) / a, 0, 1)
    return float(np.linalg.norm(p1 + d1 * s - (p2 + d2 * t)))


def _pt_tri(p, T):
    a, b, c = T
    n = np.cross(b - a, c - a)
    n /= np.linalg.norm(n)
    q = p - ((p - a) @ n) * n
    sides = [np.cross(v - u, q - u) @ n for u, v in ((a, b), (b, c), (c, a))]
    if all(x >= 0 for x in sides) or all(x <= 0 for x in sides):
        return abs(float((p - a) @ n))
    return min(float(np.linalg.norm(p - (u + np.clip((p - u) @ (v - u) / ((v - u) @ (v - u)), 0, 1) * (v - u))))
               for u, v in ((a, b), (b, c), (c, a)))


def _tri_distance_brute(S, T):
    if oracle.tri_tri(S, T):
        return 0.0
    return min([_pt_tri(p, T) for p in S] + [_pt_tri(p, S) for p in T] +
               [_seg_seg(S[i], S[(i + 1) % 3], T[j], T[(j + 1) % 3]) for i in range(3) for j in range(3)])


@pytest.mark.parametrize("Q,want", [
    ([[0, 0, 0.1], [1, 0, 0.1], [0, 1, 0.1]], 0.1),                   # parallel, 0.1 above
    ([[0.2, 0.2, -0.5], [0.2, 0.2, 0.5], [0.3, 0.3, 0.5]], 0.0),      # pierces the interior
    ([[2, 0, 0], [3, 0, 0], [2, 1, 0]], 1.0),                         # coplanar, vertex to vertex
    ([[0.25, 0.25, 0.3], [0.25, 0.25, 1.0], [0.3, 0.2, 1.0]], 0.3),   # vertex above the face
    ([[0.5, 0.5, 0.2], [1.5, 1.5, 0.2], [1.5, 1.5, 1.2]], 0.2),       # vertex above the hypotenuse
    ([[0.5, -0.5, 1e-3], [0.5, 0.5, 1e-3], [0.5, 0.0, 1.0]], 1e-3),   # edge above the face
])
def test_triangle_distance_known_answers(Q, want):
    """FCL TriangleDistance::triDistance (PQP TriDist, oracle tri_distance)"""
    Q = np.array(Q, dtype=np.float64)
    assert oracle.tri_distance(T0, Q) == pytest.approx(want, abs=1e-12)
    assert oracle.tri_distance(Q, T0) == pytest.approx(want, abs=1e-12)


def test_triangle_distance_matches_brute_force():
    """triDistance equals the exact minimum over the vertex-face and
    edge-edge distances (0 when the triangles intersect) on random pairs"""
    rng = np.random.default_rng(0)
    for _ in range(1500):
        S = rng.normal(size=(3, 3))
        T = rng.normal(size=(3, 3)) + rng.normal(size=3) * rng.uniform(0, 3)
        assert abs(oracle.tri_distance(S, T) - _tri_distance_brute(S, T)) < 1e-9


def test_mesh_octree_oracle_matches_leaf_boxes():
    """fcl::collide / fcl::distance(mesh, OcTree) in the oracle equal the
    same query against every occupied leaf as its own box (box first, as
    OcTreeMeshIntersectRecurse / OcTreeMeshDistanceRecurse run the leaf
    test), in both argument orders."""
    art = Wd.panda_articulation(False)
    mesh = next(o.geom for o in art.objects if o.link == "panda_link3")
    rng = np.random.default_rng(3)
    tree = M.OcTreeGeom(rng.uniform(-0.12, 0.12, (200, 3)), 0.02)
    leaves = np.asarray(tree.leaves)
    boxes = [(M.BoxGeom(tuple(float(v) for v in l[3:] - l[:3])), (M.IDENT[0], [float(v) for v in (l[:3] + l[3:]) * 0.5]))
             for l in leaves]
    ob = oracle.OracleWorld(art, scene=[("pcd", tree, M.IDENT), ("m", mesh, M.IDENT)] +
                            [(f"b{i}", b, c) for i, (b, c) in enumerate(boxes)])
    gt, gm = _gi(ob, tree), _gi(ob, mesh)
    gb = [_gi(ob, b) for b, _ in boxes]
    n_hit = n_far = 0
    for k in range(120):
        w, x, y, z = Wd.random_quat(rng)
        T = (M.quat_to_mat(w, x, y, z), [float(v) for v in rng.uniform(-0.3, 0.3, 3)])
        hit = Wd.collide_pair(ob, gm, T, gt, M.IDENT)
        assert hit == Wd.collide_pair(ob, gt, M.IDENT, gm, T)
        # mesh-box pairs go through FCL's BVHModel<OBBRSS> traversal (OBB
        # gates down to the triangle's own leaf box); the mesh-octree walk
        # tests every (leaf box, triangle) within libccd's reach, ungated
        # (OcTreeMeshIntersectRecurse's interleaved octree/BVH descent is not
        # restated): a gated box hit is an octree hit
        box_hits = [Wd.collide_pair(ob, g, c, gm, T) for g, (_, c) in zip(gb, boxes)]
        assert hit or not any(box_hits)
        d = Wd.distance_pair(ob, gm, T, gt, M.IDENT)
        assert d == Wd.distance_pair(ob, gt, M.IDENT, gm, T)
        assert d == min(Wd.distance_pair(ob, g, c, gm, T) for g, (_, c) in zip(gb, boxes))
        n_hit += hit
        n_far += d > 0.02
    assert n_hit > 10 and n_far > 10


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


def _box_mesh(side):
    """a box surface as a BVH mesh: 12 triangles, vertex i = (x, y, z) bits"""
    h = np.asarray(side, dtype=np.float64) / 2
    v = np.array([[x, y, z] for x in (-h[0], h[0]) for y in (-h[1], h[1]) for z in (-h[2], h[2])])
    f = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1), (2, 3, 7), (2, 7, 6), (0, 2, 6), (0, 6, 4),
         (1, 5, 7), (1, 7, 3)]
    return M.MeshGeom(v, f)


def _flatT(R=None, p=(0.0, 0.0, 0.0)):
    R = np.eye(3) if R is None else np.asarray(R)
    return np.concatenate([R.reshape(-1), np.asarray(p, dtype=np.float64)])


def _contact_pair(ob, ga, Ta, gb, Tb):
    import ctypes
    P = ctypes.POINTER(ctypes.c_double)
    depth = ctypes.c_double()
    nrm, pos = np.zeros(3), np.zeros(3)
    Ta, Tb = np.ascontiguousarray(Ta), np.ascontiguousarray(Tb)
    r = oracle.lib().orc_contact_pair(ctypes.byref(ob._w), ga, Ta.ctypes.data_as(P), gb, Tb.ctypes.data_as(P),
                                      ctypes.byref(depth), nrm.ctypes.data_as(P), pos.ctypes.data_as(P))
    return r, depth.value, nrm, pos


def test_mesh_contacts_known_answers():
    """The oracle's BVH-mesh contact restatement on plain geometry:
    sphere over a box surface mesh -> sphereTriangleIntersect's contact on the
    first hit triangle (projection of the centre, normal from the centre to
    it, stored depth -(r - d)); a small box mesh sunk 0.05 into a unit box
    mesh -> intersect_Triangle's deepest point (a bottom corner of the small
    box, depth 0.05, normal -n1 of the big box's top triangle = -z); the
    mesh-first order negates the normal; shape vs mesh through MPR
    penetration: unit normal, positive depth, mirrored by the other order."""
    big, small, ball, blk = _box_mesh((1, 1, 1)), _box_mesh((0.2, 0.2, 0.2)), M.SphereGeom(0.1), M.BoxGeom((0.2, 0.2, 0.2))
    ob = oracle.OracleWorld(Wd.panda_articulation(), scene=[(f"g{i}", g, M.IDENT) for i, g in
                                                            enumerate((big, small, ball, blk))])
    gb, gs, gp, gx = (_gi(ob, g) for g in (big, small, ball, blk))
    # sphere 0.06 above the top face, over triangle 10 (1, 5, 7): y < x
    r, d, n, p = _contact_pair(ob, gp, _flatT(p=(0.05, -0.02, 0.56)), gb, _flatT())
    assert r == 1 and abs(d - (-(0.1 - 0.06))) < 1e-12
    np.testing.assert_allclose(n, [0, 0, -1], atol=1e-12)
    np.testing.assert_allclose(p, [0.05, -0.02, 0.5], atol=1e-12)
    r2, d2, n2, p2 = _contact_pair(ob, gb, _flatT(), gp, _flatT(p=(0.05, -0.02, 0.56)))
    assert r2 == 1 and d2 == d and np.array_equal(n2, -n) and np.array_equal(p2, p)
    # mesh-mesh: the small box's bottom (z = 0.45) below the big box's top face
    c = np.cos(0.3), np.sin(0.3)
    Rz = [[c[0], -c[1], 0], [c[1], c[0], 0], [0, 0, 1]]
    Ts = _flatT(Rz, (0.13, -0.21, 0.55))
    r, d, n, p = _contact_pair(ob, gb, _flatT(), gs, Ts)
    assert r == 1 and abs(d - 0.05) < 1e-12
    np.testing.assert_allclose(n, [0, 0, -1], atol=1e-12)
    corners = (np.array(Rz) @ small.vertices.T).T + [0.13, -0.21, 0.55]
    assert abs(p[2] - 0.45) < 1e-12 and np.min(np.linalg.norm(corners - p, axis=1)) < 1e-12
    assert _contact_pair(ob, gb, _flatT(), gs, _flatT(Rz, (0.13, -0.21, 0.75)))[0] == 0
    # box shape vs mesh (MPR penetration of (box, triangle)), both orders
    r, d, n, p = _contact_pair(ob, gx, Ts, gb, _flatT())
    r2, d2, n2, p2 = _contact_pair(ob, gb, _flatT(), gx, Ts)
    assert r == r2 == 1 and d > 0 and d == d2
    assert abs(np.linalg.norm(n) - 1) < 1e-6 and np.array_equal(n2, -n) and np.array_equal(p2, p)


def test_mesh_contact_batch_consistent_with_collide():
    """The oracle's contact pass on a convex=False world reports exactly the
    pairs its collide pass does (same leaf tests decide)."""
    ow = Wd.oracle_world(3, convex=False)
    q = Wd.sample_q(ow.art, 24, 6)
    hit, depth, normal, pos = ow.contact_batch(q)
    _, masks = ow.collide_batch(q)
    bits = np.stack([(masks[:, p >> 5] >> (p & 31)) & 1 for p in range(len(ow.pairs))], 1)
    np.testing.assert_array_equal(hit, bits)
    assert hit.sum() > 0


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


def _full_mesh_world(convex):
    """Panda links as BVH meshes (convex=False) or hulls, the cfg3 boxes, a
    BVH mesh and a hull in the scene, an attached sphere, box and BVH mesh:
    (PlanningWorld, OracleWorld, base oracle world, device pair names, perm
    device pair -> oracle pair)."""
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
    return w, o2, base, names, perm


@pytest.mark.gpu
@pytest.mark.parametrize("convex", [False, True])
def test_mesh_worlds_match_oracle(convex):
    """_full_mesh_world: every pair class (mesh-mesh, mesh-box / sphere /
    convex, sphere closed form vs triangles) on both batch paths."""
    w, o2, base, names, perm = _full_mesh_world(convex)
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
@pytest.mark.parametrize("convex", [False, True])
def test_mesh_distance_matches_oracle(convex):
    """fcl::distance on BVH meshes (mesh-mesh triDistance, mesh-shape GJK
    on the triangle GJK objects) in PlanningWorld::distanceSelf /
    distanceOthers: batched minima within 1e-9 of the oracle, the same
    nearest pair, penetration (-1) / touching meshes (0) the same; scalar
    self_distance / distance_with_others on a few states."""
    w, o2, base, names, perm = _full_mesh_world(convex)
    q = np.vstack([Wd.sample_q(base.art, 400, 41), [Wd.KAT_FREE, Wd.KAT_COLLIDING]])
    ds, ps, do, po = w.distance_batch(q)
    rs, rps, ro, rpo = o2.distance_batch(q)
    on = o2.pair_names()
    for d, r, p, rp in ((ds, rs, ps, rps), (do, ro, po, rpo)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
        same = [names[a] == on[b] for a, b in zip(p, rp)]
        assert np.mean(same) > 0.99
    mesh_pairs = {n for n in names if "scene_mesh" in n or "tool" in n} | (set(names) if not convex else set())
    assert any(names[p] in mesh_pairs for p in np.concatenate([ps, po]))  # a mesh pair is the nearest somewhere
    for i in (0, 1, len(q) - 1):
        w.set_qpos_all(list(q[i]))
        a, b = w.self_distance(), w.distance_with_others()
        assert abs(a.min_distance - rs[i]) < 1e-9 and abs(b.min_distance - ro[i]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("cloud", ["floor", "blue"])
def test_mesh_robot_point_cloud_matches_oracle(cloud):
    """BVH mesh links against a point cloud (fcl::collide / fcl::distance on
    (BVHModel, OcTree): box-first MPR / GJK on every (leaf, triangle) pair):
    flags and pair bits on both batch paths bit-exact, distances within 1e-9
    of the oracle."""
    art = scenes.panda(convex=False)
    if cloud == "floor":
        w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
        scene = []
        allowed = []
    else:
        w, art = scenes.world(3, convex=False)
        scene = Wd.boxes_scene()
        allowed = [("panda_link0", "table")]
    w.add_point_cloud("scene_pcd", scenes.cloud_points(cloud), 1e-3)
    o = oracle.OracleWorld(Wd.panda_articulation(False),
                           scene=scene + [("scene_pcd", M.OcTreeGeom(scenes.cloud_points(cloud), 1e-3), M.IDENT)],
                           allowed=allowed)
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    assert names == o.pair_names()
    q = np.vstack([Wd.sample_q(o.art, 3000, 77), [scenes.FLOOR_COLLIDING, Wd.KAT_FREE]])
    fo, mo = o.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)
    k = names.index(("panda_link0", "scene_pcd")) if cloud == "floor" else names.index(("panda_hand", "scene_pcd"))
    cloud_hits = sum(int(((mo[:, p >> 5] >> (p & 31)) & 1).sum()) for p, n in enumerate(names) if n[1] == "scene_pcd")
    assert cloud_hits > 0, k
    qd = q[-40:]
    ds, ps, do, po = w.distance_batch(qd)
    rs, rps, ro, rpo = o.distance_batch(qd)
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)


@pytest.mark.gpu
def test_mesh_world_scalar_queries():
    w, _ = scenes.world(2, convex=False)
    w.set_qpos_all(Wd.KAT_COLLIDING)
    assert w.collide() and len(w.collide_full()) > 0
    assert w.collide(pymp.fcl.CollisionRequest(enable_contact=True))
    w.set_qpos_all(Wd.KAT_FREE)
    assert not w.collide() and w.collide_full() == []


def _check_scalar_contacts(w, o2, q):
    """collide_full(CollisionRequest(enable_contact=True)) per configuration
    against the oracle's contact pass: the same reported pairs, each with the
    oracle's (depth, normal, position) within 1e-9."""
    req = pymp.fcl.CollisionRequest(enable_contact=True)
    hit, rd, rn, rp = o2.contact_batch(q)
    names = o2.pair_names()
    for i in range(len(q)):
        w.set_qpos_all(list(q[i]))
        got = {(c.link_name1, c.link_name2): c.res.get_contacts()[0] for c in w.collide_full(req)}
        exp = {names[p]: p for p in np.nonzero(hit[i])[0]}
        assert set(got) == set(exp)
        for k, p in exp.items():
            c = got[k]
            assert abs(c.penetration_depth - rd[i, p]) < 1e-9, (k, c.penetration_depth, rd[i, p])
            np.testing.assert_allclose(c.normal, rn[i, p], atol=1e-9)
            np.testing.assert_allclose(c.pos, rp[i, p], atol=1e-9)
    return hit


@pytest.mark.gpu
@pytest.mark.parametrize("convex", [False, True])
def test_mesh_contacts_match_oracle(convex):
    """enable_contact=True on every BVH-mesh pair class of _full_mesh_world
    (mesh-mesh deepest points, sphere-triangle, shape-triangle MPR
    penetration, both argument orders): the device reports the pairs the
    oracle does, each contact within 1e-9 of the oracle's restatement."""
    w, o2, base, names, perm = _full_mesh_world(convex)
    q = Wd.sample_q(base.art, 6000, 31)
    _, mo = o2.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    on = o2.pair_names()
    mesh_pairs = [k for k, n in enumerate(on) if "scene_mesh" in n or "tool" in n or not convex]
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in mesh_pairs], 1), 1))[0]
    assert len(sel) >= 20
    hit = _check_scalar_contacts(w, o2, q[sel[:60]])
    assert hit[:, mesh_pairs].sum() >= 20


@pytest.mark.gpu
@pytest.mark.parametrize("cloud", ["floor", "blue"])
def test_mesh_robot_point_cloud_contacts_match_oracle(cloud):
    """enable_contact=True between BVH mesh links and a point cloud: MPR
    penetration of the first (leaf box, triangle) hit in
    OcTreeMeshIntersectRecurse's visit order, within 1e-9 of the oracle."""
    w, o = _cloud_mesh_worlds(cloud)
    q = np.vstack([Wd.sample_q(o.art, 600, 78), [scenes.FLOOR_COLLIDING]])
    _, mo = o.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    pc = [k for k, (a, b) in enumerate(o.pair_names()) if b == "scene_pcd"]
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in pc], 1), 1))[0]
    assert len(sel) >= 1
    hit = _check_scalar_contacts(w, o, q[sel[:12]])
    assert hit[:, pc].sum() >= 1


def _cloud_mesh_worlds(cloud):
    art = scenes.panda(convex=False)
    if cloud == "floor":
        w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
        scene, allowed = [], []
    else:
        w, art = scenes.world(3, convex=False)
        scene, allowed = Wd.boxes_scene(), [("panda_link0", "table")]
    w.add_point_cloud("scene_pcd", scenes.cloud_points(cloud), 1e-3)
    o = oracle.OracleWorld(Wd.panda_articulation(False),
                           scene=scene + [("scene_pcd", M.OcTreeGeom(scenes.cloud_points(cloud), 1e-3), M.IDENT)],
                           allowed=allowed)
    return w, o


def _near_cloud_contact(o, n_seg, seed):
    """Configurations straddling first contact with the cloud: segments from
    a state with no cloud pair hit to one with a hit, bisected 14 times on the
    oracle's cloud bits, then jittered by 1e-5 rad around the boundary."""
    pc = [k for k, (a, b) in enumerate(o.pair_names()) if b == "scene_pcd"]

    def cloud_hit(q):
        _, m = o.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
        return np.any(np.stack([(m[:, k >> 5] >> (k & 31)) & 1 for k in pc], 1), 1)

    q = Wd.sample_q(o.art, 4000, seed)
    h = cloud_hit(q)
    ins, outs = q[h], q[~h]
    n = min(n_seg, len(ins), len(outs))
    assert n >= 8
    lo, hi = outs[:n].copy(), ins[:n].copy()
    for _ in range(14):
        mid = (lo + hi) / 2
        hm = cloud_hit(mid)
        hi[hm], lo[~hm] = mid[hm], mid[~hm]
    rng = np.random.default_rng(seed + 1)
    return np.vstack([lo, hi] + [hi + rng.normal(0, 1e-5, hi.shape) for _ in range(6)]), pc


@pytest.mark.gpu
@pytest.mark.parametrize("cloud", ["floor", "blue"])
def test_mesh_robot_point_cloud_near_contact(cloud):
    """BVH mesh links grazing a point cloud, where OcTreeMeshIntersectRecurse's
    BV tests decide which (leaf, triangle) pairs reach MPR: flags and pair bits
    on both batch paths bit-exact with the oracle's traversal, and the first
    contact in its visit order (depth / normal / position within 1e-9)."""
    w, o = _cloud_mesh_worlds(cloud)
    q, pc = _near_cloud_contact(o, 48, 91)
    fo, mo = o.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    hits = np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in pc], 1), 1)
    assert 0 < hits.sum() < len(q)
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)
    sel = np.nonzero(hits)[0]
    _check_scalar_contacts(w, o, q[sel[::max(1, len(sel) // 24)]])


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
