"""CPU: the oracle restatement against the reference's known answers and the
committed golden vectors (regression pins; see tests/golden/gen_golden.py)."""
import json
import os

import numpy as np
import pytest

import oracle
import worlds as Wd
from oracle import model as M


@pytest.fixture(scope="module")
def ow2():
    return Wd.oracle_world(2)


def test_model_facts_match_survey(ow2, golden_dir):
    """11 objects, 1033 hull vertices, 19 SRDF-filtered pairs."""
    art = ow2.art
    facts = json.load(open(os.path.join(golden_dir, "panda_model.json")))
    assert [o.link for o in art.objects] == facts["objects"] == Wd.PANDA_LINKS
    counts = [len(o.geom.vertices) for o in art.objects]
    assert counts == [84, 133, 131, 131, 133, 117, 102, 79, 93, 15, 15] == facts["vertex_counts"]
    assert sum(counts) == 1033
    assert [list(p) for p in art.pairs] == facts["self_pairs"]
    assert art.pairs == [(0, 5), (1, 5), (2, 5), (0, 6), (1, 6), (0, 7), (1, 7), (2, 7), (0, 8), (1, 8), (2, 8),
                         (0, 9), (1, 9), (2, 9), (5, 9), (0, 10), (1, 10), (2, 10), (5, 10)]
    assert abs(facts["link0_min_z"] - (-3.25e-5)) < 1e-7
    assert art.qpos_dim == 7


def test_parent_rule_before_srdf():
    """fcl_model.cpp:282-293 leaves 46 pairs before SRDF removal."""
    from oracle import model as M
    d = Wd.panda_dir()
    art = M.Articulation(os.path.join(d, "panda.urdf"), "", Wd.PANDA_LINKS, Wd.PANDA_JOINTS)
    assert len(art.pairs) == 46


def test_detect_collision_known_answers(ow2):
    """examples/detect_collision.py:25 (free) and :31 (self-colliding)."""
    f, m = ow2.collide_batch(np.array([Wd.KAT_FREE, Wd.KAT_COLLIDING]))
    assert f.tolist() == [0, 1]
    assert ow2.decode(m[0]) == []
    assert len(ow2.decode(m[1])) > 0


@pytest.mark.parametrize("name,cfg", [("panda_self_4096", 2), ("panda_boxes_4096", 3), ("panda_convex_1024", 4),
                                      ("panda_mesh_1024", 7)])
def test_oracle_reproduces_golden(golden_dir, name, cfg):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    ow = Wd.oracle_world(cfg)
    f, m = ow.collide_batch(g["q"], nthreads=4)
    np.testing.assert_array_equal(f, g["flags"])
    np.testing.assert_array_equal(m, g["masks"])
    assert [list(p) for p in ow.pair_names()] == g["pairs"].tolist()
    # flags are exactly "any reported pair"
    np.testing.assert_array_equal(f.astype(bool), (m != 0).any(1))


def test_oracle_fk_golden(golden_dir, ow2):
    g = np.load(os.path.join(golden_dir, "panda_fk_64.npz"))
    poses, objT = ow2.fk_batch(g["q"])
    np.testing.assert_array_equal(poses, g["link_pose"])
    np.testing.assert_array_equal(objT, g["obj_T"])


def test_oracle_multithread_deterministic(ow2):
    q = Wd.sample_q(ow2.art, 512, 11)
    a = ow2.collide_batch(q, nthreads=1)
    b = ow2.collide_batch(q, nthreads=4)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_acm_allowed_pair_never_reported():
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, 256, 1)
    # allow everything with link0: its bits must vanish
    allowed = [(p[4], p[5]) for p in ow.pairs if "panda_link0" in (p[4], p[5])]
    import oracle
    ow_a = oracle.OracleWorld(ow.art, scene=ow.scene, allowed=allowed)
    f, m = ow_a.collide_batch(q)
    for row in m:
        assert all("panda_link0" not in pr for pr in ow_a.decode(row))


def test_assimp_atof_semantics():
    from oracle import model as M
    assert M.assimp_atof("0.14") == float(np.float32(0.14))
    e = M.assimp_atof("-5.6801935e-05")
    assert e == float(np.float32(e)) and abs(e + 5.6801935e-05) < 1e-11
    v = M.assimp_atof("-0.031705923")
    assert v == float(np.float32(v))  # a binary32 value
    assert abs(v + 0.031705923) < 1e-8


# ------------------------------------------------ FCL closed-form primitive pairs
def _pair_world(geoms):
    import oracle
    from oracle import model as M
    base = Wd.oracle_world(2)
    eye = (list(M.quat_to_mat(1.0, 0.0, 0.0, 0.0)), [0.0, 0.0, 0.0])
    w = oracle.OracleWorld(base.art, scene=[(f"g{i}", g, eye) for i, g in enumerate(geoms)])
    idx = [next(i for i, gg in enumerate(w.geoms) if gg is g) for g in geoms]
    return w, idx


def _T(q=(1.0, 0.0, 0.0, 0.0), p=(0.0, 0.0, 0.0)):
    from oracle import model as M
    return np.array(list(M.quat_to_mat(*q)) + list(p), dtype=np.float64)


def _collide(w, ga, Ta, gb, Tb):
    import ctypes
    import oracle
    P = ctypes.POINTER(ctypes.c_double)
    return oracle.lib().orc_collide_pair(ctypes.byref(w._w), ga, Ta.ctypes.data_as(P), gb, Tb.ctypes.data_as(P))


def test_box_box_closed_form_known_answers():
    """FCL boxBox2 (return_code != 0): face axes separate only for s2 > 0, so
    touching boxes intersect; edge axes use ODE's 1e-6 fudge."""
    from oracle import model as M
    b1, b2 = M.BoxGeom((1.0, 1.0, 1.0)), M.BoxGeom((0.5, 2.0, 0.25))
    w, (g1, g2) = _pair_world([b1, b2])
    assert _collide(w, g1, _T(), g2, _T(p=(0.7, 0.0, 0.0))) == 1
    assert _collide(w, g1, _T(), g2, _T(p=(0.75, 0.0, 0.0))) == 1       # touching faces: s2 == 0
    assert _collide(w, g1, _T(), g2, _T(p=(0.7500001, 0.0, 0.0))) == 0
    assert _collide(w, g1, _T(), g2, _T(p=(0.0, 1.4, 0.0))) == 1
    assert _collide(w, g1, _T(), g2, _T(p=(0.0, 0.0, 0.63))) == 0
    c, s = np.cos(np.pi / 8), np.sin(np.pi / 8)                          # 45 deg about z
    q45 = (c, 0.0, 0.0, s)
    # corner of the rotated unit box reaches 0.5*sqrt(2) along x
    assert _collide(w, g1, _T(), g1, _T(q=q45, p=(1.2, 0.0, 0.0))) == 1
    assert _collide(w, g1, _T(), g1, _T(q=q45, p=(1.22, 0.0, 0.0))) == 0
    assert _collide(w, g2, _T(q=q45), g1, _T(p=(0.3, 0.3, 0.3))) == 1    # argument order swapped


def test_sphere_closed_forms_known_answers():
    from oracle import model as M
    sp, sp2, bx = M.SphereGeom(0.1), M.SphereGeom(0.25), M.BoxGeom((0.4, 0.2, 1.0))
    w, (gs, gs2, gb) = _pair_world([sp, sp2, bx])
    assert _collide(w, gs, _T(), gs2, _T(p=(0.35, 0.0, 0.0))) == 1      # len == r1 + r2 touches
    assert _collide(w, gs, _T(), gs2, _T(p=(0.3500001, 0.0, 0.0))) == 0
    assert _collide(w, gs, _T(p=(0.0, 0.0, 0.0)), gb, _T()) == 1        # centre inside the box
    assert _collide(w, gs, _T(p=(0.2999, 0.0, 0.0)), gb, _T()) == 1
    assert _collide(w, gs, _T(p=(0.3001, 0.0, 0.0)), gb, _T()) == 0
    assert _collide(w, gb, _T(), gs, _T(p=(0.0, 0.1999, 0.0))) == 1    # box first: same test
    corner = 0.2 + 0.1 / np.sqrt(3) * 0.999
    assert _collide(w, gs, _T(p=(corner, 0.1 + 0.1 / np.sqrt(3) * 0.999, 0.5 + 0.1 / np.sqrt(3) * 0.999)), gb,
                    _T()) == 1
    assert _collide(w, gs, _T(p=(0.2 + 0.06, 0.1 + 0.06, 0.5 + 0.06)), gb, _T()) == 0


# ------------------------------------------------------------- GJK distance
def _qp_distance(VA, VB):
    """min |sum l_i a_i - sum m_j b_j| over the two simplices (SLSQP): an
    independent reference for the polytope distance."""
    from scipy.optimize import minimize
    na, nb = len(VA), len(VB)

    def f(x):
        d = x[:na] @ VA - x[na:] @ VB
        return d @ d

    def g(x):
        d = x[:na] @ VA - x[na:] @ VB
        return np.concatenate([2 * VA @ d, -2 * VB @ d])

    x0 = np.concatenate([np.full(na, 1 / na), np.full(nb, 1 / nb)])
    cons = [{"type": "eq", "fun": lambda x: x[:na].sum() - 1}, {"type": "eq", "fun": lambda x: x[na:].sum() - 1}]
    r = minimize(f, x0, jac=g, bounds=[(0, 1)] * (na + nb), constraints=cons, method="SLSQP",
                 options={"ftol": 1e-16, "maxiter": 500})
    return float(np.sqrt(max(r.fun, 0.0)))


def test_gjk_distance_matches_qp():
    import ctypes
    import oracle
    from oracle import model as M
    rng = np.random.default_rng(8)
    P = ctypes.POINTER(ctypes.c_double)
    for trial in range(12):
        A = rng.normal(size=(rng.integers(6, 20), 3)) * 0.1
        B = rng.normal(size=(rng.integers(6, 20), 3)) * 0.1
        gA, gB = M.ConvexGeom(A, []), M.ConvexGeom(B, [])
        w, (ia, ib) = _pair_world([gA, gB])
        off = rng.normal(size=3)
        off *= (0.3 + 0.3 * rng.random()) / np.linalg.norm(off)
        Ta, Tb = _T(), _T(p=tuple(off))
        d = oracle.lib().orc_distance_pair(ctypes.byref(w._w), ia, Ta.ctypes.data_as(P), ib, Tb.ctypes.data_as(P))
        ref = _qp_distance(A, B + off)
        if ref < 1e-9:
            assert d == -1.0
        else:
            assert abs(d - ref) < 1e-7, (trial, d, ref)


def test_gjk_distance_primitives_known_answers():
    import ctypes
    import oracle
    from oracle import model as M
    P = ctypes.POINTER(ctypes.c_double)
    b1, s1 = M.BoxGeom((1.0, 1.0, 1.0)), M.SphereGeom(0.25)
    w, (gb, gs) = _pair_world([b1, s1])
    dist = lambda ga, Ta, gb_, Tb: oracle.lib().orc_distance_pair(ctypes.byref(w._w), ga, Ta.ctypes.data_as(P), gb_,
                                                                   Tb.ctypes.data_as(P))
    # supports are libccd ccd_vec3_t values: single precision (float libccd)
    assert abs(dist(gb, _T(), gb, _T(p=(1.7, 0.0, 0.0))) - 0.7) < 1e-6       # face-face
    assert abs(dist(gb, _T(), gb, _T(p=(1.5, 1.5, 0.0))) - np.sqrt(0.5)) < 1e-6  # edge-edge
    assert abs(dist(gs, _T(), gb, _T(p=(1.0, 0.0, 0.0))) - 0.25) < 1e-6      # sphere (curved support)
    assert dist(gb, _T(), gb, _T(p=(0.9, 0.2, 0.1))) == -1.0                  # penetrating -> -1
    assert dist(gs, _T(), gs, _T(p=(0.3, 0.3, 0.0))) == -1.0


def test_distance_batch_semantics():
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, 300, 4)
    ds, ps, do, po = ow.distance_batch(q)
    f, _ = ow.collide_batch(q)
    # a penetrating pair (-1) makes the configuration collide; the converse
    # holds up to float libccd MPR's false hits, which reach up to
    # CCD_EPS^(1/4) = 1.86 cm: FCL's own collide() and
    # distance() disagree there the same way
    coll = (ds == -1.0) | (do == -1.0)
    assert not (coll & ~f.astype(bool)).any()
    odd = ~coll & f.astype(bool)
    assert (np.minimum(ds, do)[odd] < 0.0186).all() and odd.sum() <= 3
    assert ((ps >= 0) & (ps < ow.n_self_pairs)).all() and (po >= ow.n_self_pairs).all()
    free = ~coll
    assert (np.minimum(ds, do)[free] > 0).all()


# ------------------------------------------------------ MPR penetration (contacts)
def test_mpr_penetration_box_box_known_answer():
    """Two unit boxes overlapping by 0.1 along x: libccd's MPR penetration
    converges to depth 0.1 along +x (object 1 -> object 2), contact point in
    the overlap slab."""
    import ctypes
    import oracle
    from oracle import model as M
    P = ctypes.POINTER(ctypes.c_double)
    hull = M.ConvexGeom(np.array([[x, y, z] for x in (-.5, .5) for y in (-.5, .5) for z in (-.5, .5)]), [])
    w, (g,) = _pair_world([hull])
    depth = ctypes.c_double()
    nrm, pos = np.zeros(3), np.zeros(3)
    r = oracle.lib().orc_contact_pair(ctypes.byref(w._w), g, _T().ctypes.data_as(P), g,
                                      _T(p=(0.9, 0.02, 0.01)).ctypes.data_as(P), ctypes.byref(depth),
                                      nrm.ctypes.data_as(P), pos.ctypes.data_as(P))
    assert r == 1
    assert abs(depth.value - 0.1) < 1e-6
    np.testing.assert_allclose(nrm, [1.0, 0.0, 0.0], atol=1e-6)
    assert 0.4 - 1e-9 <= pos[0] <= 0.5 + 1e-9
    r = oracle.lib().orc_contact_pair(ctypes.byref(w._w), g, _T().ctypes.data_as(P), g,
                                      _T(p=(1.1, 0.0, 0.0)).ctypes.data_as(P), ctypes.byref(depth),
                                      nrm.ctypes.data_as(P), pos.ctypes.data_as(P))
    assert r == 0


def test_contact_batch_consistent_with_collide():
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, 200, 6)
    hit, depth, normal, pos = ow.contact_batch(q)
    _, masks = ow.collide_batch(q)
    bits = np.stack([(masks[:, p >> 5] >> (p & 31)) & 1 for p in range(len(ow.pairs))], 1)
    np.testing.assert_array_equal(hit, bits)  # same MPR discovery/refinement decides
    nz = depth[hit == 1] > 0
    # the normal is a libccd (single precision) unit vector
    np.testing.assert_allclose(np.linalg.norm(normal[hit == 1][nz], axis=1), 1.0, atol=1e-6)
    assert (depth >= 0).all()


def _pair(ow, ga, Ta, gb, Tb):
    import ctypes
    DP = ctypes.POINTER(ctypes.c_double)
    a = np.ascontiguousarray(Ta, dtype=np.float64)
    b = np.ascontiguousarray(Tb, dtype=np.float64)
    return oracle.lib().orc_collide_pair(ctypes.byref(ow._w), ga, a.ctypes.data_as(DP), gb, b.ctypes.data_as(DP))


def _rand_T(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    R = np.array(M.quat_to_mat(*q)).reshape(3, 3)
    return R, rng.uniform(-0.3, 0.3, 3)


def test_sphere_capsule_cylinder_closed_forms_match_geometry():
    """FCL's sphereCapsuleIntersect / sphereCylinderIntersect restatements
    against the plain geometry (sphere centre to axis segment / to the solid
    cylinder), away from touching contact, both argument orders."""
    cap, cyl, ball = M.CapsuleGeom(0.05, 0.3), M.CylinderGeom(0.06, 0.25), M.SphereGeom(0.08)
    ow = oracle.OracleWorld(Wd.panda_articulation(),
                            scene=[("cap", cap, M.IDENT), ("cyl", cyl, M.IDENT), ("ball", ball, M.IDENT)])
    gi = {id(g): k for k, g in enumerate(ow.geoms)}
    rng = np.random.default_rng(3)
    checked = {"cap": [0, 0], "cyl": [0, 0]}
    for _ in range(4000):
        Rs, ps = _rand_T(rng)
        Ro, po = _rand_T(rng)
        Ts = np.concatenate([Rs.reshape(-1), ps])
        To = np.concatenate([Ro.reshape(-1), po])
        c = Ro.T @ (ps - po)  # sphere centre in the other shape's frame
        for name, g in (("cap", cap), ("cyl", cyl)):
            if name == "cap":
                z = np.clip(c[2], -g.lz / 2, g.lz / 2)
                d = np.linalg.norm(c - [0, 0, z]) - g.radius - ball.radius
            else:
                rxy = np.hypot(c[0], c[1])
                dz = max(abs(c[2]) - g.lz / 2, 0.0)
                dr = max(rxy - g.radius, 0.0)
                d = np.hypot(dz, dr) - ball.radius
            if abs(d) < 1e-9:
                continue
            want = int(d <= 0)
            assert _pair(ow, gi[id(ball)], Ts, gi[id(g)], To) == want
            assert _pair(ow, gi[id(g)], To, gi[id(ball)], Ts) == want
            checked[name][want] += 1
    assert min(min(v) for v in checked.values()) > 100  # both outcomes exercised


# ------------------------------------------- closed-form contacts (enable_contact)
def _contact(w, ga, Ta, gb, Tb):
    import ctypes
    import oracle
    P = ctypes.POINTER(ctypes.c_double)
    depth = ctypes.c_double()
    nrm, pos = np.zeros(3), np.zeros(3)
    r = oracle.lib().orc_contact_pair(ctypes.byref(w._w), ga, Ta.ctypes.data_as(P), gb, Tb.ctypes.data_as(P),
                                      ctypes.byref(depth), nrm.ctypes.data_as(P), pos.ctypes.data_as(P))
    return r, depth.value, nrm, pos


def test_sphere_contacts_known_answers():
    """FCL 0.7.0 sphereSphereIntersect / sphereBoxIntersect contacts (plain
    geometry): normal from object 1 into object 2, depth, and the contact
    point (sphere-sphere: on the centre line at r1/(r1+r2); sphere-box: half
    way between the sphere's deepest point and the box surface)."""
    from oracle import model as M
    w, (s5, s3, box) = _pair_world([M.SphereGeom(0.5), M.SphereGeom(0.3), M.BoxGeom((1.0, 1.0, 1.0))])
    r, d, n, p = _contact(w, s5, _T(), s3, _T(p=(0.7, 0.0, 0.0)))
    assert r == 1 and abs(d - 0.1) < 1e-12
    np.testing.assert_allclose(n, [1, 0, 0], atol=1e-15)
    np.testing.assert_allclose(p, [0.4375, 0, 0], atol=1e-15)
    assert _contact(w, s5, _T(), s3, _T(p=(0.81, 0.0, 0.0)))[0] == 0
    # sphere centre outside the box: nearest point (0.5, 0, 0), distance 0.4
    r, d, n, p = _contact(w, s5, _T(p=(0.9, 0.0, 0.0)), box, _T())
    assert r == 1 and abs(d - 0.1) < 1e-12
    np.testing.assert_allclose(n, [-1, 0, 0], atol=1e-15)
    np.testing.assert_allclose(p, [0.45, 0, 0], atol=1e-12)
    # box first: flipNormal
    r, d2, n2, p2 = _contact(w, box, _T(), s5, _T(p=(0.9, 0.0, 0.0)))
    assert r == 1 and d2 == d
    np.testing.assert_array_equal(n2, -n)
    np.testing.assert_array_equal(p2, p)
    # centre inside the box: the nearest face (+x, 0.2 away), depth 0.2 + r
    r, d, n, p = _contact(w, s3, _T(p=(0.3, 0.1, 0.0)), box, _T())
    assert r == 1 and abs(d - 0.5) < 1e-12
    np.testing.assert_allclose(n, [-1, 0, 0], atol=1e-15)
    np.testing.assert_allclose(p, [0.3 - (0.3 - 0.25), 0.1, 0.0], atol=1e-12)
    # rotated box: the normal and point come back to the world frame
    q = (np.cos(0.3), 0.0, 0.0, np.sin(0.3))
    T = _T(q=q, p=(0.1, 0.2, 0.3))
    R = T[:9].reshape(3, 3)
    Ts = _T(p=tuple(R @ np.array([0.9, 0.0, 0.0]) + T[9:]))
    r, d, n, p = _contact(w, s5, Ts, box, T)
    assert r == 1 and abs(d - 0.1) < 1e-12
    np.testing.assert_allclose(n, R @ [-1, 0, 0], atol=1e-12)
    np.testing.assert_allclose(p, R @ [0.45, 0, 0] + T[9:], atol=1e-12)


def test_box_box_contact_known_answers():
    """FCL 0.7.0 boxBox2 with contacts (ODE dBoxBox): face-face contact points
    on the incident face, normal from box 1 to box 2, and FCL's stored
    penetration_depth = -(depth of the point) (the sign boxBox2 emits; with
    one requested contact ShapeShapeCollide keeps the largest value)."""
    from oracle import model as M
    w, (b1, b2) = _pair_world([M.BoxGeom((1.0, 1.0, 1.0)), M.BoxGeom((1.0, 0.5, 0.5))])
    r, d, n, p = _contact(w, b1, _T(), b1, _T(p=(0.9, 0.02, 0.01)))
    assert r == 1 and abs(d + 0.1) < 1e-12
    np.testing.assert_allclose(n, [1, 0, 0], atol=1e-15)
    assert abs(p[0] - 0.4) < 1e-12 and abs(p[1]) <= 0.5 + 1e-12 and abs(p[2]) <= 0.5 + 1e-12
    # box 2 below box 1 along z: normal -z, reference face is box 1's
    r, d, n, p = _contact(w, b1, _T(), b2, _T(p=(0.1, 0.0, -0.7)))
    assert r == 1 and abs(d + 0.05) < 1e-12
    np.testing.assert_allclose(n, [0, 0, -1], atol=1e-15)
    assert abs(p[2] + 0.45) < 1e-12
    # tilted incident box: the shallowest of the clipped points is kept
    q = (np.cos(0.1), np.sin(0.1), 0.0, 0.0)
    r, d, n, p = _contact(w, b1, _T(), b2, _T(q=q, p=(0.0, 0.0, 0.7)))
    assert r == 1 and n[2] > 0.99 and -0.2 < d < 0.0
    # edge-edge: box 2 turned 45 degrees about z and x, just touching an edge
    s = np.sqrt(0.5)
    q = (np.cos(np.pi / 8) * np.cos(np.pi / 8), np.sin(np.pi / 8) * np.cos(np.pi / 8),
         np.cos(np.pi / 8) * np.sin(np.pi / 8), -np.sin(np.pi / 8) * np.sin(np.pi / 8))
    assert _contact(w, b1, _T(), b1, _T(q=q, p=(1.4, 0.0, 0.0)))[0] == 0
    r, d, n, p = _contact(w, b1, _T(), b1, _T(q=q, p=(1.05, 0.3, 0.2)))
    assert r == 1 and d <= 0.0 and n[0] > 0.0 and s > 0
    # separated
    assert _contact(w, b1, _T(), b1, _T(p=(1.01, 0.0, 0.0)))[0] == 0


def test_closed_form_contact_batch_consistent_with_collide():
    """collision_avoidance.py:87-90's attached box in the cfg3 box scene:
    the oracle's contact pass reports exactly the pairs collide() reports
    (box-box through boxBox2's contact path, box-convex through MPR), with
    unit normals and boxBox2's non-positive stored depth."""
    base = Wd.oracle_world(3)
    pose = [0.0, 0.0, 0.14, 1.0, 0.0, 0.0, 0.0]
    T = (M.quat_to_mat(*pose[3:]), pose[:3])
    o2 = oracle.OracleWorld(base.art, scene=base.scene, attached=[("held", 8, M.BoxGeom((0.04, 0.04, 0.12)), T)],
                            allowed=[("panda_hand", "held"), ("panda_link0", "table")])
    q = Wd.sample_q(base.art, 3000, 18)
    hit, depth, normal, pos = o2.contact_batch(q)
    _, masks = o2.collide_batch(q)
    P = len(o2.pairs)
    bits = np.stack([(masks[:, p >> 5] >> (p & 31)) & 1 for p in range(P)], 1)
    np.testing.assert_array_equal(hit, bits)
    bb = [k for k, (a, b) in enumerate(o2.pair_names()) if a == "held"]  # held x scene boxes: boxBox2
    h = hit[:, bb].astype(bool)
    assert h.sum() > 0
    np.testing.assert_allclose(np.linalg.norm(normal[:, bb][h], axis=1), 1.0, atol=1e-12)
    assert (depth[:, bb][h] <= 0).all()


def test_sphere_capsule_cylinder_contacts_known_answers():
    """FCL 0.7.0 sphereCapsuleIntersect / sphereCylinderIntersect contacts
    (plain geometry; parity unpinned): normal from the sphere into the other
    shape, the capsule's point on the sphere side of the axis point, the
    cylinder's half way between the sphere's deepest point and the surface;
    the other argument order flips the normal."""
    w, (sph, cap, cyl, small) = _pair_world([M.SphereGeom(0.2), M.CapsuleGeom(0.1, 0.4), M.CylinderGeom(0.1, 0.4),
                                             M.SphereGeom(0.05)])
    r, d, n, p = _contact(w, sph, _T(p=(0.25, 0.0, 0.1)), cap, _T())
    assert r == 1 and abs(d - 0.05) < 1e-12
    np.testing.assert_allclose(n, [-1, 0, 0], atol=1e-15)
    np.testing.assert_allclose(p, [0.05, 0, 0.1], atol=1e-12)
    r, d2, n2, p2 = _contact(w, cap, _T(), sph, _T(p=(0.25, 0.0, 0.1)))
    assert r == 1 and d2 == d
    np.testing.assert_array_equal(n2, -n)
    np.testing.assert_array_equal(p2, p)
    assert _contact(w, sph, _T(p=(0.31, 0.0, 0.1)), cap, _T())[0] == 0
    # beyond the capsule's end cap: the segment end is the nearest axis point
    r, d, n, p = _contact(w, sph, _T(p=(0.0, 0.0, 0.45)), cap, _T())
    assert r == 1 and abs(d - 0.05) < 1e-12
    np.testing.assert_allclose(n, [0, 0, -1], atol=1e-15)
    r, d, n, p = _contact(w, sph, _T(p=(0.25, 0.0, 0.1)), cyl, _T())
    assert r == 1 and abs(d - 0.05) < 1e-12
    np.testing.assert_allclose(n, [-1, 0, 0], atol=1e-15)
    np.testing.assert_allclose(p, [0.075, 0, 0.1], atol=1e-12)
    # centre inside the cylinder, nearer the top cap than the barrel
    r, d, n, p = _contact(w, small, _T(p=(0.02, 0.0, 0.15)), cyl, _T())
    assert r == 1 and abs(d - 0.1) < 1e-12
    np.testing.assert_allclose(n, [0, 0, -1], atol=1e-15)
    np.testing.assert_allclose(p, [0.02, 0, 0.15], atol=1e-12)
    # nearer the barrel
    r, d, n, p = _contact(w, small, _T(p=(0.07, 0.0, 0.0)), cyl, _T())
    assert r == 1 and abs(d - 0.08) < 1e-12
    np.testing.assert_allclose(n, [-1, 0, 0], atol=1e-15)
    r, d2, n2, _ = _contact(w, cyl, _T(), small, _T(p=(0.07, 0.0, 0.0)))
    assert r == 1 and d2 == d
    np.testing.assert_array_equal(n2, -n)


@pytest.mark.parametrize("cloud", ["blue"])
def test_point_cloud_contact_batch_consistent_with_collide(cloud):
    """The oracle's contact pass on a point-cloud world reports exactly the
    pairs collide() reports: the first intersecting leaf (contact) exists
    iff some leaf intersects (boolean), and its normal is a unit vector."""
    o = Wd.oracle_cloud_world(cloud)
    q = Wd.sample_q(o.art, 600, 8)
    hit, depth, normal, pos = o.contact_batch(q)
    _, masks = o.collide_batch(q)
    P = len(o.pairs)
    bits = np.stack([(masks[:, p >> 5] >> (p & 31)) & 1 for p in range(P)], 1)
    np.testing.assert_array_equal(hit, bits)
    pc = [k for k, (a, b) in enumerate(o.pair_names()) if b == "scene_pcd"]
    h = hit[:, pc].astype(bool)
    assert h.sum() > 0
    nz = depth[:, pc][h] != 0
    np.testing.assert_allclose(np.linalg.norm(normal[:, pc][h][nz], axis=1), 1.0, atol=1e-6)
