"""fcl.Cone, fcl.Ellipsoid and fcl.TriangleP (python/pybind_fcl.hpp:95-98,
137-141, 168-175) as world geometry: FCL 0.7.0's GJKSolver_libccd has no
closed form for any of them in a shape pair, so every pair with one is libccd
MPR over supportCone / supportEllipsoid / supportTriangle (collision,
contacts: MPR penetration; distance: libccd GJK) and, with GST_INDEP,
details::GJK over getSupport's Cone / Ellipsoid / Triangle cases.  Restated in the oracle
(oracle/collide_oracle.c support_cone / support_ellipsoid,
oracle/fcl_gjk_indep.h gjk_shape_support) and on the device
(mpg_kernels.hip support_local, mpg_gjk_indep.h shape_support).

FCL is not under /root/reference, so the restatement is pinned by geometry
(known answers against the exact surfaces, beyond libccd's 1.86 cm false-hit
reach for MPR, at GJK's tolerance band for GST_INDEP, distances against the
analytic gap) -- parity with real FCL is unpinned below that; the GPU equals
the oracle bit for bit."""
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


def _dist(w, ga, Ta, gb, Tb):
    import oracle
    return float(oracle.lib().orc_distance_pair(ctypes.byref(w._w), ga, np.ascontiguousarray(Ta).ctypes.data_as(P),
                                                gb, np.ascontiguousarray(Tb).ctypes.data_as(P)))


def _shapes():
    from oracle import model as M
    return [M.EllipsoidGeom((0.3, 0.2, 0.1)), M.ConeGeom(0.2, 0.6), M.BoxGeom((1.0, 1.0, 1.0)), M.SphereGeom(0.05),
            M.CapsuleGeom(0.05, 0.3)]


def _slant_point(R, h, gap, rs):
    """Centre of a sphere of radius rs whose surface is `gap` off the cone's
    slanted side at mid-height (cone radius R, half height h, apex at +h)."""
    n = np.array([2 * h, 0.0, R]) / np.hypot(2 * h, R)
    return np.array([R / 2, 0.0, 0.0]) + n * (rs + gap)


_SLANT_TH = np.arctan2(-0.2, 0.6)  # the slant's direction (-R, 0, 2h) as a rotation of z about y
_SLANT_Q = (float(np.cos(_SLANT_TH / 2)), 0.0, float(np.sin(_SLANT_TH / 2)), 0.0)


def _cases(el, co, bx, sp, cp, gap_no, gap_yes):
    """(ga, Ta, gb, Tb, expected) at separation gap_no (False) / overlap
    gap_yes (True) along each shape's extent."""
    out = []
    for gap, want in ((gap_no, False), (-gap_yes, True)):
        # ellipsoid semi-axes 0.3 / 0.2 / 0.1 against the unit box's faces
        out += [(el, _T(), bx, _T(p=(0.8 + gap, 0.0, 0.0)), want),
                (el, _T(), bx, _T(p=(0.0, -(0.7 + gap), 0.0)), want),
                (el, _T(), bx, _T(p=(0.0, 0.0, 0.6 + gap)), want),
                # rotated ellipsoid: its 0.3 axis along y
                (el, _T(q=(np.cos(np.pi / 4), 0.0, 0.0, np.sin(np.pi / 4))), bx, _T(p=(0.0, 0.8 + gap, 0.0)), want),
                # cone apex (+0.3), base (-0.3), rim (0.2) and slant against spheres / boxes
                (co, _T(), sp, _T(p=(0.0, 0.0, 0.35 + gap)), want),
                (co, _T(), bx, _T(p=(0.0, 0.0, -(0.8 + gap))), want),
                (co, _T(), bx, _T(p=(0.7 + gap, 0.0, -0.5)), want),
                (co, _T(), sp, _T(p=tuple(_slant_point(0.2, 0.3, gap, 0.05))), want),
                # a capsule lying along the slant line (its axis rotated about y onto it)
                (co, _T(), cp, _T(q=_SLANT_Q, p=tuple(_slant_point(0.2, 0.3, gap, 0.05))), want),
                # cone against ellipsoid: apex under the ellipsoid's 0.1 axis
                (co, _T(), el, _T(p=(0.0, 0.0, 0.4 + gap)), want)]
    return out


def test_cone_ellipsoid_mpr_known_answers():
    """libccd MPR (GST_LIBCCD): no collision beyond its false-hit reach
    (3 cm), collision at 1 cm overlap, both argument orders."""
    w, (el, co, bx, sp, cp) = _pair_world(_shapes())
    for k, (ga, Ta, gb, Tb, want) in enumerate(_cases(el, co, bx, sp, cp, 0.03, 0.01)):
        assert _hit(w, ga, Ta, gb, Tb) == want, k
        assert _hit(w, gb, Tb, ga, Ta) == want, ("swapped", k)


def test_cone_ellipsoid_gjk_indep_known_answers():
    """FCL's own GJK (GST_INDEP) in double: its tolerance band, 1 mm."""
    w, (el, co, bx, sp, cp) = _pair_world(_shapes())
    w._w.gjk_solver = 1
    for k, (ga, Ta, gb, Tb, want) in enumerate(_cases(el, co, bx, sp, cp, 1e-3, 1e-3)):
        assert _hit(w, ga, Ta, gb, Tb) == want, k
        assert _hit(w, gb, Tb, ga, Ta) == want, ("swapped", k)


def test_cone_ellipsoid_distance_known_answers():
    """libccd GJK distance (float ccd_real) against the analytic gap."""
    w, (el, co, bx, sp, cp) = _pair_world(_shapes())
    for gap in (0.01, 0.05, 0.2):
        for ga, Ta, gb, Tb, _ in _cases(el, co, bx, sp, cp, gap, 0.0)[:10]:
            assert abs(_dist(w, ga, Ta, gb, Tb) - gap) < 2e-4 * (1 + gap), gap
    assert _dist(w, el, _T(), bx, _T(p=(0.79, 0.0, 0.0))) == -1.0
    assert _dist(w, co, _T(), sp, _T(p=(0.0, 0.0, 0.34))) == -1.0


def test_cone_ellipsoid_supports_are_extreme():
    """The support points the oracle's MPR uses lie on the surfaces: an
    ellipsoid with equal radii is a sphere (collision set identical to a
    sphere's MPR against a hull), and a degenerate cone direction (straight
    down) takes the base centre."""
    from oracle import model as M
    rng = np.random.default_rng(5)
    hull = M.ConvexGeom(rng.normal(size=(30, 3)) * 0.1, [])
    w, (el, sp, hv) = _pair_world([M.EllipsoidGeom((0.1, 0.1, 0.1)), M.SphereGeom(0.1), hull])
    agree = 0
    for _ in range(300):
        off = rng.normal(size=3)
        off *= rng.uniform(0.1, 0.35) / np.linalg.norm(off)
        Tb = _T(p=tuple(off))
        agree += _hit(w, el, _T(), hv, Tb) == _hit(w, sp, _T(), hv, Tb)
    assert agree >= 297  # float rounding of the two supports may flip a grazing case
    w2, (co, bx2) = _pair_world([M.ConeGeom(0.2, 0.6), M.BoxGeom((1.0, 1.0, 1.0))])
    assert _hit(w2, co, _T(), bx2, _T(p=(0.0, 0.0, -0.79)))
    assert not _hit(w2, co, _T(), bx2, _T(p=(0.0, 0.0, -0.84)))


def _tri_cases(tr, bx, sp, gap_no, gap_yes):
    """TriangleP (0,0,0), (1,0,0), (0,1,0) against a box above its face, a
    sphere off its hypotenuse and a box beside its corner."""
    out = []
    h = np.array([0.5, 0.5, 0.0]) + np.array([1.0, 1.0, 0.0]) / np.sqrt(2) * 0.05  # sphere r 0.05 off the edge
    for gap, want in ((gap_no, False), (-gap_yes, True)):
        out += [(tr, _T(), bx, _T(p=(0.2, 0.2, 0.5 + gap)), want),
                (tr, _T(), sp, _T(p=tuple(h + np.array([1.0, 1.0, 0.0]) / np.sqrt(2) * gap)), want),
                (tr, _T(), bx, _T(p=(-0.5 - gap, 0.3, 0.0)), want),
                # rotated triangle (about x by 90 deg: it stands in the xz plane)
                (tr, _T(q=(np.cos(np.pi / 4), np.sin(np.pi / 4), 0.0, 0.0)), bx, _T(p=(0.2, -0.5 - gap, 0.2)), want)]
    return out


def test_triangle_p_known_answers():
    """TriangleP: MPR beyond the false-hit reach / at 1 cm overlap, GJK
    (GST_INDEP) at 1 mm, libccd GJK distance against the gap."""
    from oracle import model as M
    w, (tr, bx, sp) = _pair_world([M.TrianglePGeom((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0)),
                                   M.BoxGeom((1.0, 1.0, 1.0)), M.SphereGeom(0.05)])
    for k, (ga, Ta, gb, Tb, want) in enumerate(_tri_cases(tr, bx, sp, 0.03, 0.01)):
        assert _hit(w, ga, Ta, gb, Tb) == want, k
        assert _hit(w, gb, Tb, ga, Ta) == want, ("swapped", k)
    for gap in (0.01, 0.1):
        for ga, Ta, gb, Tb, _ in _tri_cases(tr, bx, sp, gap, 0.0)[:4]:
            assert abs(_dist(w, ga, Ta, gb, Tb) - gap) < 2e-4 * (1 + gap), gap
    w._w.gjk_solver = 1
    for k, (ga, Ta, gb, Tb, want) in enumerate(_tri_cases(tr, bx, sp, 1e-3, 1e-3)):
        assert _hit(w, ga, Ta, gb, Tb) == want, ("indep", k)
        assert _hit(w, gb, Tb, ga, Ta) == want, ("indep swapped", k)


def test_host_types():
    """fcl.Cone / fcl.Ellipsoid exist with the reference's constructors and
    fields, and a world with them builds its descriptor (no device call)."""
    from mplib_amd import pymp
    c = pymp.fcl.Cone(0.2, 0.6)
    assert (c.radius, c.lz) == (0.2, 0.6)
    e = pymp.fcl.Ellipsoid(0.3, 0.2, 0.1)
    np.testing.assert_array_equal(e.radii, [0.3, 0.2, 0.1])
    e2 = pymp.fcl.Ellipsoid(radii=[0.1, 0.2, 0.3])
    np.testing.assert_array_equal(e2.radii, [0.1, 0.2, 0.3])
    assert pymp.fcl.CollisionObject(e, [0, 0, 1], [1, 0, 0, 0]).get_collision_geometry().kind == "Ellipsoid"
    t = pymp.fcl.TriangleP([0, 0, 0], [1, 0, 0], [0, 1, 0])
    np.testing.assert_array_equal(t.b, [1, 0, 0])
    # Halfspace / Plane: unit normal, signed distance; no device evaluation
    h = pymp.fcl.Halfspace([0.0, 0.0, 2.0], 1.0)
    np.testing.assert_array_equal(h.n, [0, 0, 1])
    assert h.d == 0.5 and h.signed_distance([0, 0, 2.0]) == 1.5 and h.distance([0, 0, -1.0]) == 1.5
    pl = pymp.fcl.Plane(1.0, 0.0, 0.0, -2.0)
    assert pl.signed_distance([0.0, 5.0, 0.0]) == 2.0
    box = pymp.fcl.CollisionObject(pymp.fcl.Box(1.0, 1.0, 1.0), [0, 0, 0], [1, 0, 0, 0])
    for g in (h, pl):
        with pytest.raises(NotImplementedError, match="not supported by the device"):
            pymp.fcl.collide(pymp.fcl.CollisionObject(g, [0, 0, 0], [1, 0, 0, 0]), box)


# ------------------------------------------------------------------ GPU
def _mixed_world():
    """cfg3 (Panda + 10 boxes) plus three ellipsoids, three cones and two
    TriangleP plates in the workspace, a cone held by the hand and an
    ellipsoid on link 6."""
    import oracle
    from oracle import model as M
    from mplib_amd import pymp, scenes
    from test_gpu_parity import _oracle_T
    w, art = scenes.world(3)
    rng = np.random.default_rng(808)
    extra = []
    for k in range(6):
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        if k < 3:
            radii = tuple(float(x) for x in rng.uniform(0.03, 0.12, 3))
            g, og, name = pymp.fcl.Ellipsoid(*radii), M.EllipsoidGeom(radii), f"ell{k}"
        else:
            r, lz = float(rng.uniform(0.04, 0.1)), float(rng.uniform(0.1, 0.3))
            g, og, name = pymp.fcl.Cone(r, lz), M.ConeGeom(r, lz), f"cone{k}"
        w.add_normal_object(name, pymp.fcl.CollisionObject(g, list(c), list(q)))
        extra.append((name, og, _oracle_T(list(c) + list(q))))
    for k in range(6, 8):  # two TriangleP plates
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        P = [tuple(float(x) for x in rng.uniform(-0.12, 0.12, 3)) for _ in range(3)]
        g, og, name = pymp.fcl.TriangleP(*[list(p) for p in P]), M.TrianglePGeom(*P), f"tri{k}"
        w.add_normal_object(name, pymp.fcl.CollisionObject(g, list(c), list(q)))
        extra.append((name, og, _oracle_T(list(c) + list(q))))
    p_tip = [0.0, 0.0, 0.15, 1.0, 0.0, 0.0, 0.0]
    p_egg = [0.0, 0.06, 0.0, 0.7071067811865476, 0.7071067811865476, 0.0, 0.0]
    w.attach_object("tip", pymp.fcl.Cone(0.03, 0.12), "panda", 8, p_tip, ["panda_hand"])
    w.attach_object("egg", pymp.fcl.Ellipsoid(0.03, 0.05, 0.08), "panda", 6, p_egg, ["panda_link6", "panda_link7"])
    base = Wd.oracle_world(3)
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + extra,
                            attached=[("tip", 8, M.ConeGeom(0.03, 0.12), _oracle_T(p_tip)),
                                      ("egg", 6, M.EllipsoidGeom((0.03, 0.05, 0.08)), _oracle_T(p_egg))],
                            allowed=[("panda_hand", "tip"), ("panda_link6", "egg"), ("panda_link7", "egg"),
                                     ("panda_link0", "table")])
    return w, o2, base


def _bits(M_, P_):
    return np.stack([(M_[:, p >> 5] >> (p & 31)) & 1 for p in P_], 1)


@pytest.mark.gpu
def test_cone_ellipsoid_world_matches_oracle():
    """Every flag and pair bit equal to the oracle's on 30000 configurations,
    through the throughput pipeline and the latency path; the new pairs are
    exercised (cone / ellipsoid against links, boxes and each other)."""
    w, o2, base = _mixed_world()
    order = {pn: k for k, pn in enumerate(o2.pair_names())}
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    assert sorted(names) == sorted(o2.pair_names())
    perm = [order[n] for n in names]
    q = Wd.sample_q(base.art, 30000, 29)
    fo, mo = o2.collide_batch(q, nthreads=8)
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(_bits(m, range(len(perm))), _bits(mo, perm))
    hit = _bits(mo, perm)
    new = [k for k, (a, b) in enumerate(names) if a in ("tip", "egg") or b[:3] in ("ell", "con", "tri")]
    assert int(hit[:, new].sum()) > 50
    for i in range(0, 300, 3):  # latency server
        f3, m3 = w.collide_batch(q[i:i + 3])
        np.testing.assert_array_equal(f3, fo[i:i + 3])


@pytest.mark.gpu
def test_cone_ellipsoid_contacts_and_distance_match_oracle():
    """enable_contact=True (MPR penetration over the new supports) within
    1e-9 of the oracle; batched distance (libccd GJK) equal to the oracle's,
    the argmin pair by name."""
    from test_gpu_parity import _check_scalar_contacts
    w, o2, base = _mixed_world()
    q = Wd.sample_q(base.art, 20000, 31)
    _, mo = o2.collide_batch(q, nthreads=8)
    names = o2.pair_names()
    new = [k for k, (a, b) in enumerate(names) if a in ("tip", "egg") or b[:3] in ("ell", "con", "tri")]
    sel = np.nonzero(_bits(mo, new).any(1))[0]
    assert len(sel) >= 20
    hit = _check_scalar_contacts(w, o2, np.concatenate([q[sel[:120]], q[:20]]))
    assert hit[:, new].sum() >= 20
    qd = q[:3000]
    ds, ps, do, po = w.distance_batch(qd)
    rs, rps, ro, rpo = o2.distance_batch(qd)
    wn = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
    assert [wn[p] for p in po] == [names[p] for p in rpo]
    assert [wn[p] for p in ps] == [names[p] for p in rps]
    assert any(names[p][1][:3] in ("ell", "con", "tri") or names[p][0] in ("tip", "egg") for p in rpo)


@pytest.mark.gpu
def test_cone_ellipsoid_gjk_indep_world_matches_oracle():
    """GST_INDEP on the mixed world: FCL's own GJK over the Cone / Ellipsoid
    getSupport cases, device equal to the oracle bit for bit."""
    import oracle
    from mplib_amd import _capi as C
    from mplib_amd.batch import DeviceWorld
    _, o2, base = _mixed_world()
    ind = oracle.OracleWorld(o2.art, scene=o2.scene, attached=o2.attached, allowed=list(o2.allowed),
                             gjk_solver="indep")
    dw = DeviceWorld(Wd.desc_arrays(ind), gjk_solver=C.GJK_INDEP)
    q = Wd.sample_q(base.art, 4096, 37)
    fo, mo = ind.collide_batch(q, nthreads=8)
    f, m = dw.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    f2, m2 = dw.collide_batch(q[:512])
    np.testing.assert_array_equal(f2, fo[:512])
    np.testing.assert_array_equal(m2, mo[:512])
    dw.close()
