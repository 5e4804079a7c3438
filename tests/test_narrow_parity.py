"""Narrow-phase parity without forward kinematics: the device's fcl::collide
of two posed geometries (mpg_debug_collide_pairs) against the oracle's
(oracle/collide_oracle.c orc_collide_pair) on poses concentrated at the
contact boundary, where single-precision libccd (the reference's build, see
DESIGN.md "Oracle variants") decides by its own rounding.  Every bit must
agree: the device restates float libccd operation by operation.

Poses: for each sample a random relative rotation and approach direction;
the translation along it at which the pair starts touching is bracketed by
bisection with the oracle, then samples are spread within +-2e-6 m of it."""
import ctypes

import numpy as np
import pytest

import oracle
from oracle import model as M
import worlds as Wd

_DP = ctypes.POINTER(ctypes.c_double)


def _T(R, p):
    return np.concatenate([np.asarray(R, float).reshape(9), np.asarray(p, float)])


def _rand_R(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    return np.array(M.quat_to_mat(*q)).reshape(3, 3)


def orc_pair(ow, ga, Ta, gb, Tb) -> int:
    a = np.ascontiguousarray(Ta, dtype=np.float64)
    b = np.ascontiguousarray(Tb, dtype=np.float64)
    return oracle.lib().orc_collide_pair(ctypes.byref(ow._w), ga, a.ctypes.data_as(_DP), gb, b.ctypes.data_as(_DP))


def _local_centre(ow, g):
    geom = ow.geoms[g]
    return np.asarray(geom.interior, float) if isinstance(geom, M.ConvexGeom) else np.zeros(3)


def boundary_poses(ow, ga, gb, n, seed, centre_a=(0.0, 0.0, 0.0), reach=0.6, spread=2e-6, per=8):
    """(Ta, Tb) rows near the contact boundary of geometry ga (random
    rotation, its interior point at centre_a) and gb (random rotation, its
    interior point moved out from centre_a along a random direction)."""
    rng = np.random.default_rng(seed)
    ca, cb = _local_centre(ow, ga), _local_centre(ow, gb)
    TA, TB = [], []
    tries = 0
    while len(TA) < n:
        tries += 1
        assert tries < 50 * n, "no boundary found"
        Ra, Rb = _rand_R(rng), _rand_R(rng)
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        Ta = _T(Ra, np.subtract(centre_a, Ra @ ca))
        pb = np.subtract(centre_a, Rb @ cb)
        lo, hi = 0.0, reach  # hit at lo, miss at hi
        if not orc_pair(ow, ga, Ta, gb, _T(Rb, pb + lo * u)):
            continue
        if orc_pair(ow, ga, Ta, gb, _T(Rb, pb + hi * u)):
            continue
        for _ in range(48):
            mid = 0.5 * (lo + hi)
            if orc_pair(ow, ga, Ta, gb, _T(Rb, pb + mid * u)):
                lo = mid
            else:
                hi = mid
        for t in lo + rng.uniform(-spread, spread, per):
            TA.append(Ta)
            TB.append(_T(Rb, pb + t * u))
    return np.array(TA[:n]), np.array(TB[:n])


def _device_world(ow):
    from mplib_amd.batch import DeviceWorld
    return DeviceWorld(Wd.desc_arrays(ow))


def _geom(ow, g):
    return next(i for i, gg in enumerate(ow.geoms) if gg is g)


def _compare(ow, dw, ga, gb, TA, TB):
    dev = dw.debug_collide_pairs(ga, gb, TA, TB)
    ref = np.array([orc_pair(ow, ga, a, gb, b) for a, b in zip(TA, TB)], np.uint8)
    return dev, ref


@pytest.mark.gpu
@pytest.mark.parametrize("la,lb", [("panda_link3", "panda_link5"), ("panda_hand", "panda_link0"),
                                   ("panda_leftfinger", "panda_link7")])
def test_mpr_convex_convex_boundary_bit_exact(la, lb):
    ow = Wd.oracle_world(2)
    objs = {o.link: o for o in ow.art.objects}
    ga, gb = _geom(ow, objs[la].geom), _geom(ow, objs[lb].geom)
    TA, TB = boundary_poses(ow, ga, gb, 4000, seed=sum(map(ord, la + lb)))
    dw = _device_world(ow)
    dev, ref = _compare(ow, dw, ga, gb, TA, TB)
    assert 0.2 < ref.mean() < 0.8  # the samples straddle the boundary
    np.testing.assert_array_equal(dev, ref)


@pytest.mark.gpu
def test_mpr_convex_box_boundary_bit_exact():
    ow = Wd.oracle_world(3)
    objs = {o.link: o for o in ow.art.objects}
    boxes = [s for s in ow.scene if isinstance(s[1], M.BoxGeom)]
    dw = _device_world(ow)
    for k, link in enumerate(["panda_link5", "panda_hand", "panda_rightfinger"]):
        ga, gb = _geom(ow, objs[link].geom), _geom(ow, boxes[k + 1][1])
        TA, TB = boundary_poses(ow, ga, gb, 3000, seed=50 + k)
        dev, ref = _compare(ow, dw, ga, gb, TA, TB)
        assert 0.2 < ref.mean() < 0.8
        np.testing.assert_array_equal(dev, ref, err_msg=link)


@pytest.mark.gpu
def test_octree_leaf_boundary_bit_exact():
    """(finger, floor octree) at the boundary of single 1 mm leaves: box-first
    float MPR on the leaf boxes behind FCL's obbDisjoint gate."""
    ow = Wd.oracle_cloud_world("floor")
    objs = {o.link: o for o in ow.art.objects}
    go = next(i for i, g in enumerate(ow.geoms) if isinstance(g, M.OcTreeGeom))
    oc = ow.geoms[go]
    dw = _device_world(ow)
    rng = np.random.default_rng(7)
    leaves = oc.leaves[rng.choice(len(oc.leaves), 60, replace=False)]
    TO = _T(np.eye(3), (0.0, 0.0, 0.0))
    for link in ["panda_leftfinger", "panda_link7"]:
        gs = _geom(ow, objs[link].geom)
        TA, TB = [], []
        for L in leaves:
            c = 0.5 * (L[:3] + L[3:])
            # approach the leaf centre from a random direction: the shape
            # starts at the leaf and moves out until it stops touching
            for _ in range(4):
                R = _rand_R(rng)
                u = rng.normal(size=3)
                u /= np.linalg.norm(u)
                lo, hi = 0.0, 0.5
                if not orc_pair(ow, gs, _T(R, c), go, TO) or orc_pair(ow, gs, _T(R, c + hi * u), go, TO):
                    continue
                for _ in range(44):
                    mid = 0.5 * (lo + hi)
                    if orc_pair(ow, gs, _T(R, c + mid * u), go, TO):
                        lo = mid
                    else:
                        hi = mid
                for t in lo + rng.uniform(-2e-6, 2e-6, 6):
                    TA.append(_T(R, c + t * u))
                    TB.append(TO)
        TA, TB = np.array(TA), np.array(TB)
        dev, ref = _compare(ow, dw, gs, go, TA, TB)
        assert 0.2 < ref.mean() < 0.8
        np.testing.assert_array_equal(dev, ref, err_msg=link)


@pytest.mark.gpu
@pytest.mark.parametrize("side", [1e-3, 0.05])
def test_mpr_box_first_boundary_bit_exact(side):
    """Box as fcl::collide's first object (the octree leaf order), small and
    medium boxes against a finger and a link hull."""
    box = M.BoxGeom((side, side, side))
    ow = oracle.OracleWorld(Wd.panda_articulation(), scene=[("b", box, M.IDENT)])
    objs = {o.link: o for o in ow.art.objects}
    dw = _device_world(ow)
    gb = _geom(ow, box)
    for k, link in enumerate(["panda_leftfinger", "panda_link7"]):
        gs = _geom(ow, objs[link].geom)
        TA, TB = boundary_poses(ow, gb, gs, 2000, seed=90 + k, reach=0.5)
        dev, ref = _compare(ow, dw, gb, gs, TA, TB)
        assert 0.2 < ref.mean() < 0.8
        np.testing.assert_array_equal(dev, ref, err_msg=link)
