"""Pins from the reference's own data: the MoveIt reasons of
data/panda/panda.srdf:44-79 (reference `data/panda/panda.srdf`), the only
collision facts the reference holds beyond examples/detect_collision.py.

* reason="Default" (4 pairs): in collision at MoveIt's default state (each
  joint 0 when 0 is inside its limits, else the middle of its range: joint4 =
  -1.5708; fingers 0).  Built without the SRDF (46 pairs after FCLModel's
  parent rule, fcl_model.cpp:114-136), the world must report exactly these 4
  there, for convex=True (hulls) and convex=False (BVH meshes).
* reason="Never" (23 pairs): MoveIt's setup assistant saw no collision over
  its random samples.  That is a sampling statistic, not a geometric fact: 22
  of the 23 pairs never collide in 2^14 uniform samples, but panda_link2 -
  panda_link6 does, in ~0.08 % of them, all with joint4 within 0.11 rad of its
  lower limit (elbow fully folded).  Those hits are real: an independent
  point-in-mesh ray cast (below, plain numpy, no oracle code) finds vertices of
  each mesh centimetres inside the other.  So the pin is: no Never pair except
  link2-link6, and every link2-link6 hit is a folded elbow whose meshes
  interpenetrate.
The oracle checks run here (CPU); the product twins run through
PlanningWorld.collide_full() and sample_pair_counts() on the GPU.
"""
import os
import re

import numpy as np
import pytest

import oracle
import worlds as Wd
from oracle import model as M

FOLDED_ELBOW = -2.95  # every link2-link6 hit has joint4 below this (limit -3.0718)


def srdf_reasons():
    txt = open(os.path.join(Wd.panda_dir(), "panda.srdf")).read()
    return {frozenset((a, b)): r for a, b, r in
            re.findall(r'<disable_collisions link1="(\w+)" link2="(\w+)" reason="(\w+)"', txt)}


def default_state(lim):
    """MoveIt's default joint values: 0 if within the bounds, else the middle."""
    return np.array([0.0 if lo <= 0.0 <= hi else 0.5 * (lo + hi) for lo, hi in lim])


def oracle_full_world(convex):
    art = M.Articulation(os.path.join(Wd.panda_dir(), "panda.urdf"), "", Wd.PANDA_LINKS, Wd.PANDA_JOINTS,
                         convex=convex, move_group=None)
    return oracle.OracleWorld(art)


def pair_hits(mask, p):
    return ((mask[:, p >> 5] >> (p & 31)) & 1).astype(bool)


def test_srdf_reason_counts():
    r = srdf_reasons()
    kinds = {k: sorted(tuple(sorted(p)) for p, v in r.items() if v == k) for k in set(r.values())}
    assert len(r) == 36 and len(kinds["Default"]) == 4 and len(kinds["Never"]) == 23 and len(kinds["Adjacent"]) == 9
    assert kinds["Default"] == [("panda_hand", "panda_link5"), ("panda_hand", "panda_link7"),
                                ("panda_leftfinger", "panda_rightfinger"), ("panda_link5", "panda_link7")]


@pytest.mark.parametrize("convex", [True, False])
def test_default_state_reports_exactly_the_default_pairs(convex):
    ow = oracle_full_world(convex)
    assert len(ow.pair_names()) == 46
    lim = ow.art.joint_limits()
    q0 = default_state(lim)
    assert q0[3] == pytest.approx(-1.5708) and np.count_nonzero(q0) == 1
    _, m = ow.collide_batch(q0[None])
    got = {frozenset(p) for p in ow.decode(m[0])}
    want = {p for p, v in srdf_reasons().items() if v == "Default"}
    assert got == want
    # Adjacent pairs are gone already by the parent rule
    names = {frozenset(p) for p in ow.pair_names()}
    assert not names & {p for p, v in srdf_reasons().items() if v == "Adjacent"}


def _inside(points, V, F):
    """Point-in-closed-mesh by the parity of ray crossings (Moller-Trumbore)."""
    d = np.array([0.5773, 0.5774, 0.5775])
    d /= np.linalg.norm(d)
    A, B, C = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    e1, e2 = B - A, C - A
    h = np.cross(d, e2)
    a = (e1 * h).sum(1)
    out = []
    for P in points:
        s = P - A
        with np.errstate(divide="ignore", invalid="ignore"):
            u = (s * h).sum(1) / a
            qv = np.cross(s, e1)
            v = (qv @ d) / a
            t = (qv * e2).sum(1) / a
        ok = (np.abs(a) > 1e-12) & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 0)
        out.append(ok.sum() % 2 == 1)
    return np.array(out, bool)


def _posed(geom, T):
    return geom.vertices @ T[:9].reshape(3, 3).T + T[9:]


def test_never_pairs_over_random_samples_bvh():
    """2^14 uniform full configurations, convex=False: no Never pair collides
    except link2-link6 at a folded elbow, whose meshes really interpenetrate."""
    ow = oracle_full_world(False)
    lim = ow.art.joint_limits()
    q = np.random.default_rng(5).uniform(lim[:, 0], lim[:, 1], size=(1 << 14, len(lim)))
    _, m = ow.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    reasons = srdf_reasons()
    names = ow.pair_names()
    hits26 = None
    for p, nm in enumerate(names):
        h = pair_hits(m, p)
        if reasons.get(frozenset(nm)) != "Never":
            continue
        if frozenset(nm) == frozenset(("panda_link2", "panda_link6")):
            hits26 = np.nonzero(h)[0]
        else:
            assert not h.any(), (nm, int(h.sum()))
    assert hits26 is not None and 0 < len(hits26) < 0.002 * len(q)
    assert (q[hits26, 3] < FOLDED_ELBOW).all()
    objs = [o.link for o in ow.art.objects]
    i2, i6 = objs.index("panda_link2"), objs.index("panda_link6")
    g2, g6 = ow.art.objects[i2].geom, ow.art.objects[i6].geom
    _, objT = ow.fk_batch(q[hits26])
    for k in range(len(hits26)):
        V2, V6 = _posed(g2, objT[k, i2]), _posed(g6, objT[k, i6])
        assert _inside(V6, V2, np.asarray(g2.faces)).any() or _inside(V2, V6, np.asarray(g6.faces)).any(), k


def test_never_pairs_over_random_samples_hulls():
    """The same with the convex hulls (convex=True): hulls only grow the
    links, and the Never pairs hit are link2-link6 alone, again at a folded
    elbow (DESIGN.md 2 records the count)."""
    ow = oracle_full_world(True)
    lim = ow.art.joint_limits()
    q = np.random.default_rng(5).uniform(lim[:, 0], lim[:, 1], size=(1 << 14, len(lim)))
    _, m = ow.collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    reasons = srdf_reasons()
    for p, nm in enumerate(ow.pair_names()):
        h = pair_hits(m, p)
        if reasons.get(frozenset(nm)) == "Never" and h.any():
            assert frozenset(nm) == frozenset(("panda_link2", "panda_link6")), (nm, int(h.sum()))
            assert h.sum() < 0.003 * len(q) and (q[h, 3] < FOLDED_ELBOW).all()


def product_full_world(convex):
    from mplib_amd import pymp, scenes
    art = pymp.articulation.ArticulatedModel(os.path.join(scenes.PANDA_DIR, "panda.urdf"), "", [0, 0, -9.81],
                                             scenes.PANDA_JOINTS, scenes.PANDA_LINKS, verbose=False, convex=convex)
    return pymp.planning_world.PlanningWorld([art], ["panda"], [], [])


@pytest.mark.gpu
@pytest.mark.parametrize("convex", [True, False])
def test_device_default_state_reports_exactly_the_default_pairs(convex):
    w = product_full_world(convex)
    assert len(w.get_collision_pair_info()) == 46
    lo, hi = w.get_full_state_limits()
    q0 = default_state(np.stack([lo, hi], 1))
    w.set_qpos_all(q0)
    got = {frozenset((r.link_name1, r.link_name2)) for r in w.collide_full()}
    assert got == {p for p, v in srdf_reasons().items() if v == "Default"}
    assert w.collide()
    f, m = w.collide_batch(q0[None])  # the batch path agrees
    info = w.get_collision_pair_info()
    assert {frozenset((info[p][3], info[p][4])) for p in range(len(info)) if pair_hits(m, p)[0]} == got


@pytest.mark.gpu
def test_device_never_pairs_over_2e20_samples_bvh():
    """sample_pair_counts(2^20) on the convex=False world: no Never pair but
    link2-link6 (folded elbow, rate < 0.2 %); the first 4096 samples' counts
    equal the oracle's on the same draws."""
    from mplib_amd import planner
    w = product_full_world(False)
    info = w.get_collision_pair_info()
    names = [frozenset((i[3], i[4])) for i in info]
    reasons = srdf_reasons()
    n = 1 << 20
    counts = np.asarray(w.sample_pair_counts(n, 77))
    for nm, c in zip(names, counts):
        if reasons.get(nm) == "Never" and nm != frozenset(("panda_link2", "panda_link6")):
            assert c == 0, (tuple(nm), int(c))
    c26 = int(counts[names.index(frozenset(("panda_link2", "panda_link6")))])
    assert 0 < c26 < 0.002 * n
    # Default pairs collide often, never-checked (Adjacent) pairs are absent
    assert all(counts[names.index(p)] > 0 for p, v in reasons.items() if v == "Default")
    ow = oracle_full_world(False)
    assert [frozenset(p) for p in ow.pair_names()] == names
    lo, hi = w.get_full_state_limits()
    k = 4096
    ck = np.asarray(w.sample_pair_counts(k, 78))
    _, mo = ow.collide_batch(planner.sample_uniform(lo, hi, k, 78), nthreads=16)
    np.testing.assert_array_equal(ck, [int(pair_hits(mo, p).sum()) for p in range(len(info))])
