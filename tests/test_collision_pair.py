"""Planner.generate_collision_pair (mplib/planner.py:118-163), batched:
random full configurations drawn on the device (mpg_sample_uniform's
splitmix64 stream, restated in mplib_amd/planner.py), evaluated like
collide_full() and counted per pair on the device (mpg_collide_count).
Checked against the oracle's collide_batch on the same samples, and the SRDF
against the reference's output format."""
import os
import tempfile
import time
import xml.etree.ElementTree as ET

import numpy as np
import pytest

import oracle
from oracle import model as M
import worlds as Wd
from mplib_amd import planner


def test_sampler_known_answers():
    # splitmix64's first output for seed 0 is 0xE220A8397B1DCDAF (the
    # generator's published reference value); u = that >> 11 times 2^-53
    u = planner.sample_uniform([0.0], [1.0], 1, 0)[0, 0]
    assert u == (0xE220A8397B1DCDAF >> 11) * 2.0 ** -53
    q = planner.sample_uniform([-1.0, 0.0, 2.0], [1.0, 0.04, 2.0], 10000, 123)
    assert q.shape == (10000, 3)
    assert (q[:, 0] >= -1).all() and (q[:, 0] < 1).all() and (q[:, 1] < 0.04).all() and (q[:, 2] == 2.0).all()
    # rows are addressable: a batch split in two equals the whole batch
    a = planner.sample_uniform([-1.0, 0.0], [1.0, 1.0], 7, 5)
    b = np.vstack([planner.sample_uniform([-1.0, 0.0], [1.0, 1.0], 3, 5),
                   planner.sample_uniform([-1.0, 0.0], [1.0, 1.0], 4, 5, offset=3)])
    np.testing.assert_array_equal(a, b)


class _FakeWorld:
    """pair table + counts, as PlanningWorld returns them"""

    def __init__(self, pairs, counts):
        self.pairs, self.counts = pairs, counts

    def sample_pair_counts(self, n, seed):
        return self.counts

    def get_collision_pair_info(self):
        return [("self", "robot", "robot", a, b, False, True) for a, b in self.pairs]


def test_srdf_format_matches_reference():
    """planner.py:137-163: every (link_i, link_j) whose count is sample_time,
    as disable_collisions with reason Default, minidom pretty-printed."""
    links = ["l0", "l1", "l2", "l3"]
    w = _FakeWorld([("l0", "l2"), ("l1", "l3"), ("l0", "l3"), ("l2", "l3")], [100, 99, 100, 0])
    d = tempfile.mkdtemp()
    path = planner.generate_collision_pair(w, links, os.path.join(d, "robot.urdf"), sample_time=100, verbose=False)
    assert path == os.path.join(d, "robot.srdf")
    root = ET.parse(path).getroot()
    assert root.tag == "robot" and root.get("name") == "robot"
    got = [(e.get("link1"), e.get("link2"), e.get("reason")) for e in root]
    assert got == [("l0", "l2", "Default"), ("l0", "l3", "Default")]
    assert open(path).read().startswith('<?xml version="1.0" ?>\n<robot name="robot">\n    <disable_collisions')


def _panda_full_worlds():
    from mplib_amd import pymp, scenes
    art = pymp.articulation.ArticulatedModel(os.path.join(scenes.PANDA_DIR, "panda.urdf"), "", [0, 0, -9.81],
                                             scenes.PANDA_JOINTS, scenes.PANDA_LINKS, verbose=False, convex=True)
    w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
    oart = M.Articulation(os.path.join(Wd.panda_dir(), "panda.urdf"), "", Wd.PANDA_LINKS, Wd.PANDA_JOINTS,
                          convex=True, move_group=None)
    return w, oracle.OracleWorld(oart)


@pytest.mark.gpu
def test_device_sampler_matches_host():
    from mplib_amd import _capi as C
    import ctypes
    lo = np.array([-2.8973, -1.7628, 0.0, -3.14159265359], np.float64)
    hi = np.array([2.8973, 1.7628, 0.04, 3.14159265359], np.float64)
    n, seed = 100003, 987654321
    out = np.zeros((n, 4), np.float64)
    C.check(C.lib().mpg_sample_uniform(lo.ctypes.data_as(ctypes.c_void_p), hi.ctypes.data_as(ctypes.c_void_p), 4, n,
                                       seed, 17, out.ctypes.data_as(ctypes.c_void_p), 0), "mpg_sample_uniform")
    np.testing.assert_array_equal(out, planner.sample_uniform(lo, hi, n, seed, offset=17))


@pytest.mark.gpu
def test_pair_counts_match_oracle():
    """2^20 random full configurations of the Panda without SRDF (the
    situation generate_collision_pair runs in: 46 pairs after the parent
    rule), every pair count equal to the oracle's on the same samples."""
    w, ow = _panda_full_worlds()
    info = w.get_collision_pair_info()
    assert [(i[3], i[4]) for i in info] == ow.pair_names()
    lo, hi = w.get_full_state_limits()
    assert len(lo) == 9 and ow.dof == 9
    n, seed = 1 << 20, 2024
    counts = np.asarray(w.sample_pair_counts(n, seed))
    q = planner.sample_uniform(lo, hi, n, seed)
    _, mo = ow.collide_batch(q, nthreads=16)
    want = np.array([int(((mo[:, p >> 5] >> (p & 31)) & 1).sum()) for p in range(len(info))])
    np.testing.assert_array_equal(counts, want)
    assert 0 < counts.sum() and (counts < n).any()


@pytest.mark.gpu
def test_generate_collision_pair_srdf_and_speed():
    """10^6 samples (the reference's default sample_time) in one device call;
    the SRDF lists exactly the pairs that collide in every sample."""
    w, ow = _panda_full_worlds()
    w.sample_pair_counts(4096, 1)  # snapshot + workspaces
    t0 = time.perf_counter()
    counts = w.sample_pair_counts(1000000, 0)
    dt = time.perf_counter() - t0
    print(f"generate_collision_pair: 10^6 samples in {dt * 1e3:.2f} ms")
    assert dt < 0.05
    d = tempfile.mkdtemp()
    path = planner.generate_collision_pair(w, Wd.PANDA_LINKS, os.path.join(d, "panda.urdf"), sample_time=1000000,
                                           verbose=False)
    always = {(e.get("link1"), e.get("link2")) for e in ET.parse(path).getroot()}
    info = w.get_collision_pair_info()
    assert always == {(i[3], i[4]) for i, c in zip(info, counts) if c == 1000000}
