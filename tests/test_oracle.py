"""CPU: the oracle restatement against the reference's known answers and the
committed golden vectors (regression pins; see tools/gen_golden.py)."""
import json
import os

import numpy as np
import pytest

import worlds as Wd


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


@pytest.mark.parametrize("name,cfg", [("panda_self_4096", 2), ("panda_boxes_4096", 3), ("panda_convex_1024", 4)])
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
