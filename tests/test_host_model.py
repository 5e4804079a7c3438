"""CPU: the C++ host (mplib_amd.pymp) builds the same model, pair table and
ACM decisions as the oracle -- no device needed for any of these."""
import numpy as np
import pytest

import worlds as Wd
from mplib_amd import pymp, scenes


@pytest.fixture(scope="module")
def art():
    return scenes.panda()


def test_panda_model(art):
    fcl = art.get_fcl_model()
    assert fcl.get_collision_link_names() == Wd.PANDA_LINKS
    assert [tuple(p) for p in fcl.get_collision_pairs()] == Wd.panda_articulation().pairs
    pin = art.get_pinocchio_model()
    assert pin.get_joint_types() == ["JointModelRZ"] * 7 + ["JointModelPY", "JointModelPrismaticUnaligned"]
    assert art.get_qpos_dim() == 7
    assert list(art.get_move_group_joint_indices()) == list(range(7))
    np.testing.assert_array_equal(scenes.joint_limits(art), Wd.panda_articulation().joint_limits()[:7])
    assert pin.get_link_names(False)[:3] == ["panda_link0", "panda_link1", "panda_link2"]
    assert pin.get_leaf_links() == ["panda_leftfinger", "panda_rightfinger"]
    assert pin.get_chain_joint_name("panda_hand") == Wd.PANDA_JOINTS[:7]


def test_convex_vertices_equal_oracle(art):
    ora = Wd.panda_articulation()
    mesh = f"{scenes.PANDA_DIR}/franka_description/meshes/collision/link3.stl.convex.stl"
    g = pymp.fcl.load_mesh_as_Convex(mesh, [1, 1, 1])
    np.testing.assert_array_equal(g.get_vertices(), ora.objects[3].geom.vertices)
    np.testing.assert_array_equal(g.get_interior_point(), np.array(ora.objects[3].geom.interior))


@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_pair_table_equals_oracle(cfg):
    w, _ = scenes.world(cfg)
    ow = Wd.oracle_world(cfg)
    info = w.get_collision_pair_info()
    assert [(i[3], i[4]) for i in info] == ow.pair_names()
    allowed = [bool(i[5]) for i in info]
    assert allowed == [frozenset((p[4], p[5])) in ow.allowed for p in ow.pairs]
    assert w.get_state_dim() == 7
    assert w.get_mask_words() == (len(info) + 31) // 32


def test_acm_semantics():
    acm = pymp.collision_matrix.AllowedCollisionMatrix()
    AC = pymp.collision_matrix.AllowedCollision
    assert acm.get_allowed_collision("a", "b") is None
    acm.set_default_entry("a", True)
    assert acm.get_allowed_collision("a", "b") == AC.ALWAYS
    acm.set_default_entry("b", False)
    assert acm.get_allowed_collision("a", "b") == AC.NEVER  # NEVER wins among defaults
    acm.set_entry("a", "b", True)
    assert acm.get_allowed_collision("b", "a") == AC.ALWAYS  # explicit entry wins, symmetric
    acm.remove_entry("a", "b")
    assert not acm.has_entry("a", "b")
    acm.set_entry("c", ["d", "e"], False)
    assert acm.get_entry("e", "c") == AC.NEVER and len(acm) == 3
    acm.set_entry(True)
    assert acm.get_entry("c", "d") == AC.ALWAYS
    acm.remove_entry("c")
    assert not acm.has_entry("c") and sorted(acm.get_all_entry_names()) == ["a", "b"]


def test_acm_change_updates_pair_table():
    w, _ = scenes.world(3)
    before = [i[5] for i in w.get_collision_pair_info()]
    w.get_allowed_collision_matrix().set_entry("panda_hand", "red_cube", True)
    after = [i[5] for i in w.get_collision_pair_info()]
    changed = [i for i, (a, b) in enumerate(zip(before, after)) if a != b]
    info = w.get_collision_pair_info()
    assert len(changed) == 1 and (info[changed[0]][3], info[changed[0]][4]) == ("panda_hand", "red_cube")


@pytest.mark.gpu  # attachObject's AttachedBody ctor evaluates the link pose (device FK)
def test_attached_body_pairs():
    w, art = scenes.world(4)
    w.attach_object("held", pymp.fcl.Box([0.04, 0.04, 0.12]), "panda", 8, [0, 0, 0.14, 1, 0, 0, 0], ["panda_hand"])
    info = w.get_collision_pair_info()
    types = [i[0] for i in info]
    assert types.count("self_attach") == 11
    assert types.count("attach_sceneobject") == 4
    # reference argument order: collide(attached_obj, link) for self_attach
    sa = [i for i in info if i[0] == "self_attach"]
    assert sa[0][3] == "panda_link0" and sa[0][4] == "held"
    # touch link allowed by the ACM (attachObject sets entry(name, touch_links))
    assert [i[5] for i in sa if i[3] == "panda_hand"] == [True]
    assert w.detach_object("held") and not w.is_normal_object_attached("held")


def test_unsupported_requests_raise():
    w, _ = scenes.world(2)
    with pytest.raises(NotImplementedError):
        w.collide(pymp.fcl.CollisionRequest(enable_cost=True))
    # GST_INDEP collides and measures unsigned distances on the device since
    # round 6 (tests/test_gjk_indep.py); its EPA (contacts, signed distances)
    # is not restated
    with pytest.raises(NotImplementedError):
        w.collide(pymp.fcl.CollisionRequest(enable_contact=True, gjk_solver_type=pymp.fcl.GJKSolverType.GST_INDEP))
    with pytest.raises(NotImplementedError):
        w.distance_full(pymp.fcl.DistanceRequest(enable_signed_distance=True,
                                                 gjk_solver_type=pymp.fcl.GJKSolverType.GST_INDEP))


def test_set_qpos_validation(art):
    with pytest.raises(RuntimeError, match="Length is not correct"):
        art.set_qpos([0.0] * 5)
    art.set_qpos([0.1] * 9, True)
    np.testing.assert_array_equal(art.get_qpos(), [0.1] * 9)
    art.set_qpos([0.0] * 7)
    np.testing.assert_array_equal(art.get_qpos(), [0.0] * 7 + [0.1, 0.1])
    art.set_qpos([0.0] * 9, True)
