"""Worlds with several articulations (reference src/planning_world.cpp:
setQposAll 250-262 splits the state across the planned articulations in
std::map name order; selfCollide 277-369 adds planned x planned link pairs and
attached bodies against every planned articulation; collideWithOthers
372-481 adds planned x unplanned link pairs and attached x unplanned).

The oracle (oracle.MultiOracleWorld) restates them on one merged kinematic
forest; the product's pair table is matched to the oracle's by (object
names, link names)."""
import os
import tempfile

import numpy as np
import pytest

import oracle
from oracle import model as M
import worlds as Wd

OFFSET_XYZ = (1.25, 0.05, 0.0)
OFFSET_RPY = (0.0, 0.0, 3.14159265358979)
B_QPOS = [0.3, -0.4, 0.2, -2.2, 0.1, 2.0, 0.6]


def offset_panda_urdf(xyz=OFFSET_XYZ, rpy=OFFSET_RPY) -> str:
    """The Panda URDF with a new root link fixed at (xyz, rpy) (MPlib 0.1.1 has
    no articulation base pose; a second robot gets its place from its URDF).
    Written next to a link to the Panda's mesh directory."""
    src = os.path.join(Wd.panda_dir(), "panda.urdf")
    d = tempfile.mkdtemp(prefix="panda_off_")
    os.symlink(os.path.join(Wd.panda_dir(), "franka_description"), os.path.join(d, "franka_description"))
    text = open(src).read()
    head = text.index(">", text.index("<robot")) + 1
    extra = ('\n  <link name="offset_base"/>\n  <joint name="offset_joint" type="fixed">\n'
             f'    <parent link="offset_base"/>\n    <child link="panda_link0"/>\n'
             f'    <origin xyz="{xyz[0]} {xyz[1]} {xyz[2]}" '
             f'rpy="{rpy[0]} {rpy[1]} {rpy[2]}"/>\n  </joint>\n')
    path = os.path.join(d, "panda.urdf")
    open(path, "w").write(text[:head] + extra + text[head:])
    return path


def oracle_panda(urdf):
    return M.Articulation(urdf, os.path.join(Wd.panda_dir(), "panda.srdf"), Wd.PANDA_LINKS, Wd.PANDA_JOINTS,
                          convex=True, move_group="panda_hand")


ATT_SIDE = (0.04, 0.05, 0.09)
ATT_POSE = (0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0)


def oracle_world(b_planned: bool, scene_boxes: int = 4):
    a = oracle_panda(os.path.join(Wd.panda_dir(), "panda.urdf"))
    b = oracle_panda(offset_panda_urdf())
    mg = b.move_group_qpos_index()
    for i, v in zip(mg, B_QPOS):
        b.current_qpos[i] = v
    scene = Wd.boxes_scene()[:scene_boxes]
    hand = Wd.PANDA_LINKS.index("panda_hand")
    name = f"a_panda_{hand}_box"  # PlanningWorld::attachBox naming (planning_world.cpp:206)
    att = [(name, "a_panda", hand, M.BoxGeom(ATT_SIDE), oracle.pose7_to_se3(ATT_POSE))]
    parts = [("a_panda", a, True), ("b_panda", b, b_planned)]
    allowed = [("panda_link0", "table")]
    # attachObject without touch links (planning_world.cpp:144-169): the links
    # selfCollide() reports against the new body at the current state become
    # its touch links, allowed in the ACM by name
    mw = oracle.MultiOracleWorld(parts, scene=scene, attached=att, allowed=allowed)
    state = [0.0] * 7 + (B_QPOS if b_planned else [])
    _, m = mw.collide_batch(np.array([state]))
    touch = [k[3] if k[2] == name else k[2] for p, k in enumerate(mw.pair_keys[:mw.n_self_pairs])
             if (int(m[0, p >> 5]) >> (p & 31)) & 1 and name in (k[2], k[3])]
    return oracle.MultiOracleWorld(parts, scene=scene, attached=att, allowed=allowed + [(name, t) for t in touch])


def test_merged_single_articulation_equals_oracle_world():
    """One planned articulation through the merged forest reproduces the
    single-articulation oracle bit for bit."""
    ow = Wd.oracle_world(3)
    mw = oracle.MultiOracleWorld([("panda", ow.art, True)], scene=ow.scene, attached=[],
                                 allowed=[tuple(p) for p in ow.allowed])
    assert mw.pair_names() == ow.pair_names()
    q = Wd.sample_q(ow.art, 3000, 5)
    f0, m0 = ow.collide_batch(q, nthreads=8)
    f1, m1 = mw.collide_batch(q, nthreads=8)
    np.testing.assert_array_equal(f0, f1)
    np.testing.assert_array_equal(m0, m1)


def test_two_articulation_oracle_kinematics():
    """The offset robot's links are the base robot's links moved by the root
    offset (FK through the merged forest), and the planned state splits in
    std::map name order."""
    mw = oracle_world(b_planned=True)
    assert mw.dof == 14
    q = Wd.sample_q(mw.parts[0][1], 4, 9)
    qq = np.concatenate([q, q[::-1]], axis=1)
    poses, _ = mw.fk_batch(qq)
    single = Wd.oracle_world(2)
    pa, _ = single.fk_batch(q)
    pb, _ = single.fk_batch(q[::-1])
    n = len(Wd.PANDA_LINKS)
    np.testing.assert_array_equal(poses[:, :n], pa)
    # robot b: base rotated by pi about z and shifted
    c, s = np.cos(OFFSET_RPY[2]), np.sin(OFFSET_RPY[2])
    xb = pb[:, :, 0] * c - pb[:, :, 1] * s + OFFSET_XYZ[0]
    np.testing.assert_allclose(poses[:, n:, 0], xb, atol=1e-12)
    # pair structure: self pairs of both + 11 x 11 planned x planned + the attached body x both
    kinds = [k[:2] for k in mw.pair_keys]
    assert kinds.count(("b_panda", "a_panda")) == 11 * 11
    assert kinds.count(("a_panda_8_box", "a_panda_8_box")) == 0


def product_world(b_planned: bool, scene_boxes: int = 4):
    from mplib_amd import pymp, scenes
    a = scenes.panda()
    b = pymp.articulation.ArticulatedModel(offset_panda_urdf(), os.path.join(scenes.PANDA_DIR, "panda.srdf"),
                                           [0, 0, -9.81], scenes.PANDA_JOINTS, scenes.PANDA_LINKS, verbose=False,
                                           convex=True)
    b.set_move_group("panda_hand")
    b.set_qpos(B_QPOS, False)
    w = pymp.planning_world.PlanningWorld([a], ["a_panda"], [], [])
    w.add_articulation("b_panda", b, b_planned)
    for name, side, pos in scenes._boxes()[:scene_boxes]:
        w.add_normal_object(name, pymp.fcl.CollisionObject(pymp.fcl.Box(list(side)), list(pos), [1, 0, 0, 0]))
    w.get_allowed_collision_matrix().set_entry("panda_link0", "table", True)
    w.attach_box(list(ATT_SIDE), "a_panda", scenes.PANDA_LINKS.index("panda_hand"), list(ATT_POSE))
    return w


@pytest.mark.gpu
@pytest.mark.parametrize("b_planned", [False, True])
def test_two_pandas_match_oracle(b_planned):
    w = product_world(b_planned)
    mw = oracle_world(b_planned)
    info = w.get_collision_pair_info()
    keys = [(i[1], i[2], i[3], i[4]) for i in info]
    assert sorted(keys) == sorted(mw.pair_keys)
    perm = [mw.pair_keys.index(k) for k in keys]  # product pair p = oracle pair perm[p]
    n = 1 << 16
    qa = Wd.sample_q(mw.parts[0][1], n, 41)
    q = np.concatenate([qa, Wd.sample_q(mw.parts[0][1], n, 42)], axis=1) if b_planned else qa
    assert w.get_state_dim() == q.shape[1]
    fo, mo = mw.collide_batch(q, nthreads=16)
    f, m = w.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    m = m.view(np.uint32)
    for p, po in enumerate(perm):
        got = (m[:, p >> 5] >> (p & 31)) & 1
        want = (mo[:, po >> 5] >> (po & 31)) & 1
        assert np.array_equal(got, want), keys[p]
    assert 0.05 < f.mean() < 0.999
    # some configurations collide only through the second robot
    arts = [p for p, k in enumerate(keys) if "b_panda" in (k[0], k[1]) and k[0] != k[1]]
    assert any(((m[:, p >> 5] >> (p & 31)) & 1).any() for p in arts)


@pytest.mark.gpu
@pytest.mark.parametrize("b_planned", [False, True])
def test_two_pandas_latency_path_matches_oracle(b_planned):
    """The planner's one-launch latency path (batches of <= 256 states: each
    lane's joint sin/cos and both objects' chains staged in LDS) on the
    two-Panda forest (18 joints, dof 7 or 14): every flag and pair bit equals
    the oracle's."""
    w = product_world(b_planned)
    mw = oracle_world(b_planned)
    keys = [(i[1], i[2], i[3], i[4]) for i in w.get_collision_pair_info()]
    perm = [mw.pair_keys.index(k) for k in keys]
    n = 2048
    qa = Wd.sample_q(mw.parts[0][1], n, 43)
    q = np.concatenate([qa, Wd.sample_q(mw.parts[0][1], n, 44)], axis=1) if b_planned else qa
    fo, mo = mw.collide_batch(q, nthreads=16)
    w.set_small_batch_max(1 << 20)
    for i in range(0, n, 200):
        f, m = w.collide_batch(q[i:i + 200])
        np.testing.assert_array_equal(f, fo[i:i + 200])
        m = m.view(np.uint32)
        for p, po in enumerate(perm):
            got = (m[:, p >> 5] >> (p & 31)) & 1
            want = (mo[i:i + 200, po >> 5] >> (po & 31)) & 1
            assert np.array_equal(got, want), keys[p]
    assert 0.05 < fo.mean() < 0.999


@pytest.mark.gpu
def test_two_pandas_planner_matches_oracle_checker():
    """RRTConnect over the two planned Pandas' 14-dof compound space: the
    device checker (speculative batches on the latency path) plans the path
    the oracle checker gives."""
    from mplib_amd import pymp
    w = product_world(True)
    mw = oracle_world(True)
    dev = pymp.ompl.OMPLPlanner(w)
    ref = pymp.ompl.OMPLPlanner(product_world(True), state_validity_checker=lambda s: mw.collide_batch(s)[0] == 0)
    start = np.array([0.0, 0.2, 0.0, -2.6, 0.0, 3.0, 0.8] + list(B_QPOS[:7]))
    goal = np.array([0.3, -0.3, 0.2, -2.0, 0.1, 2.2, 0.5] + list(B_QPOS[:7]))
    assert (mw.collide_batch(goal[None])[0] == 0).all()
    pymp.set_global_seed(11)
    s1, p1 = dev.plan(start, [goal], range=0.2, time=60.0)
    pymp.set_global_seed(11)
    s2, p2 = ref.plan(start, [goal], range=0.2, time=60.0)
    assert s1 == s2 == "Exact solution"
    assert np.array_equal(p1, p2)


FAR = (310.0, -205.5, 42.25)


@pytest.mark.gpu
def test_far_from_origin_world_matches_oracle():
    """The whole cfg3 world (robot base and boxes) moved ~370 m from the
    origin: the fp32 cull's margin grows with the world's coordinate bound
    (kFp32CullRel), so every flag and pair bit still equals the oracle's."""
    from mplib_amd import pymp, scenes
    urdf = offset_panda_urdf(FAR, (0.0, 0.0, 0.0))
    art = pymp.articulation.ArticulatedModel(urdf, os.path.join(scenes.PANDA_DIR, "panda.srdf"), [0, 0, -9.81],
                                             scenes.PANDA_JOINTS, scenes.PANDA_LINKS, verbose=False, convex=True)
    art.set_move_group("panda_hand")
    w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
    scene = []
    for name, side, pos in scenes._boxes():
        p = [pos[i] + FAR[i] for i in range(3)]
        w.add_normal_object(name, pymp.fcl.CollisionObject(pymp.fcl.Box(list(side)), p, [1, 0, 0, 0]))
        scene.append((name, M.BoxGeom(tuple(float(x) for x in side)), (list(M.IDENT[0]), [float(x) for x in p])))
    w.get_allowed_collision_matrix().set_entry("panda_link0", "table", True)
    ow = oracle.OracleWorld(oracle_panda(urdf), scene=scene, allowed=[("panda_link0", "table")])
    q = Wd.sample_q(ow.art, 1 << 17, 77)
    f, m = w.collide_batch(q)
    fo, mo = ow.collide_batch(q, nthreads=16)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m.view(np.uint32), mo)
    assert 0.05 < fo.mean() < 0.95


RAIL_AT = (300.0, -12.0, 0.5)
RAIL_JOINTS = ["rail_joint"] + Wd.PANDA_JOINTS


def rail_panda_urdf(lower: float = 0.0, upper: float = 5.0) -> str:
    """The Panda on a prismatic rail along x (limits [lower, upper] m) whose
    base sits ~300 m from the origin."""
    src = os.path.join(Wd.panda_dir(), "panda.urdf")
    d = tempfile.mkdtemp(prefix="panda_rail_")
    os.symlink(os.path.join(Wd.panda_dir(), "franka_description"), os.path.join(d, "franka_description"))
    text = open(src).read()
    head = text.index(">", text.index("<robot")) + 1
    extra = ('\n  <link name="rail_base"/>\n  <joint name="rail_joint" type="prismatic">\n'
             '    <parent link="rail_base"/>\n    <child link="panda_link0"/>\n'
             f'    <origin xyz="{RAIL_AT[0]} {RAIL_AT[1]} {RAIL_AT[2]}" rpy="0 0 0"/>\n'
             '    <axis xyz="1 0 0"/>\n'
             f'    <limit effort="100" lower="{lower}" upper="{upper}" velocity="1.0"/>\n  </joint>\n')
    path = os.path.join(d, "panda.urdf")
    open(path, "w").write(text[:head] + extra + text[head:])
    return path


@pytest.mark.gpu
def test_prismatic_rail_far_from_origin_matches_oracle():
    """a Panda on a 5 m prismatic rail ~300 m from the origin
    (the rail's travel enters the fp32 cull's coordinate bound), boxes along
    the rail; 2^16 configurations in the limits plus 4096 with the rail value
    far outside them (evaluated with every pair), every flag and pair bit vs
    the oracle."""
    from mplib_amd import pymp, scenes
    urdf = rail_panda_urdf()
    art = pymp.articulation.ArticulatedModel(urdf, os.path.join(scenes.PANDA_DIR, "panda.srdf"), [0, 0, -9.81],
                                             RAIL_JOINTS, scenes.PANDA_LINKS, verbose=False, convex=True)
    art.set_move_group("panda_hand")
    w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
    scene, allowed = [], []
    for copy, dx in (("a", 1.0), ("b", 3.5)):
        for name, side, pos in scenes._boxes():
            p = [RAIL_AT[0] + dx + pos[0], RAIL_AT[1] + pos[1], RAIL_AT[2] + pos[2]]
            w.add_normal_object(f"{name}_{copy}", pymp.fcl.CollisionObject(pymp.fcl.Box(list(side)), p, [1, 0, 0, 0]))
            scene.append((f"{name}_{copy}", M.BoxGeom(tuple(float(x) for x in side)),
                          (list(M.IDENT[0]), [float(x) for x in p])))
        w.get_allowed_collision_matrix().set_entry("panda_link0", f"table_{copy}", True)
        allowed.append(("panda_link0", f"table_{copy}"))
    oart = M.Articulation(urdf, os.path.join(Wd.panda_dir(), "panda.srdf"), Wd.PANDA_LINKS, RAIL_JOINTS, convex=True,
                          move_group="panda_hand")
    ow = oracle.OracleWorld(oart, scene=scene, allowed=allowed)
    assert w.get_state_dim() == 8 and ow.dof == 8
    lim = oart.joint_limits()[:8]
    assert np.allclose(lim[0], [0.0, 5.0])
    rng = np.random.default_rng(2024)
    q = rng.uniform(lim[:, 0], lim[:, 1], size=(1 << 16, 8))
    out = rng.uniform(lim[:, 0], lim[:, 1], size=(4096, 8))
    out[:, 0] = rng.choice([-1.0, 1.0], 4096) * rng.uniform(6.0, 40.0, 4096)  # beyond the rail's travel bound
    q = np.concatenate([q, out])
    f, m = w.collide_batch(q)
    fo, mo = ow.collide_batch(q, nthreads=16)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m.view(np.uint32), mo)
    assert 0.05 < fo[:1 << 16].mean() < 0.95
