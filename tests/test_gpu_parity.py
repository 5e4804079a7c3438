"""GPU parity: the HIP path (through the C ABI and through the pybind host)
against the CPU oracle and the golden fixtures.  Bit-exact for flags, pair
masks and FK poses (integer/boolean outputs; FK is fp64 with identical op order).
"""
import ctypes
import ctypes.util
import os

import numpy as np
import pytest

import worlds as Wd
from mplib_amd import pymp, scenes
from mplib_amd.batch import DeviceWorld, device_sincos

pytestmark = pytest.mark.gpu

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]


def libm_sincos(x):
    s, c = np.zeros_like(x), np.zeros_like(x)
    a, b = ctypes.c_double(), ctypes.c_double()
    for i, v in enumerate(x):
        _libm.sincos(float(v), ctypes.byref(a), ctypes.byref(b))
        s[i], c[i] = a.value, b.value
    return s, c


NTHREADS = min(16, os.cpu_count() or 1)
_OW = {}
_DW = {}


def ow(cfg):
    if cfg not in _OW:
        _OW[cfg] = Wd.oracle_world(cfg)
    return _OW[cfg]


def dw(cfg):
    if cfg not in _DW:
        _DW[cfg] = DeviceWorld(Wd.desc_arrays(ow(cfg)))
    return _DW[cfg]


def test_device_sincos_matches_libm():
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-4, 4, 100000), rng.uniform(-0.2, 0.2, 30000), rng.uniform(-1e3, 1e3, 30000),
                        np.array([0.0, -0.0, 0.126, 0.85546875, 2.426265, np.pi])])
    s, c = device_sincos(x)
    rs, rc = libm_sincos(x)
    assert int((s != rs).sum()) == 0 and int((c != rc).sum()) == 0


@pytest.mark.parametrize("name,cfg", [("panda_self_4096", 2), ("panda_boxes_4096", 3), ("panda_convex_1024", 4),
                                      ("panda_mesh_1024", 7)])
def test_capi_matches_golden(golden_dir, name, cfg):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    f, m = dw(cfg).collide_batch(g["q"])
    np.testing.assert_array_equal(f, g["flags"])
    np.testing.assert_array_equal(m, g["masks"])


def test_fk_bit_exact(golden_dir):
    g = np.load(os.path.join(golden_dir, "panda_fk_64.npz"))
    np.testing.assert_array_equal(dw(2).fk_batch(g["q"]), g["link_pose"])
    q = Wd.sample_q(ow(2).art, 4096, 77)
    np.testing.assert_array_equal(dw(2).fk_batch(q), ow(2).fk_batch(q)[0])


def test_debug_switches_do_not_change_results(monkeypatch):
    """The product library ignores the ablation switches (compiled in only
    under MPG_DIAG): a world created with them set still matches the oracle."""
    monkeypatch.setenv("MPG_DEBUG_CULL", "1")
    monkeypatch.setenv("MPG_DEBUG_MARGIN", "0")
    monkeypatch.setenv("MPG_DEBUG_NO_WALK", "1")
    d = DeviceWorld(Wd.desc_arrays(ow(3)))
    for n in (200, 20000):  # latency path and pipeline
        q = Wd.sample_q(ow(3).art, n, 4242 + n)
        f, m = d.collide_batch(q)
        fo, mo = ow(3).collide_batch(q, nthreads=NTHREADS)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 127, 129, 1000])
def test_ragged_batch_sizes(n):
    q = Wd.sample_q(ow(3).art, max(n, 1), 100 + n)[:n]
    f, m = dw(3).collide_batch(q)
    assert f.shape == (n,) and m.shape == (n, dw(3).mask_words)
    if n:
        fo, mo = ow(3).collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)


def test_device_pointer_path_matches_host_path():
    torch = pytest.importorskip("torch")
    q = Wd.sample_q(ow(3).art, 10000, 3)
    qd = torch.from_numpy(q).cuda()
    fd = torch.zeros(len(q), dtype=torch.uint8, device="cuda")
    md = torch.zeros((len(q), dw(3).mask_words), dtype=torch.int32, device="cuda")
    dw(3).collide_batch(qd, fd, md, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    f, m = dw(3).collide_batch(q)
    np.testing.assert_array_equal(fd.cpu().numpy(), f)
    np.testing.assert_array_equal(md.cpu().numpy().view(np.uint32), m)


# ----------------------------------------------------------------- product path
@pytest.mark.parametrize("cfg,name", [(2, "panda_self_4096"), (3, "panda_boxes_4096"), (4, "panda_convex_1024"),
                                      (7, "panda_mesh_1024")])
def test_product_world_matches_golden(golden_dir, cfg, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    w, _ = scenes.world(cfg)
    f, m = w.collide_batch(g["q"])
    np.testing.assert_array_equal(f, g["flags"])
    np.testing.assert_array_equal(m, g["masks"])


@pytest.mark.parametrize("cfg,n", [(2, 1 << 16), (3, 1 << 20), (4, 1 << 22)])
def test_product_full_size_parity(cfg, n):
    """Every flag and pair bit at the BASELINE sizes (cfg4: the whole 2^22
    batch of BASELINE.json's strong-scaling config on one GPU)."""
    w, art = scenes.world(cfg)
    q = scenes.sample_states(art, n, scenes.CFG_SEED[cfg])
    f, m = w.collide_batch(q)
    fo, mo = ow(cfg).collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    np.testing.assert_array_equal(f.astype(bool), (m != 0).any(1))


def test_scalar_api_known_answers(golden_dir):
    import json
    kat = json.load(open(os.path.join(golden_dir, "kat.json")))
    w, art = scenes.world(2)
    w.set_qpos_all(kat["free"]["q"])
    assert w.collide() is False and w.self_collide() == []
    w.set_qpos_all(kat["colliding"]["q"])
    assert w.collide() is True
    got = sorted((c.link_name1, c.link_name2) for c in w.self_collide())
    assert got == sorted(tuple(p) for p in kat["colliding"]["pairs"])
    full = w.collide_full()
    assert all(c.collision_type == "self" and c.object_name1 == "panda" for c in full)
    assert all(c.res.is_collision() for c in full)
    # FCLModel.collide_full after ArticulatedModel.set_qpos (fcl_model.cpp:182-193)
    res = art.get_fcl_model().collide_full()
    pairs = art.get_fcl_model().get_collision_pairs()
    names = art.get_fcl_model().get_collision_link_names()
    hit = sorted((names[a], names[b]) for (a, b), r in zip(pairs, res) if r.is_collision())
    assert hit == got


def test_pinocchio_link_pose_matches_oracle():
    w, art = scenes.world(2)
    q = Wd.sample_q(ow(2).art, 8, 5)
    po, _ = ow(2).fk_batch(q)
    pin = art.get_pinocchio_model()
    for i in range(len(q)):
        pin.compute_forward_kinematics(list(q[i]) + [0.0, 0.0])
        for l in range(len(Wd.PANDA_LINKS)):
            np.testing.assert_array_equal(pin.get_link_pose(l), po[i, l])


def test_scene_collide_with_others():
    w, art = scenes.world(3)
    q = Wd.sample_q(ow(3).art, 64, 21)
    fo, mo = ow(3).collide_batch(q)
    for i in range(len(q)):
        w.set_qpos_all(list(q[i]))
        got = sorted((c.link_name1, c.link_name2) for c in w.collide_full())
        assert got == sorted(ow(3).decode(mo[i]))
        assert w.collide() == bool(fo[i])


def test_attached_box_matches_oracle():
    """Attached box (Box-Convex MPR against links and hulls) vs the oracle."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(4)
    pose = [0.0, 0.0, 0.14, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("held", pymp.fcl.Box([0.04, 0.04, 0.12]), "panda", 8, pose, ["panda_hand"])
    base = ow(4)
    T = (M.quat_to_mat(1.0, 0.0, 0.0, 0.0), [0.0, 0.0, 0.14])
    o2 = oracle.OracleWorld(base.art, scene=base.scene, attached=[("held", 8, M.BoxGeom((0.04, 0.04, 0.12)), T)],
                            allowed=[("panda_hand", "held")])
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == o2.pair_names()
    q = Wd.sample_q(base.art, 20000, 8)
    f, m = w.collide_batch(q)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)


def test_acm_allow_all_clears_masks():
    w, art = scenes.world(3)
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    acm = w.get_allowed_collision_matrix()
    for a, b in names:
        acm.set_entry(a, b, True)
    q = scenes.sample_states(art, 4096, 1)
    f, m = w.collide_batch(q)
    assert not f.any() and not m.any()


def test_fcl_collide_free_function():
    import oracle
    from oracle import model as M
    hull = pymp.fcl.load_mesh_as_Convex(
        f"{scenes.PANDA_DIR}/franka_description/meshes/collision/link3.stl.convex.stl", [1, 1, 1])
    box = pymp.fcl.Box([0.1, 0.2, 0.3])
    o = ow(3)
    rng = np.random.default_rng(4)
    lib = oracle.lib()
    hits = 0
    for _ in range(200):
        p = rng.uniform(-0.2, 0.2, 3)
        qq = rng.normal(size=4)
        qq /= np.linalg.norm(qq)
        a = pymp.fcl.CollisionObject(hull, [0, 0, 0], [1, 0, 0, 0])
        b = pymp.fcl.CollisionObject(box, list(p), list(qq))
        r = pymp.fcl.collide(a, b).is_collision()
        Ta = np.array(list(M.quat_to_mat(1.0, 0.0, 0.0, 0.0)) + [0.0, 0.0, 0.0])
        Tb = np.array(list(M.quat_to_mat(*[float(v) for v in qq])) + [float(v) for v in p])
        g_hull = next(i for i, g in enumerate(o.geoms) if g is o.art.objects[3].geom)
        g_box = next(i for i, g in enumerate(o.geoms) if isinstance(g, M.BoxGeom))
        # the oracle's box geometry differs in size; build a dedicated world for the box instead
        ob = oracle.OracleWorld(o.art, scene=[("b", M.BoxGeom((0.1, 0.2, 0.3)), (list(Tb[:9]), list(Tb[9:])))])
        gb = next(i for i, g in enumerate(ob.geoms) if isinstance(g, M.BoxGeom))
        gh = next(i for i, g in enumerate(ob.geoms) if g is ob.art.objects[3].geom)
        ref = lib.orc_collide_pair(ctypes.byref(ob._w), gh, Ta.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), gb,
                                   Tb.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        assert r == bool(ref)
        hits += r
    assert 0 < hits < 200


# ------------------------------------------------------- batched motion validation
def _motion_reference(q_from, q_to, lvs, ow_):
    """OMPL DiscreteMotionValidator semantics restated in numpy (RealVector
    subspaces, weights 1) + the CPU oracle for every generated state."""
    segs, states, owner = [], [], []
    for e in range(len(q_from)):
        a, b = q_from[e], q_to[e]
        d = 0.0
        for i in range(len(a)):
            diff = a[i] - b[i]
            d += 1.0 * float(np.sqrt(diff * diff))
        m = max(1, int(np.ceil(d / lvs)))
        segs.append(m)
        for j in range(1, m + 1):
            states.append(b.copy() if j == m else a + (b - a) * (j / m))
            owner.append(e)
    flags, _ = ow_.collide_batch(np.array(states), nthreads=NTHREADS)
    valid = np.ones(len(q_from), bool)
    first = np.full(len(q_from), -1, np.int32)
    owner = np.array(owner)
    pos = 0
    for e, m in enumerate(segs):
        f = flags[pos:pos + m]
        if f.any():
            valid[e] = False
            first[e] = int(np.argmax(f)) + 1
        pos += m
    return valid, first, np.array(segs, np.int32)


def test_check_motion_batch_matches_oracle():
    w, art = scenes.world(3)
    rng = np.random.default_rng(17)
    n = 600
    q_from = scenes.sample_states(art, n, 71)
    q_to = q_from + rng.normal(scale=rng.choice([0.02, 0.3, 1.0], size=(n, 1)), size=(n, 7))
    lim = scenes.joint_limits(art)
    q_to = np.clip(q_to, lim[:, 0], lim[:, 1])
    q_to[:5] = q_from[:5]  # zero-length edges: only q_to is checked
    so2, extent = w.get_motion_space()
    assert so2 == 0 and abs(extent - float(np.sum(lim[:, 1] - lim[:, 0]))) < 1e-12
    valid, first, segs = w.check_motion_batch(q_from, q_to)
    rv, rf, rs = _motion_reference(q_from, q_to, 0.01 * extent, ow(3))
    np.testing.assert_array_equal(segs, rs)
    np.testing.assert_array_equal(valid, rv)
    np.testing.assert_array_equal(first, rf)
    assert 0 < valid.sum() < n


# ------------------------------------------ FCL closed-form pairs (attached bodies)
def _oracle_T(pose):
    from oracle import model as M
    return (M.quat_to_mat(*[float(v) for v in pose[3:]]), [float(v) for v in pose[:3]])


def test_attached_box_in_box_scene_matches_oracle():
    """collision_avoidance.py:87-90: a box attached to the hand in the box
    scene -> Box-Box pairs take FCL's boxBox2 closed form, Box-Convex MPR."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    pose = [0.0, 0.0, 0.14, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("held", pymp.fcl.Box([0.04, 0.04, 0.12]), "panda", 8, pose, ["panda_hand"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=base.scene,
                            attached=[("held", 8, M.BoxGeom((0.04, 0.04, 0.12)), _oracle_T(pose))],
                            allowed=[("panda_hand", "held"), ("panda_link0", "table")])
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == o2.pair_names()
    q = Wd.sample_q(base.art, 30000, 18)
    f, m = w.collide_batch(q)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    w.set_small_batch_max(1 << 20)  # the same batch through the one-launch latency path
    f2, m2 = w.collide_batch(q)
    np.testing.assert_array_equal(f2, fo)
    np.testing.assert_array_equal(m2, mo)
    held = [k for k, i in enumerate(w.get_collision_pair_info()) if i[3] == "held" or i[4] == "held"]
    box_box = [k for k in held if w.get_collision_pair_info()[k][0] != "self"]
    hits = [(mo[:, k >> 5] >> (k & 31)) & 1 for k in box_box]
    assert sum(int(h.sum()) for h in hits) > 0  # the closed form is exercised with both outcomes


@pytest.mark.parametrize("server", [1, 0])
@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_latency_path_matches_oracle(cfg, server, monkeypatch):
    """Host batches up to the small-batch limit run as one small_kernel launch
    (one wave per pair x 64-config tile, bounding-sphere test, MPR / closed
    forms), up to 32 states (MPG_SMALL_SERVER_MAX) through the resident
    latency server (MPG_SMALL_SERVER): bit-exact with the oracle and with the
    two-phase pipeline.  With the server on, the batches of at most 32 states
    really went through it (latency_server_stats: served, never fallen back)."""
    monkeypatch.setenv("MPG_SMALL_SERVER", str(server))
    monkeypatch.setenv("MPG_SMALL_SERVER_MAX", "32")
    w, art = scenes.world(cfg)
    q = Wd.sample_q(ow(cfg).art, 20000, 40 + cfg)
    fo, mo = ow(cfg).collide_batch(q, nthreads=NTHREADS)
    w.set_small_batch_max(1 << 20)
    f, m = w.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    w.set_small_batch_max(1024)
    for n in (1, 2, 3, 5, 17, 32, 33, 63, 64, 65, 1000, 1024, 1025):
        f, m = w.collide_batch(q[:n])
        np.testing.assert_array_equal(f, fo[:n])
        np.testing.assert_array_equal(m, mo[:n])
    # one or two states at a time (isStateValid): rows in the kernel
    # arguments, half-wave FK; colliding and free states both
    for i in range(0, 400, 2):
        f, m = w.collide_batch(q[i:i + 1])
        np.testing.assert_array_equal(f, fo[i:i + 1])
        np.testing.assert_array_equal(m, mo[i:i + 1])
        f, m = w.collide_batch(q[i:i + 2])
        np.testing.assert_array_equal(f, fo[i:i + 2])
        np.testing.assert_array_equal(m, mo[i:i + 2])
    assert 0 < fo[:400].sum() < 400
    for n in (4, 7, 16, 32):  # served batches of several states (32: with MPG_SMALL_SERVER_MAX=32)
        for i in range(0, 160, n):
            f, m = w.collide_batch(q[i:i + n])
            np.testing.assert_array_equal(f, fo[i:i + n])
            np.testing.assert_array_equal(m, mo[i:i + n])
    st = w.latency_server_stats()
    if server:
        # every host batch of <= 32 states above: 6 + 400 + (40 + 23 + 10 + 5)
        assert st["state"] == "in_use" and st["fallbacks"] == 0, st
        assert st["served"] == 484 and st["starts"] >= 1, st
    else:
        assert st == {"served": 0, "starts": 0, "fallbacks": 0, "state": "unused"}, st
    w.set_small_batch_max(0)
    f, m = w.collide_batch(q[:1000])
    np.testing.assert_array_equal(f, fo[:1000])
    np.testing.assert_array_equal(m, mo[:1000])


def test_latency_server_idle_restart_and_teardown(monkeypatch):
    """The resident server leaves after its idle time and is started again by
    the next request; worlds destroyed with their server resident; two
    worlds' servers side by side."""
    import gc
    import time as _t
    monkeypatch.setenv("MPG_SMALL_SERVER", "1")
    monkeypatch.setenv("MPG_SMALL_SERVER_IDLE_US", "200")
    w, art = scenes.world(3)
    w2, _ = scenes.world(3)
    q = Wd.sample_q(ow(3).art, 64, 77)
    fo, mo = ow(3).collide_batch(q, nthreads=NTHREADS)
    for k in range(64):
        for ww in (w, w2):
            f, m = ww.collide_batch(q[k:k + 1])
            np.testing.assert_array_equal(f, fo[k:k + 1])
            np.testing.assert_array_equal(m, mo[k:k + 1])
        if k % 8 == 0:
            _t.sleep(0.002)  # > idle: the servers have left
    for ww in (w, w2):  # every request was answered by the server, restarted after each idle exit
        st = ww.latency_server_stats()
        assert st["served"] == 64 and st["fallbacks"] == 0 and st["state"] == "in_use", st
        assert st["starts"] >= 8, st
    del w, w2
    gc.collect()


def test_spheres_closed_forms_match_oracle():
    """Sphere obstacles + an attached sphere: Sphere-Sphere and Sphere-Box
    closed forms, Sphere-Convex MPR."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    rng = np.random.default_rng(55)
    spheres = []
    for k in range(4):
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        r = float(rng.uniform(0.05, 0.15))
        w.add_normal_object(f"ball{k}", pymp.fcl.CollisionObject(pymp.fcl.Sphere(r), list(c), [1, 0, 0, 0]))
        spheres.append((f"ball{k}", M.SphereGeom(r), _oracle_T(list(c) + [1.0, 0.0, 0.0, 0.0])))
    pose = [0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("orb", pymp.fcl.Sphere(0.05), "panda", 8, pose, ["panda_hand"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + spheres,
                            attached=[("orb", 8, M.SphereGeom(0.05), _oracle_T(pose))],
                            allowed=[("panda_hand", "orb"), ("panda_link0", "table")])
    assert sorted((i[3], i[4]) for i in w.get_collision_pair_info()) == sorted(o2.pair_names())
    order = {pn: k for k, pn in enumerate(o2.pair_names())}
    perm = [order[(i[3], i[4])] for i in w.get_collision_pair_info()]
    q = Wd.sample_q(base.art, 30000, 19)
    f, m = w.collide_batch(q)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    bits = lambda M_, P: np.stack([(M_[:, p >> 5] >> (p & 31)) & 1 for p in P], 1)
    np.testing.assert_array_equal(bits(m, range(len(perm))), bits(mo, perm))
    w.set_small_batch_max(1 << 20)  # closed forms through the latency path
    f2, m2 = w.collide_batch(q)
    np.testing.assert_array_equal(f2, fo)
    np.testing.assert_array_equal(bits(m2, range(len(perm))), bits(mo, perm))
    for i in range(0, 600, 3):  # ... and through the latency server (attached sphere included)
        f3, m3 = w.collide_batch(q[i:i + 3])
        np.testing.assert_array_equal(f3, fo[i:i + 3])
        np.testing.assert_array_equal(bits(m3, range(len(perm))), bits(mo[i:i + 3], perm))


# ------------------------------------------------------------------- distance
@pytest.mark.parametrize("cfg", [3, 4])
def test_distance_batch_matches_oracle(cfg):
    """Batched distanceSelf/distanceOthers vs the oracle (the same float
    libccd GJK and closed forms restated): every distance and argmin pair
    equal, -1 exactly on penetration; a penetrating pair implies collide(),
    the converse up to float MPR's false hits (< 1.86 cm)."""
    w, art = scenes.world(cfg)
    q = scenes.sample_states(art, 4000, 90 + cfg)
    ds, ps, do, po = w.distance_batch(q)
    rs, rps, ro, rpo = ow(cfg).distance_batch(q)
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
    np.testing.assert_array_equal(ps, rps)
    np.testing.assert_array_equal(po, rpo)
    f, _ = w.collide_batch(q)
    pen = (ds == -1.0) | (do == -1.0)
    assert not (pen & ~f.astype(bool)).any()
    odd = ~pen & f.astype(bool)
    assert (np.minimum(ds, do)[odd] < 0.0186).all()


def test_scalar_distance_api():
    w, art = scenes.world(3)
    q = scenes.sample_states(art, 16, 5)
    rs, rps, ro, rpo = ow(3).distance_batch(q)
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    for i in range(len(q)):
        w.set_qpos_all(list(q[i]))
        s, o, full = w.self_distance(), w.distance_with_others(), w.distance_full()
        assert abs(s.min_distance - rs[i]) < 1e-9 and (s.link_name1, s.link_name2) == names[rps[i]]
        assert abs(o.min_distance - ro[i]) < 1e-9 and (o.link_name1, o.link_name2) == names[rpo[i]]
        assert s.distance_type == "self" and o.distance_type == "articulation_sceneobject"
        assert full.min_distance == min(s.min_distance, o.min_distance) == w.distance()
    with pytest.raises(NotImplementedError):  # FCL's own EPA (GST_INDEP signed) is not restated
        w.self_distance(pymp.fcl.DistanceRequest(enable_signed_distance=True,
                                                 gjk_solver_type=pymp.fcl.GJKSolverType.GST_INDEP))


def test_fcl_distance_free_function():
    a = pymp.fcl.CollisionObject(pymp.fcl.Box([1.0, 1.0, 1.0]), [0, 0, 0], [1, 0, 0, 0])
    b = pymp.fcl.CollisionObject(pymp.fcl.Box([1.0, 1.0, 1.0]), [1.5, 1.5, 0.0], [1, 0, 0, 0])
    # libccd's GJK in float (ccd_real_t, FCL 0.7.0): sqrt(0.5) to ~1e-8
    assert abs(pymp.fcl.distance(a, b).min_distance - np.sqrt(0.5)) < 1e-6
    c = pymp.fcl.CollisionObject(pymp.fcl.Sphere(0.25), [1.0, 0.0, 0.0], [1, 0, 0, 0])
    assert abs(pymp.fcl.distance(c, a).min_distance - 0.25) < 1e-6
    d = pymp.fcl.CollisionObject(pymp.fcl.Box([1.0, 1.0, 1.0]), [0.9, 0.2, 0.1], [1, 0, 0, 0])
    assert pymp.fcl.distance(a, d).min_distance == -1.0


# ------------------------------------------------------------------- contacts
def test_contacts_match_oracle():
    """enable_contact=True: libccd MPR penetration (depth, normal, position)
    of every reported pair equals the oracle's restatement within 1e-9 (the
    north star's bar vs FCL is 1e-5)."""
    import ctypes
    from mplib_amd import _capi
    d = dw(3)
    q = Wd.sample_q(ow(3).art, 3000, 33)
    n, P = len(q), len(ow(3).pairs)
    flags = np.zeros(n, np.uint8)
    masks = np.zeros((n, d.mask_words), np.uint32)
    depth, normal, pos = np.zeros((n, P)), np.zeros((n, P, 3)), np.zeros((n, P, 3))
    L = _capi.lib()
    v = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    _capi.check(L.mpg_collide_contacts(d.handle, v(np.ascontiguousarray(q)), n, 0, v(flags), v(masks), v(depth),
                                       v(normal), v(pos), _capi.MPG_MEM_HOST, None), "mpg_collide_contacts")
    hit, rd, rn, rp = ow(3).contact_batch(q)
    fo, mo = ow(3).collide_batch(q)
    np.testing.assert_array_equal(flags, fo)
    np.testing.assert_array_equal(masks, mo)
    h = hit.astype(bool)
    assert h.sum() > 1000
    np.testing.assert_allclose(depth[h], rd[h], atol=1e-9)
    np.testing.assert_allclose(normal[h], rn[h], atol=1e-9)
    np.testing.assert_allclose(pos[h], rp[h], atol=1e-9)
    assert not depth[~h].any() and not normal[~h].any()


def test_contacts_scalar_api():
    w, art = scenes.world(3)
    q = Wd.sample_q(ow(3).art, 32, 34)
    hit, rd, rn, rp = ow(3).contact_batch(q)
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    req = pymp.fcl.CollisionRequest(enable_contact=True)
    for i in range(len(q)):
        w.set_qpos_all(list(q[i]))
        got = {(c.link_name1, c.link_name2): c.res.get_contacts()[0] for c in w.collide_full(req)}
        exp = {names[p]: p for p in np.nonzero(hit[i])[0]}
        assert set(got) == set(exp)
        for k, p in exp.items():
            c = got[k]
            assert abs(c.penetration_depth - rd[i, p]) < 1e-9
            np.testing.assert_allclose(c.normal, rn[i, p], atol=1e-9)
            np.testing.assert_allclose(c.pos, rp[i, p], atol=1e-9)


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


def test_closed_form_contacts_attached_box_scene():
    """collision_avoidance.py:87-90's attached box with enable_contact=True:
    the held box against the scene boxes takes boxBox2's contact path
    (face-face clipping, edge-edge closest points), the other pairs MPR
    penetration; every reported contact equals the oracle's within 1e-9."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    pose = [0.0, 0.0, 0.14, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("held", pymp.fcl.Box([0.04, 0.04, 0.12]), "panda", 8, pose, ["panda_hand"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=base.scene,
                            attached=[("held", 8, M.BoxGeom((0.04, 0.04, 0.12)), _oracle_T(pose))],
                            allowed=[("panda_hand", "held"), ("panda_link0", "table")])
    q = Wd.sample_q(base.art, 30000, 18)
    _, mo = o2.collide_batch(q, nthreads=NTHREADS)
    bb = [k for k, (a, b) in enumerate(o2.pair_names()) if a == "held"]
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in bb], 1), 1))[0]
    assert len(sel) >= 20
    q = np.concatenate([q[sel[:150]], q[:20]])
    hit = _check_scalar_contacts(w, o2, q)
    assert hit[:, bb].sum() >= 20


def test_closed_form_contacts_spheres():
    """Sphere obstacles + an attached sphere with enable_contact=True:
    sphereSphereIntersect / sphereBoxIntersect contacts (both argument
    orders) and MPR for sphere-convex, vs the oracle within 1e-9."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    rng = np.random.default_rng(55)
    spheres = []
    for k in range(4):
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        r = float(rng.uniform(0.05, 0.15))
        w.add_normal_object(f"ball{k}", pymp.fcl.CollisionObject(pymp.fcl.Sphere(r), list(c), [1, 0, 0, 0]))
        spheres.append((f"ball{k}", M.SphereGeom(r), _oracle_T(list(c) + [1.0, 0.0, 0.0, 0.0])))
    pose = [0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("orb", pymp.fcl.Sphere(0.05), "panda", 8, pose, ["panda_hand"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + spheres,
                            attached=[("orb", 8, M.SphereGeom(0.05), _oracle_T(pose))],
                            allowed=[("panda_hand", "orb"), ("panda_link0", "table")])
    q = Wd.sample_q(base.art, 30000, 19)
    _, mo = o2.collide_batch(q, nthreads=NTHREADS)
    orb = [k for k, (a, b) in enumerate(o2.pair_names()) if a == "orb"]
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in orb], 1), 1))[0]
    assert len(sel) >= 20
    hit = _check_scalar_contacts(w, o2, q[sel[:150]])
    assert hit[:, orb].sum() >= 20


def test_closed_form_contacts_capsules_cylinders():
    """The capsule / cylinder world of test_capsule_cylinder_worlds_match_oracle
    with enable_contact=True: sphere-capsule / sphere-cylinder contacts (both
    argument orders, flipNormal) and MPR for convex-capsule, capsule-capsule;
    every reported contact within 1e-9 of the oracle."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    rng = np.random.default_rng(77)
    extra = []
    for k in range(6):
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        r, lz = float(rng.uniform(0.03, 0.08)), float(rng.uniform(0.1, 0.3))
        if k < 2:
            g, og, name = pymp.fcl.Capsule(r, lz), M.CapsuleGeom(r, lz), f"cap{k}"
        elif k < 4:
            g, og, name = pymp.fcl.Cylinder(r, lz), M.CylinderGeom(r, lz), f"cyl{k}"
        else:
            g, og, name = pymp.fcl.Sphere(r), M.SphereGeom(r), f"ball{k}"
        w.add_normal_object(name, pymp.fcl.CollisionObject(g, list(c), list(q)))
        extra.append((name, og, _oracle_T(list(c) + list(q))))
    p_orb = [0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0]
    p_rod = [0.0, 0.05, 0.0, 0.7071067811865476, 0.7071067811865476, 0.0, 0.0]
    w.attach_object("orb", pymp.fcl.Sphere(0.05), "panda", 8, p_orb, ["panda_hand"])
    w.attach_object("rod", pymp.fcl.Capsule(0.02, 0.2), "panda", 6, p_rod, ["panda_link6", "panda_link7"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + extra,
                            attached=[("orb", 8, M.SphereGeom(0.05), _oracle_T(p_orb)),
                                      ("rod", 6, M.CapsuleGeom(0.02, 0.2), _oracle_T(p_rod))],
                            allowed=[("panda_hand", "orb"), ("panda_link6", "rod"), ("panda_link7", "rod"),
                                     ("panda_link0", "table")])
    q = Wd.sample_q(base.art, 30000, 23)
    _, mo = o2.collide_batch(q, nthreads=NTHREADS)
    cf = [k for k, (a, b) in enumerate(o2.pair_names())
          if (a == "orb" and b[:3] in ("cap", "cyl")) or (a == "rod" and b.startswith("ball"))]
    assert cf
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in cf], 1), 1))[0]
    assert len(sel) >= 5
    hit = _check_scalar_contacts(w, o2, np.concatenate([q[sel[:150]], q[:20]]))
    assert hit[:, cf].sum() >= 5


# ------------------------------------------------------------ scale / streams
def test_chunked_batch_across_workspace_chunks():
    """Batches larger than one workspace chunk (2^20 configurations) run as
    consecutive chunks on the stream; results stay bit-exact."""
    w, art = scenes.world(2)
    q = scenes.sample_states(art, (1 << 20) + 4097, 123)
    f, m = w.collide_batch(q)
    fo, mo = ow(2).collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)


def test_concurrent_streams_do_not_share_workspace():
    torch = pytest.importorskip("torch")
    d = dw(3)
    qs = [Wd.sample_q(ow(3).art, 50000, 200 + k) for k in range(3)]
    streams = [torch.cuda.Stream() for _ in qs]
    outs = []
    for q, s in zip(qs, streams):
        qd = torch.from_numpy(q).cuda()
        fd = torch.zeros(len(q), dtype=torch.uint8, device="cuda")
        md = torch.zeros((len(q), d.mask_words), dtype=torch.int32, device="cuda")
        d.collide_batch(qd, fd, md, stream=s.cuda_stream)
        outs.append((qd, fd, md))
    torch.cuda.synchronize()
    for q, (_, fd, md) in zip(qs, outs):
        fo, mo = ow(3).collide_batch(q, nthreads=NTHREADS)
        np.testing.assert_array_equal(fd.cpu().numpy(), fo)
        np.testing.assert_array_equal(md.cpu().numpy().view(np.uint32), mo)


def test_two_threads_overlapped_launches_race_free():
    """Two host threads, each on its own torch stream, each launching
    >= 2^19-configuration batches (the overlapped two-stream path) whose input
    a copy kernel on that stream produced just before: per-call fork/join
    events keep each call's side half ordered after its own stream only
    (include/mpgpu.h thread-safety contract)."""
    import threading
    torch = pytest.importorskip("torch")
    d = dw(3)
    n = 1 << 19
    qs = [[Wd.sample_q(ow(3).art, n, 300 + 10 * t + k) for k in range(2)] for t in range(2)]
    srcs = [[torch.from_numpy(q).cuda() for q in row] for row in qs]
    torch.cuda.synchronize()
    outs = [[None, None], [None, None]]
    errs = []

    def run(t):
        try:
            s = torch.cuda.Stream()
            for k in range(2):
                with torch.cuda.stream(s):
                    qd = srcs[t][k].clone()  # produced on s right before the call
                    fd = torch.empty(n, dtype=torch.uint8, device="cuda")
                    md = torch.empty((n, d.mask_words), dtype=torch.int32, device="cuda")
                d.collide_batch(qd, fd, md, stream=s.cuda_stream)
                outs[t][k] = (qd, fd, md)
            s.synchronize()
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    torch.cuda.synchronize()
    for t in range(2):
        for k in range(2):
            fo, mo = ow(3).collide_batch(qs[t][k], nthreads=NTHREADS)
            np.testing.assert_array_equal(outs[t][k][1].cpu().numpy(), fo)
            np.testing.assert_array_equal(outs[t][k][2].cpu().numpy().view(np.uint32), mo)


def test_bench_two_ranks_gloo_one_gpu():
    """bench.py's multi-rank path (barrier, max over ranks, weak scaling) with
    two ranks sharing this box's GPU over gloo."""
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MPLIB_AMD_DIST_BACKEND="gloo")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "2", "--steps", "3", "--warmup", "1", "--per-gpu", "65536", "--cpu-sample", "0"],
                         env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["value"] > 0
    assert r["config"]["configs_per_gpu"] == 65536


@pytest.mark.gpu
def test_bench_gpus2_self_launch_gloo_one_gpu():
    """`python bench.py --gpus 2` with no launcher starts its two ranks itself
    (here sharing this box's GPU over gloo) and reports n_gpus 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MPLIB_AMD_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup",
                          "1", "--per-gpu", "65536", "--cpu-sample", "0"],
                         env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["value"] > 0


@pytest.mark.gpu
def test_bench_one_rank_nccl_gather():
    """RCCL on hardware: one rank launched by torch.distributed.run with the
    nccl backend (RCCL) initialises its communicator and times the all-gather
    of flags + pair masks and of the distance results (--gather)."""
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "MPLIB_AMD_DIST_BACKEND"}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "1", "--steps", "3", "--warmup", "1", "--per-gpu", "65536", "--cpu-sample", "0",
                          "--gather"], env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["gather_ms"] > 0
    assert r["gather_bytes_per_rank"] == 65536 * (1 + 4 * r["config"]["mask_words"])
    # and the distance results (minima + pair indices of both groups)
    assert r["gather_distance_ms"] > 0 and r["gather_distance_bytes_per_rank"] == 65536 * 24


# --------------------------------------------------------------- point clouds
@pytest.mark.parametrize("kind", ["floor", "blue"])
def test_point_cloud_world_matches_oracle(kind):
    """add_point_cloud -> fcl::OcTree: (link, cloud) pairs through the device
    octree test (grid cells -> obbDisjoint -> box-first MPR / closed forms)
    on both the pipeline and the latency path, bit-exact with the oracle."""
    w, art = scenes.cloud_world(kind)
    ow_ = Wd.oracle_cloud_world(kind)
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == ow_.pair_names()
    q = Wd.sample_q(ow_.art, 20000, 31)
    fo, mo = ow_.collide_batch(q, nthreads=NTHREADS)
    w.set_small_batch_max(0)
    f, m = w.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    w.set_small_batch_max(1 << 20)
    f, m = w.collide_batch(q)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)


def test_point_cloud_known_answers_and_unsupported_queries():
    w, art = scenes.cloud_world("floor")
    w.set_qpos_all(scenes.FLOOR_COLLIDING)
    hits = [r for r in w.collide_with_others() if r.object_name2 == "scene_pcd"]
    assert len(hits) >= 2  # detect_collision.py: several joints dip below the floor
    w.set_qpos_all(Wd.KAT_FREE)
    assert w.collide_with_others() == []
    assert w.collide(pymp.fcl.CollisionRequest(enable_contact=True)) is False
    assert w.collide_full(pymp.fcl.CollisionRequest(enable_contact=True)) == []


@pytest.mark.parametrize("cloud", ["floor", "blue"])
def test_point_cloud_contacts_match_oracle(cloud):
    """enable_contact=True against a point cloud: the first leaf of the
    traversal that intersects the shape gives the contact (leaf box first:
    boxBox2 / sphereBox flipped / MPR penetration), the tree as the
    contact's o1; equal to the oracle within 1e-9."""
    w, art = scenes.cloud_world(cloud)
    o = Wd.oracle_cloud_world(cloud)
    q = scenes.sample_states(art, 4000, 98)
    _, mo = o.collide_batch(q, nthreads=NTHREADS)
    pc = [k for k, (a, b) in enumerate(o.pair_names()) if b == "scene_pcd"]
    sel = np.nonzero(np.any(np.stack([(mo[:, k >> 5] >> (k & 31)) & 1 for k in pc], 1), 1))[0]
    assert len(sel) >= 5
    hit = _check_scalar_contacts(w, o, q[sel[:40]])
    assert hit[:, pc].sum() >= 5


@pytest.mark.parametrize("cloud,n", [("floor", 96), ("blue", 512)])
def test_point_cloud_distance_matches_oracle(cloud, n):
    """distance to a point cloud (fcl::distance(shape, OcTree): the minimum
    over the occupied leaf boxes of GJK(leaf box, shape)): batched and scalar
    distances equal the oracle's within 1e-9, argmin pair equal."""
    w, art = scenes.cloud_world(cloud)
    o = Wd.oracle_cloud_world(cloud)
    q = scenes.sample_states(art, n, 97)
    ds, ps, do, po = w.distance_batch(q)
    rs, rps, ro, rpo = o.distance_batch(q)
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
    assert (ps == rps).mean() > 0.99 and (po == rpo).mean() > 0.99
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    if cloud == "floor":  # the floor is the nearest object for most configurations
        assert np.mean([names[p][1] == "scene_pcd" for p in po]) > 0.5
    for i in range(4):
        w.set_qpos_all(list(q[i]))
        r = w.distance_with_others()
        assert abs(r.min_distance - ro[i]) < 1e-9 and (r.link_name1, r.link_name2) == names[rpo[i]]


def test_attached_box_against_point_cloud():
    """An attached box (collision_avoidance.py:87-90) against the blue-cube
    cloud: leaf boxes meet it through FCL's boxBox2 closed form."""
    import oracle
    from oracle import model as M
    w, art = scenes.cloud_world("blue")
    pose = [0.0, 0.0, 0.14, 1.0, 0.0, 0.0, 0.0]
    w.attach_object("held", pymp.fcl.Box([0.04, 0.04, 0.12]), "panda", 8, pose, ["panda_hand"])
    base = Wd.oracle_cloud_world("blue")
    o2 = oracle.OracleWorld(base.art, scene=base.scene,
                            attached=[("held", 8, M.BoxGeom((0.04, 0.04, 0.12)), _oracle_T(pose))],
                            allowed=[("panda_hand", "held"), ("panda_link0", "table")])
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == o2.pair_names()
    q = Wd.sample_q(base.art, 20000, 32)
    f, m = w.collide_batch(q)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    k = o2.pair_names().index(("held", "scene_pcd"))
    assert int(((mo[:, k >> 5] >> (k & 31)) & 1).sum()) > 0


def test_capsule_cylinder_worlds_match_oracle():
    """Capsule / cylinder obstacles and attachments: convex-capsule and
    capsule-capsule through MPR, sphere-capsule / sphere-cylinder (both
    argument orders) through FCL's closed forms."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    rng = np.random.default_rng(77)
    extra = []
    for k in range(6):
        c = rng.uniform([0.2, -0.4, 0.1], [0.7, 0.4, 0.7])
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        r, lz = float(rng.uniform(0.03, 0.08)), float(rng.uniform(0.1, 0.3))
        if k < 2:
            g, og, name = pymp.fcl.Capsule(r, lz), M.CapsuleGeom(r, lz), f"cap{k}"
        elif k < 4:
            g, og, name = pymp.fcl.Cylinder(r, lz), M.CylinderGeom(r, lz), f"cyl{k}"
        else:
            g, og, name = pymp.fcl.Sphere(r), M.SphereGeom(r), f"ball{k}"
        w.add_normal_object(name, pymp.fcl.CollisionObject(g, list(c), list(q)))
        extra.append((name, og, _oracle_T(list(c) + list(q))))
    p_orb = [0.0, 0.0, 0.12, 1.0, 0.0, 0.0, 0.0]
    p_rod = [0.0, 0.05, 0.0, 0.7071067811865476, 0.7071067811865476, 0.0, 0.0]
    w.attach_object("orb", pymp.fcl.Sphere(0.05), "panda", 8, p_orb, ["panda_hand"])
    w.attach_object("rod", pymp.fcl.Capsule(0.02, 0.2), "panda", 6, p_rod, ["panda_link6", "panda_link7"])
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=list(base.scene) + extra,
                            attached=[("orb", 8, M.SphereGeom(0.05), _oracle_T(p_orb)),
                                      ("rod", 6, M.CapsuleGeom(0.02, 0.2), _oracle_T(p_rod))],
                            allowed=[("panda_hand", "orb"), ("panda_link6", "rod"), ("panda_link7", "rod"),
                                     ("panda_link0", "table")])
    order = {pn: k for k, pn in enumerate(o2.pair_names())}
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    assert sorted(names) == sorted(o2.pair_names())
    perm = [order[n] for n in names]
    q = Wd.sample_q(base.art, 30000, 23)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    bits = lambda M_, P: np.stack([(M_[:, p >> 5] >> (p & 31)) & 1 for p in P], 1)
    for small in (0, 1 << 20):
        w.set_small_batch_max(small)
        f, m = w.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(bits(m, range(len(perm))), bits(mo, perm))
    hit = bits(mo, perm)
    # every closed-form class is exercised (oracle counts for this sample: 64, 65, 65, 63)
    for pair in [("orb", "cap0"), ("orb", "cyl2"), ("rod", "ball4"), ("rod", "cap0")]:
        assert hit[:, names.index(pair)].sum() > 0, pair
    assert int(hit.sum()) > 0


def test_big_walk_hulls_match_oracle(monkeypatch):
    """a 302-vertex cone (cell lists of ~300 rim vertices) and a
    770-vertex sphere (above the 512-vertex direction-table limit: every
    support climbs) as FCL neighbour-walk obstacles -- both batch paths and
    the latency server, every flag and pair bit vs the oracle."""
    monkeypatch.setenv("MPG_SMALL_SERVER", "1")
    o = Wd.big_hull_world()
    d = DeviceWorld(Wd.desc_arrays(o))
    for n in (300, 1 << 14):
        q = Wd.sample_q(o.art, n, 31 + n)
        f, m = d.collide_batch(q)
        fo, mo = o.collide_batch(q, nthreads=NTHREADS)
        assert fo.mean() > 0.05
        np.testing.assert_array_equal(f, fo)
        np.testing.assert_array_equal(m, mo)
        if n == 300:  # batches of 1, 3 and 16 states: the latency server's waves climb side by side
            for k in (1, 3, 16):
                for i in range(0, 300, k):
                    f, m = d.collide_batch(q[i:i + k])
                    np.testing.assert_array_equal(f, fo[i:i + k])
                    np.testing.assert_array_equal(m, mo[i:i + k])


def test_huge_walk_hull_matches_oracle(monkeypatch):
    """a watertight hull above 4096 vertices (a 6322-vertex UV
    sphere) is accepted -- its neighbour walk keeps the visited set in a
    pooled global slot instead of the per-wave LDS bitset -- and every flag
    and pair bit equals the oracle's walk on both batch paths and the
    latency server's batches of 1 and 16 states."""
    monkeypatch.setenv("MPG_SMALL_SERVER", "1")
    o = Wd.huge_hull_world()
    assert len(o.scene[0][1].vertices) > 4096
    d = DeviceWorld(Wd.desc_arrays(o))
    q = Wd.sample_q(o.art, 4000, 808)
    f, m = d.collide_batch(q)
    fo, mo = o.collide_batch(q, nthreads=NTHREADS)
    k = [i for i, pn in enumerate(o.pair_names()) if pn[1] == "huge_ball"]
    assert sum(int(((mo[:, p >> 5] >> (p & 31)) & 1).sum()) for p in k) > 20
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    for bs in (1, 16):
        for i in range(0, 160, bs):
            f, m = d.collide_batch(q[i:i + bs])
            np.testing.assert_array_equal(f, fo[i:i + bs])
            np.testing.assert_array_equal(m, mo[i:i + bs])


def test_huge_walk_hull_distance_and_contacts():
    """The 6322-vertex sphere of test_huge_walk_hull_matches_oracle through
    the PlanningWorld API: batched distances (GJK on its neighbour-walk
    support, pooled visited sets) equal the oracle's, and contacts of the
    colliding states (MPR penetration) within 1e-9."""
    o = Wd.huge_hull_world()
    V = np.asarray(o.scene[0][1].vertices, np.float64)
    F = np.asarray(o.scene[0][1].faces, np.int32)
    pos = o.scene[0][2][1]
    wxyz = Wd.random_quat(np.random.default_rng(98))  # the pose huge_hull_world draws
    w, _ = scenes.world(2)
    w.add_normal_object("huge_ball", pymp.fcl.CollisionObject(pymp.fcl.Convex(V, F, True), list(pos), list(wxyz)))
    names = [(i[3], i[4]) for i in w.get_collision_pair_info()]
    assert names == o.pair_names()
    q = Wd.sample_q(o.art, 400, 818)
    f, m = w.collide_batch(q)
    fo, mo = o.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    ds, ps, do, po = w.distance_batch(q)
    rs, rps, ro, rpo = o.distance_batch(q)
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
    k = [i for i, pn in enumerate(names) if pn[1] == "huge_ball"]
    hitq = np.nonzero(np.any(np.stack([(mo[:, p >> 5] >> (p & 31)) & 1 for p in k], 1), 1))[0]
    assert len(hitq) > 5
    hit, rd, rn, rp = o.contact_batch(q[hitq[:12]])
    req = pymp.fcl.CollisionRequest(enable_contact=True)
    for i, qi in enumerate(q[hitq[:12]]):
        w.set_qpos_all(list(qi))
        got = {(c.link_name1, c.link_name2): c.res.get_contacts()[0] for c in w.collide_full(req)}
        for p in np.nonzero(hit[i])[0]:
            c = got[names[p]]
            assert abs(c.penetration_depth - rd[i, p]) < 1e-9
            np.testing.assert_allclose(c.normal, rn[i, p], atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [5, 300, 5000])
def test_dof0_world_with_moving_links(n):
    """a world whose robot links move but whose move group
    is empty (dof 0, q = NULL): every joint is a constant, every configuration
    is the same state.  Latency path (n <= 1024, host buffers) and pipeline,
    both equal to the oracle at that state."""
    from mplib_amd import _capi as C
    o = ow(3)
    q0 = np.array(Wd.KAT_COLLIDING)
    a = Wd.desc_arrays(o)
    mg = o.art.move_group_qpos_index()
    src = list(a["joint_q_source"])
    const = list(a["joint_q_const"])
    for j, s in enumerate(src):
        if s >= 0:
            const[j] = float(q0[s])
            src[j] = -1
    a.update(joint_q_source=src, joint_q_const=const, dof=0)
    assert len(mg) == 7
    d = DeviceWorld(a)
    fl = np.full(n, 7, np.uint8)
    pm = np.zeros((n, d.mask_words), np.uint32)
    C.check(C.lib().mpg_collide_batch(d._h, None, n, fl.ctypes.data_as(ctypes.c_void_p),
                                      pm.ctypes.data_as(ctypes.c_void_p), C.MPG_MEM_HOST, None), "dof0")
    fo, mo = o.collide_batch(q0[None])
    assert fo[0] == 1
    np.testing.assert_array_equal(fl, np.repeat(fo, n))
    np.testing.assert_array_equal(pm, np.repeat(mo, n, axis=0))


def test_collide_batch_multi_one_device():
    """mpg_collide_batch_multi: one world, and two worlds of the same
    descriptor on the one device of this box (the shards run concurrently
    from two host threads), equal the single-world batch bit for bit; worlds
    of different descriptors are refused."""
    from mplib_amd.batch import collide_batch_multi
    q = Wd.sample_q(ow(3).art, 50001, 515)  # odd: ragged shards
    f, m = dw(3).collide_batch(q)
    for ws in ([dw(3)], [dw(3), DeviceWorld(Wd.desc_arrays(ow(3)))]):
        f2, m2 = collide_batch_multi(ws, q)
        np.testing.assert_array_equal(f2, f)
        np.testing.assert_array_equal(m2, m)
    fo, mo = ow(3).collide_batch(q[:3000], nthreads=NTHREADS)
    np.testing.assert_array_equal(f[:3000], fo)
    with pytest.raises(ValueError, match="descriptor"):
        collide_batch_multi([dw(3), dw(2)], q[:10])
    # same counts, another scene (red_cube moved 1 cm): refused by
    # the snapshot hash, not only by the counts
    import oracle
    scene = Wd.boxes_scene()
    name, geom, pose = scene[1]
    scene[1] = (name, geom, (pose[0], [pose[1][0] + 0.01, pose[1][1], pose[1][2]]))
    other = DeviceWorld(Wd.desc_arrays(oracle.OracleWorld(Wd.panda_articulation(), scene=scene,
                                                          allowed=[("panda_link0", "table")])))
    assert other.mask_words == dw(3).mask_words
    with pytest.raises(ValueError, match="descriptor"):
        collide_batch_multi([dw(3), other], q[:10])


def test_distance_batch_device_matches_host_path():
    """PlanningWorld.distance_batch_device (device buffers, torch's stream):
    the host path's minima, pair indices and nearest points, and
    mplib_amd.dist.distance_sharded_device (world size 1) the same."""
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    from mplib_amd import pymp, scenes
    from mplib_amd.dist import distance_sharded_device
    w, art = scenes.world(3)
    q = scenes.sample_states(art, 3000, 616)
    req = pymp.fcl.DistanceRequest(enable_signed_distance=True)
    ds, ps, do, po, qs, qo = w.distance_batch(q, request=req)
    qt = torch.from_numpy(q).cuda()
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    out, (s, c) = distance_sharded_device(w, qt, request=req, nearest_points=True)
    torch.cuda.synchronize()
    assert (s, c) == (0, len(q))
    np.testing.assert_array_equal(out["d_self"].cpu().numpy(), ds)
    np.testing.assert_array_equal(out["p_self"].cpu().numpy(), ps)
    np.testing.assert_array_equal(out["d_others"].cpu().numpy(), do)
    np.testing.assert_array_equal(out["p_others"].cpu().numpy(), po)
    np.testing.assert_array_equal(out["pts_self"].cpu().numpy(), qs)
    np.testing.assert_array_equal(out["pts_others"].cpu().numpy(), qo)
    dist.destroy_process_group()


def test_collide_batch_multi_device_one_device():
    """mpg_collide_batch_multi_device: a one-world list, and two
    worlds of the same descriptor on the one device of this box with their
    own streams and ragged shards, device-resident, gathered into one device
    buffer: equal the single-world batch bit for bit."""
    torch = pytest.importorskip("torch")
    from mplib_amd.batch import collide_batch_multi_device, shard_range_c
    q = Wd.sample_q(ow(3).art, 40001, 717)
    f, m = dw(3).collide_batch(q)
    qt = torch.from_numpy(q).cuda()
    W = dw(3).mask_words
    for ws in ([dw(3)], [dw(3), DeviceWorld(Wd.desc_arrays(ow(3)))]):
        k = len(ws)
        parts = [shard_range_c(len(q), i, k) for i in range(k)]
        qs = [qt[s:s + c] for s, c in parts]
        fl = [torch.full((c,), 7, dtype=torch.uint8, device="cuda") for _, c in parts]
        mk = [torch.full((c, W), -1, dtype=torch.int32, device="cuda") for _, c in parts]
        streams = [torch.cuda.Stream() for _ in ws]
        gf = torch.zeros(len(q), dtype=torch.uint8, device="cuda")
        gm = torch.zeros((len(q), W), dtype=torch.int32, device="cuda")
        collide_batch_multi_device(ws, qs, fl, mk, [s.cuda_stream for s in streams], gf, gm)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(torch.cat(fl).cpu().numpy(), f)
        np.testing.assert_array_equal(torch.cat(mk).cpu().numpy().view(np.uint32), m)
        np.testing.assert_array_equal(gf.cpu().numpy(), f)
        np.testing.assert_array_equal(gm.cpu().numpy().view(np.uint32), m)
        for w, s in zip(ws, streams):
            w.release_stream(s.cuda_stream)
    # flags only, default streams, no gather
    fl = [torch.zeros(len(q), dtype=torch.uint8, device="cuda")]
    collide_batch_multi_device([dw(3)], [qt], fl)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fl[0].cpu().numpy(), f)


def test_point_cloud_attached_to_the_hand():
    """VERDICT r5 missing #2: an OcTree riding on an attached body
    (attachObject takes any FCL geometry, planning_world.cpp:174-191): a
    point cloud held under panda_hand against the cfg3 boxes and the robot's
    own links -- every flag and pair bit on both batch paths and the distances
    (the octree's pose now per configuration) equal the oracle's."""
    import oracle
    from oracle import model as M
    w, art = scenes.world(3)
    pts = scenes.box_surface_points(np.random.default_rng(11), (0.06, 0.06, 0.05), 800, (0.0, 0.0, 0.0))
    res = 0.005
    pose = [0.0, 0.0, 0.16, 1.0, 0.0, 0.0, 0.0]
    touch = ["panda_hand", "panda_leftfinger", "panda_rightfinger"]
    w.attach_object("held_cloud", pymp.fcl.OcTree(pts, res), "panda", 8, pose, touch)
    base = ow(3)
    o2 = oracle.OracleWorld(base.art, scene=base.scene,
                            attached=[("held_cloud", 8, M.OcTreeGeom(pts, res), _oracle_T(pose))],
                            allowed=[(t, "held_cloud") for t in touch] + [("panda_link0", "table")])
    assert [(i[3], i[4]) for i in w.get_collision_pair_info()] == o2.pair_names()
    q = Wd.sample_q(base.art, 20000, 33)
    f, m = w.collide_batch(q)
    fo, mo = o2.collide_batch(q, nthreads=NTHREADS)
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    k = o2.pair_names().index(("held_cloud", "red_cube"))
    assert ((mo[:, k >> 5] >> (k & 31)) & 1).sum() > 0  # the held cloud does meet the scene
    w.set_small_batch_max(1 << 20)  # the latency path (small_kernel, octree class)
    f2, m2 = w.collide_batch(q[:3000])
    np.testing.assert_array_equal(f2, fo[:3000])
    np.testing.assert_array_equal(m2, mo[:3000])
    ds, ps, do, po = w.distance_batch(q[:1000])
    rs, rps, ro, rpo = o2.distance_batch(q[:1000])
    for d, r in ((ds, rs), (do, ro)):
        np.testing.assert_array_equal(d == -1.0, r == -1.0)
        np.testing.assert_allclose(d, r, rtol=0, atol=1e-9)
    assert (ps == rps).mean() > 0.99 and (po == rpo).mean() > 0.99
