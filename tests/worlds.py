"""Benchmark / parity worlds of BASELINE.json, described with the ORACLE's
independent model loader (test infrastructure).

``desc_arrays(ow)`` turns an ``oracle.OracleWorld`` into the plain-array
``mpg_world_desc`` the C ABI takes, so C-ABI tests can drive the HIP library
with a world that was NOT built by the product's own host code.

Configs (BASELINE.json / SURVEY.md 8(d)):
  cfg1  detect_collision.py single configurations (CPU known answers)
  cfg2  Panda self-collision, 2^16 configs, default_rng(0)
  cfg3  Panda + 10 boxes (collision_avoidance.py scene + 6 synthetic), 2^20, default_rng(1)
  cfg4  Panda + 4 convex hull obstacles, 2^22 sharded, default_rng(2)
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np

import oracle
from oracle import model as M

REF_DATA = "/root/reference/data/panda"
_REPO_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "panda")


def panda_dir() -> str:
    """Panda URDF/SRDF + meshes: the in-repo copy (the reference is absent on the GPU box)."""
    if os.path.exists(os.path.join(_REPO_DATA, "panda.urdf")):
        return _REPO_DATA
    return REF_DATA


PANDA_LINKS = ["panda_link0", "panda_link1", "panda_link2", "panda_link3", "panda_link4", "panda_link5",
               "panda_link6", "panda_link7", "panda_hand", "panda_leftfinger", "panda_rightfinger"]
PANDA_JOINTS = ["panda_joint1", "panda_joint2", "panda_joint3", "panda_joint4", "panda_joint5", "panda_joint6",
                "panda_joint7", "panda_finger_joint1", "panda_finger_joint2"]
# examples/detect_collision.py:25,31
KAT_FREE = [0.0, 0.19, 0.0, -2.61, 0.0, 2.94, 0.78]
KAT_COLLIDING = [0.0, 1.36, 0.0, -3.0, -3.0, 3.0, -1.0]


def panda_articulation(convex: bool = True) -> M.Articulation:
    d = panda_dir()
    return M.Articulation(os.path.join(d, "panda.urdf"), os.path.join(d, "panda.srdf"), PANDA_LINKS,
                          PANDA_JOINTS, convex=convex, move_group="panda_hand")


def _box(side, pos):
    return (M.BoxGeom(tuple(float(s) for s in side)), (list(M.IDENT[0]), [float(p) for p in pos]))


def boxes_scene() -> List[Tuple[str, object, tuple]]:
    """collision_avoidance.py:29-59 boxes (side = 2 x half_size) + 6 synthetic (default_rng(1234))."""
    scene = [("table",) + _box((0.8, 0.8, 0.05), (0.56, 0.0, -0.025)),
             ("red_cube",) + _box((0.04, 0.04, 0.12), (0.7, 0.0, 0.06)),
             ("green_cube",) + _box((0.08, 0.08, 0.01), (0.4, 0.3, 0.005)),
             ("blue_cube",) + _box((0.1, 0.4, 0.2), (0.55, 0.0, 0.1))]
    rng = np.random.default_rng(1234)
    for k in range(6):
        side = rng.uniform(0.02, 0.2, size=3)
        c = rng.uniform([0.2, -0.5, 0.05], [0.8, 0.5, 0.8])
        scene.append((f"box{k}",) + _box(side, c))
    return scene


def random_quat(rng) -> Tuple[float, float, float, float]:
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    return tuple(float(v) for v in q)  # w x y z


def convex_scene(art: M.Articulation) -> List[Tuple[str, object, tuple]]:
    """cfg4: the Panda link3/link5/hand/link0 hulls at fixed random poses (default_rng(4321))."""
    rng = np.random.default_rng(4321)
    pick = {"panda_link3": None, "panda_link5": None, "panda_hand": None, "panda_link0": None}
    for o in art.objects:
        if o.link in pick and pick[o.link] is None:
            pick[o.link] = o.geom
    scene = []
    for k, name in enumerate(["panda_link3", "panda_link5", "panda_hand", "panda_link0"]):
        pos = rng.uniform([0.3, -0.5, 0.0], [0.8, 0.5, 0.7])
        w, x, y, z = random_quat(rng)
        scene.append((f"hull{k}_{name}", pick[name], (M.quat_to_mat(w, x, y, z), [float(v) for v in pos])))
    return scene


def oracle_world(cfg: int, convex: bool = True) -> oracle.OracleWorld:
    if cfg == 7:
        return oracle_world(3, convex=False)
    art = panda_articulation(convex)
    if cfg in (1, 2):
        return oracle.OracleWorld(art)
    if cfg == 3:
        return oracle.OracleWorld(art, scene=boxes_scene(), allowed=[("panda_link0", "table")])
    if cfg == 4:
        return oracle.OracleWorld(art, scene=convex_scene(art))
    if cfg == 6:
        return oracle_cloud_world("floor")
    raise ValueError(cfg)


def oracle_cloud_world(kind: str, resolution: float = 1e-3) -> oracle.OracleWorld:
    """The oracle twin of scenes.cloud_world: the same points, the oracle's
    own octomap restatement (oracle/model.py OcTreeGeom)."""
    from mplib_amd import scenes
    art = panda_articulation()
    cloud = ("scene_pcd", M.OcTreeGeom(scenes.cloud_points(kind), resolution), M.IDENT)
    if kind == "floor":
        return oracle.OracleWorld(art, scene=[cloud])
    return oracle.OracleWorld(art, scene=boxes_scene() + [cloud], allowed=[("panda_link0", "table")])


def sample_q(art: M.Articulation, n: int, seed: int) -> np.ndarray:
    lim = art.joint_limits()[:7]
    return np.random.default_rng(seed).uniform(lim[:, 0], lim[:, 1], size=(n, 7))


CFG_SEED = {2: 0, 3: 1, 4: 2, 7: 7}
CFG_N = {2: 1 << 16, 3: 1 << 20, 4: 1 << 22}


def desc_arrays(ow: oracle.OracleWorld) -> dict:
    """mpg_world_desc arrays from an OracleWorld (moving = robot objects then
    attached bodies; static = scene objects)."""
    art = ow.art
    pin = art.pin
    J = pin.joints[1:]
    mg = art.move_group_qpos_index()
    qsrc, qconst = [], []
    for j in range(1, len(pin.joints)):
        src, const = -1, 0.0
        if j in art.user_joints:
            u = art.user_joints.index(j)
            slot = art.user_vidx[u]
            if slot in mg:
                src = mg.index(slot)
            else:
                const = art.current_qpos[slot]
        qsrc.append(src)
        qconst.append(const)
    geoms = ow.geoms
    gtype, gvs, gnv, gparam, verts, leaves, tris, cfaces = [], [], [], [], [], [], [], []
    nv = 0
    nl = 0
    nt = 0
    for g in geoms:
        if isinstance(g, M.MeshGeom):
            gtype.append(6)
            gvs.append(nv)
            gnv.append(len(g.vertices))
            nv += len(g.vertices)
            verts.append(g.vertices.reshape(-1))
            gparam += [float(nt), float(len(g.faces)), 0.0, 0.0]
            tris.append(np.asarray(g.faces, np.int32).reshape(-1))
            nt += len(g.faces)
        elif isinstance(g, M.OcTreeGeom):
            gtype.append(5)
            gvs.append(0)
            gnv.append(0)
            gparam += [float(nl), float(len(g.leaves)), g.resolution, 0.0]
            leaves.append(g.leaves.reshape(-1))
            nl += len(g.leaves)
        elif isinstance(g, M.ConvexGeom):
            gtype.append(0)
            gvs.append(nv)
            gnv.append(len(g.vertices))
            nv += len(g.vertices)
            verts.append(g.vertices.reshape(-1))
            gparam += [float(len(cfaces)), float(len(g.faces)), 0.0, 0.0]  # FCL layout faces
            for f in g.faces:
                cfaces += [len(f)] + [int(v) for v in f]
        elif isinstance(g, M.SphereGeom):
            gtype.append(2)
            gvs.append(0)
            gnv.append(0)
            gparam += [float(g.radius), 0.0, 0.0, 0.0]
        elif isinstance(g, (M.CapsuleGeom, M.CylinderGeom, M.ConeGeom)):
            gtype.append(3 if isinstance(g, M.CapsuleGeom) else M.GEOM_CONE if isinstance(g, M.ConeGeom) else 4)
            gvs.append(0)
            gnv.append(0)
            gparam += [float(g.radius), float(g.lz), 0.0, 0.0]
        elif isinstance(g, M.TrianglePGeom):
            gtype.append(M.GEOM_TRIANGLE_P)
            gvs.append(nv)
            gnv.append(3)
            nv += 3
            verts.append(g.vertices.reshape(-1))
            gparam += [0.0] * 4
        elif isinstance(g, M.EllipsoidGeom):
            gtype.append(M.GEOM_ELLIPSOID)
            gvs.append(0)
            gnv.append(0)
            gparam += [float(g.radii[0]), float(g.radii[1]), float(g.radii[2]), 0.0]
        else:
            gtype.append(1)
            gvs.append(0)
            gnv.append(0)
            gparam += [float(g.side[0]), float(g.side[1]), float(g.side[2]), 0.0]

    def gi(g):
        return next(i for i, gg in enumerate(geoms) if gg is g)

    n_obj = len(art.objects)
    n_att = len(ow.attached)
    moving_link = list(art.obj_user_link) + [a[1] for a in ow.attached]
    moving_geom = [gi(o.geom) for o in art.objects] + [gi(a[2]) for a in ow.attached]
    moving_offset = [c for o in art.objects for c in list(o.origin[0]) + list(o.origin[1])]
    moving_offset += [c for a in ow.attached for c in list(a[3][0]) + list(a[3][1])]

    def oid(kind, idx):
        if kind == oracle.KIND_ROBOT:
            return idx
        if kind == oracle.KIND_ATTACHED:
            return n_obj + idx
        return n_obj + n_att + idx

    frames = [pin.frames[f] for f in art.link_frames]
    return dict(
        joint_type=[j.jtype for j in J], joint_parent=[j.parent for j in J],
        joint_axis=[c for j in J for c in j.axis],
        joint_placement=[c for j in J for c in list(j.placement[0]) + list(j.placement[1])],
        joint_q_source=qsrc, joint_q_const=qconst, dof=len(mg),
        link_parent=[f.parent for f in frames],
        link_placement=[c for f in frames for c in list(f.placement[0]) + list(f.placement[1])],
        geom_type=gtype, geom_vertex_start=gvs, geom_vertex_count=gnv, geom_param=gparam,
        vertices=np.concatenate(verts) if verts else np.zeros(0),
        moving_link=moving_link, moving_geom=moving_geom, moving_offset=moving_offset,
        static_geom=[gi(s[1]) for s in ow.scene],
        static_transform=[c for s in ow.scene for c in list(s[2][0]) + list(s[2][1])],
        pair_a=[oid(p[0], p[1]) for p in ow.pairs], pair_b=[oid(p[2], p[3]) for p in ow.pairs],
        pair_allowed=[1 if frozenset((p[4], p[5])) in ow.allowed else 0 for p in ow.pairs],
        octree_leaf=np.concatenate(leaves) if leaves else np.zeros(0),
        mesh_triangle=np.concatenate(tris) if tris else np.zeros(0, np.int32),
        convex_face=np.asarray(cfaces, np.int32),
        joint_lower=[j.lower[0] if j.nq == 1 else -np.inf for j in J],
        joint_upper=[j.upper[0] if j.nq == 1 else np.inf for j in J],
    )


def collide_pair(ow: oracle.OracleWorld, ga: int, Ta, gb: int, Tb) -> bool:
    """The oracle's fcl::collide on two posed geometries of ow (SE3 tuples)."""
    import ctypes
    DP = ctypes.POINTER(ctypes.c_double)
    a = np.ascontiguousarray(oracle._se3_flat(Ta), dtype=np.float64)
    b = np.ascontiguousarray(oracle._se3_flat(Tb), dtype=np.float64)
    return bool(oracle.lib().orc_collide_pair(ctypes.byref(ow._w), ga, a.ctypes.data_as(DP), gb,
                                              b.ctypes.data_as(DP)))


def distance_pair(ow: oracle.OracleWorld, ga: int, Ta, gb: int, Tb) -> float:
    """The oracle's fcl::distance on two posed geometries of ow (SE3 tuples)."""
    import ctypes
    DP = ctypes.POINTER(ctypes.c_double)
    a = np.ascontiguousarray(oracle._se3_flat(Ta), dtype=np.float64)
    b = np.ascontiguousarray(oracle._se3_flat(Tb), dtype=np.float64)
    return float(oracle.lib().orc_distance_pair(ctypes.byref(ow._w), ga, a.ctypes.data_as(DP), gb,
                                                b.ctypes.data_as(DP)))


def distance_pair_ex(ow: oracle.OracleWorld, ga: int, Ta, gb: int, Tb, signed: bool = False,
                     nearest_points: bool = False, distance_tolerance: float = 1e-6):
    """The oracle's fcl::distance of two posed geometries with
    DistanceRequest(nearest_points, signed, distance_tolerance): (distance,
    nearest_points[0], nearest_points[1]); RuntimeError where FCL throws."""
    import ctypes
    DP = ctypes.POINTER(ctypes.c_double)
    flat = lambda T: np.ascontiguousarray(T if np.ndim(T) == 1 else oracle._se3_flat(T), dtype=np.float64)  # noqa: E731
    a, b = flat(Ta), flat(Tb)
    pts = np.zeros(6)
    st = ctypes.c_int(0)
    mode = (1 if signed else 0) | (2 if nearest_points else 0)
    d = float(oracle.lib().orc_distance_pair_ex(ctypes.byref(ow._w), ga, a.ctypes.data_as(DP), gb,
                                                b.ctypes.data_as(DP), mode, ctypes.c_double(distance_tolerance),
                                                pts.ctypes.data_as(DP), ctypes.byref(st)))
    if st.value:
        raise RuntimeError("FCL throws on this configuration")
    return d, pts[:3], pts[3:]


def cone_hull(n_rim: int = 300, r: float = 0.12, h: float = 0.25):
    """A watertight triangulated cone: n_rim rim vertices (z = 0), apex, base
    centre.  Its flat base keeps every rim vertex in the walk cells around
    -z (lists of >= 256 entries)."""
    t = 2 * np.pi * np.arange(n_rim) / n_rim
    V = [[r * np.cos(a), r * np.sin(a), 0.0] for a in t] + [[0.0, 0.0, h], [0.0, 0.0, 0.0]]
    apex, ctr = n_rim, n_rim + 1
    F = [(i, (i + 1) % n_rim, apex) for i in range(n_rim)] + [(ctr, (i + 1) % n_rim, i) for i in range(n_rim)]
    return M.ConvexGeom(np.asarray(V, np.float64), F)


def uv_sphere_hull(stacks: int = 24, slices: int = 32, r: float = 0.1):
    """A watertight UV sphere of (stacks - 1) * slices + 2 vertices (770 by
    default: more than the 512-vertex direction-table limit)."""
    V = [[0.0, 0.0, r]]
    for i in range(1, stacks):
        th = np.pi * i / stacks
        for j in range(slices):
            ph = 2 * np.pi * j / slices
            V.append([r * np.sin(th) * np.cos(ph), r * np.sin(th) * np.sin(ph), r * np.cos(th)])
    V.append([0.0, 0.0, -r])
    bot = len(V) - 1

    def ring(i, j):
        return 1 + (i - 1) * slices + j % slices

    F = [(0, ring(1, j), ring(1, j + 1)) for j in range(slices)]
    for i in range(1, stacks - 1):
        for j in range(slices):
            a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j), ring(i + 1, j + 1)
            F += [(a, c, b), (b, c, d)]
    F += [(ring(stacks - 1, j), bot, ring(stacks - 1, j + 1)) for j in range(slices)]
    return M.ConvexGeom(np.asarray(V, np.float64), F)


def huge_hull_world() -> oracle.OracleWorld:
    """Panda + a 6322-vertex UV sphere: an FCL neighbour-walk hull above the
    device's 4096-vertex LDS visited set (wave_walk's pooled global set)."""
    art = panda_articulation()
    rng = np.random.default_rng(98)
    w, x, y, z = random_quat(rng)
    return oracle.OracleWorld(art, scene=[("huge_ball", uv_sphere_hull(80, 80, 0.12),
                                           (M.quat_to_mat(w, x, y, z), [0.4, -0.2, 0.45]))])


def big_hull_world() -> oracle.OracleWorld:
    """Panda + a 302-vertex cone + a 770-vertex sphere (FCL neighbour-walk
    hulls beyond the round-2 device limits), at fixed random poses."""
    art = panda_articulation()
    rng = np.random.default_rng(99)
    scene = []
    for name, g, pos in (("cone", cone_hull(), (0.45, 0.15, 0.3)), ("ball", uv_sphere_hull(), (0.35, -0.3, 0.5))):
        w, x, y, z = random_quat(rng)
        scene.append((name, g, (M.quat_to_mat(w, x, y, z), list(pos))))
    return oracle.OracleWorld(art, scene=scene)
