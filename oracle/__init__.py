"""ORACLE -- CPU parity checker for the mplib_amd batched collide path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package.  The shipped
product (``mplib_amd``) never imports, links or executes anything under
``oracle/``; it fails loudly when its HIP library is missing instead.

* ``oracle/model.py``          -- independent URDF/SRDF/STL -> model restatement
* ``oracle/collide_oracle.c``  -- C restatement of the FK + FCL/libccd MPR +
                                  PlanningWorld pair loops (built into
                                  ``oracle/build/liboracle.so`` by ``make -C oracle``)

Parity status (see DESIGN.md section "Oracle"): the reference (KolinGuo/MPlib
0.1.1) ships no golden vectors for this path and its third-party arithmetic
(FCL 0.7.0, libccd 2.1, pinocchio 2.6.21, Eigen 3.4.0) is absent from this
image, so the restatement is pinned by the reference's own known answers
(examples/detect_collision.py:25,31), the Panda model facts in SURVEY.md 8(a),
and -- for sin/cos -- bit-for-bit agreement with the host libm.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import model as M

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the C restatement (gcc -O2 -ffp-contract=off)."""
    src = os.path.join(_HERE, "collide_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_collide_batch.restype = ctypes.c_int
        _lib.orc_fk_batch.restype = ctypes.c_int
        _lib.orc_collide_pair.restype = ctypes.c_int
        _lib.orc_distance_pair.restype = ctypes.c_double
        _lib.orc_distance_batch.restype = ctypes.c_int
        _lib.orc_distance_batch_ex.restype = ctypes.c_int
        _lib.orc_distance_pair_ex.restype = ctypes.c_double
        _lib.orc_contact_pair.restype = ctypes.c_int
        _lib.orc_contact_batch.restype = ctypes.c_int
        _lib.orc_tri_tri.restype = ctypes.c_int
        _lib.orc_sphere_tri.restype = ctypes.c_int
        _lib.orc_tri_distance.restype = ctypes.c_double
    return _lib


# Oracle variants (DESIGN.md "Oracle variants"): the same restatement built with
# one open arithmetic choice switched, to count how many flags / pair bits each
# choice can change.  Test infrastructure like the rest of this package.
VARIANTS = {
    "ccd_double": ["-DORC_CCD_DOUBLE"],          # libccd built with ENABLE_DOUBLE_PRECISION=ON
    "fcl_linear": ["-DORC_FCL_LINEAR"],          # linear first-maximum convex support (no neighbour walk)
    "pin_cross": ["-DORC_PIN_REVOLUTE_CROSS"],   # column-wise SE3 x TransformRevolute with a cross product
    "eigen_slice": ["-DORC_EIGEN_ORDER=1"],      # Eigen 3.4 SSE2 slice-vectorised 3x3 products
    "eigen_tree": ["-DORC_EIGEN_ORDER=2"],       # Eigen redux-tree order for every coefficient
    "hist": ["-DORC_HIST"],                      # diagnostics: support calls per MPR (orc_hist_read)
}
_variant_libs: Dict[str, ctypes.CDLL] = {}


def variant_lib(name: str):
    """Build (once) and load oracle/build/variants/liboracle_<name>.so.
    ``name`` is a '+'-joined list of VARIANTS keys."""
    if name not in _variant_libs:
        flags = []
        for part in name.split("+"):
            flags += VARIANTS[part]
        src = os.path.join(_HERE, "collide_oracle.c")
        out = os.path.join(_HERE, "build", "variants", f"liboracle_{name}.so")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
            subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-std=c99",
                                   "-D_POSIX_C_SOURCE=200809L", *flags, "-shared", "-o", out, src, "-lm", "-lpthread"])
        L = ctypes.CDLL(out)
        L.orc_collide_batch.restype = ctypes.c_int
        L.orc_fk_batch.restype = ctypes.c_int
        _variant_libs[name] = L
    return _variant_libs[name]


def fcl_convex_neighbors(nv: int, faces) -> Tuple[List[int], bool]:
    """FCL 0.7.0 ``Convex::FindVertexNeighbors`` encoding [ext]: entry i
    (i < nv) is the offset of vertex i's record = [count, sorted neighbours...];
    each face contributes its consecutive edges (and the closing edge).
    Second value: ``ValidateTopology`` passed (every edge shared by exactly two
    faces, every vertex in some face) -- FCL walks neighbours only then."""
    nb = [set() for _ in range(nv)]
    edge_faces: Dict[Tuple[int, int], int] = {}
    for f in faces:
        prev = f[-1]
        for v in f:
            nb[v].add(prev)
            nb[prev].add(v)
            e = (min(v, prev), max(v, prev))
            edge_faces[e] = edge_faces.get(e, 0) + 1
            prev = v
    out = [0] * nv
    for i in range(nv):
        out[i] = len(out)
        out.append(len(nb[i]))
        out.extend(sorted(nb[i]))
    ok = all(len(s) > 0 for s in nb) and all(c == 2 for c in edge_faces.values())
    return out, ok


def tri_tri(P, Q) -> bool:
    """FCL Intersect::intersect_Triangle on two triangles ([3, 3] each)."""
    a = np.ascontiguousarray(P, dtype=np.float64).reshape(9)
    b = np.ascontiguousarray(Q, dtype=np.float64).reshape(9)
    return bool(lib().orc_tri_tri(a.ctypes.data_as(_DP), b.ctypes.data_as(_DP)))


def tri_distance(P, Q) -> float:
    """FCL TriangleDistance::triDistance (PQP TriDist) of two triangles ([3, 3] each)."""
    a = np.ascontiguousarray(P, dtype=np.float64).reshape(9)
    b = np.ascontiguousarray(Q, dtype=np.float64).reshape(9)
    return float(lib().orc_tri_distance(a.ctypes.data_as(_DP), b.ctypes.data_as(_DP)))


def sphere_tri(radius: float, centre, P) -> bool:
    """FCL sphereTriangleIntersect: a sphere at `centre` vs world triangle P."""
    T = np.zeros(12)
    T[[0, 4, 8]] = 1.0
    T[9:] = centre
    a = np.ascontiguousarray(P, dtype=np.float64).reshape(9)
    return bool(lib().orc_sphere_tri(ctypes.c_double(radius), T.ctypes.data_as(_DP), a.ctypes.data_as(_DP)))


_IP = ctypes.POINTER(ctypes.c_int)
_DP = ctypes.POINTER(ctypes.c_double)


class _World(ctypes.Structure):
    _fields_ = [
        ("nj", ctypes.c_int), ("nq_pin", ctypes.c_int),
        ("jtype", _IP), ("jparent", _IP), ("jidx_q", _IP),
        ("jaxis", _DP), ("jplace", _DP),
        ("n_user_joints", ctypes.c_int), ("user_joint", _IP),
        ("nq_user", ctypes.c_int), ("qpos_template", _DP),
        ("dof", ctypes.c_int), ("mg_index", _IP),
        ("n_links", ctypes.c_int), ("link_parent", _IP), ("link_place", _DP),
        ("n_geom", ctypes.c_int), ("geom_type", _IP), ("geom_vstart", _IP), ("geom_nv", _IP),
        ("geom_param", _DP), ("geom_interior", _DP), ("verts", _DP),
        ("n_obj", ctypes.c_int), ("obj_link", _IP), ("obj_geom", _IP), ("obj_origin", _DP),
        ("n_att", ctypes.c_int), ("att_link", _IP), ("att_geom", _IP), ("att_pose", _DP),
        ("n_scene", ctypes.c_int), ("scene_geom", _IP), ("scene_tf", _DP),
        ("n_pairs", ctypes.c_int),
        ("pa_kind", _IP), ("pa_idx", _IP), ("pb_kind", _IP), ("pb_idx", _IP), ("p_allowed", _IP),
        ("oct_leaf", _DP),
        ("mesh_tri", _IP),
        ("conv_nbr", _IP),
        ("bvh", ctypes.c_void_p),
        ("gjk_solver", ctypes.c_int),
    ]


class Stats(ctypes.Structure):
    _fields_ = [("support_calls", ctypes.c_longlong), ("vertex_dots", ctypes.c_longlong),
                ("refine_iters", ctypes.c_longlong), ("mpr_runs", ctypes.c_longlong)]


def _se3_flat(T) -> List[float]:
    return list(T[0]) + list(T[1])


def pose7_to_se3(pose) -> tuple:
    """``posevec_to_transform`` / CollisionObject(p, wxyz) (src/math_utils.cpp:12-18)."""
    p = pose[:3]
    w, x, y, z = pose[3:7]
    return (M.quat_to_mat(float(w), float(x), float(y), float(z)), [float(v) for v in p])


KIND_ROBOT, KIND_ATTACHED, KIND_SCENE = 0, 1, 2


class OracleWorld:
    """A PlanningWorld with one planned articulation, static scene objects,
    attached bodies and an allowed-collision set, evaluated on the CPU.

    Pair-table order follows ``PlanningWorldTpl::selfCollide`` then
    ``collideWithOthers`` (src/planning_world.cpp:277-481); each pair keeps the
    reference's (o1, o2) argument order for ``fcl::collide``.
    """

    def __init__(self, art: M.Articulation, scene: Sequence[Tuple[str, object, tuple]] = (),
                 attached: Sequence[Tuple[str, int, object, tuple]] = (),
                 allowed: Sequence[Tuple[str, str]] = (), gjk_solver: str = "libccd"):
        if gjk_solver not in ("libccd", "indep"):
            raise ValueError(gjk_solver)
        self.gjk_solver = gjk_solver      # CollisionRequest::gjk_solver_type (GST_LIBCCD / GST_INDEP)
        self.art = art
        self.scene = list(scene)          # (name, geom, SE3)
        self.attached = list(attached)    # (name, user link index, geom, SE3 pose)
        self.allowed = {frozenset(p) for p in allowed}
        self._build()

    # ------------------------------------------------------------------
    def _geom_index(self, g, geoms, verts) -> int:
        for i, gg in enumerate(geoms):
            if gg is g:
                return i
        geoms.append(g)
        return len(geoms) - 1

    def _build(self):
        art = self.art
        pin = art.pin
        geoms: List[object] = []
        obj_geom = [self._geom_index(o.geom, geoms, None) for o in art.objects]
        att_geom = [self._geom_index(a[2], geoms, None) for a in self.attached]
        scene_geom = [self._geom_index(s[1], geoms, None) for s in self.scene]
        gtype, gvstart, gnv, gparam, ginterior, verts = [], [], [], [], [], []
        leaves = []
        tris = []
        nbr_all: List[int] = []
        ntris = 0
        nverts = 0
        nleaves = 0
        for g in geoms:
            if isinstance(g, M.ConvexGeom):
                gtype.append(M.GEOM_CONVEX)
                gvstart.append(nverts)
                gnv.append(len(g.vertices))
                nverts += len(g.vertices)
                verts.append(np.asarray(g.vertices, dtype=np.float64).reshape(-1))
                enc, ok = fcl_convex_neighbors(len(g.vertices), g.faces)
                gparam += [float(len(nbr_all)) if ok else -1.0, 0.0, 0.0, 0.0]
                if ok:
                    nbr_all += enc
                ginterior += g.interior
            elif isinstance(g, M.MeshGeom):
                gtype.append(M.GEOM_MESH)
                gvstart.append(nverts)
                gnv.append(len(g.vertices))
                nverts += len(g.vertices)
                verts.append(np.asarray(g.vertices, dtype=np.float64).reshape(-1))
                gparam += [float(ntris), float(len(g.faces)), 0.0, 0.0]
                ginterior += [0.0] * 3
                tris.append(np.asarray(g.faces, dtype=np.int32).reshape(-1))
                ntris += len(g.faces)
            elif isinstance(g, M.BoxGeom):
                gtype.append(M.GEOM_BOX)
                gvstart.append(0)
                gnv.append(0)
                gparam += [float(g.side[0]), float(g.side[1]), float(g.side[2]), 0.0]
                ginterior += [0.0] * 3
            elif isinstance(g, M.OcTreeGeom):
                gtype.append(M.GEOM_OCTREE)
                gvstart.append(0)
                gnv.append(0)
                gparam += [float(nleaves), float(len(g.leaves)), g.resolution, 0.0]
                ginterior += [0.0] * 3
                leaves.append(np.asarray(g.leaves, dtype=np.float64).reshape(-1))
                nleaves += len(g.leaves)
            elif isinstance(g, M.TrianglePGeom):
                gtype.append(M.GEOM_TRIANGLE_P)
                gvstart.append(nverts)
                gnv.append(3)
                nverts += 3
                verts.append(g.vertices.reshape(-1))
                gparam += [0.0] * 4
                ginterior += [0.0] * 3
            elif isinstance(g, M.EllipsoidGeom):
                gtype.append(M.GEOM_ELLIPSOID)
                gvstart.append(0)
                gnv.append(0)
                gparam += [float(g.radii[0]), float(g.radii[1]), float(g.radii[2]), 0.0]
                ginterior += [0.0] * 3
            elif isinstance(g, (M.CapsuleGeom, M.CylinderGeom, M.ConeGeom)):
                gtype.append(M.GEOM_CAPSULE if isinstance(g, M.CapsuleGeom) else
                             M.GEOM_CONE if isinstance(g, M.ConeGeom) else M.GEOM_CYLINDER)
                gvstart.append(0)
                gnv.append(0)
                gparam += [float(g.radius), float(g.lz), 0.0, 0.0]
                ginterior += [0.0] * 3
            elif isinstance(g, M.SphereGeom):
                gtype.append(M.GEOM_SPHERE)
                gvstart.append(0)
                gnv.append(0)
                gparam += [float(g.radius), 0.0, 0.0, 0.0]
                ginterior += [0.0] * 3
            else:
                raise TypeError(f"oracle: unsupported geometry {type(g)}")
        pairs, self.n_self_pairs = self._pair_table()
        self.pairs = pairs
        self.W = max(1, (len(pairs) + 31) // 32)
        allowed = [1 if frozenset((p[4], p[5])) in self.allowed else 0 for p in pairs]

        nj = len(pin.joints) - 1
        J = pin.joints[1:]
        self._keep = []

        def ia(x):
            a = np.ascontiguousarray(np.asarray(x, dtype=np.int32).reshape(-1) if len(x) else np.zeros(1, np.int32))
            self._keep.append(a)
            return a.ctypes.data_as(_IP)

        def da(x):
            a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1) if len(x) else np.zeros(1))
            self._keep.append(a)
            return a.ctypes.data_as(_DP)

        mg = art.move_group_qpos_index()
        w = _World()
        w.nj = nj
        w.nq_pin = pin.nq
        w.jtype = ia([j.jtype for j in J])
        w.jparent = ia([j.parent for j in J])
        w.jidx_q = ia([j.idx_q for j in J])
        w.jaxis = da([c for j in J for c in j.axis])
        w.jplace = da([c for j in J for c in _se3_flat(j.placement)])
        w.n_user_joints = len(art.user_joints)
        w.user_joint = ia(art.user_joints)
        w.nq_user = art.nv
        w.qpos_template = da(art.current_qpos)
        w.dof = len(mg)
        w.mg_index = ia(mg)
        frames = [pin.frames[f] for f in art.link_frames]
        w.n_links = len(frames)
        w.link_parent = ia([f.parent for f in frames])
        w.link_place = da([c for f in frames for c in _se3_flat(f.placement)])
        w.n_geom = len(geoms)
        w.geom_type = ia(gtype)
        w.geom_vstart = ia(gvstart)
        w.geom_nv = ia(gnv)
        w.geom_param = da(gparam)
        w.geom_interior = da(ginterior)
        w.verts = da(np.concatenate(verts) if verts else [])
        w.n_obj = len(art.objects)
        w.obj_link = ia(art.obj_user_link)
        w.obj_geom = ia(obj_geom)
        w.obj_origin = da([c for o in art.objects for c in _se3_flat(o.origin)])
        w.n_att = len(self.attached)
        w.att_link = ia([a[1] for a in self.attached])
        w.att_geom = ia(att_geom)
        w.att_pose = da([c for a in self.attached for c in _se3_flat(a[3])])
        w.n_scene = len(self.scene)
        w.scene_geom = ia(scene_geom)
        w.scene_tf = da([c for s in self.scene for c in _se3_flat(s[2])])
        w.n_pairs = len(pairs)
        w.pa_kind = ia([p[0] for p in pairs])
        w.pa_idx = ia([p[1] for p in pairs])
        w.pb_kind = ia([p[2] for p in pairs])
        w.pb_idx = ia([p[3] for p in pairs])
        w.p_allowed = ia(allowed)
        w.oct_leaf = da(np.concatenate(leaves) if leaves else [])
        w.mesh_tri = ia(np.concatenate(tris) if tris else [])
        w.conv_nbr = ia(nbr_all)
        w.bvh = None
        w.gjk_solver = 1 if getattr(self, "gjk_solver", "libccd") == "indep" else 0
        if lib().orc_bvh_build(ctypes.byref(w)):  # FCL BVHModel<OBBRSS> trees, octree nodes, shape OBBs
            raise ValueError("octree leaves off FCL's root-BV halving grid")
        self._w = w
        self.geoms = geoms
        self.dof = len(mg)

    def __del__(self):
        try:
            if getattr(self, "_w", None) is not None and self._w.bvh:
                lib().orc_bvh_free(ctypes.byref(self._w))
        except Exception:  # interpreter shutdown
            pass

    def bvh_nodes(self, geom: int):
        """The FCL BVHModel<OBBRSS> tree (OBB half) the oracle built for a mesh
        geometry: (boxes[n, 15] = axis row-major 9, To 3, extent 3,
        links[n, 3] = first_child, first_prim, num_prim)."""
        out15, out3 = np.zeros(15), np.zeros(3, np.int32)
        n = lib().orc_bvh_node(ctypes.byref(self._w), geom, -1, out15.ctypes.data_as(_DP), out3.ctypes.data_as(_IP))
        boxes, links = np.zeros((max(n, 0), 15)), np.zeros((max(n, 0), 3), np.int32)
        for k in range(max(n, 0)):
            lib().orc_bvh_node(ctypes.byref(self._w), geom, k, out15.ctypes.data_as(_DP), out3.ctypes.data_as(_IP))
            boxes[k], links[k] = out15, out3
        return boxes, links

    def _pair_table(self):
        """(pairs, n_self) in PlanningWorldTpl::selfCollide then
        collideWithOthers order for one planned articulation
        (src/planning_world.cpp:277-481); entries (ka, ia, kb, ib, name1,
        name2) keep fcl::collide's (o1, o2) argument order."""
        art = self.art
        names = [o.link for o in art.objects]
        pairs = []
        for a, b in art.pairs:
            pairs.append((KIND_ROBOT, a, KIND_ROBOT, b, names[a], names[b]))
        for k, att in enumerate(self.attached):
            for i in range(len(art.objects)):
                pairs.append((KIND_ATTACHED, k, KIND_ROBOT, i, names[i], att[0]))
        for k in range(len(self.attached)):
            for k2 in range(k):
                pairs.append((KIND_ATTACHED, k, KIND_ATTACHED, k2, self.attached[k][0], self.attached[k2][0]))
        n_self = len(pairs)
        for s, sc in enumerate(self.scene):
            for i in range(len(art.objects)):
                pairs.append((KIND_ROBOT, i, KIND_SCENE, s, names[i], sc[0]))
        for k, att in enumerate(self.attached):
            for s, sc in enumerate(self.scene):
                pairs.append((KIND_ATTACHED, k, KIND_SCENE, s, att[0], sc[0]))
        return pairs, n_self

    # ------------------------------------------------------------------
    def collide_batch(self, q: np.ndarray, nthreads: int = 1, want_stats: bool = False, variant: str = ""):
        """flags[n], masks[n, W].  ``variant`` names an oracle-variant build
        (``variant_lib``) used only by the variant study."""
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, self.dof)
        n = q.shape[0]
        flags = np.zeros(n, dtype=np.uint8)
        masks = np.zeros((n, self.W), dtype=np.uint32)
        st = Stats()
        rc = (variant_lib(variant) if variant else lib()).orc_collide_batch(ctypes.byref(self._w), q.ctypes.data_as(_DP), ctypes.c_long(n),
                                     flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                     masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                     ctypes.c_int(self.W), ctypes.c_int(nthreads), ctypes.byref(st))
        if rc != 0:
            raise RuntimeError("orc_collide_batch failed")
        if want_stats:
            return flags, masks, {k: getattr(st, k) for k, _ in Stats._fields_}
        return flags, masks

    def fk_batch(self, q: np.ndarray):
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, self.dof)
        n = q.shape[0]
        poses = np.zeros((n, self._w.n_links, 7))
        objT = np.zeros((n, self._w.n_obj, 12))
        rc = lib().orc_fk_batch(ctypes.byref(self._w), q.ctypes.data_as(_DP), ctypes.c_long(n),
                                poses.ctypes.data_as(_DP), objT.ctypes.data_as(_DP))
        if rc != 0:
            raise RuntimeError("orc_fk_batch failed")
        return poses, objT

    def distance_batch(self, q: np.ndarray):
        """PlanningWorld::distanceSelf / distanceOthers per configuration:
        (d_self, pair_self, d_others, pair_others); -1 = penetrating pair,
        DBL_MAX / -1 = empty group."""
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, self.dof)
        n = q.shape[0]
        ds, do = np.zeros(n), np.zeros(n)
        ps, po = np.zeros(n, np.int32), np.zeros(n, np.int32)
        rc = lib().orc_distance_batch(ctypes.byref(self._w), q.ctypes.data_as(_DP), ctypes.c_long(n),
                                      ctypes.c_int(self.n_self_pairs), ds.ctypes.data_as(_DP), ps.ctypes.data_as(_IP),
                                      do.ctypes.data_as(_DP), po.ctypes.data_as(_IP))
        if rc != 0:
            raise RuntimeError("orc_distance_batch failed")
        return ds, ps, do, po

    def distance_batch_ex(self, q: np.ndarray, signed: bool = False, nearest_points: bool = False,
                          distance_tolerance: float = 1e-6, indep: bool = False):
        """distance_batch with DistanceRequest(enable_signed_distance,
        enable_nearest_points, distance_tolerance): (d_self, pair_self,
        pts_self[n, 6], d_others, pair_others, pts_others[n, 6]); pts =
        DistanceResult::nearest_points of the group's minimum pair, world frame
        (oracle/collide_oracle.c pair_distance says which point is which).
        RuntimeError where FCL throws (FCL_THROW_FAILED_AT_THIS_CONFIGURATION).
        indep: DistanceRequest(gjk_solver_type=GST_INDEP) -- FCL's own GJK
        (fcl_gjk_indep.h gjk_indep_distance), unsigned shape pairs only."""
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, self.dof)
        n = q.shape[0]
        ds, do = np.zeros(n), np.zeros(n)
        ps, po = np.zeros(n, np.int32), np.zeros(n, np.int32)
        qs, qo = np.zeros((n, 6)), np.zeros((n, 6))
        mode = (1 if signed else 0) | (2 if nearest_points else 0) | (4 if indep else 0)
        rc = lib().orc_distance_batch_ex(ctypes.byref(self._w), q.ctypes.data_as(_DP), ctypes.c_long(n),
                                         ctypes.c_int(self.n_self_pairs), ctypes.c_int(mode),
                                         ctypes.c_double(distance_tolerance),
                                         ds.ctypes.data_as(_DP), ps.ctypes.data_as(_IP), qs.ctypes.data_as(_DP),
                                         do.ctypes.data_as(_DP), po.ctypes.data_as(_IP), qo.ctypes.data_as(_DP))
        if rc == -3:
            raise RuntimeError("FCL throws on this configuration (libccd EPA: FCL_THROW_FAILED_AT_THIS_CONFIGURATION)")
        if rc != 0:
            raise RuntimeError("orc_distance_batch_ex failed")
        return ds, ps, qs, do, po, qo

    @staticmethod
    def epa_stats():
        """(largest EPA polytope in vertices, convexity-guard stops) over the
        distance calls since the last read (oracle/fcl_gjk_dist.h)."""
        g = ctypes.c_int(0)
        m = lib().orc_epa_stats(ctypes.byref(g))
        return int(m), int(g.value)

    def contact_batch(self, q: np.ndarray):
        """fcl::collide with CollisionRequest(enable_contact=True) on every pair:
        (hit[n, P], depth[n, P], normal[n, P, 3], pos[n, P, 3])."""
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, self.dof)
        n, P = q.shape[0], len(self.pairs)
        hit = np.zeros((n, P), np.uint8)
        depth = np.zeros((n, P))
        normal = np.zeros((n, P, 3))
        pos = np.zeros((n, P, 3))
        lib().orc_contact_batch(ctypes.byref(self._w), q.ctypes.data_as(_DP), ctypes.c_long(n),
                                hit.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), depth.ctypes.data_as(_DP),
                                normal.ctypes.data_as(_DP), pos.ctypes.data_as(_DP))
        return hit, depth, normal, pos

    def pair_names(self) -> List[Tuple[str, str]]:
        return [(p[4], p[5]) for p in self.pairs]

    def decode(self, mask_row) -> List[Tuple[str, str]]:
        out = []
        for p, pr in enumerate(self.pairs):
            if (int(mask_row[p >> 5]) >> (p & 31)) & 1:
                out.append((pr[4], pr[5]))
        return out


class _MergedArticulation:
    """Several articulations as ONE kinematic forest for the C restatement:
    each articulation's pinocchio joints, frames, user joints/links, user qpos
    and collision objects appended with their indices offset (a root joint's
    parent stays the universe, so oMi = liMi as in its own model).  The move
    group -- setQposAll's state -- is the planned articulations' move groups
    concatenated in the given (std::map name) order; unplanned articulations
    and non-move-group joints keep their current qpos."""

    def __init__(self, parts):
        from types import SimpleNamespace
        joints, names, frames, objects = [None], ["universe"], [M.PinFrame("universe", "FIXED_JOINT", 0, M.IDENT)], []
        self.user_joints, self.link_frames, self.obj_user_link, self.current_qpos = [], [], [], []
        self.obj_base, self.user_link_base, self.qpos_base = {}, {}, {}
        nq = nv = 0
        mg = []
        for name, art, planned in parts:
            jo, fo = len(joints) - 1, len(frames) - 1  # art joint j >= 1 -> jo + j; frame f >= 1 -> fo + f
            for j in art.pin.joints[1:]:
                joints.append(M.PinJoint(j.name, j.jtype, j.parent + jo if j.parent > 0 else 0, j.placement, j.axis,
                                         j.idx_q + nq, j.nq, j.nv, j.lower, j.upper))
                names.append(j.name)
            for f in art.pin.frames[1:]:
                frames.append(M.PinFrame(f.name, f.ftype, f.parent + jo if f.parent > 0 else 0, f.placement))
            self.qpos_base[name] = len(self.current_qpos)
            self.user_link_base[name] = len(self.link_frames)
            self.obj_base[name] = len(objects)
            self.user_joints += [j + jo if j > 0 else 0 for j in art.user_joints]
            self.link_frames += [f + fo if f > 0 else 0 for f in art.link_frames]
            self.obj_user_link += [self.user_link_base[name] + u for u in art.obj_user_link]
            objects += art.objects
            if planned:
                mg += [self.qpos_base[name] + i for i in art.move_group_qpos_index()]
            self.current_qpos += list(art.current_qpos)
            nq += art.pin.nq
            nv += art.pin.nv
        self.pin = SimpleNamespace(joints=joints, names=names, frames=frames, nq=nq, nv=nv)
        self.objects = objects
        self.nv = len(self.current_qpos)
        self._mg = mg

    def move_group_qpos_index(self):
        return list(self._mg)


class MultiOracleWorld(OracleWorld):
    """PlanningWorld with several articulations (reference
    src/planning_world.cpp:250-481): ``arts`` = [(name, Articulation,
    planned)] -- the planned ones in std::map (name) order, the unplanned in
    the order collideWithOthers iterates them; ``attached`` = [(name,
    art name, user link index, geom, pose)].  Pairs are matched with the
    product by (object names, link names), see ``pair_keys``."""

    def __init__(self, arts, scene=(), attached=(), allowed=()):
        self.parts = list(arts)
        merged = _MergedArticulation(self.parts)
        self.att_art = [a[1] for a in attached]
        att = [(a[0], merged.user_link_base[a[1]] + a[2], a[3], a[4]) for a in attached]
        super().__init__(merged, scene=scene, attached=att, allowed=allowed)

    def _pair_table(self):
        m = self.art
        planned = [(n, a) for n, a, p in self.parts if p]
        unplanned = [(n, a) for n, a, p in self.parts if not p]
        pairs, keys = [], []

        def add(ka, ia, kb, ib, n1, n2, on1, on2):
            pairs.append((ka, ia, kb, ib, n1, n2))
            keys.append((on1, on2, n1, n2))

        def links(a):
            return [o.link for o in a.objects]

        for ai, (an, A) in enumerate(planned):  # selfCollide
            base, ln = m.obj_base[an], links(A)
            for a, b in A.pairs:
                add(KIND_ROBOT, base + a, KIND_ROBOT, base + b, ln[a], ln[b], an, an)
            for bn, B in planned[:ai]:
                b0, ln2 = m.obj_base[bn], links(B)
                for i in range(len(ln)):
                    for j in range(len(ln2)):
                        add(KIND_ROBOT, base + i, KIND_ROBOT, b0 + j, ln[i], ln2[j], an, bn)
            for k, att in enumerate(self.attached):
                for i in range(len(ln)):
                    add(KIND_ATTACHED, k, KIND_ROBOT, base + i, ln[i], att[0], an, att[0])
        for k in range(len(self.attached)):
            for k2 in range(k):
                n1, n2 = self.attached[k][0], self.attached[k2][0]
                add(KIND_ATTACHED, k, KIND_ATTACHED, k2, n1, n2, n1, n2)
        n_self = len(pairs)
        for an, A in planned:  # collideWithOthers
            base, ln = m.obj_base[an], links(A)
            for bn, B in unplanned:
                b0, ln2 = m.obj_base[bn], links(B)
                for i in range(len(ln)):
                    for j in range(len(ln2)):
                        add(KIND_ROBOT, base + i, KIND_ROBOT, b0 + j, ln[i], ln2[j], an, bn)
            for s, sc in enumerate(self.scene):
                for i in range(len(ln)):
                    add(KIND_ROBOT, base + i, KIND_SCENE, s, ln[i], sc[0], an, sc[0])
        for k, att in enumerate(self.attached):
            for bn, B in unplanned:
                b0, ln2 = m.obj_base[bn], links(B)
                for i in range(len(ln2)):
                    add(KIND_ATTACHED, k, KIND_ROBOT, b0 + i, att[0], ln2[i], att[0], bn)
            for s, sc in enumerate(self.scene):
                add(KIND_ATTACHED, k, KIND_SCENE, s, att[0], sc[0], att[0], sc[0])
        self.pair_keys = keys
        return pairs, n_self
