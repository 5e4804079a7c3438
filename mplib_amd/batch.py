"""Batched state-validity checking through the C ABI (include/mpgpu.h).

``DeviceWorld`` owns one immutable device snapshot (``mpg_world``) built from
a plain-array world description and evaluates ``collide()`` /
``collideFull()`` for a whole batch of joint configurations in one launch.
Inputs may be host numpy arrays (copied through staging buffers) or device
tensors (any object exposing ``data_ptr()``, e.g. a torch tensor on the
world's device; the launch is enqueued on the given stream and not
synchronised).

Reference semantics: ``flags[i] == PlanningWorld.collide()`` after
``set_qpos_all(q[i])`` (src/planning_world.h:248-250, cpp:250-262), and bit p
of ``pair_mask[i]`` is set iff pair p is in ``collide_full()``'s result
(src/planning_world.cpp:484-490, ACM-filtered by :265-274).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np

from . import _capi as C

_DESC_INT_FIELDS = ["joint_type", "joint_parent", "joint_q_source", "link_parent", "geom_type",
                    "geom_vertex_start", "geom_vertex_count", "moving_link", "moving_geom", "static_geom",
                    "pair_a", "pair_b"]
_DESC_F64_FIELDS = ["joint_axis", "joint_placement", "joint_q_const", "link_placement", "geom_param",
                    "vertices", "moving_offset", "static_transform"]


class DeviceWorld:
    """An ``mpg_world`` snapshot on one device."""

    def __init__(self, arrays: Dict[str, np.ndarray], device: int = 0, gjk_tolerance: float = 1e-6,
                 gjk_solver: int = C.GJK_LIBCCD):
        L = C.lib()
        self._keep = []

        def ip(name):
            a = np.ascontiguousarray(np.asarray(arrays[name], dtype=np.int32).reshape(-1))
            if a.size == 0:
                a = np.zeros(1, np.int32)
            self._keep.append(a)
            return a.ctypes.data_as(C._I32P)

        def fp(name):
            a = np.ascontiguousarray(np.asarray(arrays[name], dtype=np.float64).reshape(-1))
            if a.size == 0:
                a = np.zeros(1, np.float64)
            self._keep.append(a)
            return a.ctypes.data_as(C._F64P)

        d = C.WorldDesc()
        d.n_joints = len(arrays["joint_type"])
        d.dof = int(arrays["dof"])
        d.n_links = len(arrays["link_parent"])
        d.n_geoms = len(arrays["geom_type"])
        d.n_vertices = int(np.asarray(arrays["vertices"]).size // 3)
        d.n_moving = len(arrays["moving_link"])
        d.n_static = len(arrays["static_geom"])
        d.n_pairs = len(arrays["pair_a"])
        for f in _DESC_INT_FIELDS:
            setattr(d, f, ip(f))
        for f in _DESC_F64_FIELDS:
            setattr(d, f, fp(f))
        al = np.ascontiguousarray(np.asarray(arrays["pair_allowed"], dtype=np.uint8).reshape(-1))
        if al.size == 0:
            al = np.zeros(1, np.uint8)
        self._keep.append(al)
        d.pair_allowed = al.ctypes.data_as(C._U8P)
        d.gjk_tolerance = gjk_tolerance
        d.gjk_solver = int(gjk_solver)
        leaves = np.ascontiguousarray(np.asarray(arrays.get("octree_leaf", np.zeros(0)), dtype=np.float64).reshape(-1))
        d.n_octree_leaves = leaves.size // 6
        if leaves.size == 0:
            leaves = np.zeros(6)
        self._keep.append(leaves)
        d.octree_leaf = leaves.ctypes.data_as(C._F64P)
        tris = np.ascontiguousarray(np.asarray(arrays.get("mesh_triangle", np.zeros(0)), dtype=np.int32).reshape(-1))
        d.n_mesh_triangles = tris.size // 3
        if tris.size == 0:
            tris = np.zeros(3, np.int32)
        self._keep.append(tris)
        d.mesh_triangle = tris.ctypes.data_as(C._I32P)
        faces = np.ascontiguousarray(np.asarray(arrays.get("convex_face", np.zeros(0)), dtype=np.int32).reshape(-1))
        d.n_convex_face_ints = faces.size
        if faces.size == 0:
            faces = np.zeros(1, np.int32)
        self._keep.append(faces)
        d.convex_face = faces.ctypes.data_as(C._I32P)
        for f in ("joint_lower", "joint_upper"):  # optional: NULL = unbounded
            if f in arrays and arrays[f] is not None:
                a = np.ascontiguousarray(np.asarray(arrays[f], dtype=np.float64).reshape(-1))
                self._keep.append(a)
                setattr(d, f, a.ctypes.data_as(C._F64P))
        h = ctypes.c_void_p()
        C.check(L.mpg_world_create(ctypes.byref(d), device, ctypes.byref(h)), "mpg_world_create")
        self._keep = []
        self._h = h
        info = C.WorldInfo()
        C.check(L.mpg_world_get_info(h, ctypes.byref(info)), "mpg_world_get_info")
        self.n_pairs = info.n_pairs
        self.mask_words = info.mask_words
        self.dof = info.dof
        self.n_links = info.n_links
        self.device = info.device
        self.block_size = info.block_size

    def close(self):
        if getattr(self, "_h", None):
            C.lib().mpg_world_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_small_batch_max(self, n: int):
        """Host batches of at most n configurations take the one-launch latency path (0 disables)."""
        C.check(C.lib().mpg_set_small_batch_max(self._h, int(n)), "mpg_set_small_batch_max")

    def release_stream(self, stream: int):
        """Drop the workspace / side stream kept for a caller stream (call before destroying it)."""
        C.check(C.lib().mpg_release_stream(self._h, ctypes.c_void_p(int(stream))), "mpg_release_stream")

    # ------------------------------------------------------------------
    def collide_batch(self, q, flags=None, pair_mask=None, stream: Optional[int] = None):
        """Host path (numpy): returns (flags[n] u8, pair_mask[n, W] u32).
        Device path (tensors with data_ptr()): fills the given device buffers
        on ``stream`` and returns them without synchronising."""
        if hasattr(q, "data_ptr"):
            n = q.shape[0] if q.dim() > 1 else q.numel() // self.dof
            if flags is None:
                raise ValueError("device path needs preallocated flags (and optionally pair_mask)")
            C.check(C.lib().mpg_collide_batch(self._h, ctypes.c_void_p(q.data_ptr()), n,
                                              ctypes.c_void_p(flags.data_ptr()),
                                              ctypes.c_void_p(pair_mask.data_ptr() if pair_mask is not None else 0),
                                              C.MPG_MEM_DEVICE, ctypes.c_void_p(stream or 0)), "mpg_collide_batch")
            return flags, pair_mask
        qa = np.ascontiguousarray(np.asarray(q, dtype=np.float64)).reshape(-1, self.dof)
        n = qa.shape[0]
        fl = np.zeros(n, np.uint8)
        pm = np.zeros((n, self.mask_words), np.uint32)
        C.check(C.lib().mpg_collide_batch(self._h, qa.ctypes.data_as(ctypes.c_void_p), n,
                                          fl.ctypes.data_as(ctypes.c_void_p), pm.ctypes.data_as(ctypes.c_void_p),
                                          C.MPG_MEM_HOST, ctypes.c_void_p(stream or 0)), "mpg_collide_batch")
        return fl, pm

    def debug_collide_pairs(self, geom_a: int, geom_b: int, Ta, Tb) -> np.ndarray:
        """Narrow phase only: fcl::collide(geometry geom_a at Ta[i], geom_b at
        Tb[i]) (SE3 rows of 12 doubles) -> uint8 hits (mpg_debug_collide_pairs)."""
        A = np.ascontiguousarray(Ta, dtype=np.float64).reshape(-1, 12)
        B = np.ascontiguousarray(Tb, dtype=np.float64).reshape(-1, 12)
        n = len(A)
        hit = np.zeros(n, np.uint8)
        C.check(C.lib().mpg_debug_collide_pairs(self._h, int(geom_a), int(geom_b), n, A.ctypes.data_as(ctypes.c_void_p),
                                                B.ctypes.data_as(ctypes.c_void_p), hit.ctypes.data_as(ctypes.c_void_p)),
                "mpg_debug_collide_pairs")
        return hit

    def fk_batch(self, q) -> np.ndarray:
        """[n, n_links, 7] link poses (p, wxyz) -- getLinkPose for every user link."""
        qa = np.ascontiguousarray(np.asarray(q, dtype=np.float64)).reshape(-1, self.dof)
        n = qa.shape[0]
        out = np.zeros((n, self.n_links, 7))
        C.check(C.lib().mpg_fk_batch(self._h, qa.ctypes.data_as(ctypes.c_void_p), n,
                                     out.ctypes.data_as(ctypes.c_void_p), C.MPG_MEM_HOST, None), "mpg_fk_batch")
        return out


def device_sincos(x, device: int = 0):
    xa = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    s = np.zeros_like(xa)
    c = np.zeros_like(xa)
    C.check(C.lib().mpg_debug_sincos(xa.ctypes.data_as(ctypes.c_void_p), xa.size, s.ctypes.data_as(ctypes.c_void_p),
                                     c.ctypes.data_as(ctypes.c_void_p), device), "mpg_debug_sincos")
    return s, c


def collide_batch_multi(worlds, q):
    """One host batch over several DeviceWorlds (built from the same
    descriptor, one per GPU): mpg_collide_batch_multi checks contiguous shards
    concurrently.  Returns (flags[n] u8, pair_mask[n, W] u32)."""
    worlds = list(worlds)
    if not worlds:
        raise ValueError("no worlds")
    w0 = worlds[0]
    q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, w0.dof)
    n = q.shape[0]
    flags = np.zeros(n, np.uint8)
    masks = np.zeros((n, w0.mask_words), np.uint32)
    hs = (ctypes.c_void_p * len(worlds))(*[w.handle for w in worlds])
    C.check(C.lib().mpg_collide_batch_multi(hs, len(worlds), q.ctypes.data, n, flags.ctypes.data, masks.ctypes.data),
            "mpg_collide_batch_multi")
    return flags, masks


def shard_range_c(n: int, k: int, parts: int):
    """mpg_shard_range: (start, count) of part k of n configurations."""
    start, count = ctypes.c_int64(), ctypes.c_int64()
    C.check(C.lib().mpg_shard_range(int(n), int(k), int(parts), ctypes.byref(start), ctypes.byref(count)),
            "mpg_shard_range")
    return start.value, count.value


def collide_batch_multi_device(worlds, qs, flags, masks=None, streams=None, gather_flags=None, gather_masks=None):
    """mpg_collide_batch_multi_device: shard k already on worlds[k]'s device
    (torch tensors or raw device pointers via .data_ptr()): qs[k] [count, dof]
    float64, flags[k] [count] uint8, masks[k] [count, W] int32/uint32 or None;
    streams[k] a stream handle (int) or None.  gather_flags / gather_masks:
    tensors on worlds[0]'s device receiving every shard in order.  Enqueues
    only (no synchronisation)."""
    worlds = list(worlds)
    k = len(worlds)
    handle = lambda w: w.handle if hasattr(w, "handle") else w.device_handle()  # noqa: E731  (DeviceWorld / PlanningWorld)
    if not (len(qs) == len(flags) == k) or (masks is not None and len(masks) != k):
        raise ValueError("one q / flags (/ masks) buffer per world")
    P = ctypes.c_void_p
    ptr = lambda t: P(t.data_ptr() if t is not None else 0)  # noqa: E731
    hs = (P * k)(*[handle(w) for w in worlds])
    qa = (P * k)(*[ptr(t) for t in qs])
    fa = (P * k)(*[ptr(t) for t in flags])
    ma = (P * k)(*[ptr(t) for t in masks]) if masks is not None else None
    sa = (P * k)(*[P(int(s or 0)) for s in streams]) if streams is not None else None
    counts = (ctypes.c_int64 * k)(*[int(t.shape[0]) for t in qs])
    C.check(C.lib().mpg_collide_batch_multi_device(hs, k, qa, counts, fa, ma, sa, ptr(gather_flags),
                                                   ptr(gather_masks)), "mpg_collide_batch_multi_device")
