"""ctypes binding of the C ABI declared in include/mpgpu.h.

This is the exact binding a maintainer would add to the reference's Python
side.  It loads ``mplib_amd/lib/libmpgpu.so`` (built
in-tree by ``make -C mplib_amd``) and fails loudly when the library is
missing: there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmpgpu.so")

MPG_OK, MPG_E_INVALID, MPG_E_UNSUPPORTED, MPG_E_HIP, MPG_E_NOMEM, MPG_E_FAILED = 0, 1, 2, 3, 4, 5
MPG_MEM_HOST, MPG_MEM_DEVICE = 0, 1
STAGES = ("cull", "bucket", "narrow")  # MPG_STAGE_* order

(JOINT_RX, JOINT_RY, JOINT_RZ, JOINT_REVOLUTE_UNALIGNED, JOINT_PX, JOINT_PY, JOINT_PZ,
 JOINT_PRISMATIC_UNALIGNED, JOINT_RUBX, JOINT_RUBY, JOINT_RUBZ, JOINT_RUB_UNALIGNED) = range(12)
GEOM_CONVEX, GEOM_BOX, GEOM_SPHERE, GEOM_CAPSULE, GEOM_CYLINDER, GEOM_OCTREE, GEOM_MESH, GEOM_ELLIPSOID, GEOM_CONE = range(9)
GJK_LIBCCD, GJK_INDEP = 0, 1

_I32P = ctypes.POINTER(ctypes.c_int32)
_F64P = ctypes.POINTER(ctypes.c_double)
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U32P = ctypes.POINTER(ctypes.c_uint32)


class WorldDesc(ctypes.Structure):
    """``mpg_world_desc`` (include/mpgpu.h)."""
    _fields_ = [
        ("n_joints", ctypes.c_int32), ("joint_type", _I32P), ("joint_parent", _I32P),
        ("joint_axis", _F64P), ("joint_placement", _F64P),
        ("joint_q_source", _I32P), ("joint_q_const", _F64P), ("dof", ctypes.c_int32),
        ("n_links", ctypes.c_int32), ("link_parent", _I32P), ("link_placement", _F64P),
        ("n_geoms", ctypes.c_int32), ("geom_type", _I32P), ("geom_vertex_start", _I32P),
        ("geom_vertex_count", _I32P), ("geom_param", _F64P), ("n_vertices", ctypes.c_int64),
        ("vertices", _F64P),
        ("n_moving", ctypes.c_int32), ("moving_link", _I32P), ("moving_geom", _I32P),
        ("moving_offset", _F64P),
        ("n_static", ctypes.c_int32), ("static_geom", _I32P), ("static_transform", _F64P),
        ("n_pairs", ctypes.c_int32), ("pair_a", _I32P), ("pair_b", _I32P), ("pair_allowed", _U8P),
        ("gjk_tolerance", ctypes.c_double),
        ("n_octree_leaves", ctypes.c_int64), ("octree_leaf", _F64P),
        ("n_mesh_triangles", ctypes.c_int64), ("mesh_triangle", _I32P),
        ("n_convex_face_ints", ctypes.c_int64), ("convex_face", _I32P),
        ("joint_lower", _F64P), ("joint_upper", _F64P),
        ("gjk_solver", ctypes.c_int32),
    ]


MPG_DISTANCE_SIGNED, MPG_DISTANCE_NEAREST_POINTS, MPG_DISTANCE_GJK_INDEP = 1, 2, 4


class DistanceRequest(ctypes.Structure):
    """mpg_distance_request (include/mpgpu.h): DistanceRequest's flags and
    distance_tolerance."""
    _fields_ = [("flags", ctypes.c_int32), ("distance_tolerance", ctypes.c_double)]


class WorldInfo(ctypes.Structure):
    _fields_ = [("n_pairs", ctypes.c_int32), ("mask_words", ctypes.c_int32), ("dof", ctypes.c_int32),
                ("n_links", ctypes.c_int32), ("device", ctypes.c_int32), ("block_size", ctypes.c_int32),
                ("snapshot_bytes", ctypes.c_int64)]


#: every symbol include/mpgpu.h declares, with (restype, argtypes)
SIGNATURES = {
    "mpg_world_create": (ctypes.c_int, [ctypes.POINTER(WorldDesc), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "mpg_world_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "mpg_world_get_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(WorldInfo)]),
    "mpg_set_small_batch_max": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "mpg_release_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mpg_collide_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "mpg_sample_uniform": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                          ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int]),
    "mpg_collide_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "mpg_collide_batch_multi": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_void_p,
                                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "mpg_shard_range": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(ctypes.c_int64)]),
    "mpg_collide_batch_multi_device": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32,
                                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                      ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                      ctypes.c_void_p]),
    "mpg_collide_link_poses": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "mpg_check_motion_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_uint32, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "mpg_distance_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p]),
    "mpg_distance_batch_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_void_p]),
    "mpg_distance_batch_req": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p]),
    "mpg_collide_contacts": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "mpg_fk_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_void_p]),
    "mpg_profile_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mpg_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "mpg_debug_collide_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mpg_debug_sincos": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]),
    "mpg_fcl_bvh_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mpg_latency_server_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_int32)]),
    "mpg_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "mpg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mpg_last_error": (ctypes.c_char_p, []),
    "mpg_last_error_copy": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "mpg_version": (ctypes.c_char_p, []),
}

_lib = None


class MpgError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libmpgpu.so; raise ImportError if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"mplib_amd: HIP library {LIB_PATH} is missing -- run `make -C mplib_amd` "
                              "(there is no CPU fallback)")
        try:  # share torch's HIP runtime when torch is present (see mplib_amd/__init__.py)
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != MPG_OK:
        msg = lib().mpg_last_error().decode(errors="replace")
        if rc == MPG_E_UNSUPPORTED:
            raise NotImplementedError(f"{what}: {msg}")
        if rc == MPG_E_INVALID:
            raise ValueError(f"{what}: {msg}")
        raise MpgError(f"{what} failed (status {rc}): {msg}")
