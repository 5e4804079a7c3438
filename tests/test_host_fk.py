"""CPU: the product FK (mplib_amd/csrc/mpg_fk.h, the same code the HIP kernel
runs) compiled for the host equals the oracle bit-for-bit."""
import ctypes
import os

import numpy as np

import worlds as Wd
from native.host_shim import lib


def host_fk(d, q):
    keep = []

    def I(a):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.int32))
        keep.append(a)
        return a.ctypes.data_as(ctypes.c_void_p)

    def F(a):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
        keep.append(a)
        return a.ctypes.data_as(ctypes.c_void_p)

    nl = len(d["link_parent"])
    out = np.zeros((len(q), nl, 7))
    lib().host_fk(len(d["joint_type"]), I(d["joint_type"]), I(d["joint_parent"]), I(d["joint_q_source"]),
                  F(d["joint_q_const"]), F(d["joint_axis"]), F(d["joint_placement"]), int(d["dof"]), nl,
                  I(d["link_parent"]), F(d["link_placement"]), F(q), ctypes.c_long(len(q)),
                  out.ctypes.data_as(ctypes.c_void_p))
    return out


def test_host_fk_equals_oracle():
    ow = Wd.oracle_world(2)
    q = Wd.sample_q(ow.art, 20000, 7)
    po, _ = ow.fk_batch(q)
    np.testing.assert_array_equal(host_fk(Wd.desc_arrays(ow), q), po)


def test_host_fk_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "panda_fk_64.npz"))
    ow = Wd.oracle_world(2)
    np.testing.assert_array_equal(host_fk(Wd.desc_arrays(ow), g["q"]), g["link_pose"])


def test_host_fk_extreme_angles():
    """Angles outside the URDF limits and near the glibc branch points."""
    ow = Wd.oracle_world(2)
    rng = np.random.default_rng(9)
    q = np.concatenate([rng.uniform(-30, 30, (2000, 7)),
                        np.full((1, 7), 0.85546875), np.full((1, 7), 2.426265), np.zeros((1, 7))])
    po, _ = ow.fk_batch(q)
    np.testing.assert_array_equal(host_fk(Wd.desc_arrays(ow), q), po)
