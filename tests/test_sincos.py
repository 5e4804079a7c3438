"""CPU: the product's restatement of glibc sin/cos (mplib_amd/csrc/mpg_math.h),
compiled for the host, is bit-identical to the host libm.

* kFma=false == glibc sincos() (generic build, no FMA ifunc variant) -- what
  pinocchio's SINCOS and GCC-folded sin/cos pairs call.
* kFma=true  == glibc sin()/cos() on FMA+AVX2 hosts (__sin_fma/__cos_fma).
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

from native.host_shim import lib

_m = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_m.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
_m.sin.argtypes = _m.cos.argtypes = [ctypes.c_double]
_m.sin.restype = _m.cos.restype = ctypes.c_double

HAS_FMA = "fma" in open("/proc/cpuinfo").read().split()


def host(x, fma, fused=False):
    x = np.ascontiguousarray(x, dtype=np.float64)
    s, c = np.zeros_like(x), np.zeros_like(x)
    lib().host_sincos(x.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(x.size), s.ctypes.data_as(ctypes.c_void_p),
                      c.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(2 if fused else 1 if fma else 0))
    return s, c


def samples():
    rng = np.random.default_rng(3)
    return np.concatenate([rng.uniform(-4, 4, 60000), rng.uniform(-0.2, 0.2, 20000),
                           rng.uniform(-1000, 1000, 20000), rng.uniform(-1e-7, 1e-7, 2000),
                           np.array([0.0, -0.0, 0.126, -0.126, 0.85546875, 2.426265, np.pi / 2, -np.pi, 1e5])])


def test_generic_matches_libm_sincos():
    x = samples()
    s, c = host(x, fma=False)
    bad = 0
    for i in range(x.size):
        rs, rc = ctypes.c_double(), ctypes.c_double()
        _m.sincos(float(x[i]), ctypes.byref(rs), ctypes.byref(rc))
        bad += (rs.value != s[i]) + (rc.value != c[i])
    assert bad == 0


@pytest.mark.skipif(not HAS_FMA, reason="glibc selects the FMA sin/cos variant only on FMA hosts")
def test_fma_variant_matches_libm_sin_cos():
    x = samples()
    s, c = host(x, fma=True)
    bad = sum((_m.sin(float(x[i])) != s[i]) + (_m.cos(float(x[i])) != c[i]) for i in range(x.size))
    assert bad == 0


def test_fused_sincos_equals_separate():
    """mpg_sincos (selects instead of branches, used by the FK) is bit-identical
    to the separate generic mpg_sin/mpg_cos, including the case boundaries,
    tiny, huge, signed-zero and non-finite arguments."""
    rng = np.random.default_rng(4)
    edges = np.array([0x3e400000, 0x3e500000, 0x3feb6000, 0x400368fd, 0x419921FB], dtype=np.uint64) << np.uint64(32)
    around = (edges[:, None].astype(np.int64) + np.arange(-3, 4)[None, :]).astype(np.uint64).reshape(-1).view(np.float64)
    x = np.concatenate([samples(), rng.uniform(-1e6, 1e6, 20000), rng.uniform(-3.0, 3.0, 200000), around, -around,
                        np.array([np.inf, -np.inf, np.nan, 1e9, -1e9, 5e-324, 0.12599999999999998, 0.126])])
    s0, c0 = host(x, fma=False)
    s1, c1 = host(x, fma=False, fused=True)
    np.testing.assert_array_equal(s1.view(np.uint64)[~np.isnan(s0)], s0.view(np.uint64)[~np.isnan(s0)])
    np.testing.assert_array_equal(c1.view(np.uint64)[~np.isnan(c0)], c0.view(np.uint64)[~np.isnan(c0)])
    assert np.array_equal(np.isnan(s0), np.isnan(s1)) and np.array_equal(np.isnan(c0), np.isnan(c1))
