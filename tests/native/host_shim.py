"""Build tests/native/host_fk.cpp (product headers compiled for the host)."""
import ctypes
import os
import subprocess
import tempfile

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def _build(src, stem):
    """Compile src into a per-process file: pytest-xdist workers build the
    same shim at once, and a shared output path could be loaded half-written."""
    out = os.path.join(tempfile.gettempdir(), "%s_%d_%d.so" % (stem, os.getuid(), os.getpid()))
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", out, src])
    return ctypes.CDLL(out)


def lib():
    global _lib
    if _lib is None:
        _lib = _build(os.path.join(_HERE, "host_fk.cpp"), "mplib_amd_host_fk")
    return _lib


_walk = None


def walk_lib():
    """tests/native/walk_cells.cpp: mpg_hullcells.h's walk-hull tables on the host."""
    global _walk
    if _walk is None:
        _walk = _build(os.path.join(_HERE, "walk_cells.cpp"), "mplib_amd_walk_cells")
    return _walk
