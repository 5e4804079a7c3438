"""Build tests/native/host_fk.cpp (product headers compiled for the host)."""
import ctypes
import os
import subprocess
import tempfile

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        out = os.path.join(tempfile.gettempdir(), "mplib_amd_host_fk_%d.so" % os.getuid())
        src = os.path.join(_HERE, "host_fk.cpp")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", out, src])
        _lib = ctypes.CDLL(out)
    return _lib


_walk = None


def walk_lib():
    """tests/native/walk_cells.cpp: mpg_hullcells.h's walk-hull tables on the host."""
    global _walk
    if _walk is None:
        out = os.path.join(tempfile.gettempdir(), "mplib_amd_walk_cells_%d.so" % os.getuid())
        src = os.path.join(_HERE, "walk_cells.cpp")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", out, src])
        _walk = ctypes.CDLL(out)
    return _walk
