"""mplib_amd -- MI355X-native batched state-validity checking for MPlib.

``mplib_amd.pymp`` mirrors the reference's ``mplib.pymp`` module
(submodules ``fcl``, ``pinocchio``, ``articulation``, ``collision_matrix``,
``planning_world`` and ``set_global_seed``); every kinematics / collision
evaluation runs on the GPU through the C ABI in ``include/mpgpu.h``
(``mplib_amd/lib/libmpgpu.so``).  There is no CPU fallback: importing
``pymp`` fails if the libraries have not been built (``make -C mplib_amd``).
"""
# PyTorch (used by callers for device buffers, streams and torch.distributed)
# bundles its own libamdhip64.so.7 with the same soname as /opt/rocm's.  Two
# HIP runtimes in one process do not share devices, so when torch is installed
# it is loaded first and libmpgpu.so binds to that already-loaded runtime.
try:  # pragma: no cover - depends on the environment
    import torch as _torch  # noqa: F401
except ImportError:  # torch-free deployments use /opt/rocm's runtime
    _torch = None

from . import pymp  # noqa: F401,E402  (raises ImportError when the build is missing)
from .pymp import articulation, collision_matrix, fcl, pinocchio, planning_world, set_global_seed  # noqa: F401

__version__ = "0.1.0"
