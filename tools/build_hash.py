"""Hash of what libmpgpu.so is compiled from (kernel sources, headers and the
Makefile's HIP flags): profiles/pmc_cfg*.json are keyed by it, so a rebuild of
the same sources (the driver rebuilds in its own container) still matches,
and any kernel change invalidates the recorded counters."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = ("mplib_amd/csrc/mpg_kernels.hip", "mplib_amd/csrc/mpg_math.h", "mplib_amd/csrc/mpg_fk.h",
         "mplib_amd/csrc/mpg_sincostab.h", "mplib_amd/csrc/mpg_broadphase.h", "mplib_amd/csrc/mpg_hullcells.h",
         "include/mpgpu.h")


def build_hash() -> str:
    h = hashlib.sha256()
    for f in FILES:
        h.update(f.encode())
        h.update(open(os.path.join(ROOT, f), "rb").read())
    for line in open(os.path.join(ROOT, "mplib_amd", "Makefile")):
        if line.startswith("HIPFLAGS"):
            h.update(line.encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(build_hash())
