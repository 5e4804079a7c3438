"""Host-side cost of reading pinned buffers and of writing fresh numpy
outputs (round 6 host pipeline diagnosis).  Prints one JSON line."""
import ctypes
import json
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
NB = 20 << 20
res = {}


def timeit(fn, reps=10):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e3


dst = np.empty(NB, np.uint8)
dst.fill(0)
for name, flags in (("default", 0x0), ("mapped", 0x2), ("mapped_coherent", 0x2 | 0x40000000),
                    ("mapped_noncoherent", 0x2 | 0x80000000), ("wc", 0x2 | 0x4)):
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(NB), ctypes.c_uint(flags))
    if rc:
        res[name] = f"rc {rc}"
        continue
    ctypes.memset(p, 1, NB)
    res[name + "_read_ms"] = timeit(lambda: ctypes.memmove(dst.ctypes.data, p, NB))
    res[name + "_write_ms"] = timeit(lambda: ctypes.memmove(p, dst.ctypes.data, NB))
    hip.hipHostFree(p)
src = np.ones(NB, np.uint8)
def fresh():
    a = np.empty(NB, np.uint8)
    ctypes.memmove(a.ctypes.data, src.ctypes.data, NB)
    return a


res["fresh_numpy_dst_ms"] = timeit(fresh)
res["fresh_numpy_zeros_ms"] = timeit(lambda: np.zeros(NB, np.uint8))
res["reused_dst_ms"] = timeit(lambda: ctypes.memmove(dst.ctypes.data, src.ctypes.data, NB))
print(json.dumps(res))
