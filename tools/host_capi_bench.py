"""mpg_collide_batch(MPG_MEM_HOST) through the C ABI on the cfg3 2^20 batch:
caller-owned output buffers reused across calls (a C++ caller) vs fresh
numpy outputs per call (the pymp route).  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import worlds as Wd  # noqa: E402
from mplib_amd import _capi as C, scenes  # noqa: E402
from mplib_amd.batch import DeviceWorld  # noqa: E402

n = 1 << 20
ow = Wd.oracle_world(3)
d = DeviceWorld(Wd.desc_arrays(ow))
_, art = scenes.world(3)
q = scenes.sample_states(art, n, scenes.CFG_SEED[3])
W = d.mask_words
fl = np.zeros(n, np.uint8)
pm = np.zeros((n, W), np.uint32)


def call(f, m):
    C.check(C.lib().mpg_collide_batch(d.handle, q.ctypes.data_as(ctypes.c_void_p), n, f.ctypes.data_as(ctypes.c_void_p),
                                      m.ctypes.data_as(ctypes.c_void_p), C.MPG_MEM_HOST, None), "mpg_collide_batch")


def fresh():
    f = np.empty(n, np.uint8)
    m = np.empty((n, W), np.uint32)
    call(f, m)
    return f, m


res = {}
for name, fn in (("reused_outputs", lambda: call(fl, pm)), ("fresh_outputs", fresh),
                 ("reused_outputs_again", lambda: call(fl, pm))):
    for _ in range(3):
        fn()
    t = []
    for _ in range(20):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    res[name + "_ms"] = float(np.median(t) * 1e3)
    res[name + "_cfg_s"] = n / float(np.median(t))
print(json.dumps(res))
