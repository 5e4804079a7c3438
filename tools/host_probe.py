"""Host-buffer path probe (round 6): what the numpy-in / numpy-out cfg3 path
costs today, and the PCIe / host-memcpy rates a pipelined path is bounded by.
Prints one JSON line."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mplib_amd import scenes  # noqa: E402

res = {}
w, art = scenes.world(3)
n = 1 << 20
q = scenes.sample_states(art, n, scenes.CFG_SEED[3])
for _ in range(3):
    w.collide_batch(q)
t = []
for _ in range(10):
    t0 = time.perf_counter()
    w.collide_batch(q)
    t.append(time.perf_counter() - t0)
res["host_path_ms"] = float(np.median(t) * 1e3)
res["host_path_cfg_s"] = n / float(np.median(t))

dev = torch.device("cuda:0")
nb = 56 << 20
d = torch.empty(nb, dtype=torch.uint8, device=dev)
d2 = torch.empty(nb, dtype=torch.uint8, device=dev)
hp = torch.empty(nb, dtype=torch.uint8).pin_memory()
hp2 = torch.empty(nb, dtype=torch.uint8).pin_memory()
hpage = torch.empty(nb, dtype=torch.uint8)
hpage.fill_(1)


def rate(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nb * reps / (time.perf_counter() - t0) / 1e9


res["h2d_pinned_GBs"] = rate(lambda: d.copy_(hp, non_blocking=True))
res["d2h_pinned_GBs"] = rate(lambda: hp.copy_(d, non_blocking=True))
res["h2d_pageable_GBs"] = rate(lambda: d.copy_(hpage))
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def both():
    with torch.cuda.stream(s1):
        d.copy_(hp, non_blocking=True)
    with torch.cuda.stream(s2):
        hp2.copy_(d2, non_blocking=True)


res["duplex_each_GBs"] = rate(both)

# host memcpy pageable -> pinned with k threads (ctypes.memmove releases the GIL)
src = np.ones(nb, dtype=np.uint8)
dst_addr = hp.data_ptr()
for k in (1, 2, 4, 8, 16):
    def cp():
        step = nb // k
        ths = [threading.Thread(target=ctypes.memmove, args=(dst_addr + i * step, src.ctypes.data + i * step, step))
               for i in range(k)]
        [x.start() for x in ths]
        [x.join() for x in ths]
    cp()
    t0 = time.perf_counter()
    for _ in range(5):
        cp()
    res[f"memcpy_{k}t_GBs"] = nb * 5 / (time.perf_counter() - t0) / 1e9
# registration cost of a fresh pageable buffer
buf = np.ones(nb, dtype=np.uint8)
hip = ctypes.CDLL("libamdhip64.so")
t0 = time.perf_counter()
rc = hip.hipHostRegister(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(nb), 0)
res["host_register_56MB_ms"] = (time.perf_counter() - t0) * 1e3
res["host_register_rc"] = rc
hip.hipHostUnregister(ctypes.c_void_p(buf.ctypes.data))
res["nproc"] = os.cpu_count()
res["affinity"] = len(os.sched_getaffinity(0))
print(json.dumps(res))
