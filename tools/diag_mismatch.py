#!/usr/bin/env python3
"""GPU diagnostic: run a world on the device and the oracle, save the
mismatching configurations (q rows, device / oracle masks) to
gpurun_out/diag_<name>.npz for offline analysis with the oracle variants.
usage: python tools/diag_mismatch.py floor|blue|cfg3 [n] [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mplib_amd import scenes  # noqa: E402
import worlds as Wd  # noqa: E402

kind = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 31
if kind in ("floor", "blue"):
    w, art = scenes.cloud_world(kind)
    ow = Wd.oracle_cloud_world(kind)
else:
    cfg = int(kind[3:])
    w, art = scenes.world(cfg)
    ow = Wd.oracle_world(cfg)
q = Wd.sample_q(ow.art, n, seed)
fo, mo = ow.collide_batch(q, nthreads=16)
w.set_small_batch_max(0)
f, m = w.collide_batch(q)
bad = np.nonzero((m.view(np.uint32) != mo).any(axis=1))[0]
print(kind, "mismatching configs:", len(bad), bad[:20].tolist())
for i in bad[:20]:
    x = m[i].view(np.uint32) ^ mo[i]
    bits = [32 * k + b for k in range(len(x)) for b in range(32) if (int(x[k]) >> b) & 1]
    print(i, "pairs", bits, "device", [int((int(m[i].view(np.uint32)[p >> 5]) >> (p & 31)) & 1) for p in bits])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"diag_{kind}.npz"), q=q[bad], dev=m[bad].view(np.uint32), orc=mo[bad], idx=bad)
