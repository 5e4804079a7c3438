#!/usr/bin/env python3
"""Latency-path A/B (host buffers, the planner's regime): median round trip of
PlanningWorld.collide_batch for N states (cfg3) under the current environment
(MPG_OWN_STREAM, MPG_SMALL_HOST_SC, MPG_SMALL_INLINE_SC), and the bare floors:
an empty torch op + synchronize on the default and on a side stream."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402
from mplib_amd import scenes  # noqa: E402


def med(fn, reps=400):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts) * 1e6), 1)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    x = torch.zeros(16, device="cuda")
    s = torch.cuda.Stream()
    floor = med(lambda: (x.add_(1), torch.cuda.synchronize()))
    with torch.cuda.stream(s):
        floor_s = med(lambda: (x.add_(1), s.synchronize()))
    w, art = scenes.world(3)
    out = {"tag": tag, "torch_add_sync_us": floor, "torch_add_sync_side_stream_us": floor_s}
    sizes = [int(v) for v in os.environ.get("LAT_N", "1,8,64,256").split(",")]
    for n in sizes:
        q = scenes.sample_states(art, n, 3)
        out[f"n{n}_us"] = med(lambda: w.collide_batch(q))
    print(out, flush=True)


if __name__ == "__main__":
    main()
