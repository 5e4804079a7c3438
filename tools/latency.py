#!/usr/bin/env python3
"""Round-trip latency of small collide batches (host buffers), the planner's
regime: median wall time of PlanningWorld.collide_batch for N states, next to
the latency of bare primitives (one empty launch + sync, small copies)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402
from mplib_amd import scenes  # noqa: E402


def med(fn, reps=200):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


def main():
    x = torch.zeros(16, device="cuda")
    torch.cuda.synchronize()
    print("torch add+sync us", med(lambda: (x.add_(1), torch.cuda.synchronize())))
    h = torch.zeros(64, dtype=torch.float64)
    hp = torch.zeros(64, dtype=torch.float64).pin_memory()
    d = torch.zeros(64, dtype=torch.float64, device="cuda")
    print("H2D pageable 512B us", med(lambda: (d.copy_(h), torch.cuda.synchronize())))
    print("H2D pinned 512B us", med(lambda: (d.copy_(hp, non_blocking=True), torch.cuda.synchronize())))
    print("D2H 512B us", med(lambda: h.copy_(d)))
    for cfg in (3, 4):
        w, art = scenes.world(cfg)
        for n in (1, 2, 8, 64, 512, 4096):
            q = scenes.sample_states(art, n, 3)
            print(f"cfg{cfg} collide_batch N={n} us", round(med(lambda: w.collide_batch(q)), 1), flush=True)
        w.profile_enable(True)
        q = scenes.sample_states(art, 8, 3)
        for _ in range(100):
            w.collide_batch(q)
        print("stages (ms, launches, units) over 100 calls of N=8:", w.profile_read())


if __name__ == "__main__":
    main()
