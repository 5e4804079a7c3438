#!/usr/bin/env python3
"""Throughput of the widened rows on one GPU, cfg3 world:
batched distance, batched motion validation, collide with contacts.
Host-buffer APIs (PCIe-inclusive), so these are end-to-end call rates."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (share the HIP runtime)
from mplib_amd import pymp, scenes


def timeit(fn, reps=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main():
    w, art = scenes.world(3)
    out = {}
    q = scenes.sample_states(art, 1 << 18, 7)
    dt = timeit(lambda: w.distance_batch(q))
    out["distance_batch"] = {"configs": len(q), "s": dt, "configs_per_s": len(q) / dt}
    dt = timeit(lambda: w.collide_batch(q))
    out["collide_batch_host_buffers"] = {"configs": len(q), "s": dt, "configs_per_s": len(q) / dt}
    rng = np.random.default_rng(3)
    a = scenes.sample_states(art, 1 << 14, 8)
    lim = scenes.joint_limits(art)
    b = np.clip(a + rng.normal(scale=0.3, size=a.shape), lim[:, 0], lim[:, 1])
    res = {}

    def motion():
        res["r"] = w.check_motion_batch(a, b)

    dt = timeit(motion)
    segs = int(res["r"][2].sum())
    out["check_motion_batch"] = {"edges": len(a), "states": segs, "s": dt, "edges_per_s": len(a) / dt,
                                 "states_per_s": segs / dt}
    from mplib_amd.batch import DeviceWorld  # noqa: F401
    req = pymp.fcl.CollisionRequest(enable_contact=True)
    qs = scenes.sample_states(art, 256, 9)

    def scalar_contacts():
        for i in range(len(qs)):
            w.set_qpos_all(list(qs[i]))
            w.collide_full(req)

    dt = timeit(scalar_contacts, reps=1)
    out["scalar_collide_full_with_contacts"] = {"calls": len(qs), "s": dt, "calls_per_s": len(qs) / dt}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
