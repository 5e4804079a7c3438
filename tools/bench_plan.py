#!/usr/bin/env python3
"""cfg5 (BASELINE.json configs[4]): RRTConnect plan() end-to-end in the cfg3
scene with batched device validity, next to the same planner driven by the CPU
oracle (test infrastructure, one host thread, OMPL's serial growTree loop).

Per goal (scenes.PLAN_GOALS) and seed: wall time of OMPLPlanner.plan(), its
iterations, validity batches and states checked.  Paths must be identical
between the two checkers (same seed, same tree).
usage: python tools/bench_plan.py [--seeds 16] [--cpu-seeds 4] [--out file]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401  (share the HIP runtime)
from mplib_amd import pymp, scenes  # noqa: E402


def run(p, goal, seed, spec=True):
    p.set_speculative_connect(spec)
    pymp.set_global_seed(seed)
    t0 = time.perf_counter()
    status, path = p.plan(scenes.PLAN_START, [goal], range=0.1, time=60.0)
    dt = time.perf_counter() - t0
    return status, path, dt, p.get_last_plan_stats()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=16)
    ap.add_argument("--cpu-seeds", type=int, default=4)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    w, _ = scenes.world(3)
    dev = pymp.ompl.OMPLPlanner(w)
    run(dev, scenes.PLAN_GOALS["near"], 0)  # warm-up: snapshot upload, staging buffers
    import worlds as Wd  # CPU baseline checker (oracle; test infrastructure)
    ow = Wd.oracle_world(3)
    cpu = pymp.ompl.OMPLPlanner(scenes.world(3)[0], state_validity_checker=lambda s: ow.collide_batch(s)[0] == 0)
    out = {"workload": "cfg5: RRTConnect plan(), Panda + 10 boxes (cfg3 scene), range 0.1, start test_basic.py qpos",
           "goals": {}}
    for name, goal in scenes.PLAN_GOALS.items():
        rows = {"gpu": [], "gpu_serial": [], "cpu": []}
        paths = {}
        for seed in range(a.seeds):
            for kind, spec in (("gpu", True), ("gpu_serial", False)):
                st, path, dt, s = run(dev, goal, seed, spec)
                rows[kind].append(dict(seed=seed, status=st, ms=dt * 1e3, **{k: s[k] for k in (
                    "iterations", "batches", "states_checked")}))
                paths[(kind, seed)] = path
        for seed in range(min(a.cpu_seeds, a.seeds)):
            st, path, dt, s = run(cpu, goal, seed, False)
            rows["cpu"].append(dict(seed=seed, status=st, ms=dt * 1e3, **{k: s[k] for k in (
                "iterations", "batches", "states_checked")}))
            assert np.array_equal(path, paths[("gpu", seed)]), "GPU and CPU-oracle planners diverged"
        summ = {}
        for kind, r in rows.items():
            ms = np.array([x["ms"] for x in r])
            summ[kind] = {"plans": len(r), "solved": sum(x["status"] == "Exact solution" for x in r),
                          "median_ms": float(np.median(ms)), "mean_ms": float(ms.mean()),
                          "plans_per_s": float(len(r) / (ms.sum() / 1e3)),
                          "mean_iterations": float(np.mean([x["iterations"] for x in r])),
                          "mean_batches": float(np.mean([x["batches"] for x in r])),
                          "mean_states": float(np.mean([x["states_checked"] for x in r])),
                          "us_per_batch": float(ms.sum() * 1e3 / sum(x["batches"] for x in r))}
        summ["speedup_gpu_vs_cpu_on_common_seeds"] = float(
            sum(x["ms"] for x in rows["cpu"]) / sum(x["ms"] for x in rows["gpu"][:len(rows["cpu"])]))
        out["goals"][name] = {"goal": goal, "summary": summ, "runs": rows}
        print(name, json.dumps(summ), flush=True)
    out["cpu_baseline"] = {"kind": "port", "cores": 1,
                           "what": "same planner, oracle/collide_oracle.c as the checker through a Python callback, "
                                   "one validity batch per growTree (OMPL's serial loop)"}
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
