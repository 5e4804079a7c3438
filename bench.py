#!/usr/bin/env python3
"""bench.py -- batched PlanningWorld::collide() throughput on MI355X.

Metric (BASELINE.json): configs/sec of full collide() (self + world) for the
Panda 7-DoF + 10 boxes world (cfg3), 2^20 uniform-random configurations per
GPU per step, weak scaling over 1/2/4/8 GPUs (one process per GPU).

A step = one pass of the hot path (FK + all 129 pairs + ACM filter) over one
2^20-configuration batch that is already resident in HBM: one
mpg_collide_batch call (cull -> bucket -> narrow kernels on one stream)
writing flags[N] (u8) and pair_mask[N, 5] (u32).

Other workloads (not the headline): --cfg 2 / 4 (self-only / convex
obstacles), --cfg 6 (the detect_collision.py floor point cloud as an
fcl::OcTree), --cfg 7 (cfg3 with the Panda links as BVH triangle meshes,
convex=False), --cfg 5 (RRTConnect plan() end to end: a step is one plan()).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-sample S] [--cfg C]
        torchrun --nproc-per-node N bench.py --gpus N ...
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
STAGES = ("cull", "bucket", "narrow")  # MPG_STAGE_* (include/mpgpu.h)
KERNEL_NAME = {"cull": "cull_kernel", "bucket": "pair_scan/chunk_scan/scatter",
               "narrow": "narrow stage (narrow_kernel + closed_form_kernel instances)"}
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X spec (vector FP64; FMA counted as 2)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--cfg", type=int, default=3,
                   help="2, 3, 4: BASELINE collide configs; 5: RRTConnect plan(); 6: floor point cloud; "
                        "7: cfg3 with BVH mesh links (convex=False)")
    p.add_argument("--goal", default="far", help="cfg5 goal (scenes.PLAN_GOALS)")
    p.add_argument("--cpu-plans", type=int, default=4, help="cfg5: plans timed with the CPU oracle checker")
    p.add_argument("--per-gpu", type=int, default=0, help="configs per GPU per step (default: BASELINE size)")
    p.add_argument("--cpu-sample", type=int, default=1 << 17,
                   help="configs timed on the CPU oracle for cpu_baseline (rank 0, N=1 only; 0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=1)
    p.add_argument("--gather", action="store_true", help="also time an all-gather of the results to every rank")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") across GPUs; MPLIB_AMD_DIST_BACKEND=gloo rehearses the
    # multi-rank flow with several ranks sharing one GPU (tests / 1-GPU boxes)
    backend = os.environ.get("MPLIB_AMD_DIST_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if backend != "nccl":
        local = 0
    torch.cuda.set_device(local)
    os.environ["MPLIB_AMD_DEVICE"] = str(local)

    from mplib_amd import scenes

    cfg = args.cfg
    if cfg == 5:
        return plan_main(args, world, rank, local, backend)
    n = args.per_gpu or (scenes.CFG_N[cfg] if cfg != 4 else (1 << 22) // max(world, 1))
    w, art = scenes.world(cfg)
    dim = w.get_state_dim()
    W = w.get_mask_words()
    n_pairs = len(w.get_collision_pair_info())
    # this rank's shard of synthetic uniform states (rank 0 = the BASELINE seed)
    q_host = scenes.sample_states(art, n, scenes.CFG_SEED[cfg] + 1000 * rank)
    q = torch.from_numpy(q_host).to(f"cuda:{local}")
    flags = torch.empty(n, dtype=torch.uint8, device=q.device)
    masks = torch.empty((n, W), dtype=torch.int32, device=q.device)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    def step():
        w.collide_batch_device(q.data_ptr(), n, flags.data_ptr(), masks.data_ptr(), sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    w.profile_enable(True)  # HIP events around each device stage, on the launch stream
    w.profile_read()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    prof = w.profile_read()
    w.profile_enable(False)
    # per-launch averages of each stage
    st = {k: {"ms_per_launch": v[0] / max(v[1], 1), "launches_per_step": v[1] / args.steps,
              "units_per_launch": v[2] / max(v[1], 1)} for k, v in prof.items()}
    if world > 1:
        t = torch.tensor([elapsed, step_ms] + [st[k]["ms_per_launch"] for k in STAGES], dtype=torch.float64,
                         device=q.device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms = float(t[0]), float(t[1])
        for i, k in enumerate(STAGES):
            st[k]["ms_per_launch"] = float(t[2 + i])

    gather_ms = None
    if args.gather and world > 1 and backend == "nccl":
        out = torch.empty(n * world, dtype=torch.uint8, device=q.device)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        dist.all_gather_into_tensor(out, flags)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    total = n * world * args.steps
    value = total / elapsed
    # algorithmic bytes per unit (DESIGN.md "Roofline"):
    #   cull:   per configuration  q row in + flag + pair-mask zeroing (8*dof + 1 + 4W)
    #           + survivor words out (4W)
    #   narrow: per candidate      candidate index + q row + mask word read-modify-write + flag
    bytes_per_unit = {"cull": 8 * dim + 1 + 4 * W + 4 * W, "narrow": 4 + 8 * dim + 8 + 1,
                      "bucket": 4 * W * 3 + 4 * (n_pairs + 1)}
    dom = max(("cull", "narrow"), key=lambda k: st[k]["ms_per_launch"])
    units = st[dom]["units_per_launch"]
    achieved_gbps = bytes_per_unit[dom] * units / (st[dom]["ms_per_launch"] * 1e-3) / 1e9
    traffic = None
    pmc_file = os.path.join(ROOT, "profiles", f"pmc_cfg{cfg}.json")
    if os.path.exists(pmc_file):
        try:
            pm = json.load(open(pmc_file))
            if pm.get("configs_per_launch") == int(st["cull"]["units_per_launch"]) and dom in pm.get("hbm_bytes_per_launch", {}):
                traffic = pm["hbm_bytes_per_launch"][dom]
        except Exception:
            traffic = None

    result = {
        "metric": "configs/sec full collide() Panda-7DoF+10 boxes" if cfg == 3 else f"configs/sec collide() cfg{cfg}",

        "value": value,
        "unit": "configs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (uniform in URDF joint limits)",
        "config": {"workload": f"cfg{cfg} {scenes.CFG_NAME[cfg]}: {n} configs/GPU/step, {n_pairs} pairs, "
                               f"full self+world collide() with ACM filter",
                   "configs_per_gpu": n, "pairs": n_pairs, "parallelism": f"dp{world} (config shards, no "
                                                                          "data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved_gbps / HBM_PEAK_GBPS, "traffic": traffic,
                     "kernel": KERNEL_NAME[dom], "kernel_ms": st[dom]["ms_per_launch"],
                     "units_per_launch": units, "unit_kind": "configs" if dom == "cull" else "candidates",
                     "algorithmic_bytes_per_unit": bytes_per_unit[dom],
                     "note": "the path is fp32/fp64-VALU and latency bound, not HBM bound (DESIGN.md); "
                             "HBM fraction reported as mandated"},
        "stages": {k: {"ms_per_step": st[k]["ms_per_launch"] * st[k]["launches_per_step"],
                       "units_per_launch": st[k]["units_per_launch"]} for k in STAGES},
        "step_ms_events": step_ms,
    }
    if gather_ms is not None:
        result["gather_ms"] = gather_ms

    if rank == 0 and world == 1 and args.cpu_sample > 0:
        k = args.cpu_sample if cfg != 7 else min(args.cpu_sample, 1 << 13)  # the mesh oracle is ~100x slower
        result["cpu_baseline"] = cpu_baseline(cfg, q_host[:k], flags, masks, args.cpu_threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def plan_main(args, world, rank, local, backend):
    """cfg5: RRTConnect plan() in the cfg3 scene, device validity (speculative
    connect batches, latency path).  A step = one plan() from PLAN_START to
    PLAN_GOALS[goal] with range 0.1 and seed = step index (+1000 * rank:
    ranks are independent replicas)."""
    import torch
    import torch.distributed as dist
    from mplib_amd import pymp, scenes

    goal = scenes.PLAN_GOALS[args.goal]
    # plan() prints MPlib's messages ("invalid start state!! ...") on the C
    # stdout, as the reference does: send them to stderr, keep stdout one line
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    w, _ = scenes.world(3)
    planner = pymp.ompl.OMPLPlanner(w)

    def one(seed):
        pymp.set_global_seed(seed)
        return planner.plan(scenes.PLAN_START, [goal], range=0.1, time=60.0)

    for i in range(args.warmup):
        one(10_000 + i)
    w.profile_enable(True)
    w.profile_read()
    stats, paths, solved = [], {}, 0
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        st, path = one(1000 * rank + i)
        solved += st == "Exact solution"
        paths[i] = path
        stats.append(planner.get_last_plan_stats())
    elapsed = time.perf_counter() - t0
    prof = w.profile_read()
    w.profile_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    mean = lambda k: float(np.mean([s[k] for s in stats]))  # noqa: E731
    ms, launches, units = prof["narrow"]  # the latency path records its kernel as the narrow stage
    kern_ms = ms / max(launches, 1)
    states_per_launch = mean("states_checked") / max(mean("batches"), 1.0)
    bytes_per_state = 8 * w.get_state_dim() + len(w.get_collision_pair_info())  # q row in + hit bytes out
    achieved = bytes_per_state * states_per_launch / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    result = {
        "metric": "plans/sec RRTConnect plan() cfg5 (Panda + 10 boxes)", "value": args.steps * world / elapsed,
        "unit": "plans/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic RRTConnect queries: seeds 0..steps-1, start tests/test_basic.py qpos, goal = IK of a "
                "panda_hand pose (scenes.PLAN_GOALS)",
        "config": {"workload": f"cfg5 RRTConnect {args.goal} goal, range 0.1, cfg3 scene", "goal": list(goal),
                   "parallelism": f"replicas x{world}"},
        "solved": solved, "mean_iterations": mean("iterations"), "mean_batches": mean("batches"),
        "mean_states_checked": mean("states_checked"), "mean_check_ms": mean("check_seconds") * 1e3,
        "roofline": {"bound": "latency", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": "small_kernel",
                     "kernel_ms": kern_ms, "units_per_launch": states_per_launch, "unit_kind": "states",
                     "algorithmic_bytes_per_unit": bytes_per_state,
                     "note": "one validity batch per planner iteration: round-trip latency, not bandwidth, "
                             "bounds a plan"},
    }
    if rank == 0 and world == 1 and args.cpu_plans > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import worlds as Wd  # test fixture module: the oracle-built cfg3 world
        ow = Wd.oracle_world(3)
        cpu = pymp.ompl.OMPLPlanner(scenes.world(3)[0], state_validity_checker=lambda s: ow.collide_batch(s)[0] == 0)
        cpu.set_speculative_connect(False)  # OMPL's serial loop: one batch per growTree
        k = min(args.cpu_plans, args.steps)
        same = True
        t0 = time.perf_counter()
        for i in range(k):
            pymp.set_global_seed(i)
            st, path = cpu.plan(scenes.PLAN_START, [goal], range=0.1, time=60.0)
            same &= bool(np.array_equal(path, paths[i]))
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": k / dt, "unit": "plans/s", "cores": 1, "kind": "port",
                                  "sample": f"seeds 0..{k - 1}: the same planner with oracle/collide_oracle.c as "
                                            f"its checker, one batch per growTree call, {dt:.1f} s",
                                  "gpu_matches_cpu_on_sample": same}
    sys.stdout.flush()
    os.dup2(saved_stdout, 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(cfg, q_sample, flags, masks, threads):
    """The CPU restatement of MPlib's PlanningWorld::collide (oracle/) timed on
    this host on a bounded sample; also cross-checks the GPU results on it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import worlds as Wd  # test fixture module: oracle-built world of the same config

    ow = Wd.oracle_world(cfg)
    ow.collide_batch(q_sample[:256], nthreads=threads)  # warm
    t0 = time.perf_counter()
    fo, mo = ow.collide_batch(q_sample, nthreads=threads)
    dt = time.perf_counter() - t0
    k = len(q_sample)
    parity = bool(np.array_equal(fo, flags[:k].cpu().numpy()) and
                  np.array_equal(mo, masks[:k].cpu().numpy().view(np.uint32)))
    return {"value": k / dt, "unit": "configs/s", "cores": threads, "kind": "port",
            "sample": f"first {k} configs of the rank-0 batch, oracle/collide_oracle.c (C restatement of "
                      f"FK + FCL/libccd MPR + PlanningWorld loops), {threads} thread(s), {dt:.1f} s",
            "gpu_matches_cpu_on_sample": parity}


if __name__ == "__main__":
    main()
