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
        python bench.py --host ...          (the batch in host memory: numpy in / numpy out, PCIe timed)
        python bench.py --capi-multi N ...  (one process, N GPUs through mpg_collide_batch_multi_device)
`python bench.py --gpus N` (N > 1) without a launcher starts the N ranks
itself (torch.distributed.run as a child process, one process per GPU, RCCL);
under a launcher whose WORLD_SIZE differs from --gpus it exits non-zero.
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
PCIE_PEAK_GBPS = 63.0  # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s spec
# VALU issue: a wave issues one VALU instruction per 2 cycles on its SIMD
# (MI355X_MICROARCH.md "Wave scheduling"); 1024 SIMDs at 2.4 GHz.  FP64 VALU
# instructions run at half the FP32 rate (78.6 TF vs 157.3 TF vector, spec):
# they occupy the issue port twice as long.
SIMDS, CLOCK_HZ, VALU_ISSUE_CYCLES = 1024, 2.4e9, 2
STAGES = ("cull", "bucket", "narrow")  # MPG_STAGE_* (include/mpgpu.h)
KERNEL_NAME = {"cull": "cull_kernel", "bucket": "pair_scan/chunk_scan/scatter",
               "narrow": "narrow stage (narrow_kernel + closed_form_kernel instances)"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--cfg", type=int, default=3,
                   help="2, 3, 4: BASELINE collide configs; 5: RRTConnect plan(); 6: floor point cloud; "
                        "7: cfg3 with BVH mesh links (convex=False)")
    p.add_argument("--goal", default="far", help="cfg5 goal (scenes.PLAN_GOALS)")
    p.add_argument("--spec-nodes", type=int, default=None, help="cfg5: outcome-tree nodes explored before each batch")
    p.add_argument("--cpu-plans", type=int, default=-1,
                   help="cfg5: plans timed with the CPU oracle checker (-1: the same seeds as the GPU run, 0: none)")
    p.add_argument("--per-gpu", type=int, default=0, help="configs per GPU per step (default: BASELINE size)")
    p.add_argument("--cpu-sample", type=int, default=1 << 20,
                   help="configs timed on the CPU oracle for cpu_baseline on all the box's cores (rank 0, N=1 only; "
                        "0 = skip); a quarter of them on one core")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the all-core CPU baseline (0: the box's share, OMP_NUM_THREADS or nproc)")
    p.add_argument("--gather", action="store_true", help="also time an all-gather of the results to every rank")
    p.add_argument("--capi-multi", type=int, default=0, metavar="N",
                   help="one process drives N GPUs through the C entry mpg_collide_batch_multi_device "
                        "(device-resident shards, one host thread per GPU; --gather adds the peer-copy gather "
                        "into GPU 0); not under a launcher")
    p.add_argument("--host", action="store_true",
                   help="the batch in host memory: numpy in, numpy out through PlanningWorld.collide_batch "
                        "(mpg_collide_batch with MPG_MEM_HOST, PCIe both ways inside the timed step)")
    return p.parse_args()


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: start N ranks (one
    process per GPU) with torch.distributed.run as a child process and return
    its exit code.  Nothing here has touched the GPU (the ranks do that)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if args.capi_multi:
        if launched or args.gpus != 1:
            sys.exit("bench.py: --capi-multi N runs in one process (no launcher, no --gpus)")
        return capi_multi_main(args)
    if not launched and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") across GPUs; MPLIB_AMD_DIST_BACKEND=gloo rehearses the
    # multi-rank flow with several ranks sharing one GPU (tests / 1-GPU boxes)
    backend = os.environ.get("MPLIB_AMD_DIST_BACKEND", "nccl")
    if launched:  # a process group whenever a launcher started us (RCCL initialises even at N=1)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if os.environ.get("MPLIB_AMD_BENCH_DRYRUN") == "1":
        return dryrun_main(args, world, rank, launched)
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
    if args.host:
        return host_main(args, world, rank, local, backend, cfg, n, w, q_host, dim, W, n_pairs)
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
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    prof = w.profile_read()
    w.profile_enable(False)
    # per-launch averages of each stage
    st = {k: {"ms_per_launch": v[0] / max(v[1], 1), "launches_per_step": v[1] / args.steps,
              "units_per_launch": v[2] / max(v[1], 1)} for k, v in prof.items()}
    if dist.is_initialized():
        t = torch.tensor([elapsed, step_ms] + [st[k]["ms_per_launch"] for k in STAGES], dtype=torch.float64,
                         device=q.device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms = float(t[0]), float(t[1])
        for i, k in enumerate(STAGES):
            st[k]["ms_per_launch"] = float(t[2 + i])

    gather_ms = gather_dist_ms = None
    if args.gather and dist.is_initialized() and backend == "nccl":
        # every rank's flags + pair masks to every rank, device to device
        # (RCCL all-gather over xGMI; mplib_amd.dist.collide_sharded_device's
        # collective), timed apart from the check: not part of `value`
        all_f = torch.empty(n * world, dtype=torch.uint8, device=q.device)
        all_m = torch.empty((n * world, W), dtype=torch.int32, device=q.device)
        dist.all_gather_into_tensor(all_f, flags)
        dist.all_gather_into_tensor(all_m, masks)
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            dist.all_gather_into_tensor(all_f, flags)
            dist.all_gather_into_tensor(all_m, masks)
        torch.cuda.synchronize()
        g1 = time.perf_counter()
        # the distance results (PlanningWorld::distanceSelf / distanceOthers
        # minima + pair indices, mplib_amd.dist.distance_sharded_device): one
        # device pass over this rank's batch, then the same all-gather timed
        dres = {"d_self": torch.empty(n, dtype=torch.float64, device=q.device),
                "p_self": torch.empty(n, dtype=torch.int32, device=q.device),
                "d_others": torch.empty(n, dtype=torch.float64, device=q.device),
                "p_others": torch.empty(n, dtype=torch.int32, device=q.device)}
        w.distance_batch_device(q.data_ptr(), n, dres["d_self"].data_ptr(), dres["p_self"].data_ptr(),
                                dres["d_others"].data_ptr(), dres["p_others"].data_ptr(), 0, 0,
                                torch.cuda.current_stream(q.device).cuda_stream, None)
        dall = {k: torch.empty((n * world,), dtype=v.dtype, device=q.device) for k, v in dres.items()}
        torch.cuda.synchronize()
        dist.barrier()
        g2 = time.perf_counter()
        for _ in range(args.steps):
            for k in dres:
                dist.all_gather_into_tensor(dall[k], dres[k])
        torch.cuda.synchronize()
        t = torch.tensor([(g1 - g0) * 1e3 / args.steps, (time.perf_counter() - g2) * 1e3 / args.steps],
                         dtype=torch.float64, device=q.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather_ms, gather_dist_ms = float(t[0]), float(t[1])

    total = n * world * args.steps
    value = total / elapsed
    roofline, valu = rooflines(st, cfg, dim, W)

    result = {
        "metric": "configs/sec full collide() Panda-7DoF+10 boxes" if cfg == 3 else f"configs/sec collide() cfg{cfg}",

        "value": value,
        "unit": "configs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        # cfg4 is quoted on a fixed 2^22 batch split over the ranks
        "scaling": "strong" if cfg == 4 and not args.per_gpu else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (uniform in URDF joint limits)",
        "config": {"workload": f"cfg{cfg} {scenes.CFG_NAME[cfg]}: {n} configs/GPU/step, {n_pairs} pairs, "
                               f"full self+world collide() with ACM filter",
                   "configs_per_gpu": n, "pairs": n_pairs, "mask_words": W, "parallelism": f"dp{world} (config shards, no "
                                                                          "data-path collective)"},
        "roofline": roofline,
        "valu_roofline": valu,
        "lib_hash": lib_hash(),
        "stages": {k: {"ms_per_step": st[k]["ms_per_launch"] * st[k]["launches_per_step"],
                       "units_per_launch": st[k]["units_per_launch"]} for k in STAGES},
        "step_ms_events": step_ms,
    }
    if gather_ms is not None:
        result["gather_ms"] = gather_ms
        result["gather_bytes_per_rank"] = n * (1 + 4 * W)
        result["gather_distance_ms"] = gather_dist_ms
        result["gather_distance_bytes_per_rank"] = n * 24

    if rank == 0 and world == 1 and args.cpu_sample > 0:
        k = args.cpu_sample if cfg != 7 else min(args.cpu_sample, 1 << 13)  # the mesh oracle is ~100x slower
        threads = args.cpu_threads or box_threads()
        result["cpu_baseline"] = cpu_baseline(cfg, q_host[:k], flags, masks, threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def capi_multi_main(args):
    """--capi-multi N: the in-process multi-GPU route a C++ caller of the C
    ABI takes (include/mpgpu.h mpg_collide_batch_multi_device): N worlds, one
    per GPU, each GPU's shard (the BASELINE size per GPU, weak scaling; cfg4
    the fixed 2^22 batch split) resident in its HBM, one host thread per GPU
    enqueueing its shard on its own stream; a step = one call + the
    synchronisation of every GPU.  --gather: every shard's flags and mask rows
    also copied into GPU 0 (peer copies over xGMI) inside the step."""
    import torch
    from mplib_amd import scenes
    from mplib_amd.batch import collide_batch_multi_device

    N, cfg = args.capi_multi, args.cfg
    if torch.cuda.device_count() < N:
        sys.exit(f"bench.py: --capi-multi {N} but {torch.cuda.device_count()} GPUs")
    n = args.per_gpu or (scenes.CFG_N[cfg] if cfg != 4 else (1 << 22) // N)
    worlds, qs, fl, mk, streams = [], [], [], [], []
    for k in range(N):
        os.environ["MPLIB_AMD_DEVICE"] = str(k)  # the snapshot is built on GPU k
        w, art = scenes.world(cfg)
        w.device_handle()
        dev = torch.device("cuda", k)
        worlds.append(w)
        qs.append(torch.from_numpy(scenes.sample_states(art, n, scenes.CFG_SEED[cfg] + 1000 * k)).to(dev))
        fl.append(torch.empty(n, dtype=torch.uint8, device=dev))
        mk.append(torch.empty((n, w.get_mask_words()), dtype=torch.int32, device=dev))
        streams.append(torch.cuda.Stream(device=dev))
    W, dim, n_pairs = worlds[0].get_mask_words(), worlds[0].get_state_dim(), len(worlds[0].get_collision_pair_info())
    gf = gm = None
    if args.gather:
        gf = torch.empty(n * N, dtype=torch.uint8, device="cuda:0")
        gm = torch.empty((n * N, W), dtype=torch.int32, device="cuda:0")
    sptr = [s.cuda_stream for s in streams]

    def step():
        collide_batch_multi_device(worlds, qs, fl, mk, sptr, gf, gm)

    def sync_all():
        for k in range(N):
            torch.cuda.synchronize(k)

    for _ in range(args.warmup):
        step()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync_all()
    elapsed = time.perf_counter() - t0
    worlds[0].profile_enable(True)
    worlds[0].profile_read()
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        step()
    sync_all()
    prof = worlds[0].profile_read()
    worlds[0].profile_enable(False)
    st = {k: {"ms_per_launch": v[0] / max(v[1], 1), "launches_per_step": v[1] / prof_steps,
              "units_per_launch": v[2] / max(v[1], 1)} for k, v in prof.items()}
    roofline, valu = rooflines(st, cfg, dim, W)
    ok = True
    if N > 1 or args.gather:  # shard 0 against a plain single-world call on the same data
        f0 = torch.empty_like(fl[0])
        m0 = torch.empty_like(mk[0])
        worlds[0].collide_batch_device(qs[0].data_ptr(), n, f0.data_ptr(), m0.data_ptr(),
                                       torch.cuda.current_stream(0).cuda_stream)
        sync_all()
        ok = bool(torch.equal(f0, fl[0]) and torch.equal(m0, mk[0]))
        if args.gather:
            ok &= bool(torch.equal(gf[:n], fl[0]) and torch.equal(gm[:n], mk[0]))
    result = {
        "metric": "configs/sec full collide() Panda-7DoF+10 boxes" if cfg == 3 else f"configs/sec collide() cfg{cfg}",
        "value": n * N * args.steps / elapsed, "unit": "configs/s", "n_gpus": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if cfg == 4 and not args.per_gpu else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (uniform in URDF joint limits)",
        "config": {"workload": f"cfg{cfg} {scenes.CFG_NAME[cfg]}: {n} configs/GPU/step, {n_pairs} pairs, "
                               f"full self+world collide() with ACM filter",
                   "configs_per_gpu": n, "pairs": n_pairs, "mask_words": W,
                   "parallelism": f"capi-multi x{N}: one process, one host thread per GPU "
                                  f"(mpg_collide_batch_multi_device){', gather into GPU 0' if args.gather else ''}"},
        "shard0_matches_single_world_call": ok,
        "roofline": roofline, "valu_roofline": valu, "lib_hash": lib_hash(),
    }
    print(json.dumps(result), flush=True)


def host_main(args, world, rank, local, backend, cfg, n, w, q_host, dim, W, n_pairs):
    """--host: the same workload with the batch in host memory, as a caller of
    the reference's API holds it: numpy in, numpy out through
    PlanningWorld.collide_batch -> mpg_collide_batch(MPG_MEM_HOST), the
    pipelined host path (input chunks over PCIe while earlier chunks compute,
    only the colliding configurations' mask rows back).  A step = one call,
    both PCIe directions and the allocation of the returned arrays included."""
    import torch
    import torch.distributed as dist
    for _ in range(args.warmup):
        w.collide_batch(q_host)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    per_call = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        flags, masks = w.collide_batch(q_host)
        per_call.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the per-stage kernel times (HIP events on the launch streams) from a
    # few more calls, outside the timed region: the events cost host time in
    # the launching thread, which the pipeline would show
    w.profile_enable(True)
    w.profile_read()
    for _ in range(max(1, min(args.steps, 5))):
        w.collide_batch(q_host)
    prof = w.profile_read()
    w.profile_enable(False)
    prof_steps = max(1, min(args.steps, 5))
    st = {k: {"ms_per_launch": v[0] / max(v[1], 1), "launches_per_step": v[1] / prof_steps,
              "units_per_launch": v[2] / max(v[1], 1)} for k, v in prof.items()}
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    rate = float(flags.mean())
    # bytes that cross PCIe per step: the q rows in, the flags and the packed
    # mask rows of the colliding configurations out
    pcie_bytes = n * (8 * dim) + n + n * rate * 4 * W
    step_s = elapsed / args.steps
    roofline, valu = rooflines(st, cfg, dim, W)
    result = {
        "metric": ("configs/sec full collide() Panda-7DoF+10 boxes" if cfg == 3 else f"configs/sec collide() cfg{cfg}")
        + ", host buffers (numpy in/out, PCIe included)",
        "value": n * world * args.steps / elapsed, "unit": "configs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (uniform in URDF joint limits)",
        "config": {"workload": f"cfg{cfg} {scenes_name(cfg)}: {n} configs/GPU/step in host memory, {n_pairs} pairs, "
                               f"full self+world collide() with ACM filter",
                   "configs_per_gpu": n, "pairs": n_pairs, "mask_words": W, "memory": "host (pageable numpy)",
                   "parallelism": f"dp{world}"},
        "call_ms_median": float(np.median(per_call) * 1e3),
        "collision_rate": rate,
        "pcie": {"bound": "pcie", "achieved": pcie_bytes / step_s / 1e9, "peak": PCIE_PEAK_GBPS, "unit": "GB/s",
                 "frac": pcie_bytes / step_s / 1e9 / PCIE_PEAK_GBPS, "bytes_per_step": pcie_bytes,
                 "bytes_per_config": pcie_bytes / n,
                 "note": "q rows in (8*dof B) + flags (1 B) + packed mask rows of colliding configurations "
                         "(4W B each) out; peak = PCIe Gen5 x16 spec (MI355X_MICROARCH.md), one link shared by "
                         "both directions on this box (profiles/r06a/host_probe.json)"},
        "roofline": roofline,
        "valu_roofline": valu,
        "lib_hash": lib_hash(),
        "stages": {k: {"ms_per_step": st[k]["ms_per_launch"] * st[k]["launches_per_step"],
                       "units_per_launch": st[k]["units_per_launch"]} for k in STAGES},
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        k = args.cpu_sample if cfg != 7 else min(args.cpu_sample, 1 << 13)
        threads = args.cpu_threads or box_threads()
        result["cpu_baseline"] = cpu_baseline(cfg, q_host[:k], flags, masks, threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def scenes_name(cfg):
    from mplib_amd import scenes
    return scenes.CFG_NAME[cfg]


def rooflines(st, cfg, dim, W):
    """(roofline, valu_roofline) of the dominant kernel from the per-stage
    profile `st` (HIP events on the launch stream) and, when it was collected
    with this library build, profiles/pmc_cfg<cfg>.json."""
    # roofline of the dominant kernel (DESIGN.md "Measurement"): achieved =
    # SURVEY.md 8(d)'s algorithmic bytes per configuration (q row 8*dof + flag 1
    # + pair mask 4W: 77 B for cfg3) x the configurations one launch covers,
    # over that kernel's average duration (HIP events on its launch stream)
    bytes_per_config = 8 * dim + 1 + 4 * W
    dom = max(("cull", "narrow"), key=lambda k: st[k]["ms_per_launch"])
    cfg_per_launch = st["cull"]["units_per_launch"]  # both stages run once per batch part
    kernel_s = st[dom]["ms_per_launch"] * 1e-3
    achieved_gbps = bytes_per_config * cfg_per_launch / kernel_s / 1e9
    traffic, valu = None, None
    pm = pmc_record(cfg)
    if pm is not None and pm.get("configs_per_launch") == int(cfg_per_launch):
        k = pm.get("kernels", {}).get(dom, {})
        traffic = k.get("hbm_bytes")
        if "SQ_INSTS_VALU" in k:
            f64 = sum(k.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                                "SQ_INSTS_VALU_TRANS_F64"))
            # the PMC kernel is the dominant stage's main kernel (narrow_kernel / cull_kernel); its duration is
            # the live event time of the stage launch
            issue_cyc = (k["SQ_INSTS_VALU"] + f64) * VALU_ISSUE_CYCLES / SIMDS  # per SIMD
            clk = k.get("clock_ghz")
            # the measured clock (GRBM_GUI_ACTIVE / 8 / dispatch time in the PMC pass), else the nominal one
            hz = clk * 1e9 if clk else CLOCK_HZ
            frac_live = issue_cyc / (hz * kernel_s)
            # the same kernel alone in the PMC pass: VALU issue cycles over its own active cycles
            frac_pmc = issue_cyc / (k["GRBM_GUI_ACTIVE"] / 8.0) if k.get("GRBM_GUI_ACTIVE") else None
            valu = {"bound": "valu", "achieved": frac_live, "peak": 1.0, "unit": "issue-port fraction",
                    "frac": frac_live, "frac_alone": frac_pmc, "clock_ghz": clk,
                    "clock_source": "GRBM_GUI_ACTIVE/8/dispatch ns (PMC pass)" if clk else "nominal 2.4 GHz",
                    "pmc_dispatch_ms": k.get("pmc_dispatch_ns", 0.0) / 1e6 or None,
                    "valu_insts_per_launch": k["SQ_INSTS_VALU"],
                    "fp64_insts_per_launch": f64,
                    "lane_activity": (k["SQ_THREAD_CYCLES_VALU"] / (64.0 * k["SQ_ACTIVE_INST_VALU"])
                                      if k.get("SQ_ACTIVE_INST_VALU") else None),
                    "wait_frac": (k["SQ_WAIT_ANY"] / k["SQ_WAVE_CYCLES"] if k.get("SQ_WAVE_CYCLES") else None),
                    "note": "VALU instructions x 2 issue cycles (fp64 counted twice) per SIMD over the measured "
                            "clock x the kernel's live duration (frac) and over its active cycles when it runs "
                            "alone in the PMC pass (frac_alone); "
                            "PMC counts from " + pm.get("source", "?")}

    roofline = {"bound": "hbm", "achieved": achieved_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved_gbps / HBM_PEAK_GBPS, "traffic": traffic,
                "kernel": KERNEL_NAME[dom], "kernel_ms": st[dom]["ms_per_launch"],
                "units_per_launch": cfg_per_launch, "unit_kind": "configs",
                "algorithmic_bytes_per_unit": bytes_per_config,
                "note": "SURVEY.md 8(d) bytes per configuration; the path is VALU and latency bound, not HBM "
                        "bound (DESIGN.md), see valu_roofline"}
    return roofline, valu


def dryrun_main(args, world, rank, launched):
    """MPLIB_AMD_BENCH_DRYRUN=1 (CPU tests of the rank fan-out, gloo): the
    launch, process group, barrier and max-over-ranks reduction of a real run,
    no device work; rank 0 prints a line with value null."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(rank)], dtype=torch.float64)
    if launched:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry run (no device work)", "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "max_rank": int(t[0]),
                          "backend": dist.get_backend() if launched else None}), flush=True)
    if launched:
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
    if args.spec_nodes is not None:
        planner.set_speculation_nodes(args.spec_nodes)

    def one(seed):
        pymp.set_global_seed(seed)
        return planner.plan(scenes.PLAN_START, [goal], range=0.1, time=60.0)

    for i in range(args.warmup):
        one(10_000 + i)
    w.profile_enable(True)
    w.profile_read()
    stats, paths, solved = [], {}, 0
    if dist.is_initialized():
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
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    mean = lambda k: float(np.mean([s[k] for s in stats]))  # noqa: E731
    # the latency path records each batch as one narrow-stage entry: a
    # small_kernel launch (event time) or a batch served by the resident
    # lat_server_kernel (host post -> done time)
    ms, launches, units = prof["narrow"]
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
        "mean_spec_nodes": mean("spec_nodes"), "mean_spec_wait_nodes": mean("spec_wait_nodes"),
        "mean_spec_ms": mean("t_spec") * 1e3,
        "roofline": {"bound": "latency", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": "lat_server_kernel (<=32 states) / small_kernel",
                     "kernel_ms": kern_ms, "units_per_launch": states_per_launch, "unit_kind": "states",
                     "algorithmic_bytes_per_unit": bytes_per_state,
                     "note": "one validity batch per planner iteration: round-trip latency, not bandwidth, "
                             "bounds a plan"},
    }
    # the validity round trip the planner pays per batch: one state, host buffers
    one = np.array([scenes.PLAN_START])
    for _ in range(20):
        w.collide_batch(one)
    rt = []
    for _ in range(300):
        t1 = time.perf_counter()
        w.collide_batch(one)
        rt.append(time.perf_counter() - t1)
    result_rt = {"one_state_round_trip_us_median": float(np.median(rt) * 1e6),
                 "one_state_round_trip_us_p90": float(np.percentile(rt, 90) * 1e6)}
    if rank == 0 and world == 1 and args.cpu_plans != 0:
        import ctypes
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle  # test infrastructure: the CPU baseline's checker
        import worlds as Wd  # test fixture module: the oracle-built cfg3 world
        ow = Wd.oracle_world(3)
        cpu = pymp.ompl.OMPLPlanner(scenes.world(3)[0])
        # C-level checker (oracle orc_validity_batch): no Python per validity call, as OMPL's
        # C++ StateValidityChecker would be called by the reference
        cpu.set_native_state_validity_checker(ctypes.cast(oracle.lib().orc_validity_batch, ctypes.c_void_p).value,
                                              ctypes.addressof(ow._w))
        cpu.set_speculative_connect(False)  # OMPL's serial loop: one batch per growTree
        k = args.steps if args.cpu_plans < 0 else min(args.cpu_plans, args.steps)
        same = True
        t0 = time.perf_counter()
        for i in range(k):
            pymp.set_global_seed(i)
            st, path = cpu.plan(scenes.PLAN_START, [goal], range=0.1, time=60.0)
            same &= bool(np.array_equal(path, paths[i]))
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": k / dt, "unit": "plans/s", "cores": 1, "kind": "port",
                                  "sample": f"seeds 0..{k - 1}: the same planner with oracle/collide_oracle.c "
                                            f"(orc_validity_batch, called from C++) as its checker, OMPL's serial "
                                            f"loop (one check per growTree step), {dt:.1f} s",
                                  "cpu_model": cpu_model(), "gpu_matches_cpu_on_sample": same}
    result.update(result_rt)
    sys.stdout.flush()
    os.dup2(saved_stdout, 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def lib_hash() -> str:
    """Hash of the sources and HIP flags libmpgpu.so is built from
    (tools/build_hash.py): profiles are keyed by it."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_hash import build_hash
    return build_hash()


def pmc_record(cfg):
    """profiles/pmc_cfg<cfg>.json (tools/pmc_summary.py) when it was collected
    with this very library build, else None."""
    f = os.path.join(ROOT, "profiles", f"pmc_cfg{cfg}.json")
    try:
        pm = json.load(open(f))
    except (OSError, ValueError):
        return None
    return pm if pm.get("lib_hash") == lib_hash() else None


def box_threads() -> int:
    """The host cores this job may use: OMP_NUM_THREADS (16 per GPU on the
    GPU pool) or nproc."""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "0"))) if os.environ.get("OMP_NUM_THREADS") else \
            len(os.sched_getaffinity(0))
    except (ValueError, AttributeError):
        return os.cpu_count() or 1


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, q_sample, flags, masks, threads):
    """The CPU restatement of MPlib's PlanningWorld::collide (oracle/) timed on
    this host: one core (the reference's execution model) on a bounded sample,
    and `threads` cores on the whole sample; also cross-checks the GPU results."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import worlds as Wd  # test fixture module: oracle-built world of the same config

    ow = Wd.oracle_world(cfg)
    k = len(q_sample)
    k1 = max(256, k // 4)
    ow.collide_batch(q_sample[:256], nthreads=1)  # warm
    t0 = time.perf_counter()
    ow.collide_batch(q_sample[:k1], nthreads=1)
    dt1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    fo, mo = ow.collide_batch(q_sample, nthreads=threads)
    dt = time.perf_counter() - t0
    as_np = lambda x: x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)  # noqa: E731
    parity = bool(np.array_equal(fo, as_np(flags[:k])) and np.array_equal(mo, as_np(masks[:k]).view(np.uint32)))
    return {"value": k / dt, "unit": "configs/s", "cores": threads, "kind": "port",
            "single_core": {"value": k1 / dt1, "unit": "configs/s", "cores": 1,
                            "sample": f"first {k1} configs, {dt1:.1f} s"},
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "sample": f"first {k} configs of the rank-0 batch, oracle/collide_oracle.c (C restatement of "
                      f"FK + FCL/libccd MPR + PlanningWorld loops) on {threads} threads, {dt:.1f} s",
            "gpu_matches_cpu_on_sample": parity}


if __name__ == "__main__":
    main()
