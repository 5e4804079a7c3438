"""Multi-GPU sharding of the batched validity check.

``isValid`` is a pure function of the state (src/ompl_planner.h:59-62), so a
batch splits into contiguous configuration ranges, one process per GPU, with
no collective in the data path.  ``collide_sharded`` runs this rank's range
and, when asked, all-gathers flags and pair masks so every rank holds the
whole result (RCCL all-gather over xGMI with the ``nccl`` backend; gloo on
CPU in the tests).  ``collide_sharded_device`` is the same split with the
batch, the results and the gather all resident on the GPU (no host copy):
each rank launches its slice of a device tensor through
``collide_batch_device`` and RCCL all-gathers flags and pair masks into
device tensors.  ``distance_sharded_device`` does the same for
PlanningWorld::distanceSelf / distanceOthers (src/planning_world.cpp:493-720):
each rank's ``distance_batch_device`` slice, then the per-group minima and
their pair indices all-gathered.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """(start, count) of rank's contiguous share of n items; the first n % world
    ranks take one extra."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(int(n), world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def collide_sharded(compute, states: np.ndarray, group=None, gather: bool = True, device: Optional[str] = None):
    """Check this rank's shard of ``states`` and optionally gather every shard.

    compute: a PlanningWorld (its ``collide_batch`` is used) or any callable
             ``states -> (flags u8 [n], masks u32 [n, W])``.
    Returns (flags, masks) for the whole batch when ``gather`` else for the
    shard, plus the shard's (start, count).
    """
    import torch
    import torch.distributed as dist

    fn: Callable = compute.collide_batch if hasattr(compute, "collide_batch") else compute
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    states = np.ascontiguousarray(states, dtype=np.float64)
    start, count = shard_range(len(states), rank, world)
    flags, masks = fn(states[start:start + count])
    flags = np.asarray(flags, dtype=np.uint8).reshape(count)
    masks = np.asarray(masks, dtype=np.uint32).reshape(count, -1)
    if not gather or world == 1:
        return flags, masks, (start, count)
    W = masks.shape[1]
    cap = -(-len(states) // world)  # shards differ by at most one row: pad to the largest
    if device is None:
        device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    buf = torch.zeros((cap, 1 + 4 * W), dtype=torch.uint8, device=device)
    row = np.concatenate([flags[:, None], masks.view(np.uint8).reshape(count, 4 * W)], axis=1)
    buf[:count] = torch.from_numpy(row).to(device)
    out = torch.empty((world * cap, 1 + 4 * W), dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.cpu().numpy().reshape(world, cap, 1 + 4 * W)
    parts = [out[r, :shard_range(len(states), r, world)[1]] for r in range(world)]
    full = np.concatenate(parts, axis=0)
    all_flags = np.ascontiguousarray(full[:, 0])
    all_masks = np.ascontiguousarray(full[:, 1:]).view(np.uint32).reshape(len(states), W)
    return all_flags, all_masks, (start, count)


def _gather_rows(parts, n, cap, group):
    """all_gather_into_tensor of each [cap, ...] tensor in parts over the group,
    the padding rows of the short shards dropped: [n, ...] each."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = []
    for t in parts:
        full = torch.empty((world * cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(full, t, group=group)
        out.append(full)
    if world * cap != n:
        keep = torch.cat([torch.arange(r * cap, r * cap + shard_range(n, r, world)[1], device=parts[0].device)
                          for r in range(world)])
        out = [t.index_select(0, keep) for t in out]
    return out


def collide_sharded_device(compute, states, group=None, gather: bool = True, mask_words: Optional[int] = None):
    """Device-resident sharded check.

    states:  torch float64 tensor [n, dim] on this rank's device, the same
             batch on every rank (e.g. broadcast by the caller).
    compute: a PlanningWorld (``collide_batch_device`` on torch's current
             stream) or a callable ``(states_slice, flags_out, masks_out)``
             filling the given output tensors (``mask_words`` then required).
    Returns (flags uint8 [n], masks int32 [n, W]) for the whole batch when
    ``gather`` (all_gather_into_tensor over the group: RCCL on GPUs) else for
    the shard, and the shard's (start, count).
    """
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if states.dtype != torch.float64 or states.dim() != 2:
        raise ValueError("states must be a float64 tensor [n, dim]")
    states = states.contiguous()
    n, dev = states.shape[0], states.device
    start, count = shard_range(n, rank, world)
    if hasattr(compute, "collide_batch_device"):
        W = compute.get_mask_words()

        def run(q, f, m):
            if q.shape[0]:
                compute.collide_batch_device(q.data_ptr(), q.shape[0], f.data_ptr(), m.data_ptr(),
                                             torch.cuda.current_stream(dev).cuda_stream)
    else:
        if mask_words is None:
            raise ValueError("mask_words is required with a callable compute")
        W, run = int(mask_words), compute
    cap = -(-n // world) if world > 1 else n  # shards differ by at most one row: pad to the largest
    flags = torch.zeros(cap, dtype=torch.uint8, device=dev)
    masks = torch.zeros((cap, W), dtype=torch.int32, device=dev)
    run(states[start:start + count], flags[:count], masks[:count])
    if not gather or world == 1:
        return flags[:count], masks[:count], (start, count)
    all_f, all_m = _gather_rows([flags, masks], n, cap, group)
    return all_f, all_m, (start, count)


def distance_sharded_device(compute, states, group=None, gather: bool = True, request=None,
                            nearest_points: bool = False):
    """Device-resident sharded distanceSelf / distanceOthers.

    states:  torch float64 tensor [n, dim] on this rank's device, the same
             batch on every rank.
    compute: a PlanningWorld (``distance_batch_device`` on torch's current
             stream, with ``request``: a DistanceRequest or None) or a callable
             ``(states_slice, d_self, p_self, d_others, p_others, pts_self,
             pts_others)`` filling the given tensors (pts_* None unless
             nearest_points).
    Returns a dict of tensors -- d_self / d_others float64 [n] (DBL_MAX for an
    empty group), p_self / p_others int32 [n] (the minimum's pair index, -1
    for none), and with nearest_points pts_self / pts_others float64 [n, 6] --
    for the whole batch when ``gather`` (RCCL all-gather on GPUs) else for the
    shard, and the shard's (start, count).
    Configurations where FCL throws (signed distance: libccd's EPA,
    FCL_THROW_FAILED_AT_THIS_CONFIGURATION) come back from the device as NaN
    distances with p = -2 (MPG_DISTANCE_FCL_THROWS), and p = -3 when the EPA
    polytope outgrew the device's capacity (MPG_DISTANCE_EPA_CAPACITY); this
    helper raises RuntimeError for either (after the gather, on every rank),
    as the host-buffer API does, so no negative index reaches a pair table.
    """
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if states.dtype != torch.float64 or states.dim() != 2:
        raise ValueError("states must be a float64 tensor [n, dim]")
    states = states.contiguous()
    n, dev = states.shape[0], states.device
    start, count = shard_range(n, rank, world)
    cap = -(-n // world) if world > 1 else n
    out = {"d_self": torch.zeros(cap, dtype=torch.float64, device=dev),
           "p_self": torch.full((cap,), -1, dtype=torch.int32, device=dev),
           "d_others": torch.zeros(cap, dtype=torch.float64, device=dev),
           "p_others": torch.full((cap,), -1, dtype=torch.int32, device=dev)}
    if nearest_points:
        out["pts_self"] = torch.zeros((cap, 6), dtype=torch.float64, device=dev)
        out["pts_others"] = torch.zeros((cap, 6), dtype=torch.float64, device=dev)
    sl = {k: v[:count] for k, v in out.items()}
    q = states[start:start + count]
    if hasattr(compute, "distance_batch_device"):
        if count:
            ptr = lambda k: sl[k].data_ptr() if k in sl else 0  # noqa: E731
            compute.distance_batch_device(q.data_ptr(), count, ptr("d_self"), ptr("p_self"), ptr("d_others"),
                                          ptr("p_others"), ptr("pts_self"), ptr("pts_others"),
                                          torch.cuda.current_stream(dev).cuda_stream, request)
    else:
        compute(q, sl["d_self"], sl["p_self"], sl["d_others"], sl["p_others"], sl.get("pts_self"),
                sl.get("pts_others"))
    if not gather or world == 1:
        _raise_on_sentinels(sl["p_self"], start)
        return sl, (start, count)
    keys = list(out)
    res = dict(zip(keys, _gather_rows([out[k] for k in keys], n, cap, group)))
    _raise_on_sentinels(res["p_self"], 0)
    return res, (start, count)


MPG_DISTANCE_FCL_THROWS, MPG_DISTANCE_EPA_CAPACITY = -2, -3  # include/mpgpu.h


def _raise_on_sentinels(p_self, offset: int):
    """The device marks a failed configuration in both groups' pair index
    (mpg_distance_batch_req); one small device reduction finds the first."""
    bad = (p_self < -1).nonzero()
    if bad.numel() == 0:
        return
    i = int(bad[0, 0])
    code = int(p_self[i])
    if code == MPG_DISTANCE_FCL_THROWS:
        raise RuntimeError(f"configuration {offset + i}: FCL's libccd EPA throws here "
                           "(FCL_THROW_FAILED_AT_THIS_CONFIGURATION)")
    raise RuntimeError(f"configuration {offset + i}: EPA polytope beyond the device capacity (code {code})")
