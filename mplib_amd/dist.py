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
device tensors.
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
    all_f = torch.empty(world * cap, dtype=torch.uint8, device=dev)
    all_m = torch.empty((world * cap, W), dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(all_f, flags, group=group)
    dist.all_gather_into_tensor(all_m, masks, group=group)
    if world * cap != n:  # drop the padding rows of the short shards
        keep = torch.cat([torch.arange(r * cap, r * cap + shard_range(n, r, world)[1], device=dev)
                          for r in range(world)])
        all_f, all_m = all_f.index_select(0, keep), all_m.index_select(0, keep)
    return all_f, all_m, (start, count)
