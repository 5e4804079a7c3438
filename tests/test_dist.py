"""CPU: configuration sharding + gather over torch.distributed (gloo,
world_size 2, 127.0.0.1), the same code path bench.py / multi-GPU callers use
with RCCL.  The per-rank compute is the CPU oracle here (no GPU in this
container); on the GPU box it is PlanningWorld.collide_batch."""
import os
import socket

import numpy as np
import pytest

from mplib_amd.dist import shard_range


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 64, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == n
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    import worlds as Wd
    from mplib_amd.dist import collide_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ow = Wd.oracle_world(3)
    f, m, (s, c) = collide_sharded(lambda x: ow.collide_batch(x, nthreads=1), q)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), flags=f, masks=m, start=s, count=c)
    dist.barrier()
    dist.destroy_process_group()


def test_collide_sharded_gloo_world2(tmp_path):
    mp = pytest.importorskip("torch.multiprocessing")
    import worlds as Wd
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, 1001, 31)  # odd size: ragged shards
    mp.start_processes(_worker, args=(2, _free_port(), q, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    fo, mo = ow.collide_batch(q, nthreads=4)
    for r in range(2):
        d = np.load(tmp_path / f"r{r}.npz")
        np.testing.assert_array_equal(d["flags"], fo)
        np.testing.assert_array_equal(d["masks"], mo)
    assert int(np.load(tmp_path / "r0.npz")["count"]) == 501


def _worker_device(rank, world, port, q, out_dir):
    """collide_sharded_device's split + gather with CPU tensors over gloo; the
    per-rank compute (the oracle) writes into the given output slices."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    import torch.distributed as dist
    import worlds as Wd
    from mplib_amd.dist import collide_sharded_device
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ow = Wd.oracle_world(3)
    W = ow.W

    def compute(qs, f, m):
        fo, mo = ow.collide_batch(qs.numpy(), nthreads=1)
        f.copy_(torch.from_numpy(fo))
        m.copy_(torch.from_numpy(mo.view(np.int32)))

    f, m, (s, c) = collide_sharded_device(compute, torch.from_numpy(q), mask_words=W)
    fs, ms, _ = collide_sharded_device(compute, torch.from_numpy(q), gather=False, mask_words=W)
    np.savez(os.path.join(out_dir, f"d{rank}.npz"), flags=f.numpy(), masks=m.numpy(), start=s, count=c,
             shard_flags=fs.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1001, 1000])
def test_collide_sharded_device_gloo_world2(tmp_path, n):
    mp = pytest.importorskip("torch.multiprocessing")
    import worlds as Wd
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, n, 37)  # 1001: ragged shards, padding dropped after the gather
    mp.start_processes(_worker_device, args=(2, _free_port(), q, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    fo, mo = ow.collide_batch(q, nthreads=4)
    for r in range(2):
        d = np.load(tmp_path / f"d{r}.npz")
        np.testing.assert_array_equal(d["flags"], fo)
        np.testing.assert_array_equal(d["masks"].view(np.uint32), mo)
        s, c = int(d["start"]), int(d["count"])
        np.testing.assert_array_equal(d["shard_flags"], fo[s:s + c])
    assert 0.0 < fo.mean() < 1.0


def _worker_distance(rank, world, port, q, out_dir):
    """distance_sharded_device's split + gather (gloo, CPU tensors); the
    per-rank compute is the oracle's distance_batch_ex with nearest points."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    import torch.distributed as dist
    import worlds as Wd
    from mplib_amd.dist import distance_sharded_device
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ow = Wd.oracle_world(3)

    def compute(qs, ds, ps, do, po, pts_s, pts_o):
        r = ow.distance_batch_ex(qs.numpy(), signed=True)
        for t, v in zip((ds, ps, pts_s, do, po, pts_o), r):
            t.copy_(torch.from_numpy(np.asarray(v)))

    out, (s, c) = distance_sharded_device(compute, torch.from_numpy(q), nearest_points=True)
    sh, _ = distance_sharded_device(compute, torch.from_numpy(q), gather=False, nearest_points=True)
    np.savez(os.path.join(out_dir, f"x{rank}.npz"), start=s, count=c, shard_d=sh["d_self"].numpy(),
             **{k: v.numpy() for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_distance_sharded_device_gloo_world2(tmp_path):
    """The distance results (per-group minima, pair indices, nearest points)
    split over two ranks and all-gathered equal the unsharded batch."""
    mp = pytest.importorskip("torch.multiprocessing")
    import worlds as Wd
    ow = Wd.oracle_world(3)
    q = Wd.sample_q(ow.art, 301, 43)  # ragged shards
    mp.start_processes(_worker_distance, args=(2, _free_port(), q, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ds, ps, qs, do, po, qo = ow.distance_batch_ex(q, signed=True)
    for r in range(2):
        d = np.load(tmp_path / f"x{r}.npz")
        np.testing.assert_array_equal(d["d_self"], ds)
        np.testing.assert_array_equal(d["p_self"], ps)
        np.testing.assert_array_equal(d["d_others"], do)
        np.testing.assert_array_equal(d["p_others"], po)
        np.testing.assert_array_equal(d["pts_self"], qs)
        np.testing.assert_array_equal(d["pts_others"], qo)
        s, c = int(d["start"]), int(d["count"])
        np.testing.assert_array_equal(d["shard_d"], ds[s:s + c])
    assert (np.minimum(ds, do) < 0).any()


def test_distance_sharded_device_raises_on_fcl_throw_sentinels(tmp_path):
    """the device marks a configuration where FCL throws with p =
    -2 (MPG_DISTANCE_FCL_THROWS) and NaN distances, p = -3 past the EPA
    capacity; distance_sharded_device raises instead of handing back a
    negative pair index (one rank, gloo)."""
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    from mplib_amd.dist import distance_sharded_device
    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        for code, what in ((-2, "throws"), (-3, "capacity")):
            def compute(q, ds, ps, do, po, pts_s, pts_o, code=code):
                ds.fill_(0.5)
                do.fill_(0.25)
                ps.fill_(3)
                po.fill_(7)
                ps[5] = code
                po[5] = code
                ds[5] = float("nan")
                do[5] = float("nan")
            with pytest.raises(RuntimeError, match=f"configuration 5: .*{what}"):
                distance_sharded_device(compute, torch.zeros((9, 7), dtype=torch.float64))

        def clean(q, ds, ps, do, po, pts_s, pts_o):
            ds.fill_(0.5)
            do.fill_(0.25)
            ps.fill_(-1)
            po.fill_(2)
        out, (s, c) = distance_sharded_device(clean, torch.zeros((9, 7), dtype=torch.float64))
        assert (s, c) == (0, 9) and int(out["p_self"][0]) == -1
    finally:
        dist.destroy_process_group()
