"""World-size-2 gloo tests of the frame-sharding / timing-reduction logic (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drnmi.dist import max_over_ranks, shard_range, sum_over_ranks


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = list(shard_range(37, rank, world))
        mine = torch.zeros(37, dtype=torch.int64)
        mine[frames] = 1
        sum_over_ranks(mine)
        slowest = max_over_ranks(0.5 + rank)
        hist = torch.full((19, 19), rank + 1, dtype=torch.int64)
        sum_over_ranks(hist)
        q.put((rank, mine.tolist(), slowest, int(hist[0, 0])))
    finally:
        dist.destroy_process_group()


def test_shard_range_balanced():
    for total in (0, 1, 7, 64, 1001):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert sum(len(r) for r in rs) == total
            assert max(len(r) for r in rs) - min(len(r) for r in rs) <= 1
            flat = [i for r in rs for i in r]
            assert flat == list(range(total))
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_gloo_world2_shards_cover_once_and_reduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, cover, slowest, h00 in out:
        assert cover == [1] * 37          # every frame processed by exactly one rank
        assert slowest == 1.5             # max over ranks
        assert h00 == 3                   # 1 + 2 summed


def _reducer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from drnmi.parallel import BucketReducer
        sizes = [300, 50, 700, 10, 10, 400, 1000, 3]          # "parameters" in backward order
        params = [torch.empty(n) for n in sizes]
        flat = torch.arange(sum(sizes), dtype=torch.float32) * (rank + 1)
        r = BucketReducer(flat, params, bucket_cap_bytes=1024 * 4)    # 1024-element buckets
        bounds = [(s, e) for s, e, _ in r.buckets]
        r.mark_ready(params[:2])
        early = list(r.launch_order)                          # nothing complete yet
        r.mark_ready(params[2:3])                             # closes bucket 0 (>= 1024 elements)
        after_first = list(r.launch_order)
        r.mark_ready(params[3:])
        r.finalize()
        q.put((rank, bounds, early, after_first, flat.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bucket_reducer():
    """Buckets are contiguous slices in backward order, launched as soon as complete, and the
    result is the SUM over ranks (the runner pre-scales by 1/world, so this is DDP's mean)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = 2473
    expect = [3.0 * i for i in range(total)]
    for rank, bounds, early, after_first, flat in out:
        assert bounds[0] == (0, 1050) and bounds[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
        assert early == [] and after_first == [0]
        assert flat == expect
