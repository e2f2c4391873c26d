"""CPU, world_size 2 over gloo: the N>1 path of bench.py shards the frame stream by index
with no data exchange; each rank's shard parsed on its own equals the matching slice of the
single-process result, and the max-over-ranks timing reduction works."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_records(rank: int, n: int, rotate: int):
    import bench
    from halo_amd import synth
    from oracle import oracle

    netif = oracle.NetIf.make()
    recs = []
    for b in range(rotate):
        first = bench.shard_first_index(rank, b, n, rotate)
        lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=3, first_index=first)
        data = oracle.synth_batch(synth.SEED, first, lay["lens"], lay["kinds"], netif, offsets_dw=lay["offsets_dw"])
        r, _ = oracle.rx_batch(data, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"])
        recs.append(r)
    return np.concatenate(recs)


def _worker(rank, world, port, n, rotate, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench

    d = bench.Dist()
    assert d.world == world and d.rank == rank
    recs = _shard_records(rank, n, rotate)
    t = torch.from_numpy(recs.view(np.uint8).copy())
    gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gathered, dst=0)
    slowest = d.max(float(rank + 1))
    d.barrier()
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in gathered]), slowest))
    d.close()


def test_two_rank_shards_equal_single_process():
    n, rotate, world = 300, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, rotate, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, slowest = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = np.concatenate([_shard_records(r, n, rotate) for r in range(world)]).view(np.uint8)
    assert np.array_equal(got, single.reshape(-1))
    assert slowest == float(world)
    # shards are disjoint slices of one global stream: rank 1 batch 0 starts after rank 0's batches
    import bench

    assert bench.shard_first_index(1, 0, n, rotate) == bench.shard_first_index(0, rotate - 1, n, rotate) + n


def _config4_worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from halo_amd import synth
    from oracle import oracle

    d = bench.Dist()
    first, per = bench.config4_shard(rank, world, total)
    # the shard the config-4 run generates on this rank: make_batches' layout, rotate = 1
    assert bench.shard_first_index(rank, 0, per, 1) == first
    netif = oracle.NetIf.make()
    lay = synth.layout(per, length=64, mutate_shift=4, first_index=first)
    data = oracle.synth_batch(synth.SEED, first, lay["lens"], lay["kinds"], netif, offsets_dw=lay["offsets_dw"])
    recs, _ = oracle.rx_batch(data, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"])
    t = torch.from_numpy(recs.view(np.uint8).copy())
    gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gathered, dst=0)
    kms = d.gather(0.25 * (rank + 1))  # every rank's own launch time, in rank order
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in gathered]), kms))
    d.close()


def test_config4_strong_shards_over_two_ranks():
    """bench.py --gpus N's config-4 run: ranks own contiguous equal slices of one frame stream;
    concatenated, the two ranks' records equal the single-process parse of the whole stream, and
    every rank's kernel time reaches rank 0 in rank order."""
    import bench
    from halo_amd import synth
    from oracle import oracle

    total, world = 4096, 2
    for w in (1, 2, 4, 8):  # the partition the driver's 1/2/4/8-GPU runs use
        shards = [bench.config4_shard(r, w) for r in range(w)]
        assert shards[0][0] == 0 and sum(c for _, c in shards) == bench.CONFIG4_FRAMES
        assert all(shards[r][0] + shards[r][1] == shards[r + 1][0] for r in range(w - 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, kms = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    netif = oracle.NetIf.make()
    lay = synth.layout(total, length=64, mutate_shift=4, first_index=0)
    data = oracle.synth_batch(synth.SEED, 0, lay["lens"], lay["kinds"], netif, offsets_dw=lay["offsets_dw"])
    whole, _ = oracle.rx_batch(data, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"])
    assert np.array_equal(got, whole.view(np.uint8).reshape(-1))
    assert kms == [0.25, 0.5]
