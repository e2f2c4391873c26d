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


def _config4_worker(rank, world, port, per, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from halo_amd import synth
    from oracle import oracle

    d = bench.Dist()
    first, per = bench.config4_shard(rank, per)
    assert bench.shard_first_index(rank, 0, per, 1) == first
    netif = oracle.NetIf.make()
    lay = synth.layout(per, length=64, mutate_shift=4, first_index=first)
    data = oracle.synth_batch(synth.SEED, first, lay["lens"], lay["kinds"], netif, offsets_dw=lay["offsets_dw"])
    recs, _ = oracle.rx_batch(data, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"])
    t = torch.from_numpy(recs.view(np.uint8).copy())
    gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gathered, dst=0)
    kms = d.gather(0.25 * (rank + 1))  # every rank's own launch time, in rank order
    ids = d.gather_obj({"rank": rank, "pci_bus_id": f"0000:{rank:02x}:00.0"})  # per-rank facts, rank order
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in gathered]), kms, ids))
    d.close()


def test_config4_weak_shards_over_two_ranks():
    """bench.py --gpus N's config-4 run: every rank owns one contiguous 16M-frame slice of the frame
    stream (8 ranks = config 4's 128M); concatenated, the two ranks' records equal the
    single-process parse of the whole stream, and every rank's kernel time and identity reach rank 0
    in rank order."""
    import bench
    from halo_amd import synth
    from oracle import oracle

    for w in (1, 2, 4, 8):  # the partition the driver's 1/2/4/8-GPU runs use
        shards = [bench.config4_shard(r) for r in range(w)]
        assert shards[0][0] == 0 and all(c == bench.CONFIG4_PER_GPU for _, c in shards)
        assert all(shards[r][0] + shards[r][1] == shards[r + 1][0] for r in range(w - 1))
    assert sum(c for _, c in (bench.config4_shard(r) for r in range(8))) == bench.CONFIG4_FRAMES
    # bench.py's defaults make each rank's shard exactly one config-4 shard
    import sys

    argv, sys.argv = sys.argv, ["bench.py"]
    try:
        a = bench.parse_args()
    finally:
        sys.argv = argv
    assert a.frames * a.rotate == bench.CONFIG4_PER_GPU
    per, world = 2048, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, kms, ids = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    netif = oracle.NetIf.make()
    lay = synth.layout(per * world, length=64, mutate_shift=4, first_index=0)
    data = oracle.synth_batch(synth.SEED, 0, lay["lens"], lay["kinds"], netif, offsets_dw=lay["offsets_dw"])
    whole, _ = oracle.rx_batch(data, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"])
    assert np.array_equal(got, whole.view(np.uint8).reshape(-1))
    assert kms == [0.25, 0.5]
    assert [i["rank"] for i in ids] == [0, 1] and len({i["pci_bus_id"] for i in ids}) == 2


@pytest.mark.parametrize("length,size_mode", [(64, 0), (0, 1)])
def test_shard_batch_views_equal_separate_batches(length, size_mode):
    """shard_batches' rebasing: batch b of a rank's contiguous shard, with its byte base moved to its
    first frame and its offsets rebased, is frame for frame the batch make_batches generates on its
    own for the same global indices (lengths, kinds, relative offsets)."""
    import bench
    from halo_amd import synth

    n, rotate, rank = 1000, 4, 3
    first = bench.shard_first_index(rank, 0, n * rotate, 1)
    kw = dict(length=length or 64, size_mode=size_mode, proto_mode=3 if size_mode else 0)
    whole = synth.layout(n * rotate, first_index=first, **kw)
    for b in range(rotate):
        lo = b * n
        sep = synth.layout(n, first_index=bench.shard_first_index(rank, b, n, rotate), **kw)
        o0 = int(whole["offsets_dw"][lo])
        assert np.array_equal(whole["offsets_dw"][lo:lo + n] - np.uint32(o0), sep["offsets_dw"])
        assert np.array_equal(whole["lens"][lo:lo + n], sep["lens"])
        assert np.array_equal(whole["kinds"][lo:lo + n], sep["kinds"])


def test_rank_plan_and_launcher(monkeypatch):
    """--gpus N > 1 without WORLD_SIZE starts torch.distributed.run as a child (never an exec) with
    N ranks on 127.0.0.1 and passes its exit code through; a WORLD_SIZE that disagrees with --gpus is
    refused; --gpus 1 without a launcher runs in-process."""
    import subprocess

    import bench

    assert bench.rank_plan(1, {}) == "single"
    assert bench.rank_plan(2, {}) == "spawn"
    assert bench.rank_plan(8, {"WORLD_SIZE": "8"}) == "ranks"
    assert bench.rank_plan(1, {"WORLD_SIZE": "1"}) == "ranks"
    assert bench.rank_plan(4, {"WORLD_SIZE": "2"}) == "mismatch"
    assert bench.rank_plan(1, {"WORLD_SIZE": "2"}) == "mismatch"
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    assert bench.launch_ranks(2, ["--gpus", "2", "--steps", "5"]) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "5"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_refuses_world_size_mismatch():
    """A launcher whose WORLD_SIZE is not --gpus: bench.py exits 2 before touching the GPU."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
