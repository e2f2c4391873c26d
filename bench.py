#!/usr/bin/env python3
"""bench.py — device-resident rx parse + checksum throughput (BASELINE.json metric).

Headline workload (BASELINE.json configs[1]): 1M synthetic 64 B IPv4/UDP frames resident in
HBM, protocol.CheckSumEnable = true, parsed Ethernet -> IPv4 -> UDP with both checksums
verified, one 32 B result record per frame. A step is one launch of the hot-path kernel over
one batch of 1M frames. Batches rotate over --rotate distinct slices of the synthetic stream
so the working set (8 x 102 MB) exceeds the 256 MB Infinity Cache and every step streams
from HBM.

Multi-GPU (--gpus N, one process per GPU): BASELINE config 4, the scaling run. Every rank owns
one contiguous 16M-frame slice of the 64 B frame stream (rank r: global frames [r*16M, (r+1)*16M),
so N = 8 covers config 4's 128M frames) and runs exactly the N=1 headline step on it: one
1M-frame launch per step, rotating over its 16 batches (weak scaling: the work per GPU is fixed).
No data-path collective: the gloo group carries only the barriers, the max-over-ranks wall time
and per-rank facts (launch duration, PCI bus id, the shard's own validation). value = N x 1M x
steps / max wall time. When --gpus N > 1 is given without a launcher around it (WORLD_SIZE unset),
bench.py starts torch.distributed.run as a CHILD process (never an exec) before anything touches
the GPU, and exits with its return code; rank 0's JSON line is the child's stdout. A WORLD_SIZE
that disagrees with --gpus is refused (exit 2).

Extra fields: roofline (dominant kernel, algorithmic bytes / HIP-event kernel time vs the
8 TB/s HBM3E spec peak), cpu_baseline (the C oracle, a scalar port of the Go path, timed on
this host's cores on a bounded sample), secondary (1500 B, IMIX, 9000 B jumbo, and the
cache-resident variant of the headline; N=1 only).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpps + Gbit/s device-resident parse+cksum, 64B & 1500B frames, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RESULT_BYTES = 32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)  # 22 ms timed region at N=1: launch jitter < 1 %
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--frames", type=int, default=1 << 20, help="frames per batch per GPU")
    p.add_argument("--rotate", type=int, default=16,
                   help="distinct batches cycled through (frames x rotate = one GPU's shard: 16M = config 4 / 8)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-secondary", action="store_true")
    p.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                   help="the full record (prose, probe tables, curves); stdout carries the compact line")
    return p.parse_args()


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, x: float) -> float:
        if not self.pg:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def gather(self, x: float) -> list:
        """x from every rank, in rank order."""
        if not self.pg:
            return [x]
        import torch

        parts = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
        self.pg.all_gather(parts, torch.tensor([x], dtype=torch.float64))
        return [float(t.item()) for t in parts]

    def gather_obj(self, x) -> list:
        """A small JSON-able object from every rank, in rank order (gloo, host memory only)."""
        if not self.pg:
            return [x]
        parts = [None] * self.world
        self.pg.all_gather_object(parts, x)
        return parts

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def rank_plan(gpus: int, env) -> str:
    """How this invocation runs: "single" (N = 1, no launcher), "ranks" (one rank of a launched
    N-rank job whose WORLD_SIZE equals --gpus), "spawn" (--gpus N > 1 and no launcher: start
    torch.distributed.run as a child) or "mismatch" (a launcher whose WORLD_SIZE is not --gpus)."""
    world = env.get("WORLD_SIZE")
    if world is None:
        return "spawn" if gpus > 1 else "single"
    return "ranks" if int(world) == gpus else "mismatch"


def launch_ranks(gpus: int, argv: list) -> int:
    """Run this script as an N-rank job under torch.distributed.run in a CHILD process and return its
    exit code. Called before anything in this process touches the GPU (no exec: the box forbids
    replacing a process that has initialised it). Rank 0's JSON line reaches our stdout directly."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[launcher] --gpus {gpus} without WORLD_SIZE: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def shard_first_index(rank: int, batch: int, n: int, rotate: int) -> int:
    """Global index of the first frame of `batch` on `rank`: ranks own disjoint, contiguous
    slices of the synthetic stream (index sharding) and never exchange data."""
    return (rank * rotate + batch) * n


def shard_batches(dev, netif, *, rank: int, n: int, rotate: int):
    """One rank's shard of the 64 B frame stream — global frames [rank*n*rotate, (rank+1)*n*rotate)
    — generated as ONE contiguous ragged batch on the rank's GPU, and the `rotate` n-frame batches
    the timed steps cycle through as views of it (batch b = frames shard_first_index(rank, b, ..),
    byte base at its first frame, offsets rebased to it). Frame i depends only on (seed, i), so
    the views hold exactly the frames make_batches generates for the same indices."""
    import numpy as np
    import torch

    from halo_amd import synth

    first = shard_first_index(rank, 0, n * rotate, 1)
    lay = synth.layout(n * rotate, length=64, first_index=first)
    shard = synth.frames_device(lay, netif, device=dev)
    shard["layout"] = lay
    batches = []
    for b in range(rotate):
        lo = b * n
        assert first + lo == shard_first_index(rank, b, n, rotate)
        o0 = int(lay["offsets_dw"][lo])
        offs = (lay["offsets_dw"][lo:lo + n] - np.uint32(o0)).astype(np.uint32)
        sub = {"n": n, "lens": lay["lens"][lo:lo + n], "offsets_dw": offs, "kinds": lay["kinds"][lo:lo + n],
               "seed": lay["seed"], "first_index": first + lo}
        batches.append({"bytes": shard["bytes"][4 * o0:], "offsets_dw": torch.from_numpy(offs.view(np.int32)).to(dev),
                        "lens": shard["lens"][lo:lo + n], "layout": sub})
    return batches, shard


def validate_shard(batches, netif, dev, rank: int, flips: int = 64) -> dict:
    """After the timed steps, on the rank's own device, through the product entry point:
    (1) every batch of the shard parsed once more with a status histogram — the histogram must sum
        to the shard's frame count and every (clean, synthetic) frame must be OK;
    (2) a known-answer probe: one bit flipped in each of `flips` seeded frames of batch 0 (a byte in
        [14, 64): IPv4 header or UDP segment, so the IPv4 header or UDP checksum must catch it) must
        turn exactly those frames to a failing status and leave every other frame OK. The flips are
        undone afterwards. No oracle: the expected answers follow from the one's-complement sum."""
    import numpy as np
    import torch

    from halo_amd import protocol

    n = batches[0]["layout"]["n"]
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=dev)
    ok = torch.zeros((), dtype=torch.int64, device=dev)
    for b in batches:
        protocol.parse_frames_batch(b["bytes"], b["offsets_dw"], b["lens"], netif=netif, max_len_hint=64, out=out,
                                    hist=hist)
        ok += (out[:, 0] == 0).sum()
    h = hist.cpu().numpy().astype(np.int64)
    frames = n * len(batches)
    rng = np.random.default_rng(0x464C4950 + rank)
    idx = np.sort(rng.choice(n, size=min(flips, n), replace=False))
    pos = batches[0]["layout"]["offsets_dw"][idx].astype(np.int64) * 4 + rng.integers(14, 64, idx.size)
    bit = (1 << rng.integers(0, 8, idx.size)).astype(np.uint8)
    b0 = batches[0]["bytes"]
    pos_d, bit_d = torch.from_numpy(pos).to(dev), torch.from_numpy(bit).to(dev)
    b0[pos_d] ^= bit_d
    protocol.parse_frames_batch(b0, batches[0]["offsets_dw"], batches[0]["lens"], netif=netif, max_len_hint=64,
                                out=out)
    st = out[:, 0].cpu().numpy()
    b0[pos_d] ^= bit_d
    torch.cuda.synchronize()
    flipped = np.zeros(n, bool)
    flipped[idx] = True
    probe = {"flipped": int(idx.size), "rejected": int((st[flipped] != 0).sum()),
             "others_ok": bool((st[~flipped] == 0).all())}
    res = {"frames": frames, "hist_sum": int(h.sum()), "ok_frames": int(ok.item()), "hist_ok": int(h[0]),
           "flip_probe": probe}
    res["valid"] = bool(res["hist_sum"] == frames and res["ok_frames"] == frames and res["hist_ok"] == frames
                        and probe["rejected"] == probe["flipped"] and probe["others_ok"])
    return res


def device_identity(gpu: int) -> dict:
    """PCI bus id (hipDeviceGetPCIBusId) and name of the device this rank runs on."""
    import ctypes

    import torch

    buf = ctypes.create_string_buffer(64)
    rc = bench_lib().halo_bench_pci_bus_id(gpu, buf, len(buf))
    return {"device": gpu, "pci_bus_id": buf.value.decode() if rc == 0 else f"error {rc}",
            "name": torch.cuda.get_device_name(gpu)}


def make_batches(dev, netif, *, n, rotate, rank, length=64, size_mode=0, proto_mode=0, strided=False,
                 mutate_shift=0):
    from halo_amd import synth

    batches = []
    for b in range(rotate):
        first = shard_first_index(rank, b, n, rotate)
        lay = synth.layout(n, length=length, size_mode=size_mode, proto_mode=proto_mode, first_index=first,
                           ragged=not strided, mutate_shift=mutate_shift)
        fr = synth.frames_device(lay, netif, device=dev, stride=length if strided else 0)
        fr["layout"] = lay
        batches.append(fr)
    return batches


def frame_bytes(fr) -> int:
    return int(fr["layout"]["lens"].astype("int64").sum())


_BENCH_LIB = None


def bench_lib():
    """tools/libhalo_bench.so: the native step loop (built on demand if missing)."""
    global _BENCH_LIB
    if _BENCH_LIB is None:
        import ctypes
        import importlib.util

        spec = importlib.util.spec_from_file_location("halo_build", os.path.join(ROOT, "halo_amd", "build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        if not os.path.exists(mod.BENCH_OUT):
            mod.build_bench()
        L = ctypes.CDLL(mod.BENCH_OUT)
        vp = ctypes.c_void_p
        L.halo_bench_steps.restype = ctypes.c_int
        L.halo_bench_steps.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_uint32, vp, ctypes.c_uint32, vp, vp, ctypes.c_int, ctypes.c_int, vp,
                                       ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
        L.halo_bench_tx_steps.restype = ctypes.c_int
        L.halo_bench_tx_steps.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_uint32,
                                          ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int, vp,
                                          ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
        i32, u32 = ctypes.c_int, ctypes.c_uint32
        tail = [i32, i32, vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
        L.halo_bench_flow_steps.restype = ctypes.c_int
        L.halo_bench_flow_steps.argtypes = [i32, vp, u32, u32, u32, vp, u32, vp] + tail
        L.halo_bench_flow_compact_steps.restype = ctypes.c_int
        L.halo_bench_flow_compact_steps.argtypes = [i32, vp, u32, u32, u32, vp, u32, vp] + tail
        L.halo_bench_route_steps.restype = ctypes.c_int
        L.halo_bench_route_steps.argtypes = [i32, vp, vp, u32, vp] + tail
        L.halo_bench_xxh3_steps.restype = ctypes.c_int
        L.halo_bench_xxh3_steps.argtypes = [i32, vp, vp, vp, u32, vp] + tail
        L.halo_bench_xxh3_probe_steps.restype = ctypes.c_int
        L.halo_bench_xxh3_probe_steps.argtypes = [i32, vp, vp, vp, u32, vp] + tail
        u64 = ctypes.c_uint64
        L.halo_bench_read_peak.restype = ctypes.c_int
        L.halo_bench_read_peak.argtypes = [vp, u64, vp] + tail
        L.halo_bench_read_probe.restype = ctypes.c_int
        L.halo_bench_read_probe.argtypes = [vp, u64, vp, i32] + tail
        L.halo_bench_read_probe_name.restype = ctypes.c_char_p
        L.halo_bench_read_probe_name.argtypes = [i32]
        L.halo_bench_rx_flow_steps.restype = ctypes.c_int
        L.halo_bench_rx_flow_steps.argtypes = [i32, vp, vp, vp, u32, u32, vp, u32, vp, u32, u32, vp, u32, vp] + tail
        L.halo_bench_stream_rw.restype = ctypes.c_int
        L.halo_bench_stream_rw.argtypes = [vp, vp, i32, u64, u64, vp] + tail
        L.halo_bench_stream_rw_v.restype = ctypes.c_int
        L.halo_bench_stream_rw_v.argtypes = [vp, vp, i32, u64, u64, vp, i32] + tail
        L.halo_bench_stream_rw_name.restype = ctypes.c_char_p
        L.halo_bench_stream_rw_name.argtypes = [i32]
        L.halo_bench_ring_scan_steps.restype = ctypes.c_int
        L.halo_bench_ring_scan_steps.argtypes = [i32, vp, u64, u64, u32, vp, vp, vp, vp, u64] + tail
        L.halo_bench_pci_bus_id.restype = ctypes.c_int
        L.halo_bench_pci_bus_id.argtypes = [i32, ctypes.c_char_p, i32]
        L.halo_bench_ring_polls.restype = ctypes.c_int
        L.halo_bench_ring_polls.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp, vp, i32, i32, vp,
                                            ctypes.POINTER(ctypes.c_uint32)]
        L.halo_bench_steps_queues.restype = ctypes.c_int
        L.halo_bench_steps_queues.argtypes = [i32, vp, vp, vp, u32, u32, vp, u32, vp, i32] + tail
        L.halo_bench_multi_steps.restype = ctypes.c_int
        L.halo_bench_multi_steps.argtypes = [i32, vp, vp, vp, u32, u32, u32, vp, u32, vp, vp] + tail
        L.halo_bench_host_calls.restype = ctypes.c_int
        L.halo_bench_host_calls.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp, i32, i32, vp,
                                            ctypes.POINTER(ctypes.c_uint32)]
        L.halo_bench_cpu_calls.restype = ctypes.c_int
        L.halo_bench_cpu_calls.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp, i32, i32, vp,
                                           ctypes.POINTER(ctypes.c_uint32)]
        L.halo_bench_gather_probe.restype = ctypes.c_int
        L.halo_bench_gather_probe.argtypes = [vp, vp, i32, u32, vp] + tail
        L.halo_bench_tx_layout_probe.restype = ctypes.c_int
        L.halo_bench_tx_layout_probe.argtypes = [vp, vp, u32, u32, vp, u32, u32, vp, vp, u32, vp, u32] + tail
        _BENCH_LIB = L
    return _BENCH_LIB


def time_steps(batches, out, netif, *, flags, hint, steps, warmup, d: Dist, strided_len: int = 0, hist=None):
    """`steps` hot-path launches, one per batch (cycling), issued back to back by the native loop
    on torch's current stream. Barrier + device sync on both sides. One HIP event pair on that
    stream brackets the timed region. Returns (max-over-ranks wall seconds, average launch
    duration in ms = event elapsed / steps)."""
    import ctypes

    import torch

    from halo_amd import _lib

    nb = len(batches)
    arr = lambda xs: (ctypes.c_void_p * nb)(*xs)  # noqa: E731
    b_bytes = arr([b["bytes"].data_ptr() for b in batches])
    b_offs = None if strided_len else arr([b["offsets_dw"].data_ptr() for b in batches])
    b_lens = None if strided_len else arr([b["lens"].data_ptr() for b in batches])
    region = ctypes.c_float()
    wall = ctypes.c_double()
    torch.cuda.synchronize()
    d.barrier()
    rc = bench_lib().halo_bench_steps(nb, b_bytes, b_offs, b_lens, batches[0]["layout"]["n"], strided_len,
                                      strided_len, flags, ctypes.addressof(netif), hint, out.data_ptr(),
                                      None if hist is None else hist.data_ptr(), warmup, steps, torch.cuda.current_stream().cuda_stream, ctypes.byref(region),
                                      ctypes.byref(wall))
    _lib.check("halo_bench_steps", rc)
    torch.cuda.synchronize()
    d.barrier()
    return d.max(wall.value), region.value / steps


CONFIG4_FRAMES = 128 << 20  # BASELINE configs[3]: 128M x 64 B IPv4/UDP, sharded by index over 8 GPUs
CONFIG4_PER_GPU = CONFIG4_FRAMES // 8  # one GPU's shard: 16M frames = bench.py's default frames x rotate


def config4_shard(rank: int, per: int = CONFIG4_PER_GPU):
    """(first global frame index, frame count) of `rank`'s config-4 shard: contiguous, disjoint,
    equal ranges; ranks 0..7 together cover config 4's [0, 128M)."""
    return rank * per, per


def config4_one_gpu(dev, netif, d: Dist, steps: int, warmup: int) -> dict:
    """All of BASELINE config 4 on ONE GPU: the 128M x 64 B frames (8 GB + 4 GB of records) in one
    launch per step — what one GPU does with the whole job, beside the N-rank curve."""
    import torch

    per = CONFIG4_FRAMES
    log(f"[rank {d.rank}] config4 on one GPU: generating {per} frames of 64 B")
    fr = make_batches(dev, netif, n=per, rotate=1, rank=0)
    out = torch.empty((per, RESULT_BYTES), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    wall, kms = time_steps(fr, out, netif, flags=1, hint=64, steps=steps, warmup=warmup, d=d)
    fb = frame_bytes(fr[0])
    alg = fb + per * (4 + 2 + RESULT_BYTES)
    res = {"workload": f"config4 whole on one GPU: {per >> 20}M x 64B IPv4/UDP frames in one launch per step, "
                       "CheckSumEnable=true, 32B record/frame",
           "frames": per, "steps": steps, "value": round(per * steps / wall / 1e6, 2), "unit": "Mpps",
           "gbit_s": round(fb * steps * 8 / wall / 1e9, 2), "ms_per_step": round(wall / steps * 1e3, 4),
           "kernel_ms": round(kms, 5), "roofline": roofline(alg, kms), "alg_bytes_per_launch": alg}
    del fr, out
    torch.cuda.empty_cache()
    return res


TX_BENCH_STEPS = 0x01 | 0x04 | 0x10  # NatChangeDst + NatChangeSrc + eth_tx DPDK fill
TX_WRITE_BYTES = 20  # header dwords 6..10 rewritten per UDP frame (addresses, ports, both checksums)


def tx_ops_for(n: int):
    """Per-frame halo_tx_op_t records for the transmit bench: seeded addresses and ports per frame.
    No TTL step: repeated passes over the same batches must do identical work (a TTL step would
    move frames to the TTL-exceeded branch after <= 255 passes)."""
    import numpy as np

    from halo_amd import protocol

    rng = np.random.default_rng(0x5458)
    ops = protocol.tx_ops(n, TX_BENCH_STEPS)
    ops["dst_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ops["src_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ops["dst_port"] = rng.integers(1, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
    ops["src_port"] = rng.integers(1, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
    return ops


def time_tx_steps(batches, ops_dev, res_dev, *, flags, hint, steps, warmup, d: Dist):
    """time_steps for halo_tx_fixup_batch_device (frames rewritten in place each launch)."""
    import ctypes

    import torch

    from halo_amd import _lib

    nb = len(batches)
    arr = lambda xs: (ctypes.c_void_p * nb)(*xs)  # noqa: E731
    region, wall = ctypes.c_float(), ctypes.c_double()
    torch.cuda.synchronize()
    d.barrier()
    rc = bench_lib().halo_bench_tx_steps(nb, arr([b["bytes"].data_ptr() for b in batches]),
                                         arr([b["offsets_dw"].data_ptr() for b in batches]),
                                         arr([b["lens"].data_ptr() for b in batches]), batches[0]["layout"]["n"],
                                         ops_dev.data_ptr(), flags, hint, res_dev.data_ptr(), warmup, steps,
                                         torch.cuda.current_stream().cuda_stream, ctypes.byref(region),
                                         ctypes.byref(wall))
    _lib.check("halo_bench_tx_steps", rc)
    torch.cuda.synchronize()
    d.barrier()
    return d.max(wall.value), region.value / steps


def cpu_rate(fn, units: int, seconds: float, unit: str, sample: str):
    """The oracle restatement of a row-f2..f4 function, one host thread, repeated for ~`seconds`."""
    fn()  # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(units * passes / el / 1e6, 3), "unit": unit, "cores": 1, "kind": "port",
            "sample": f"{sample}; {passes} passes in {el:.1f}s, oracle/*.c -O2, one thread"}


def time_native(fn, *args, steps, warmup, d: Dist):
    """One of the row-f3 native loops (halo_bench_flow_steps / halo_bench_xxh3_steps)."""
    import ctypes

    import torch

    from halo_amd import _lib

    region, wall = ctypes.c_float(), ctypes.c_double()
    torch.cuda.synchronize()
    d.barrier()
    rc = fn(*args, warmup, steps, torch.cuda.current_stream().cuda_stream, ctypes.byref(region), ctypes.byref(wall))
    _lib.check(fn.__name__, rc)
    torch.cuda.synchronize()
    d.barrier()
    return d.max(wall.value), region.value / steps


def time_torch_loop(fn, steps: int, warmup: int, d: Dist):
    """Launch fn() `steps` times back to back on torch's current stream (the stream the product
    call is given) and time the region with one HIP event pair on that stream: (max-over-ranks
    wall seconds, ms per launch)."""
    import torch

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    d.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    d.barrier()
    return d.max(wall), e0.elapsed_time(e1) / steps


def tx_build_secondary(dev, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8f f2, the Build* half: NetIf.TxUdp -> TxIpv4 -> TxEthernet for a batch of descriptors
    (halo_tx_build_batch_device): 1M 64 B UDP frames (22 B payloads, the headline's frame) and
    256k 1514 B ones (1472 B payloads, the largest BuildUdpPkt accepts), CheckSumEnable on, the
    iphId sequence carried across launches."""
    import numpy as np
    import torch

    from halo_amd import protocol
    from halo_amd._lib import BUILD_DESC_DTYPE, NetIf

    res = {}
    netif = NetIf.make(mac="02:00:00:00:00:01", ip="192.168.100.1")
    for name, n, plen, stride in (("tx_build_udp_1M_64B", 1 << 20, 22, 64),
                                  ("tx_build_udp_256k_1514B", 1 << 18, 1472, 1516)):
        rng = np.random.default_rng(0x4255)
        desc = np.zeros(n, BUILD_DESC_DTYPE)
        desc["payload_off"] = np.arange(n, dtype=np.uint64) * plen
        desc["payload_len"] = plen
        desc["proto"] = 17
        desc["src_port"] = rng.integers(1, 1 << 16, n)
        desc["dst_port"] = rng.integers(1, 1 << 16, n)
        desc["src_ip"] = netif.ip
        desc["dst_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        desc["dst_mac"] = np.frombuffer(bytes.fromhex("aaaaaaaaaaaa"), np.uint8)
        desc_d = torch.from_numpy(desc.view(np.uint8)).to(dev)
        pay_d = torch.randint(0, 256, (n * plen,), dtype=torch.uint8, device=dev)
        b = protocol.TxBuilder(n, device=dev, ip_id=1)
        frames = torch.empty((n, stride), dtype=torch.uint8, device=dev)
        lens = torch.empty(n, dtype=torch.int16, device=dev)
        rcode = torch.empty(n, dtype=torch.uint8, device=dev)
        st = max(5, steps // 5) if plen > 64 else steps
        w, k = time_torch_loop(lambda: b.build(desc_d, pay_d, netif=netif, out_stride=stride, frames=frames,
                                               lens=lens, result=rcode, max_payload_hint=plen), st, warmup, d)
        flen = 14 + 20 + 8 + plen
        assert int((rcode != 0).sum()) == 0 and int((lens != flen).sum()) == 0
        alg = n * (40 + plen + flen + 2 + 1)  # descriptor + payload in; frame + length + result out
        res[name] = {"frames": n, "mpps": round(n * st / w / 1e6, 1), "gbit_s": round(n * flen * st * 8 / w / 1e9, 1),
                     "kernel_ms": round(k, 5), "roofline": roofline(alg, k, load_traffic(name)),
                     "alg_bytes_per_launch": alg,
                     "what": "TxUdp -> BuildUdpPkt -> TxIpv4 (BuildIpv4Pkt, iphId) -> TxEthernet (BuildEthFrm)"}
        # the same byte shape with no work: descriptors + payloads in, the frame slots + lengths +
        # results out (coalesced 16-byte loads and stores)
        with_probe(res[name]["roofline"], size_matched_probe(dev, n * (40 + plen), n * (stride + 3), d, nbuf=1,
                                                             steps=20), k)
        if plen > 64:
            # the same bytes at the same addresses (1514 B frames in 1516 B slots, payloads packed
            # 1472 B apart, the build's grid and lanes) with no build work: what the layout costs
            sink = torch.zeros(16, dtype=torch.int32, device=dev)
            _, kl = time_native(bench_lib().halo_bench_tx_layout_probe, desc_d.data_ptr(), pay_d.data_ptr(), plen, plen,
                                frames.data_ptr(), stride, flen, lens.data_ptr(), rcode.data_ptr(), n,
                                sink.data_ptr(), 0, steps=20, warmup=3, d=d)
            res[name]["roofline"]["layout_matched_probe_ms"] = round(kl, 5)
            res[name]["roofline"]["frac_of_layout_matched"] = round(kl / k, 4)
        if with_cpu:
            from oracle import oracle as O

            m = min(n, 1 << 16)
            hd, hp = desc[:m].copy(), pay_d[:m * plen].cpu().numpy()
            res[name]["cpu_baseline"] = cpu_rate(
                lambda: O.tx_build_batch(hd, hp, bytes(netif.mac), 1, stride, 1), m, 2.0, "Mpps",
                f"{m} descriptors of the same batch (oracle/halo_tx_oracle.c ora_tx_build_batch)")
        del desc_d, pay_d, frames, lens, rcode, b
        torch.cuda.empty_cache()
    return res


def lo_drain_secondary(dev, netif, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8a row a12: PacketHandle's LoChan drain over 1M TxIpv4 loopback copies (50 B IPv4/UDP
    packets addressed to the NetIf itself), HALO_RX_L3_START, CheckSumEnable on."""
    import numpy as np
    import torch

    from halo_amd import protocol
    from halo_amd._lib import BUILD_DESC_DTYPE

    n, plen = 1 << 20, 22
    rng = np.random.default_rng(0x4C4F)
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["payload_off"] = np.arange(n, dtype=np.uint64) * plen
    desc["payload_len"] = plen
    desc["proto"] = 17
    desc["src_port"] = rng.integers(1, 1 << 16, n)
    desc["dst_port"] = rng.integers(1, 1 << 16, n)
    desc["src_ip"] = desc["dst_ip"] = netif.ip
    desc["mode"] = protocol.TX_BUILD_LOOPBACK
    b = protocol.TxBuilder(n, device=dev)
    pk, ln, _ = b.build(torch.from_numpy(desc.view(np.uint8)).to(dev),
                        torch.randint(0, 256, (n * plen,), dtype=torch.uint8, device=dev), netif=netif,
                        out_stride=64)  # 50 B packets in 64 B slots (out_stride >= 60)
    # packed back to back at 4-byte aligned starts, as the batched drain packs LoChan's slices
    # (go/gpurx PackAligned, halo_amd.engine lo_drain): 52-byte pitch for the 50 B packets
    pk = pk.reshape(n, 64)[:, :52].contiguous().reshape(-1)
    offs = torch.arange(n, dtype=torch.int32, device=dev) * 13
    out = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=dev)
    w, k = time_torch_loop(lambda: protocol.parse_ipv4_packets_batch(pk, offs, ln, netif=netif,
                                                                     max_len_hint=64, out=out), steps, warmup, d)
    recs = protocol.records(out)
    assert np.all(recs["status"] == 0) and np.all(recs["flags"] & 4)
    alg = n * (50 + 6 + RESULT_BYTES)
    r = {"frames": n, "mpps": round(n * steps / w / 1e6, 1), "kernel_ms": round(k, 5),
         "roofline": roofline(alg, k, load_traffic("lo_drain_1M_50B")), "alg_bytes_per_launch": alg,
         "what": "LoChan drain: ParseIpv4Pkt -> own-address filter -> RxUdp verify (engine/engine.go:353-381); "
                 "packets packed at a 52-byte pitch (4-byte aligned starts, as PackAligned lays them out)"}
    if with_cpu:
        from oracle import oracle as O

        m = 1 << 18
        host = pk[:m * 52].cpu().numpy()
        hoffs = np.arange(m, dtype=np.uint32) * 13
        hl = ln[:m].cpu().numpy().view(np.uint16)
        r["cpu_baseline"] = cpu_rate(lambda: O.rx_batch(host, hl, O.NetIf.make(), 1 | 0x10, offsets_dw=hoffs), m, 2.0,
                                     "Mpps", f"{m} packets of the batch (oracle/halo_rx_oracle.c, HALO_RX_L3_START)")
    return r


def flow_hash_secondary(batches, out_records, netif, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8f f3 on the headline frames: parse each rotating batch once, then hash every record's NAT
    flow key (NatWanFlowHash, symmetric NAT) with the hashmap bucket for a 2^20-entry table."""
    import ctypes

    import torch

    from halo_amd import protocol

    n = batches[0]["layout"]["n"]
    recs = []
    for b in batches:
        o = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=out_records.device)
        protocol.parse_frames_batch(b["bytes"], b["offsets_dw"], b["lens"], netif=netif, max_len_hint=64, out=o)
        recs.append(o)
    h = torch.empty(n, dtype=torch.int64, device=out_records.device)
    bk = torch.empty(n, dtype=torch.int32, device=out_records.device)
    arr = (ctypes.c_void_p * len(recs))(*[r.data_ptr() for r in recs])
    w, k = time_native(bench_lib().halo_bench_flow_steps, len(recs), arr, n, 1, 0, h.data_ptr(), 1 << 20,
                       bk.data_ptr(), steps=steps, warmup=warmup, d=d)
    alg = n * (20 + 8 + 4)  # record bytes 0..19 in, 8 B hash + 4 B bucket out
    res = {"mpps": round(n * steps / w / 1e6, 1), "kernel_ms": round(k, 5),
           "roofline": roofline(alg, k, load_traffic("flow_hash_config2")), "alg_bytes_per_launch": alg,
           "what": "NatWanFlowHash (13 B key) XXH3-64 + hash % 2^20 per record"}
    # the same keys from compact 16 B records (halo_flow_hash_compact_device): every fetched byte used
    from halo_amd import _lib
    from halo_amd._lib import HALO_RX_RECORD_COMPACT

    crecs = []
    for b in batches:
        o = torch.empty((n, 16), dtype=torch.uint8, device=out_records.device)
        _lib.check("halo_rx_parse_batch_device", _lib.lib.halo_rx_parse_batch_device(
            b["bytes"].data_ptr(), b["offsets_dw"].data_ptr(), b["lens"].data_ptr(), n, 1 | HALO_RX_RECORD_COMPACT,
            ctypes.byref(netif), 64, o.data_ptr(), None, torch.cuda.current_stream().cuda_stream))
        crecs.append(o)
    carr = (ctypes.c_void_p * len(crecs))(*[r.data_ptr() for r in crecs])
    wc, kc = time_native(bench_lib().halo_bench_flow_compact_steps, len(crecs), carr, n, 1, 0, h.data_ptr(), 1 << 20,
                         bk.data_ptr(), steps=steps, warmup=warmup, d=d)
    algc = n * (16 + 8 + 4)
    res["compact_records"] = {"mpps": round(n * steps / wc / 1e6, 1), "kernel_ms": round(kc, 5),
                              "roofline": roofline(algc, kc, load_traffic("flow_hash_config2_compact")),
                              "alg_bytes_per_launch": algc,
                              "what": "the same keys from HALO_RX_RECORD_COMPACT records (16 B: the key fields only)"}
    del crecs
    # size-matched probes: the bytes the memory system must move (whole 32 B / 16 B records in,
    # hash + bucket out), streamed with no work, over as many rotating buffers
    with_probe(res["roofline"], size_matched_probe(dev_of(out_records), n * 32, n * 12, d, nbuf=len(batches)), k)
    with_probe(res["compact_records"]["roofline"],
               size_matched_probe(dev_of(out_records), n * 16, n * 12, d, nbuf=len(batches)), kc)
    if with_cpu:
        from oracle import oracle as O

        host = protocol.records(recs[0])
        res["cpu_baseline"] = cpu_rate(lambda: O.flow_hash_batch(host, 1, 0, 1 << 20), n, 2.0, "Mkeys/s",
                                       f"{n} records of batch 0 (oracle/halo_xxh3_oracle.c)")
    del recs
    return res


def rx_flow_fused_secondary(batches, out, netif, steps, warmup, d: Dist, rx_ms: float, flow_ms: float):
    """The headline parse with every record's NAT flow key hashed in the same pass
    (halo_rx_parse_flow_batch_device), against the two separate launches it replaces."""
    import ctypes

    import torch

    n = batches[0]["layout"]["n"]
    nb = len(batches)
    arr = lambda xs: (ctypes.c_void_p * nb)(*xs)  # noqa: E731
    h = torch.empty(n, dtype=torch.int64, device=out.device)
    bk = torch.empty(n, dtype=torch.int32, device=out.device)
    w, k = time_native(bench_lib().halo_bench_rx_flow_steps, nb, arr([b["bytes"].data_ptr() for b in batches]),
                       arr([b["offsets_dw"].data_ptr() for b in batches]),
                       arr([b["lens"].data_ptr() for b in batches]), n, 1, ctypes.addressof(netif), 64,
                       out.data_ptr(), 1, 0, h.data_ptr(), 1 << 20, bk.data_ptr(), steps=steps, warmup=warmup, d=d)
    alg = frame_bytes(batches[0]) + n * (4 + 2 + RESULT_BYTES + 8 + 4)
    return {"mpps": round(n * steps / w / 1e6, 1), "kernel_ms": round(k, 5),
            "separate_ms": round(rx_ms + flow_ms, 5), "speedup_vs_separate": round((rx_ms + flow_ms) / k, 3),
            "roofline": roofline(alg, k), "alg_bytes_per_launch": alg,
            "what": "config-2 parse + NatWanFlowHash XXH3-64 + 2^20-bucket index of every record in one pass "
                    "(records, hashes and buckets identical to the two separate launches)"}


def xxh3_secondary(dev, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8f f3, GetHashCodeXXH3 over KCP-segment-sized strings (24..1400 B, unaligned offsets)."""
    import ctypes

    import numpy as np
    import torch

    n = 1 << 20
    rng = np.random.default_rng(0x4B4350)
    bs = []
    for _ in range(2):
        lens = rng.integers(24, 1401, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 1)
        total = int(offs[-1]) + int(lens[-1]) + 8
        data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
        bs.append((data, torch.from_numpy(offs.view(np.int64)).to(dev), torch.from_numpy(lens.view(np.int32)).to(dev),
                   int(lens.astype(np.int64).sum())))
    h = torch.empty(n, dtype=torch.int64, device=dev)
    arr = lambda xs: (ctypes.c_void_p * len(xs))(*xs)  # noqa: E731
    w, k = time_native(bench_lib().halo_bench_xxh3_steps, len(bs), arr([b[0].data_ptr() for b in bs]),
                       arr([b[1].data_ptr() for b in bs]), arr([b[2].data_ptr() for b in bs]), n, h.data_ptr(),
                       steps=steps, warmup=warmup, d=d)
    alg = bs[0][3] + n * (8 + 4 + 8)
    res = {"strings": n, "mstrings_per_s": round(n * steps / w / 1e6, 1),
           "gbytes_per_s": round(bs[0][3] * steps / w / 1e9, 1), "kernel_ms": round(k, 4),
           "roofline": roofline(alg, k, load_traffic("xxh3_kcp_1M")), "alg_bytes_per_launch": alg}
    # the same kernel's loads, windows, runs and control flow with the hashing replaced by XORs
    # (flow_hash.hip built as HALO_XXH3_PROBE into tools/libhalo_bench.so): its access-pattern floor
    _, kp = time_native(bench_lib().halo_bench_xxh3_probe_steps, len(bs), arr([b[0].data_ptr() for b in bs]),
                        arr([b[1].data_ptr() for b in bs]), arr([b[2].data_ptr() for b in bs]), n, h.data_ptr(),
                        steps=steps, warmup=warmup, d=d)
    res["roofline"]["load_pattern_probe_ms"] = round(kp, 5)
    res["roofline"]["frac_of_load_pattern_probe"] = round(kp / k, 4)
    if with_cpu:
        from oracle import oracle as O

        m = 1 << 16
        offs_h = bs[0][1][:m].cpu().numpy().view(np.uint64)
        lens_h = bs[0][2][:m].cpu().numpy().view(np.uint32)
        data_h = bs[0][0][:int(offs_h[-1]) + int(lens_h[-1])].cpu().numpy()
        res["cpu_baseline"] = cpu_rate(lambda: O.xxh3_batch(data_h, offs_h, lens_h), m, 2.0, "Mstrings/s",
                                       f"first {m} strings of batch 0 (oracle/halo_xxh3_oracle.c)")
    del bs
    return res


def route_secondary(dev, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8f f4, FindRoute on the GPU: a 500k-prefix table (BGP-like length mix, 1 in 8 prefixes
    with a second ECMP next hop, a default route), 4M uniformly random destination addresses per
    launch, route id out."""
    import ctypes

    import numpy as np
    import torch

    from halo_amd.route import RouteTable

    rng = np.random.default_rng(0x524F5554)
    n_pfx = 500_000
    plen = rng.choice([8, 12, 16, 18, 19, 20, 21, 22, 23, 24, 24, 24, 24, 24, 24, 25, 26, 27, 28, 30, 32], n_pfx)
    mask = ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF).astype(np.uint32)
    dst = rng.integers(0, 1 << 32, n_pfx, dtype=np.uint64).astype(np.uint32) & mask
    t = RouteTable(dev.index or 0)
    t.AddRoute(t.entry(0, 0, 0xC0A86401, 0))
    for k in range(n_pfx):
        e = t.entry(int(dst[k]), int(mask[k]), k + 2, k & 3)
        t.AddRoute(e)
        if k % 8 == 0:
            t.AddRoute(t.entry(int(dst[k]), int(mask[k]), k + 3, k & 3))
    t0 = time.perf_counter()
    t.sync()
    sync_s = time.perf_counter() - t0
    n = 4 << 20
    bs = [torch.from_numpy(rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
          for _ in range(4)]
    out = torch.empty(n, dtype=torch.int32, device=dev)
    arr = (ctypes.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
    w, k = time_native(bench_lib().halo_bench_route_steps, len(bs), t._t, arr, n, out.data_ptr(), steps=steps,
                       warmup=warmup, d=d)
    alg = n * (4 + 4)
    res = {"lookups": n, "mlookups_per_s": round(n * steps / w / 1e6, 1), "kernel_ms": round(k, 4),
           "roofline": roofline(alg, k, load_traffic("route_lpm_4M")), "alg_bytes_per_launch": alg,
           "table": f"{n_pfx} prefixes + default, DIR-24-8 (64 MB first level)", "sync_s": round(sync_s, 3),
           "note": "alg bytes = address in + route id out; each lookup also reads 1-2 random 4 B table "
                   "entries (tbl24 stays resident in the 256 MB Infinity Cache)"}
    t.close()
    # the lookups' own access pattern with no lookup logic: tbl[ip >> 8] over a 64 MB table, one
    # random 4-byte read per address (what DIR-24-8's first level costs), same addresses, same count
    tbl = torch.randint(0, 1 << 30, (1 << 24,), dtype=torch.int32, device=dev)
    _, kg = time_native(bench_lib().halo_bench_gather_probe, tbl.data_ptr(), arr, len(bs), n, out.data_ptr(),
                        steps=steps, warmup=warmup, d=d)
    res["roofline"]["gather_probe_ms"] = round(kg, 5)
    res["roofline"]["frac_of_gather_probe"] = round(kg / k, 4)
    res["gather_probe"] = "one random 4 B read of a 2^24-entry table per address (tbl[ip >> 8]) + 4 B out"
    del tbl
    if with_cpu:
        from oracle import oracle as O

        ot = O.RouteTable()
        ot.add((0, 0, 0xC0A86401, 0))
        for k in range(n_pfx):
            ot.add((int(dst[k]), int(mask[k]), k + 2, k & 3))
            if k % 8 == 0:
                ot.add((int(dst[k]), int(mask[k]), k + 3, k & 3))
        ips_h = bs[0][: 1 << 20].cpu().numpy().view(np.uint32)
        res["cpu_baseline"] = cpu_rate(lambda: ot.find_batch(ips_h), 1 << 20, 2.0, "Mlookups/s",
                                       "1M random addresses, the same table in the binary trie of "
                                       "oracle/halo_route_oracle.c (the reference's structure)")
    del bs
    return res


def ring_secondary(dev, netif, steps, warmup, d: Dist, with_cpu: bool = False):
    """§8f f1 and BASELINE config 1: halo's SPSC packet ring (mem/ring_buffer.go) drained by the GPU.

    (a) ring_scan_device: the record walk alone on a device-resident span of 1M 64 B records;
    (b) ring_e2e: a producer fills a registered 128 MiB ring with 1M 64 B frames (untimed), the
        consumer polls (span DMA + walk + parse + records back) and commits (timed);
    (c) config1_wire_1k: 1k x 64 B frames through an engine.Wire-sized ring (8 MiB), poll + commit
        per batch, beside the oracle's PacketHandle loop over the same ring on one core."""
    import ctypes

    import numpy as np
    import torch

    from halo_amd import _lib
    from halo_amd.ring import RingBuffer, RingConsumer

    res = {}
    n = 1 << 20
    fr = make_batches(dev, netif, n=n, rotate=1, rank=0)[0]
    lay = fr["layout"]
    host = fr["bytes"].cpu().numpy()
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    lens = lay["lens"]
    del fr
    ring = RingBuffer(128 << 20)
    assert ring.write_batch(host, offs, lens) == n
    used = ring.head - ring.tail

    # (a) the walk alone, device-resident
    span = torch.from_numpy(ring.data[:used].copy()).to(dev)
    d_off = torch.empty(n, dtype=torch.int32, device=dev)
    d_len = torch.empty(n, dtype=torch.int16, device=dev)
    info = torch.zeros(24, dtype=torch.uint8, device=dev)
    ws_bytes = _lib.lib.halo_rx_ring_scan_workspace(used, 1514)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    arr = (ctypes.c_void_p * 1)(span.data_ptr())
    w, k = time_native(bench_lib().halo_bench_ring_scan_steps, 1, arr, used, ring.size, 1514, d_off.data_ptr(),
                       d_len.data_ptr(), info.data_ptr(), ws.data_ptr(), ws_bytes, steps=steps, warmup=warmup, d=d)
    got_n = int(info.cpu().numpy().view(_lib.RING_SCAN_DTYPE)[0]["n_frames"])
    alg = used + n * 6  # the span read once, (u32 offset + u16 length) written per frame
    res["ring_scan_device_1M_64B"] = {
        "records": got_n, "mrecords_per_s": round(n * steps / w / 1e6, 1), "kernel_ms": round(k, 4),
        "roofline": roofline(alg, k, load_traffic("ring_scan_1M_64B")), "alg_bytes_per_launch": alg,
        "what": "record boundaries of a 68 MB ring span (3 kernels: every tile walks from its guessed entry, "
                "one workgroup links and verifies the tiles, every tile copies its records out)"}
    # the same bytes moved by a no-work kernel: the span in, 6 B per record out
    with_probe(res["ring_scan_device_1M_64B"]["roofline"], size_matched_probe(dev, used, n * 6, d, nbuf=1), k)
    assert got_n == n, got_n
    del span, d_off, d_len, ws
    torch.cuda.empty_cache()

    # (a') the walk over an IMIX ring (64 / 570 / 1500 B 7:4:1, TCP / UDP / ICMP): 256k records, 92 MB
    ni = 1 << 18
    fi = make_batches(dev, netif, n=ni, rotate=1, rank=0, size_mode=1, proto_mode=3)[0]
    li = fi["layout"]
    hi = fi["bytes"].cpu().numpy()
    del fi
    ring_i = RingBuffer(128 << 20)
    assert ring_i.write_batch(hi, li["offsets_dw"].astype(np.uint64) * 4, li["lens"]) == ni
    used_i = ring_i.head - ring_i.tail
    span = torch.from_numpy(ring_i.data[:used_i].copy()).to(dev)
    del ring_i, hi
    d_off = torch.empty(ni, dtype=torch.int32, device=dev)
    d_len = torch.empty(ni, dtype=torch.int16, device=dev)
    info = torch.zeros(24, dtype=torch.uint8, device=dev)
    ws_bytes = _lib.lib.halo_rx_ring_scan_workspace(used_i, 1514)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    arr = (ctypes.c_void_p * 1)(span.data_ptr())
    w, k = time_native(bench_lib().halo_bench_ring_scan_steps, 1, arr, used_i, 128 << 20, 1514, d_off.data_ptr(),
                       d_len.data_ptr(), info.data_ptr(), ws.data_ptr(), ws_bytes, steps=steps, warmup=warmup, d=d)
    got_i = int(info.cpu().numpy().view(_lib.RING_SCAN_DTYPE)[0]["n_frames"])
    assert got_i == ni, got_i
    alg = used_i + ni * 6
    res["ring_scan_device_imix_256k"] = {
        "records": got_i, "mrecords_per_s": round(ni * steps / w / 1e6, 1), "kernel_ms": round(k, 4),
        "span_bytes": used_i, "roofline": roofline(alg, k, load_traffic("ring_scan_imix_256k")),
        "alg_bytes_per_launch": alg, "what": "the same walk over a 256k-record IMIX ring (64/570/1500 B 7:4:1)"}
    with_probe(res["ring_scan_device_imix_256k"]["roofline"], size_matched_probe(dev, used_i, ni * 6, d, nbuf=1), k)
    del span, d_off, d_len, ws
    torch.cuda.empty_cache()

    # (b) end to end from the ring in host memory
    cons = RingConsumer(ring, capacity=1514, max_frames=n + 64, register=True)
    times, ok = [], True
    for s in range(max(3, steps // 20) + 1):
        if s:
            assert ring.write_batch(host, offs, lens) == n
        t0 = time.perf_counter()
        recs, inf, _ = cons.poll(netif)
        cons.commit()
        el = time.perf_counter() - t0
        ok = ok and inf["n_frames"] == n and bool((recs["status"] == 0).all())
        if s:
            times.append(el)
    el = float(np.median(times))
    fb = int(lens.astype(np.int64).sum())
    res["ring_e2e_64B_1M_registered"] = {
        "frames": n, "mpps": round(n / el / 1e6, 1), "gbit_s": round(fb * 8 / el / 1e9, 1),
        "ms_per_batch": round(el * 1e3, 3), "ok": ok, "ring_bytes": used,
        "what": "poll (raw span DMA + GPU record walk + parse in place + records DMA) + commit; median of batches"}
    cons.close()
    del ring

    # (c) BASELINE config 1: 1k x 64 B frames through an engine.Wire-sized ring, poll + commit per
    # batch from native code (tools/bench_loop.hip halo_bench_ring_polls: the calls a cgo
    # PacketHandle makes, no Python between batches); the Python-loop figure beside it
    m = 1000
    host_m = _lib.host_array(int(offs[m - 1] + lens[m - 1]) + 16)
    host_m[:] = host[:host_m.size]

    def wire_polls(persistent: bool) -> dict:
        wring = RingBuffer(8 << 20)
        wcons = RingConsumer(wring, capacity=1514, max_frames=4096, register=True, persistent=persistent)
        us = np.zeros(2000, np.float64)
        bad = ctypes.c_uint32()
        _lib.check("halo_bench_ring_polls", bench_lib().halo_bench_ring_polls(
            wring.mem.ctypes.data, wcons._h, host_m.ctypes.data, offs.ctypes.data, lens.ctypes.data, m, 1,
            ctypes.addressof(netif), wcons._out.ctypes.data, 100, us.size, us.ctypes.data, ctypes.byref(bad)))
        st = wcons.stats()
        el = float(np.median(us)) * 1e-6
        times = []
        for s in range(201):
            assert wring.write_batch(host, offs[:m], lens[:m]) == m
            t0 = time.perf_counter()
            recs, inf, _ = wcons.poll(netif)
            wcons.commit()
            if s:
                times.append(time.perf_counter() - t0)
            assert inf["n_frames"] == m and bool((recs["status"] == 0).all())
        wcons.close()
        polls = max(1, int(st["small_polls"]))
        out = {"frames": m, "mpps": round(m / el / 1e6, 3), "us_per_batch": round(el * 1e6, 2),
               "us_p10": round(float(np.percentile(us, 10)), 2), "us_p90": round(float(np.percentile(us, 90)), 2),
               "bad_batches": int(bad.value), "python_loop_us_per_batch": round(float(np.median(times)) * 1e6, 1),
               "per_poll_us": {"walk": round(st["walk_ns"] / polls / 1e3, 2),
                               "wait": round(st["wait_ns"] / polls / 1e3, 2)}}
        if persistent:
            out["per_poll_us"]["consumer_gpu"] = round(st["service_gpu_ns"] / max(1, int(st["service_requests"])) / 1e3, 2)
            out["consumer_launches"] = int(st["service_launches"])
        return out

    res["config1_wire_1k_64B"] = wire_polls(True)
    res["config1_wire_1k_64B"]["what"] = (
        "engine.Wire ring (8 MiB) attached HALO_RING_PERSISTENT, 1k x 64 B UDP, poll + commit per batch from a "
        "native loop (2000 batches, median; the producer's WritePacket calls are untimed). The host reads the 1k "
        "length fields (walk); the resident consumer (8 workgroups waiting on a pinned control block) parses "
        "the frames in place in the registered ring over PCIe and writes the records into the registered result "
        "array (wait); no launch or stream synchronisation per poll")
    res["config1_wire_1k_64B"]["launch_per_poll"] = wire_polls(False)
    res["config1_wire_1k_64B"]["launch_per_poll"]["what"] = "the same ring attached without HALO_RING_PERSISTENT: one rx launch + one stream synchronisation per poll"
    if with_cpu:
        from oracle import oracle as O

        onet = O.NetIf.make()
        oring = O.Ring(8 << 20)
        total, passes = 0.0, 0
        while total < 2.0:
            for k in range(m):
                oring.write(host[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes())
            t0 = time.perf_counter()
            recs, _, _, _ = oring.packet_handle(onet, 1, capacity=1514, max_frames=m, actions=True)
            total += time.perf_counter() - t0
            passes += 1
            assert len(recs) == m
        res["config1_wire_1k_64B"]["cpu_baseline"] = {
            "value": round(m * passes / total / 1e6, 3), "unit": "Mpps", "cores": 1, "kind": "port",
            "sample": f"{passes} passes of the same 1k frames: ReadPacket -> RxEthernet -> RxIpv4 -> RxUdp per frame "
                      "(oracle/halo_ring_oracle.c + halo_rx_oracle.c -O2, one thread; the reference is Go)"}
    return res


DROPIN_SIZES = (1, 32, 99, 256, 1024, 4096)  # frames per call: single-frame Parse*, .., PacketHandle's 99


def dropin_small_batch(dev, netif, with_cpu: bool = True) -> dict:
    """The drop-in surface at the reference's own cadence. go/gpurx Ctx.ParseBatch —
    what the batched PacketHandle (go/engine, DrainEvery 99 caps a batch at 99 polls) and, with one
    frame, the single-frame Parse* wrappers call — is halo_rx_parse_batch_host + halo_rx_dispatch over
    frames in pageable host memory (Go slices). Timed per call from native code
    (tools/bench_loop.hip halo_bench_host_calls) at 1..4096 config-2 frames per call, on the
    launched path (chunked DMA + kernel + D2H + stream synchronisation) and on the resident path
    (halo_rx_host_ctx_set_resident: frames packed into pinned staging, one request to a resident
    consumer). Beside it, the reference's cost for the same frames: the one-core C port's per-frame
    time x frames (the Go loop has no per-batch cost), and the batch size where the GPU call
    becomes cheaper (crossover)."""
    import ctypes

    import numpy as np

    from halo_amd import synth
    from halo_amd._lib import RESULT_DTYPE
    from halo_amd.engine import HostBatcher

    mmax = max(DROPIN_SIZES)
    lay = synth.layout(mmax, length=64)
    host = synth.frames_device(lay, netif, device=dev)["bytes"].cpu().numpy().copy()  # pageable, like Go's heap
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    lens = np.ascontiguousarray(lay["lens"])
    out = np.zeros(mmax, RESULT_DTYPE)
    acts = np.zeros(mmax, np.uint8)
    res = {"what": "halo_rx_parse_batch_host + halo_rx_dispatch per call over m pageable 64 B frames "
                   "(go/gpurx Ctx.ParseBatch; m = 1 is the single-frame Parse* path), native loop, "
                   "per-call wall time (median / p10 / p90 of the calls)"}
    for path in ("launched", "resident"):
        hb = HostBatcher(dev.index or 0)
        if path == "resident":
            hb.set_resident(mmax)
        curve = {}
        for m in DROPIN_SIZES:
            iters = 2000 if m <= 256 else 400
            us = np.zeros(iters, np.float64)
            bad = ctypes.c_uint32()
            st0 = hb.stats()
            from halo_amd import _lib

            _lib.check("halo_bench_host_calls", bench_lib().halo_bench_host_calls(
                hb._ctx, host.ctypes.data, offs.ctypes.data, lens.ctypes.data, m, 1, ctypes.addressof(netif),
                out.ctypes.data, acts.ctypes.data, 50, iters, us.ctypes.data, ctypes.byref(bad)))
            st1 = hb.stats()
            med = float(np.median(us))
            pt = {"us_median": round(med, 2), "us_p10": round(float(np.percentile(us, 10)), 2),
                  "us_p90": round(float(np.percentile(us, 90)), 2), "mpps": round(m / med, 3),
                  "bad_calls": int(bad.value)}
            if path == "resident":
                calls = max(1, st1["resident_calls"] - st0["resident_calls"])
                pt["per_call_us"] = {k: round((st1[k + "_ns"] - st0[k + "_ns"]) / calls / 1e3, 2)
                                     for k in ("pack", "wait", "service_gpu")}
                pt["resident_calls"] = st1["resident_calls"] - st0["resident_calls"]
            curve[str(m)] = pt
        hb.close()
        res[path] = curve
    # the CPU entry point (libhalo_rx_cpu.so, include/halo_rx_cpu.h) in the same native per-call loop
    from halo_amd import _lib
    from halo_amd import cpu as cpu_entry

    fn = ctypes.cast(cpu_entry.lib.halo_rx_parse_batch_cpu, ctypes.c_void_p).value
    curve = {}
    for m in DROPIN_SIZES:
        iters = 2000 if m <= 256 else 400
        us = np.zeros(iters, np.float64)
        bad = ctypes.c_uint32()
        _lib.check("halo_bench_cpu_calls", bench_lib().halo_bench_cpu_calls(
            fn, host.ctypes.data, offs.ctypes.data, lens.ctypes.data, m, 1, ctypes.addressof(netif), out.ctypes.data,
            acts.ctypes.data, 50, iters, us.ctypes.data, ctypes.byref(bad)))
        med = float(np.median(us))
        curve[str(m)] = {"us_median": round(med, 3), "us_p10": round(float(np.percentile(us, 10)), 3),
                         "us_p90": round(float(np.percentile(us, 90)), 3), "mpps": round(m / med, 3),
                         "bad_calls": int(bad.value)}
    res["cpu_entry"] = curve
    ms = np.array(DROPIN_SIZES, np.float64)
    t_res = np.array([res["resident"][str(m)]["us_median"] for m in DROPIN_SIZES])
    t_cpu = np.array([curve[str(m)]["us_median"] for m in DROPIN_SIZES])
    b, a = np.polyfit(ms, t_res, 1)
    c = float(np.polyfit(ms, t_cpu, 1)[0])
    res["cpu_entry_ns_per_frame"] = round(c * 1e3, 2)
    res["cpu_entry_crossover_frames"] = round(float(a / (c - b)), 1) if c > b else None
    if with_cpu:
        from oracle import oracle as O

        O.build()
        onet = O.NetIf.make()
        O.rx_batch(host, lens, onet, 1, offsets_dw=lay["offsets_dw"])  # warm
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            O.rx_batch(host, lens, onet, 1, offsets_dw=lay["offsets_dw"])
            passes += 1
        ns = (time.perf_counter() - t0) / (passes * mmax) * 1e9
        res["cpu_port_ns_per_frame"] = round(ns, 2)
        res["cpu_port_us_per_call"] = {str(m): round(m * ns / 1e3, 3) for m in DROPIN_SIZES}
        res["cpu_note"] = ("oracle/halo_rx_oracle.c -O2 on one core over the same frames (the reference is Go, "
                           "one goroutine per NetIf; its loop has no per-batch cost, so a call of m frames costs "
                           "m x the per-frame time)")
        # crossover: fit the resident curve t(m) = a + b m and solve a + b m = c m (c = CPU per frame)
        ms = np.array(DROPIN_SIZES, np.float64)
        t = np.array([res["resident"][str(m)]["us_median"] for m in DROPIN_SIZES])
        b, a = np.polyfit(ms, t, 1)
        c = ns / 1e3
        res["resident_fit_us"] = {"fixed": round(float(a), 3), "per_frame": round(float(b), 5)}
        res["crossover_frames"] = round(float(a / (c - b)), 1) if c > b else None
        beats = [m for m in DROPIN_SIZES if res["resident"][str(m)]["us_median"] < m * c]
        res["smallest_measured_batch_faster_than_cpu"] = min(beats) if beats else None
    return res


STATUS_NAMES = ("OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
                "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM")


def queues_secondary(batches, netif, steps: int, warmup: int, d: Dist, headline_ms: float) -> dict:
    """The headline step with 2 and 4 launches in flight (step k on stream k % q, each stream its own
    record array): what a caller that keeps several batches queued, one per NIC queue, gets from the
    same one-batch launches. The headline itself is one stream, one launch after the other."""
    import ctypes

    import torch

    from halo_amd import protocol

    n = batches[0]["layout"]["n"]
    nb = len(batches)
    arr = lambda xs: (ctypes.c_void_p * len(xs))(*xs)  # noqa: E731
    res = {}
    for q in (2, 4):
        outs = [torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=batches[0]["bytes"].device) for _ in range(q)]
        w, k = time_native(bench_lib().halo_bench_steps_queues, nb, arr([b["bytes"].data_ptr() for b in batches]),
                           arr([b["offsets_dw"].data_ptr() for b in batches]),
                           arr([b["lens"].data_ptr() for b in batches]), n, 1, ctypes.addressof(netif), 64,
                           arr([o.data_ptr() for o in outs]), q, steps=steps, warmup=warmup, d=d)
        # each stream's record array holds the last batch that stream parsed: the same bytes as one
        # ordinary launch over that batch
        ok = True
        ref = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=outs[0].device)
        for j in range(q):
            # (halo_bench_steps_queues numbers warm-up and timed steps from 0 each: step k -> stream
            # k % q, batch k % nb)
            timed = [kk for kk in range(steps) if kk % q == j]
            last = timed[-1] if timed else max(kk for kk in range(warmup) if kk % q == j)
            b = batches[last % nb]
            protocol.parse_frames_batch(b["bytes"], b["offsets_dw"], b["lens"], netif=netif, max_len_hint=64, out=ref)
            ok = ok and bool(torch.equal(ref, outs[j]))
        res[f"queues_{q}"] = {"mpps": round(n * steps / w / 1e6, 1), "ms_per_batch": round(k, 5),
                              "vs_headline_per_batch": round(headline_ms / k, 4), "ok": ok}
        assert ok, f"queues_{q}: records differ from a single launch"
        del outs, ref
    res["what"] = ("config 2's one-batch launches with 2 / 4 in flight on as many streams (each its own record "
                   "array); ms_per_batch = event region / steps")
    return res


def batch_stream_secondary(batches, netif, steps: int, warmup: int, d: Dist, headline_ms: float, k: int = 8) -> dict:
    """The headline's batch stream, k batches per launch (halo_rx_parse_batches_device): each
    batch keeps its own records (k record arrays), the batches rotate as in the headline."""
    import ctypes

    import torch

    n = batches[0]["layout"]["n"]
    nb = len(batches)
    arr = lambda xs: (ctypes.c_void_p * len(xs))(*xs)  # noqa: E731
    outs = [torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=batches[0]["bytes"].device) for _ in range(k)]
    st = max(10, steps // k)
    w, km = time_native(bench_lib().halo_bench_multi_steps, nb, arr([b["bytes"].data_ptr() for b in batches]),
                        arr([b["offsets_dw"].data_ptr() for b in batches]), arr([b["lens"].data_ptr() for b in batches]),
                        n, k, 1, ctypes.addressof(netif), 64, arr([o.data_ptr() for o in outs]), None, steps=st,
                        warmup=max(2, warmup // k), d=d)
    # the last launch's k record arrays against one ordinary launch per batch (launch t, slot j ->
    # batch (t k + j) mod nb: halo_bench_multi_steps)
    from halo_amd import protocol

    ref = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=outs[0].device)
    ok = True
    for j in range(k):
        b = batches[((st - 1) * k + j) % nb]
        protocol.parse_frames_batch(b["bytes"], b["offsets_dw"], b["lens"], netif=netif, max_len_hint=64, out=ref)
        ok = ok and bool(torch.equal(ref, outs[j]))
    assert ok, "batch stream: records differ from one launch per batch"
    del ref
    fb = frame_bytes(batches[0])
    alg = k * (fb + n * (4 + 2 + RESULT_BYTES))
    res = {"batches_per_launch": k, "frames_per_launch": k * n, "launches": st, "ok": ok,
           "mpps": round(k * n * st / w / 1e6, 1),
           "kernel_ms": round(km, 5), "ms_per_batch": round(km / k, 5),
           "vs_headline_per_batch": round(headline_ms / (km / k), 4),
           "roofline": roofline(alg, km, frame_bytes=k * fb), "alg_bytes_per_launch": alg,
           "kernel": "rx_lane_multi_kernel<0> (the lane kernel's window code, k batches' windows in one grid)",
           "what": f"config 2's rotating 1M-frame batches handed over {k} per call (halo_rx_parse_batches_device); "
                   "records per batch identical to the headline's one-launch-per-batch steps"}
    del outs
    return res


MEASURED_READ_GBS = None  # set by measure_read_peak() on this box
MEASURED_READ_PROBES = {}  # every probe shape's GB/s


def measure_read_peak(dev, d: Dist, gib: int = 4):
    """Read-only streaming kernels over `gib` GiB (16x the Infinity Cache): this box's achievable
    HBM read bandwidth, the second peak SURVEY.md §8d asks the roofline to be reported against —
    the fastest of a family of probe shapes (one 64 KB tile per block or persistent blocks; 64 to
    1024 threads; 4 to 16 16-byte loads in flight per lane; plain and non-temporal loads), each
    timed over 20 launches."""
    import torch

    global MEASURED_READ_GBS
    nbytes = gib << 30
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    buf.fill_(1)
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    L = bench_lib()
    v = 0
    while L.halo_bench_read_probe_name(v) is not None:
        w, k = time_native(L.halo_bench_read_probe, buf.data_ptr(), nbytes, sink.data_ptr(), v, steps=20, warmup=3,
                           d=d)
        MEASURED_READ_PROBES[L.halo_bench_read_probe_name(v).decode()] = round(nbytes / (k * 1e-3) / 1e9, 1)
        v += 1
    MEASURED_READ_GBS = max(MEASURED_READ_PROBES.values())
    del buf
    torch.cuda.empty_cache()
    return MEASURED_READ_GBS


LAST_PROBE_SHAPES = {}  # the last size_matched_probe: ms per shape


def size_matched_probe(dev, read_bytes: int, write_bytes: int, d: Dist, nbuf: int = 8, steps: int = 50):
    """Speed-of-light for a kernel's byte shape on this box: kernels that stream `read_bytes` in
    (tiles of 16-byte loads) and write `write_bytes` out (coalesced 16-byte stores) over `nbuf`
    rotating buffers, doing no other work (tools/bench_loop.hip stream_rw_kernel). Every shape of
    the family (16 / 32 / 64 KB tiles, plain and non-temporal) is timed; returns the fastest one's
    average launch duration in ms (one shape alone was not a ceiling at 16M frames)."""
    import ctypes

    import torch

    r16, w16 = (read_bytes + 15) // 16 * 16, (write_bytes + 15) // 16 * 16
    srcs = [torch.ones(r16, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    dsts = [torch.empty(w16, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    arr = lambda xs: (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs])  # noqa: E731
    L = bench_lib()
    LAST_PROBE_SHAPES.clear()
    v = 0
    while L.halo_bench_stream_rw_name(v) is not None:
        _, k = time_native(L.halo_bench_stream_rw_v, arr(srcs), arr(dsts), nbuf, r16, w16, sink.data_ptr(), v,
                           steps=steps, warmup=5, d=d)
        LAST_PROBE_SHAPES[L.halo_bench_stream_rw_name(v).decode()] = round(k, 5)
        v += 1
    del srcs, dsts, sink
    torch.cuda.empty_cache()
    return min(LAST_PROBE_SHAPES.values())


def dev_of(t):
    return t.device


def with_probe(r: dict, probe_ms: float, kernel_ms: float) -> dict:
    r["size_matched_probe_ms"] = round(probe_ms, 5)
    r["frac_of_size_matched"] = round(probe_ms / kernel_ms, 4)
    if LAST_PROBE_SHAPES:
        r["size_matched_shape"] = min(LAST_PROBE_SHAPES, key=LAST_PROBE_SHAPES.get)
        r["size_matched_shapes_ms"] = dict(LAST_PROBE_SHAPES)
    return r


def roofline(alg_bytes_per_launch, kernel_ms, traffic=None, frame_bytes=None):
    """`frame_bytes` (the frames' own bytes per launch, SURVEY §8d's primary R): also report the
    R-only fraction beside the (R + M + W) one."""
    achieved = alg_bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    session = None
    if isinstance(traffic, dict):  # load_traffic: the bytes and the profiling session they come from
        traffic, session = traffic["bytes"], traffic["session"]
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}
    if session:
        r["traffic_session"] = session
    if frame_bytes:
        r["frac_frames_only"] = round(frame_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if MEASURED_READ_GBS:
        r["peak_measured_read"] = MEASURED_READ_GBS
        r["frac_of_measured"] = round(achieved / MEASURED_READ_GBS, 4)
    return r


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if any, with the
    profiling session they come from: {"bytes": B, "session": "r5t"} or None."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        b = d.get(workload, {}).get("hbm_bytes_per_launch")
        return None if b is None else {"bytes": b, "session": d.get("sessions", {}).get(workload)}
    except Exception:
        return None


def e2e_host(dev, netif, steps: int):
    """PCIe-inclusive rate of halo_rx_parse_batch_host on packed host batches."""
    import numpy as np
    import torch

    from halo_amd import _lib
    from halo_amd.engine import HostBatcher

    res = {}
    for name, kw, n in [("e2e_host_config2_64B_1M", dict(length=64), 1 << 20),
                        ("e2e_host_imix_4M", dict(size_mode=1, proto_mode=3), 4 << 20)]:
        fr = make_batches(dev, netif, n=n, rotate=1, rank=0, **kw)[0]
        lay = fr["layout"]
        # every array is registered below: each on pages of its own (_lib.host_array)
        def own_pages(a):
            b = _lib.host_array(a.shape, a.dtype)
            b[...] = a
            return b

        host = own_pages(fr["bytes"].cpu().numpy())
        offs = own_pages(lay["offsets_dw"].astype(np.uint64) * 4)
        hb = HostBatcher(dev.index or 0)
        out = _lib.host_array(n, _lib.RESULT_DTYPE)
        out.view(np.uint8)[:] = 0  # touched once: no page faults in the timed loop
        lens = own_pages(np.ascontiguousarray(lay["lens"]))
        modes = [("_registered", True, True,
                  "zero-copy: frames and record array registered; the kernel reads the frames in place "
                  "over PCIe and writes the records straight into the caller's array"),
                 ("_registered_dma", True, False,
                  "registered, zero-copy off: one DMA per chunk from the caller's frames, records DMA'd back"),
                 ("_pageable", False, False, "pageable: runtime-staged DMA per chunk, records DMA'd back")]
        for suffix, registered, zero_copy, path in modes:
            pinned = (host, offs, lens, out) if registered else ()
            hb.set_zero_copy(zero_copy)
            out.view(np.uint8)[:] = 0
            with contextlib.ExitStack() as regs:  # unregistered on exit, checked, even on error
                for a in pinned:
                    regs.enter_context(_lib.registered(a))
                hb.parse(host, offs, lens, netif, 1, out=out)  # warm
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    hb.parse(host, offs, lens, netif, 1, out=out)
                el = (time.perf_counter() - t0) / steps
            fb = int(lay["lens"].astype(np.int64).sum())
            res[name + suffix] = {
                "frames": n, "mpps": round(n / el / 1e6, 1), "gbit_s": round(fb * 8 / el / 1e9, 1),
                "ms_per_batch": round(el * 1e3, 3), "ok": int((out["status"] == 0).sum()) == n, "path": path}
        hb.close()
        del fr
        torch.cuda.empty_cache()
    return res


def cgroup_cpu_quota():
    """CPUs' worth of time the process's cgroup allows (cgroup v2 cpu.max "quota period"), or None
    when unlimited or unknown: on the GPU box the affinity mask lists every CPU of the machine while
    the quota is the box's share for one GPU."""
    try:
        cg = "/sys/fs/cgroup"
        for ln in open("/proc/self/cgroup"):
            parts = ln.strip().split(":", 2)
            if len(parts) == 3 and parts[0] == "0":
                cand = os.path.join(cg, parts[2].lstrip("/"), "cpu.max")
                if os.path.exists(cand):
                    cg = os.path.dirname(cand)
                break
        if os.path.exists(os.path.join(cg, "cpu.max")):
            q, per = open(os.path.join(cg, "cpu.max")).read().split()[:2]
            return None if q == "max" else round(int(q) / int(per), 2)
        v1 = os.path.join(cg, "cpu")  # cgroup v1: cfs quota / period
        q = int(open(os.path.join(v1, "cpu.cfs_quota_us")).read())
        per = int(open(os.path.join(v1, "cpu.cfs_period_us")).read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(fr, seconds: float, rotate: int):
    """The C oracle (scalar restatement of the Go path) on the host over the SAME workload the GPU
    line rotates through: the rank's whole shard (`rotate` batches, 16M x 64 B = 1.07 GB of frames +
    512 MB of records at the defaults), so no pass is served from the CPU caches.
    One thread (the reference's one goroutine per NetIf), the box's CPU share for one GPU
    (OMP_NUM_THREADS) and every CPU in the affinity mask, index-sharded over the threads."""
    import resource

    import numpy as np

    from oracle import oracle

    oracle.build()
    lay = fr["layout"]
    host = fr["bytes"].cpu().numpy()
    n = lay["n"]
    out = np.zeros(n, dtype=oracle.RESULT_DTYPE)  # touched once, reused by every pass
    netif = oracle.NetIf.make()
    res = {}
    affinity = len(os.sched_getaffinity(0))
    share = max(1, min(affinity, int(os.environ.get("OMP_NUM_THREADS") or affinity)))
    every = max(1, min(affinity, n // 4096, 1024))
    for threads in sorted({1, share, every}):
        oracle.rx_batch(host, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"], threads=threads, out=out)  # warm
        passes, t0, c0 = 0, time.perf_counter(), resource.getrusage(resource.RUSAGE_SELF)
        while True:
            oracle.rx_batch(host, lay["lens"], netif, 1, offsets_dw=lay["offsets_dw"], threads=threads, out=out)
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2 or (threads > 1 and el >= 2.0):
                break
        c1 = resource.getrusage(resource.RUSAGE_SELF)
        busy = (c1.ru_utime - c0.ru_utime) + (c1.ru_stime - c0.ru_stime)  # CPU seconds of every thread
        res[threads] = (passes * n / el / 1e6, passes, el, round(busy / el, 1))
    one, mt, sh = res[1], res[every], res[share]
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    shard = f"{n / 2 ** 20:g}M x {int(lay['lens'][0])}B UDP frames ({rotate} batches, the GPU line's rotation)"
    quota = cgroup_cpu_quota()
    entry = cpu_entry_rate(host, lay, seconds=min(2.0, seconds / 2), threads=share)
    return {"value": round(one[0], 3), "unit": "Mpps", "cores": 1, "kind": "port",
            "sample": f"{shard}, {one[1]} passes in {one[2]:.1f}s, oracle/halo_rx_oracle.c -O2, one thread; "
                      f"cpu={model}",
            "multi_thread": {"value": round(mt[0], 3), "threads": every, "passes": mt[1],
                             "cpus_in_affinity": affinity, "cpu_quota_cores": quota, "cores_busy": mt[3],
                             "cpu_model": model,
                             "note": "the same shard index-sharded over threads = len(sched_getaffinity); "
                                     "the process's cgroup CPU quota (cpu_quota_cores) caps what they get"},
            "multi_thread_share": {"value": round(sh[0], 3), "threads": share, "passes": sh[1], "cores_busy": sh[3],
                                   "note": "the box's CPU share for one GPU (OMP_NUM_THREADS)"},
            "cpu_entry": entry}


def cpu_entry_rate(host, lay, seconds: float, threads: int) -> dict:
    """The product's own CPU entry point (halo_rx_parse_batch_cpu, libhalo_rx_cpu.so) over the same
    shard: one thread, and `threads` threads on contiguous index ranges (ctypes drops the GIL for
    the call). Not the baseline (that is the port above); the fastest CPU path this build ships."""
    import ctypes
    import threading

    import numpy as np

    from halo_amd import cpu as cpu_entry
    from halo_amd._lib import RESULT_DTYPE, NetIf

    n = lay["n"]
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    lens = np.ascontiguousarray(lay["lens"])
    out = np.zeros(n, dtype=RESULT_DTYPE)
    netif = NetIf.make()
    L = cpu_entry.lib

    errors = []

    def run(lo, hi):
        rc = L.halo_rx_parse_batch_cpu(host.ctypes.data, offs.ctypes.data + 8 * lo, lens.ctypes.data + 2 * lo, hi - lo,
                                       1, netif, out.ctypes.data + 32 * lo, None)
        if rc != 0:
            errors.append(rc)

    res = {}
    for t in sorted({1, threads}):
        cuts = [n * k // t for k in range(t + 1)]
        run(0, n)  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            ths = [threading.Thread(target=run, args=(cuts[k], cuts[k + 1])) for k in range(t)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        res[t] = round(passes * n / el / 1e6, 3)
    if errors:
        raise RuntimeError(f"halo_rx_parse_batch_cpu failed: {errors[:4]}")
    # every synthetic frame is a clean IPv4/UDP frame: OK, EtherType 0x0800, protocol 17 (a record the
    # call never wrote would still read zero)
    ok = bool(np.all((out["status"] == 0) & (out["ethertype"] == 0x0800) & (out["ip_proto"] == 17)))
    return {"value": res[1], "unit": "Mpps", "threads": 1, "value_threads": res[threads], "threads_n": threads,
            "ok": ok, "note": "halo_rx_parse_batch_cpu (include/halo_rx_cpu.h) over the same shard"}


WIRE_OVERHEAD = 24  # bytes per frame on the wire beyond the L2 buffer: preamble + SFD 8, FCS 4, IFG 12
LINE_LIMIT = 7680  # bytes: the final stdout line stays under 8 KB, what the driver parses
# per-entry numbers the stdout line keeps; everything else (prose, probe tables, per-size curves'
# percentiles) goes to the detail file only
_KEEP_NUM = ("mpps", "mstrings_per_s", "mlookups_per_s", "mrecords_per_s", "gbit_s", "gbit_s_wire", "kernel_ms", "ms_per_batch",
             "us_per_batch", "ok", "speedup_vs_separate", "vs_headline", "vs_headline_per_batch", "failing_frac",
             "crossover_frames", "cpu_port_ns_per_frame", "cpu_entry_ns_per_frame", "cpu_entry_crossover_frames", "value", "unit", "ms_per_step")
_KEEP_ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_session", "frac_frames_only",
              "peak_measured_read", "frac_of_measured", "size_matched_probe_ms", "frac_of_size_matched",
              "frac_of_gather_probe", "frac_of_load_pattern_probe", "frac_of_layout_matched")
_SAMPLE_MAX = 200


def _compact_roofline(r: dict) -> dict:
    return {k: r[k] for k in _KEEP_ROOF if k in r}


def _compact_cpu(c: dict) -> dict:
    out = {k: c[k] for k in ("value", "unit", "cores", "kind") if k in c}
    if "sample" in c:
        out["sample"] = str(c["sample"])[:_SAMPLE_MAX]
    for k in ("multi_thread", "multi_thread_share", "cpu_entry"):
        if isinstance(c.get(k), dict):
            out[k] = {kk: c[k][kk] for kk in ("value", "threads", "cpus_in_affinity", "cpu_quota_cores", "cores_busy",
                                              "value_threads", "threads_n") if kk in c[k]}
    return out


def _compact_entry(e):
    """Numbers only: the whitelisted scalars of an entry, its roofline's fractions, its CPU baseline's
    value, and the same for every nested entry (compact records, launch-per-poll, per-size curves)."""
    if not isinstance(e, dict):
        return e if isinstance(e, (int, float, bool)) else None
    if e and all(k.isdigit() and isinstance(v, dict) for k, v in e.items()):  # a per-size curve: medians only
        return {k: v.get("us_median") for k, v in e.items()}
    out = {}
    for k, v in e.items():
        if k == "roofline" and isinstance(v, dict):
            out[k] = {kk: v[kk] for kk in ("frac", "frac_of_size_matched", "frac_of_gather_probe",
                                             "frac_of_load_pattern_probe", "frac_of_layout_matched",
                                             "traffic_session") if kk in v}
        elif k == "cpu_baseline" and isinstance(v, dict):
            out[k] = {kk: v[kk] for kk in ("value", "unit", "cores") if kk in v}
        elif isinstance(v, dict):
            c = _compact_entry(v)
            if c:
                out[k] = c
        elif k in _KEEP_NUM and isinstance(v, (int, float, bool, str)) and not (isinstance(v, str) and len(v) > 16):
            out[k] = v
    return out


def compact_line(line: dict, limit: int = LINE_LIMIT) -> dict:
    """The stdout JSON line the driver parses: the headline keys, `roofline`, `cpu_baseline`,
    `config4_128M_one_gpu` and, per secondary, its numbers only. Prose fields (what / note / sample
    beyond 200 chars / path / mix) and probe tables stay in the detail file. If the result would still
    exceed `limit` bytes, secondaries are dropped largest first (named in `secondary_dropped`)."""
    out = {}
    for k, v in line.items():
        if k == "roofline":
            out[k] = _compact_roofline(v)
        elif k == "cpu_baseline":
            out[k] = None if v is None else _compact_cpu(v)
        elif k == "per_rank":
            out[k] = [{"rank": r.get("rank"), "pci_bus_id": r.get("pci_bus_id"), "kernel_ms": r.get("kernel_ms"),
                       "valid": (r.get("validation") or {}).get("valid")} for r in v]
        elif k == "config4_128M_one_gpu" and isinstance(v, dict):
            c = {kk: v[kk] for kk in ("frames", "steps", "value", "unit", "gbit_s", "ms_per_step", "kernel_ms",
                                      "alg_bytes_per_launch") if kk in v}
            c["roofline"] = _compact_roofline(v.get("roofline", {}))
            out[k] = c
        elif k == "secondary" and isinstance(v, dict):
            out[k] = {name: _compact_entry(e) for name, e in v.items()}
        elif k in ("note", "whole_shard_launch") and isinstance(v, dict):
            out[k] = _compact_entry(v)
        else:
            out[k] = v
    while len(json.dumps(out)) > limit and out.get("secondary"):
        name = max(out["secondary"], key=lambda n: len(json.dumps(out["secondary"][n])))
        del out["secondary"][name]
        out.setdefault("secondary_dropped", []).append(name)
    return out


def emit_line(line: dict, detail_path: str) -> str:
    """Write the full record to `detail_path` (a JSON file) and print the compact line on stdout."""
    try:
        os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
        with open(detail_path, "w") as f:
            json.dump(line, f, indent=1)
        log(f"[bench] full record: {detail_path}")
    except OSError as e:
        log(f"[bench] could not write {detail_path}: {e}")
    s = json.dumps(compact_line(line))
    print(s, flush=True)
    return s


def main():
    args = parse_args()
    plan = rank_plan(args.gpus, os.environ)
    if plan == "spawn":  # nothing has touched the GPU in this process: run the N ranks as a child job
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if plan == "mismatch":
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}: refusing to report a "
            "line whose n_gpus is not the job's rank count")
        sys.exit(2)
    import numpy as np  # noqa: F401
    import torch

    d = Dist()
    # one process per GPU; ranks beyond the visible devices share them (rehearsals on fewer GPUs:
    # the line's distinct_devices says so)
    gpu = d.local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(gpu))
    netif = NetIf.make()  # eth0 of example.UsePcapDev (example/example.go:768-773)
    measure_read_peak(dev, d)
    n = args.frames
    shard_frames = n * args.rotate

    # The headline step on every rank (config 2 at N = 1; config 4's scaling curve at N > 1): one
    # n-frame launch per step over the rank's own shard of the global stream, batches rotating.
    log(f"[rank {d.rank}] generating a {shard_frames}-frame shard of 64 B (global frames "
        f"{shard_first_index(d.rank, 0, shard_frames, 1)}..) as {args.rotate} x {n}-frame batches")
    batches, shard = shard_batches(dev, netif, rank=d.rank, n=n, rotate=args.rotate)
    out = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    wall, kern_ms = time_steps(batches, out, netif, flags=1, hint=64, steps=args.steps, warmup=args.warmup, d=d)
    per_rank_kms = d.gather(kern_ms)
    frames_total = n * args.steps * d.world
    mpps = frames_total / wall / 1e6
    fbytes = frame_bytes(batches[0])
    gbit = fbytes * args.steps * d.world * 8 / wall / 1e9
    # the same frames as wire bits: + 24 B each for preamble + SFD (8), FCS (4), inter-frame gap (12)
    gbit_wire = (fbytes + WIRE_OVERHEAD * n) * args.steps * d.world * 8 / wall / 1e9
    alg = fbytes + n * (4 + 2 + RESULT_BYTES)  # frames + dword offset + u16 len + record
    # every rank checks its own shard on its own device after the timed region, and says which device
    ident = device_identity(gpu)
    ident["rank"] = d.rank
    ident["kernel_ms"] = round(kern_ms, 5)
    ident["validation"] = validate_shard(batches, netif, dev, d.rank)
    ranks = d.gather_obj(ident)
    distinct = len({r["pci_bus_id"] for r in ranks}) == d.world
    if d.world == 1:
        workload = ("config2: 1M x 64B IPv4/UDP frames resident in HBM, CheckSumEnable=true, ragged ring-record "
                    "layout (u32 dword offsets + u16 lens), 32B record/frame")
    else:
        workload = (f"config4: 64B IPv4/UDP frames index-sharded over {d.world} GPUs, {shard_frames >> 20}M frames "
                    f"per GPU ({d.world * shard_frames >> 20}M in all; 128M at N=8), each GPU parsing {n >> 20}M "
                    "frames per step (the N=1 headline step), CheckSumEnable=true, 32B record/frame")
    line = {
        "metric": METRIC, "value": round(mpps, 2), "unit": "Mpps", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": workload, "frames_per_gpu_per_step": n, "frame_bytes": 64,
                   "rotating_batches": args.rotate, "frames_per_gpu": shard_frames,
                   "frames_total": shard_frames * d.world,
                   "parallelism": f"index-sharded x{d.world}, no collective"},
        "gbit_s": round(gbit, 2),
        "gbit_s_wire": round(gbit_wire, 2),
        "kernel_ms": round(max(per_rank_kms), 5),
        "per_rank_kernel_ms": [round(k, 5) for k in per_rank_kms],
        "kernel": "rx_lane_kernel<0, 0> (lane per frame, ragged, no fused pass)",
        "roofline": roofline(alg, kern_ms, load_traffic("config2"), frame_bytes=fbytes),
        "alg_bytes_per_launch": alg,
        "per_rank": ranks,
        "distinct_devices": distinct,
        "validated": all(r["validation"]["valid"] for r in ranks),
        "cpu_baseline": None,
    }
    if d.world > 1:
        # the same shards, each parsed whole in ONE launch per step (16M frames per GPU per launch)
        sh_out = torch.empty((shard_frames, RESULT_BYTES), dtype=torch.uint8, device=dev)
        st = max(5, args.steps // 5)
        w2, k2 = time_steps([shard], sh_out, netif, flags=1, hint=64, steps=st, warmup=2, d=d)
        ks = d.gather(k2)
        line["whole_shard_launch"] = {
            "value": round(shard_frames * d.world * st / w2 / 1e6, 2), "unit": "Mpps", "steps": st,
            "ms_per_step": round(w2 / st * 1e3, 4), "per_rank_kernel_ms": [round(k, 5) for k in ks],
            "what": f"each GPU's {shard_frames >> 20}M-frame shard in one launch per step"}
        del sh_out
        if not distinct:
            line["note"] = ("ranks shared a device (fewer GPUs than ranks): a rehearsal of the N-rank path, "
                            "not a scaling point")
        d.close()
        if d.rank == 0:
            emit_line(line, args.detail)
        sys.exit(0 if line["validated"] else 3)
    del shard
    line["roofline"]["note"] = ("achieved = (frame bytes + 6 B metadata + 32 B record) per launch / average "
                                "launch duration (one HIP event pair over the timed region / steps); "
                                "peak = HBM3E spec; traffic = HBM request bytes per launch from profiles/pmc_summary.json "
                                "(rocprofv3 --pmc TCC_EA0_RDREQ_{32,64,128}B and TCC_EA0_WRREQ/_64B, each "
                                "request at its size; the same kernel and workload, tools/prof_kernels.py); "
                                "size_matched_probe_ms = a no-work kernel streaming "
                                "the same bytes in and out with perfect access patterns over the same number of "
                                "rotating buffers (frac_of_size_matched = probe / kernel time)")
    line["roofline"]["peak_measured_read_probes"] = MEASURED_READ_PROBES
    if d.world == 1 and not args.no_secondary:
        with_probe(line["roofline"], size_matched_probe(dev, fbytes + 6 * n, RESULT_BYTES * n, d, nbuf=args.rotate),
                   kern_ms)

    if d.world == 1 and not args.no_secondary:
        sec = {}
        # cache-resident variant of the headline (one batch, 102 MB < 256 MB Infinity Cache)
        w1, k1 = time_steps(batches[:1], out, netif, flags=1, hint=64, steps=args.steps, warmup=args.warmup, d=d)
        sec["config2_mall_resident"] = {"mpps": round(n * args.steps / w1 / 1e6, 1), "kernel_ms": round(k1, 5),
                                        "roofline": roofline(alg, k1)}
        # the same headline workload writing the compact 16 B record (verdict + 5-tuple only)
        from halo_amd._lib import HALO_RX_RECORD_COMPACT

        wc, kc = time_steps(batches, out, netif, flags=1 | HALO_RX_RECORD_COMPACT, hint=64, steps=args.steps,
                            warmup=args.warmup, d=d)
        algc = fbytes + n * (4 + 2 + 16)
        sec["config2_compact_record16"] = {"mpps": round(n * args.steps / wc / 1e6, 1), "kernel_ms": round(kc, 5),
                                           "roofline": roofline(algc, kc)}
        # the headline with the §5 metrics output on: every launch counts into a status histogram
        hist = torch.zeros(14, dtype=torch.int32, device=dev)
        wh, kh = time_steps(batches, out, netif, flags=1, hint=64, steps=args.steps, warmup=args.warmup, d=d,
                            hist=hist)
        hsum = int(hist.sum().item())
        sec["config2_status_histogram"] = {
            "mpps": round(n * args.steps / wh / 1e6, 1), "kernel_ms": round(kh, 5), "roofline": roofline(alg, kh),
            "vs_headline": round(kern_ms / kh, 4), "hist_frames": hsum, "hist_ok": int(hist[0].item()),
            "what": "the headline step with d_status_hist (block-aggregated in LDS, then fence-free self-completing (arrivals, count) words: one level of 16-block runs for grids up to 16384 blocks, a two-level tree above; the lane grid halved up to 1M frames)"}
        assert hsum == n * (args.steps + args.warmup) and int(hist[0].item()) == hsum
        # the batch stream handed over 8 batches per launch (halo_rx_parse_batches_device): the ramp
        # and tail of a 1M-frame launch paid once per 8M frames
        sec["config2_batch_stream"] = batch_stream_secondary(batches, netif, args.steps, args.warmup, d, kern_ms)
        sec["config2_queues"] = queues_secondary(batches, netif, args.steps, args.warmup, d, kern_ms)

        # forward / transmit rewrite (§8f row f2) on the headline frames: DNAT + SNAT + DPDK fill
        import numpy as np

        ops_h = tx_ops_for(n)
        ops_d = torch.from_numpy(ops_h.view(np.uint8)).to(dev)
        res_d = torch.empty(n, dtype=torch.uint8, device=dev)
        wt, kt = time_tx_steps(batches, ops_d, res_d, flags=1, hint=64, steps=args.steps, warmup=args.warmup, d=d)
        algt = fbytes + n * (4 + 2 + 16 + 1 + TX_WRITE_BYTES)
        sec["tx_fixup_config2_nat_dpdk"] = {
            "mpps": round(n * args.steps / wt / 1e6, 1), "kernel_ms": round(kt, 5),
            "roofline": roofline(algt, kt, load_traffic("tx_config2")), "alg_bytes_per_launch": algt,
            "steps": "NatChangeDst + NatChangeSrc + eth_tx DPDK fill, per-frame addresses/ports"}
        # the probe moves what the memory system must: the frames + metadata + ops in, and one
        # 64-byte write per frame (the kernel's TCC_EA0_WRREQ_64B count, profiles/r03/r3f/) + results
        with_probe(sec["tx_fixup_config2_nat_dpdk"]["roofline"],
                   size_matched_probe(dev, fbytes + n * (4 + 2 + 16), n * (64 + 1), d, nbuf=args.rotate), kt)
        if not args.no_cpu:
            from oracle import oracle as O

            m = 1 << 18
            lay0 = batches[0]["layout"]
            host = batches[0]["bytes"][:int(lay0["offsets_dw"][m]) * 4].cpu().numpy()
            sec["tx_fixup_config2_nat_dpdk"]["cpu_baseline"] = cpu_rate(
                lambda: O.tx_batch(host, lay0["offsets_dw"][:m], lay0["lens"][:m], ops_h[:m], flags=1), m, 2.0, "Mpps",
                f"{m} x 64B frames of batch 0, same ops (oracle/halo_tx_oracle.c)")
        del ops_d, res_d
        sec["flow_hash_config2_nat_wan"] = flow_hash_secondary(batches, out, netif, args.steps, args.warmup, d,
                                                               with_cpu=not args.no_cpu)
        sec["rx_flow_fused_config2_nat_wan"] = rx_flow_fused_secondary(
            batches, out, netif, args.steps, args.warmup, d, kern_ms, sec["flow_hash_config2_nat_wan"]["kernel_ms"])
        del batches
        torch.cuda.empty_cache()
        sec.update(tx_build_secondary(dev, args.steps, args.warmup, d, with_cpu=not args.no_cpu))
        sec["lo_drain_1M_50B"] = lo_drain_secondary(dev, netif, args.steps, args.warmup, d, with_cpu=not args.no_cpu)
        torch.cuda.empty_cache()
        sec["xxh3_kcp_segments_1M"] = xxh3_secondary(dev, max(5, args.steps // 10), 2, d, with_cpu=not args.no_cpu)
        torch.cuda.empty_cache()
        sec["route_lpm_500k_prefixes"] = route_secondary(dev, max(10, args.steps // 4), 3, d, with_cpu=not args.no_cpu)
        torch.cuda.empty_cache()
        line["config4_128M_one_gpu"] = config4_one_gpu(dev, netif, d, max(20, args.steps // 4), 3)
        # SURVEY §8d's mutation set: 1/64 of the frames with one bit flipped in [14, L)
        bm = make_batches(dev, netif, n=n, rotate=8, rank=0, mutate_shift=6)
        om = torch.empty((n, RESULT_BYTES), dtype=torch.uint8, device=dev)
        hm = torch.zeros(14, dtype=torch.int32, device=dev)
        wm, km = time_steps(bm, om, netif, flags=1, hint=64, steps=args.steps, warmup=args.warmup, d=d, hist=hm)
        fbm = frame_bytes(bm[0])
        hmn = hm.cpu().numpy().astype(np.int64)
        sec["config2_mutated_1in64"] = {
            "mpps": round(n * args.steps / wm / 1e6, 1), "kernel_ms": round(km, 5),
            "roofline": roofline(fbm + n * (6 + RESULT_BYTES), km, frame_bytes=fbm),
            "failing_frac": round(float(hmn[1:].sum() / hmn.sum()), 5),
            "status_hist": {STATUS_NAMES[i]: int(hmn[i]) for i in range(14) if hmn[i]},
            "what": "config 2 with 1/64 of the frames mutated (one random bit flipped in [14, L) after the checksums "
                    "were filled, SURVEY §8d), 8 rotating batches, status histogram on"}
        del bm, om
        torch.cuda.empty_cache()
        for name, kw, hint, strided_len, flags in [
            ("config4_shard_16M_64B", dict(length=64), 64, 0, 1),
            ("1500B_udp_1M", dict(length=1500), 1500, 0, 1 | _lib.HALO_RX_UNIFORM_LEN),
            ("config3_imix_16M", dict(size_mode=1, proto_mode=3), 1500, 0, 1),
            ("config5_jumbo_9000B_tcp_4M_ext", dict(length=9000, proto_mode=1, strided=True), 0, 9000, 3),
        ]:
            nn = (16 << 20) if ("imix" in name or "config4" in name) else ((4 << 20) if "jumbo" in name else n)
            rot = 2 if nn * (kw.get("length", 352)) < (1 << 31) else 1
            log(f"[secondary] {name}: {rot} x {nn} frames")
            bs = make_batches(dev, netif, n=nn, rotate=rot, rank=0, **kw)
            o2 = torch.empty((nn, RESULT_BYTES), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            steps = max(5, args.steps // 5)
            w2, k2 = time_steps(bs, o2, netif, flags=flags, hint=hint, steps=steps, warmup=2, d=d,
                                strided_len=strided_len)
            fb = frame_bytes(bs[0])
            meta = 0 if strided_len else 6
            a2 = fb + nn * (meta + RESULT_BYTES)
            sec[name] = {"frames": nn, "mpps": round(nn * steps / w2 / 1e6, 1),
                         "gbit_s": round(fb * steps * 8 / w2 / 1e9, 1),
                         "gbit_s_wire": round((fb + WIRE_OVERHEAD * nn) * steps * 8 / w2 / 1e9, 1),
                         "kernel_ms": round(k2, 4),
                         "roofline": roofline(a2, k2, load_traffic(name), frame_bytes=fb)}
            if "imix" in name:
                sec[name]["mix"] = ("sizes 64/570/1500 B at 7:4:1; protocols UDP 50 / TCP 40 / ICMP 10 % "
                                    "(synth proto_mode 3, per frame from the seed)")
            if "config4" in name:
                sec[name]["what"] = ("one GPU's shard of BASELINE config 4 (128M x 64 B over 8 GPUs = 16M per GPU, "
                                     "index-sharded, no collective); the scaling run itself is bench.py --gpus N")
            del bs, o2
            torch.cuda.empty_cache()
            if not strided_len:
                with_probe(sec[name]["roofline"], size_matched_probe(dev, fb + nn * meta, nn * RESULT_BYTES, d,
                                                                     nbuf=rot, steps=steps), k2)
        # end to end from host memory: pinned H2D -> kernel -> D2H, double
        # buffered in 64 MB chunks by halo_rx_parse_batch_host; the frame buffer is registered
        # (pinned in place) so each chunk is one DMA straight from it
        sec.update(e2e_host(dev, netif, steps=max(3, args.steps // 40)))
        # the drop-in surface at small batch sizes (go/gpurx ParseBatch, single-frame Parse*)
        sec["dropin_small_batch"] = dropin_small_batch(dev, netif, with_cpu=not args.no_cpu)
        # halo's SPSC packet ring as the source (BASELINE config 1 over a Wire)
        sec.update(ring_secondary(dev, netif, max(10, args.steps // 4), 3, d, with_cpu=not args.no_cpu))
        torch.cuda.empty_cache()
        line["secondary"] = sec
    if d.world == 1 and not args.no_cpu:  # rank 0 at N=1 only
        _, cshard = shard_batches(dev, netif, rank=0, n=n, rotate=args.rotate)
        torch.cuda.synchronize()
        log("[cpu baseline] timing the oracle on the host over the rotated shard")
        line["cpu_baseline"] = cpu_baseline(cshard, args.cpu_seconds, args.rotate)
        del cshard
    d.close()
    if d.rank == 0:
        emit_line(line, args.detail)
    if not line["validated"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
