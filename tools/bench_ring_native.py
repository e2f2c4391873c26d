#!/usr/bin/env python3
"""BASELINE config 1's poll loop in native code (tools/bench_loop.hip halo_bench_ring_polls): an
engine.Wire-sized ring (8 MiB), m x 64 B frames per batch, poll + commit per batch, no Python in
between. Prints one JSON line (median / p10 / p90 microseconds per batch). Run it under
`rocprofv3 --kernel-trace --hip-runtime-trace --stats` for the per-batch breakdown.

    python tools/bench_ring_native.py [--frames 1000] [--iters 2000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(m: int = 1000, iters: int = 2000, warmup: int = 50, small_poll=None, register_out: bool = True,
        persistent: bool = False) -> dict:
    import ctypes

    import numpy as np
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    dev = torch.device("cuda", 0)
    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    netif = NetIf.make()
    fr = bench.make_batches(dev, netif, n=m, rotate=1, rank=0)[0]
    host = _lib.host_array(fr["bytes"].numel())
    host[:] = fr["bytes"].cpu().numpy()
    offs = fr["layout"]["offsets_dw"].astype(np.uint64) * 4
    lens = np.ascontiguousarray(fr["layout"]["lens"])
    ring = RingBuffer(8 << 20)
    cons = RingConsumer(ring, capacity=1514, max_frames=4096, register=True, small_poll=small_poll,
                        persistent=persistent)
    out = cons._out if register_out else np.zeros(cons.max_frames, _lib.RESULT_DTYPE)
    us = np.zeros(iters, np.float64)
    bad = ctypes.c_uint32()
    L = bench.bench_lib()
    rc = L.halo_bench_ring_polls(ring.mem.ctypes.data, cons._h, host.ctypes.data, offs.ctypes.data, lens.ctypes.data, m,
                                 1, ctypes.addressof(netif), out.ctypes.data, warmup, iters, us.ctypes.data,
                                 ctypes.byref(bad))
    _lib.check("halo_bench_ring_polls", rc)
    st = cons.stats()
    cons.close()
    sp = max(1, st["small_polls"])
    return {"frames": m, "persistent": persistent, "iters": iters, "bad_batches": int(bad.value), "us_median": round(float(np.median(us)), 2),
            "us_p10": round(float(np.percentile(us, 10)), 2), "us_p90": round(float(np.percentile(us, 90)), 2),
            "mpps": round(m / float(np.median(us)), 3),
            "per_small_poll_us": {"walk": round(st["walk_ns"] / sp / 1e3, 2), "wait": round(st["wait_ns"] / sp / 1e3, 2),
                                  "service_gpu": round(st["service_gpu_ns"] / max(1, st["service_requests"]) / 1e3, 2)},
            "small_polls": st["small_polls"], "service_requests": st["service_requests"],
            "service_launches": st["service_launches"]}


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=1000)
    p.add_argument("--iters", type=int, default=2000)
    p.add_argument("--sweep", action="store_true")
    p.add_argument("--persistent", action="store_true")
    a = p.parse_args()
    if a.sweep:
        for persistent in (False, True):
            for m in (1, 64, 256, 1000, 4000):
                print(json.dumps(run(m, a.iters, persistent=persistent)), flush=True)
    else:
        print(json.dumps(run(a.frames, a.iters, persistent=a.persistent)), flush=True)
