#!/usr/bin/env python3
"""Sweep lanes-per-frame (G) per workload on the GPU: kernel time (HIP events), GB/s of
algorithmic bytes, and a bit-identity check of every variant against the first one.

    python tools/tune.py [--quick]
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    quick = "--quick" in sys.argv
    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    netif = NetIf.make()
    d = bench.Dist()
    workloads = [
        ("64B", dict(length=64), 1 << 20, 8, [1, -1, -2]),
        ("64B4M", dict(length=64), 4 << 20, 2, [1]),
        ("64B16M", dict(length=64), 16 << 20, 1, [1]),
        ("64B128M", dict(length=64), 128 << 20, 1, [1]),
        ("128B", dict(length=128), 1 << 20, 8, [1, 4, -1, -2]),
        ("570B", dict(length=570), 1 << 20, 2, [4, 8, -1, -2]),
        ("1500B", dict(length=1500), 1 << 20, 2, [4, 8, -1, -2]),
        ("imix", dict(size_mode=1, proto_mode=3), 16 << 20, 1, [-1, -2, 1, 4]),
        ("jumbo9000", dict(length=9000, proto_mode=1, strided=True), 4 << 20, 1, [8, 16, -1, -2]),
    ]
    if quick:
        workloads = workloads[:2] + workloads[3:5]
    if "--only" in sys.argv:
        keep = sys.argv[sys.argv.index("--only") + 1].split(",")
        workloads = [w for w in workloads if w[0] in keep]
    if "--variants" in sys.argv:  # e.g. --variants=-2 (one kernel variant for every workload)
        only = [int(x) for x in sys.argv[sys.argv.index("--variants") + 1].split(",")]
        workloads = [(a, b, c, d, only) for a, b, c, d, _ in workloads]
    if "--spec" in sys.argv:  # e.g. --spec imix:-2,1500B:8 (workloads and one variant each)
        spec = dict(x.split(":") for x in sys.argv[sys.argv.index("--spec") + 1].split(","))
        workloads = [(a, b, c, d, [int(spec[a])]) for a, b, c, d, _ in workloads if a in spec]
    res = {}
    for name, kw, n, rot, gs in workloads:
        bs = bench.make_batches(dev, netif, n=n, rotate=rot, rank=0, **kw)
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        strided = kw.get("strided", False)
        flags = 3 if strided else 1
        meta = 0 if strided else 6
        alg = bench.frame_bytes(bs[0]) + n * (meta + 32)
        ref = None
        res[name] = {}
        for g in gs:
            # the last of the 20 steps parses batch 19 % rot: the same batch for every variant
            wall, kms = bench.time_steps(bs, out, netif, flags=flags | _lib.variant_flags(g), hint=0, steps=20,
                                         warmup=3, d=d,
                                         strided_len=kw["length"] if strided else 0)
            h = torch.sum(out.view(torch.int64).view(-1, 4) * torch.arange(1, 5, device=dev)).item()
            if ref is None:
                ref = h
            ok = h == ref
            res[name][g] = {"kernel_ms": round(kms, 4),
                            "GBps": round(alg / kms / 1e6, 1), "Mpps": round(n / kms / 1e3, 1), "same": ok}
            print(f"{name:10s} V={g:2d} {kms*1e3:9.1f} us  {alg / kms / 1e6:8.1f} GB/s  "
                  f"{n / kms / 1e3:9.1f} Mpps  {'ok' if ok else 'MISMATCH'}", flush=True)
        del bs, out
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "tune.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
