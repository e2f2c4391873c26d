"""Zero-copy probe (tools only): the rx kernels reading frames straight from pinned host memory
over PCIe (records to device or to pinned host memory) against an SDMA H2D copy of the same
bytes. Decides whether the host path should DMA chunks or let the kernel read them in place."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from halo_amd import _lib  # noqa: E402
from halo_amd._lib import NetIf  # noqa: E402


def main():
    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    netif = NetIf.make()
    d = bench.Dist()
    for name, kw, n in [("64B_1M", dict(length=64), 1 << 20), ("imix_4M", dict(size_mode=1, proto_mode=3), 4 << 20)]:
        fr = bench.make_batches(dev, netif, n=n, rotate=1, rank=0, **kw)[0]
        nb = fr["bytes"].numel()
        fbytes = bench.frame_bytes(fr)
        host = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
        host.copy_(fr["bytes"])
        out_d = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        out_h = torch.empty((n, 32), dtype=torch.uint8, pin_memory=True)
        torch.cuda.synchronize()
        # SDMA copy of the frame bytes, then of the records back
        for _ in range(2):
            t0 = time.perf_counter()
            fr["bytes"].copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            out_h.copy_(out_d, non_blocking=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        print(f"{name}: SDMA H2D {nb / 1e6:.1f} MB {(t1 - t0) * 1e3:.3f} ms = {nb / (t1 - t0) / 1e9:.1f} GB/s; "
              f"D2H records {(t2 - t1) * 1e3:.3f} ms", flush=True)
        ref = None
        for label, bsrc, out in [("device", fr, out_d), ("host-frames", dict(fr, bytes=host), out_d),
                                 ("host-frames+records", dict(fr, bytes=host), out_h)]:
            wall, kms = bench.time_steps([bsrc], out, netif, flags=1, hint=0, steps=10, warmup=2, d=d)
            h = int(out.to(dev).view(torch.int64).sum().item())
            ref = h if ref is None else ref
            print(f"{name}: kernel reading {label}: {kms:.3f} ms = {fbytes / kms / 1e6:.1f} GB/s of frames, "
                  f"{n / kms / 1e3:.1f} Mpps  {'same' if h == ref else 'MISMATCH'}", flush=True)
        del fr, host, out_d, out_h
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
