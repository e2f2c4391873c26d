#!/usr/bin/env python3
"""A few ring e2e polls (1M x 64 B frames, registered 128 MiB ring) for a rocprofv3 timeline (tools only)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    n = 1 << 20
    fr = bench.make_batches(dev, NetIf.make(), n=n, rotate=1, rank=0)[0]
    host = fr["bytes"].cpu().numpy()
    offs = fr["layout"]["offsets_dw"].astype(np.uint64) * 4
    lens = fr["layout"]["lens"]
    ring = RingBuffer(128 << 20)
    cons = RingConsumer(ring, capacity=1514, max_frames=n + 64, register=True)
    for s in range(6):
        assert ring.write_batch(host, offs, lens) == n
        t0 = time.perf_counter()
        _, inf, _ = cons.poll(NetIf.make())
        cons.commit()
        print(f"poll {s}: {(time.perf_counter() - t0) * 1e3:.3f} ms, {inf['n_frames']} frames", flush=True)
    cons.close()


if __name__ == "__main__":
    main()
