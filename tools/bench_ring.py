#!/usr/bin/env python3
"""Only bench.py's ring rows (SURVEY §8f row f1 / BASELINE config 1): quick iteration on the ring path."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sweep(dev, netif):
    """Poll latency vs batch size, small path vs pipelined path (64 B frames, registered ring)."""
    import time

    import numpy as np

    import bench
    from halo_amd.ring import RingBuffer, RingConsumer

    fr = bench.make_batches(dev, netif, n=1 << 18, rotate=1, rank=0)[0]
    host = fr["bytes"].cpu().numpy()
    offs = fr["layout"]["offsets_dw"].astype(np.uint64) * 4
    lens = fr["layout"]["lens"]
    for m in (1, 100, 1000, 4000, 16000, 64000, 250000):
        row = {"frames": m}
        for name, small in (("small", 16 << 20), ("pipelined", 0)):
            ring = RingBuffer(64 << 20)
            cons = RingConsumer(ring, capacity=1514, max_frames=1 << 18, small_poll=small)
            times = []
            for s in range(41 if m < 100000 else 11):
                assert ring.write_batch(host, offs[:m], lens[:m]) == m
                t0 = time.perf_counter()
                _, inf, _ = cons.poll(netif)
                cons.commit()
                el = time.perf_counter() - t0
                assert inf["n_frames"] == m
                if s:
                    times.append(el)
            row[name + "_us"] = round(float(np.median(times)) * 1e6, 1)
            cons.close()
        print(json.dumps(row), flush=True)


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    if "--sweep" in sys.argv:
        return sweep(torch.device("cuda", 0), NetIf.make())
    res = bench.ring_secondary(torch.device("cuda", 0), NetIf.make(), int(sys.argv[1]) if len(sys.argv) > 1 else 50,
                               3, bench.Dist(), with_cpu="--cpu" in sys.argv)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
