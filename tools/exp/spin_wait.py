"""Tools only: the headline region at the driver's size (20 steps, 5 warm-up) with the region's end
waited for by hipStreamSynchronize alone or by polling the closing event first (HALO_BENCH_SPIN=1),
interleaved rounds; wall us per step against the HIP-event us per launch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    import torch

    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    netif = NetIf.make()
    d = bench.Dist()
    n = 1 << 20
    batches, _ = bench.shard_batches(dev, netif, rank=0, n=n, rotate=16)
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    res = {}
    for rnd in range(8):
        for mode in ("0", "1"):
            os.environ["HALO_BENCH_SPIN"] = mode
            for steps in (20, 1000):
                w, k = bench.time_steps(batches, out, netif, flags=1, hint=64, steps=steps, warmup=5, d=d)
                res.setdefault(f"spin{mode}_steps{steps}", []).append((round(w / steps * 1e6, 2), round(k * 1e3, 2)))
    print(json.dumps({"wall_us_per_step, event_us_per_launch": res}), flush=True)


if __name__ == "__main__":
    main()
