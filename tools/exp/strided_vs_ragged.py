"""Tools only: the headline's 1M x 64 B batches parsed through the ragged layout (u32 dword offsets +
u16 lengths, the headline) and through the strided one (stride 64, one length: no metadata loads),
same frames, same native step loop; how much of the launch the metadata chain costs."""
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
    for rnd in range(3):
        for name, sl in (("ragged", 0), ("strided64", 64)):
            w, k = bench.time_steps(batches, out, netif, flags=1, hint=64, steps=1000, warmup=50, d=d, strided_len=sl)
            res.setdefault(name, []).append(round(k * 1e3, 2))
    print(json.dumps({"us_per_launch": res}), flush=True)


if __name__ == "__main__":
    main()
