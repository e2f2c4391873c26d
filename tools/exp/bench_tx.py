#!/usr/bin/env python3
"""Only bench.py's TX row (config 2 frames, DNAT + SNAT + DPDK fill): quick A/B of tx_fixup.hip (tools only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    d = bench.Dist()
    n = 1 << 20
    batches = bench.make_batches(dev, NetIf.make(), n=n, rotate=8, rank=0)
    ops_d = torch.from_numpy(bench.tx_ops_for(n).view(np.uint8)).to(dev)
    res_d = torch.empty(n, dtype=torch.uint8, device=dev)
    _, kt = bench.time_tx_steps(batches, ops_d, res_d, flags=1, hint=64, steps=100, warmup=10, d=d)
    print(json.dumps({"tx_kernel_ms": round(kt, 5)}), flush=True)


if __name__ == "__main__":
    main()
