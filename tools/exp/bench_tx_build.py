#!/usr/bin/env python3
"""Only bench.py's tx build rows (halo_tx_build_batch_device), for A/B of tx_build.hip (tools only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench
    from halo_amd import _lib

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    d = bench.Dist()
    r = bench.tx_build_secondary(dev, 100, 10, d, with_cpu=False)
    print(json.dumps({k: v["kernel_ms"] for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
