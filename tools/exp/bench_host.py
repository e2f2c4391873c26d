#!/usr/bin/env python3
"""Only bench.py's host-memory rows (halo_rx_parse_batch_host): quick A/B of host_path.hip (tools only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    r = bench.e2e_host(torch.device("cuda", 0), NetIf.make(), 10)
    print(json.dumps({k: v["ms_per_batch"] for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
