#!/usr/bin/env python3
"""Only bench.py's ring rows (SURVEY §8f row f1 / BASELINE config 1): quick iteration on the ring path."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    res = bench.ring_secondary(torch.device("cuda", 0), NetIf.make(), int(sys.argv[1]) if len(sys.argv) > 1 else 50,
                               3, bench.Dist(), with_cpu="--cpu" in sys.argv)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
