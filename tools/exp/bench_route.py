#!/usr/bin/env python3
"""Only bench.py's route row (500k prefixes, 4M lookups): quick A/B of route_lpm.hip (tools only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench
    from halo_amd import _lib

    _lib.check("init", _lib.lib.halo_rx_init(0))
    r = bench.route_secondary(torch.device("cuda", 0), 20, 3, bench.Dist())
    print(json.dumps({"kernel_ms": r["kernel_ms"], "mlookups_per_s": r["mlookups_per_s"]}), flush=True)


if __name__ == "__main__":
    main()
