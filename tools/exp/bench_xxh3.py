#!/usr/bin/env python3
"""Only bench.py's XXH3 rows (KCP segments + the NAT flow keys): quick A/B of flow_hash.hip (tools only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench
    from halo_amd import _lib

    _lib.check("init", _lib.lib.halo_rx_init(0))
    r = bench.xxh3_secondary(torch.device("cuda", 0), 20, 3, bench.Dist())
    print(json.dumps({"kernel_ms": r["kernel_ms"], "mstrings_per_s": r["mstrings_per_s"],
                      "frac": r["roofline"]["frac"]}), flush=True)


if __name__ == "__main__":
    main()
