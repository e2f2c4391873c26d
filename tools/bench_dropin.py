"""The drop-in surface's per-call latency curve alone (bench.py dropin_small_batch): python
tools/bench_dropin.py [--no-cpu] -> one JSON object on stdout."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    torch.cuda.set_device(0)
    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    print(json.dumps(bench.dropin_small_batch(torch.device("cuda", 0), NetIf.make(),
                                              with_cpu="--no-cpu" not in sys.argv)), flush=True)


if __name__ == "__main__":
    main()
