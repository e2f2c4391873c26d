#!/usr/bin/env python3
"""The stream kernel's read contract under a FETCH_SIZE pass (tools only):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- python3 tools/exp/gap_fetch.py

Launches the stream kernel 10 times on 256k IMIX frames packed densely, then 10 times on the same
frames with a 20 KB hole in the middle of every 64-frame window (windows that still pass the 2x
density test, as tests/test_gpu_stream.py::test_dense_windows_with_page_holes). If the hole pages
were read, the second layout's FETCH_SIZE would be about 2x the first's (the holes add ~80 MB to
~90 MB of frames); printed beside it are the bytes each layout must read.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from halo_amd import _lib, protocol, synth
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    n = 1 << 18
    lay = synth.layout(n, size_mode=1, proto_mode=3, first_index=7)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    blob = fr["bytes"].cpu().numpy()
    src = lay["offsets_dw"].astype(np.int64) * 4
    lens = lay["lens"].astype(np.int64)
    report = {}
    for name, hole in (("dense", 0), ("holes_20KB_per_window", 4096 + 1024)):
        gaps = np.zeros(n, np.int64)
        gaps[32::64] = hole
        offs = np.zeros(n, np.int64)
        pos = 0
        for k in range(n):
            pos += 4 * int(gaps[k])
            offs[k] = pos
            pos += (int(lens[k]) + 3) & ~3
        data = np.zeros(pos + 64, np.uint8)
        for k in range(n):
            data[offs[k]:offs[k] + lens[k]] = blob[src[k]:src[k] + lens[k]]
        buf = torch.from_numpy(data).to(dev)
        o = torch.from_numpy((offs // 4).astype(np.uint32).view(np.int32)).to(dev)
        ln = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev)
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        fw = protocol.flags_word(True, False, -2)  # the stream kernel
        torch.cuda.synchronize()
        for _ in range(10):
            _lib.check("parse", _lib.lib.halo_rx_parse_batch_device(_lib.ptr(buf), _lib.ptr(o), _lib.ptr(ln), n, fw,
                                                                    NetIf.make(), 1500, _lib.ptr(out), None, None))
        torch.cuda.synchronize()
        report[name] = {"frame_bytes": int(lens.sum()), "span_bytes": int(pos), "metadata_bytes": 6 * n,
                        "record_bytes": 32 * n}
        del buf
    print(json.dumps(report), flush=True)


if __name__ == "__main__":
    main()
