"""Histogram-on vs off launch time of the config-2 batch (1M x 64 B), per library variant.
usage: python tools/exp/bench_hist.py [reps] [other libhalo_rx.so to time instead]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from halo_amd import _lib, protocol, synth  # noqa: E402
from halo_amd._lib import NetIf  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    other = ctypes.CDLL(sys.argv[2]) if len(sys.argv) > 2 else None
    if other is not None:
        other.halo_rx_parse_batch_device.argtypes = _lib.lib.halo_rx_parse_batch_device.argtypes
        other.halo_rx_init(0)
    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    import os
    n = int(os.environ.get("HIST_FRAMES", 1 << 20))
    lay = synth.layout(n, length=64)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    hist = torch.zeros(16, dtype=torch.int32, device=dev)
    def parse(h):
        if other is None:
            protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                        max_len_hint=64, out=out, hist=h)
            return
        rc = other.halo_rx_parse_batch_device(
            _lib.ptr(fr["bytes"]), _lib.ptr(fr["offsets_dw"]), _lib.ptr(fr["lens"]), n, 1, NetIf.make(), 64,
            _lib.ptr(out), _lib.ptr(h), torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc

    for h in (None, hist, None, hist):
        for _ in range(20):
            parse(h)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            parse(h)
        e1.record()
        torch.cuda.synchronize()
        print(f"hist={'on ' if h is not None else 'off'} {e0.elapsed_time(e1) / reps * 1000:.2f} us/launch", flush=True)
    total = int(hist.sum().item())
    import os
    if os.environ.get("HIST_NOCHECK"):
        print("total", total)
    else:
        assert total == 2 * (reps + 20) * n, total
    print("hist exact", np.asarray(hist.cpu())[:2])


if __name__ == "__main__":
    main()
