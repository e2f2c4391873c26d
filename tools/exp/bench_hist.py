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
    lay = synth.layout(1 << 20, length=64)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    out = torch.empty((1 << 20, 32), dtype=torch.uint8, device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    def parse(h):
        if other is None:
            protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                        max_len_hint=64, out=out, hist=h)
            return
        rc = other.halo_rx_parse_batch_device(
            _lib.ptr(fr["bytes"]), _lib.ptr(fr["offsets_dw"]), _lib.ptr(fr["lens"]), 1 << 20, 1, NetIf.make(), 64,
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
    assert total == 2 * (reps + 20) * (1 << 20), total
    print("hist exact", np.asarray(hist.cpu())[:2])


if __name__ == "__main__":
    main()
