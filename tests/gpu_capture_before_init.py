"""Run by tests/test_gpu_hist_tree.py in a process of its own (the trees are made once per process):
a histogram-on parse captured before halo_rx_init must return HALO_E_NOMEM (a capture cannot
allocate), and after halo_rx_init a captured graph counts exactly — before and after
halo_rx_release, which hands the keys back but keeps the trees the graph points at.
Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from halo_amd import _lib, protocol, synth
    from halo_amd._lib import NetIf

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n = 70001
    lay = synth.layout(n, length=64, mutate_shift=3)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    netif = NetIf.make()
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=netif, max_len_hint=64)
    torch.cuda.synchronize()
    want = np.bincount(protocol.records(out)["status"], minlength=14).astype(np.int64)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    res = {"want_failing": int(want[1:].sum())}

    def call(stream):
        return _lib.lib.halo_rx_parse_batch_device(
            _lib.ptr(fr["bytes"]), _lib.ptr(fr["offsets_dw"]), _lib.ptr(fr["lens"]), n, 1, netif, 64, _lib.ptr(out),
            _lib.ptr(hist), ctypes.c_void_p(stream.cuda_stream))

    # 1. captured before the trees exist: refused, nothing recorded, the capture ends cleanly
    s = torch.cuda.Stream()
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0, stream=s, capture_error_mode="thread_local"):
        res["rc_capture_before_init"] = call(s)
    torch.cuda.synchronize()
    res["hist_after_refused"] = int(hist.sum().item())
    del g0

    # 2. halo_rx_init makes the trees; a capture now records the parse
    res["rc_init"] = _lib.lib.halo_rx_init(0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        res["rc_capture_after_init"] = call(s)
    torch.cuda.synchronize()
    hist.zero_()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    res["replay3_exact"] = bool(np.array_equal(hist.cpu().numpy().astype(np.int64), 3 * want))

    # 3. release: keys handed back, trees kept; the same graph still counts exactly, and so does an
    # ordinary histogram-on call
    res["rc_release"] = _lib.lib.halo_rx_release(0)
    res["claimed_after_release"] = _lib.lib.halo_rx_debug_hist_keys(0, 0, 0)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    res["replay_after_release_exact"] = bool(np.array_equal(hist.cpu().numpy().astype(np.int64), 5 * want))
    protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=netif, max_len_hint=64, out=out,
                                hist=hist)
    torch.cuda.synchronize()
    res["eager_after_release_exact"] = bool(np.array_equal(hist.cpu().numpy().astype(np.int64), 6 * want))
    res["claimed_end"] = _lib.lib.halo_rx_debug_hist_keys(0, 0, 0)
    del g
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
