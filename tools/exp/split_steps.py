"""Tools only: one 1M-frame batch per step split over 1, 2, 4 streams (halo_bench_split_steps), 16
rotating batches as the headline; per-step time and a record check against one launch."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    import torch

    from halo_amd import _lib, protocol
    from halo_amd._lib import NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    netif = NetIf.make()
    d = bench.Dist()
    L = bench.bench_lib()
    vp, i32, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32
    L.halo_bench_split_steps.restype = i32
    L.halo_bench_split_steps.argtypes = [i32, vp, vp, vp, u32, u32, vp, u32, vp, i32, i32, i32, vp,
                                         ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
    n = 1 << 20
    batches, _ = bench.shard_batches(dev, netif, rank=0, n=n, rotate=16)
    arr = lambda xs: (ctypes.c_void_p * len(xs))(*xs)  # noqa: E731
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    ref = torch.empty_like(out)
    res = {}
    for rnd in range(2):
        for parts in (1, 2, 4):
            w, k = bench.time_native(L.halo_bench_split_steps, len(batches), arr([b["bytes"].data_ptr() for b in batches]),
                                     arr([b["offsets_dw"].data_ptr() for b in batches]),
                                     arr([b["lens"].data_ptr() for b in batches]), n, 1, ctypes.addressof(netif), 64,
                                     out.data_ptr(), parts, steps=1000, warmup=50, d=d)
            last = batches[999 % 16]
            protocol.parse_frames_batch(last["bytes"], last["offsets_dw"], last["lens"], netif=netif, max_len_hint=64,
                                        out=ref)
            res[f"parts{parts}_r{rnd}"] = {"us_per_step": round(k * 1e3, 2), "wall_us_per_step": round(w / 1000 * 1e6, 2),
                                           "ok": bool(torch.equal(ref, out))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
