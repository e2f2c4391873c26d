"""Phase timeline of the ring walk's guess kernel from a HALO_GUESS_TRACE build (tools only):
per tile the start, bytes in, tables built, guess chosen, walk done, records kept, in us.
The trace hooks were taken out of the product source in round 6; build the traced library from
the last revision that had them:
    tools/exp/build_rev.sh 9391269 gtrace -DHALO_GUESS_TRACE=1
usage: python tools/exp/guess_trace.py tools/exp/libhalo_rx_gtrace.so [frames] [length]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from halo_amd import _lib  # noqa: E402
from halo_amd._lib import NetIf  # noqa: E402
from halo_amd.ring import RingBuffer  # noqa: E402


def main():
    lib = ctypes.CDLL(sys.argv[1])
    lib.halo_rx_ring_scan_device.argtypes = _lib.lib.halo_rx_ring_scan_device.argtypes
    lib.halo_rx_ring_scan_workspace.restype = ctypes.c_uint64
    lib.halo_rx_ring_scan_workspace.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    length = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    assert lib.halo_rx_init(0) == 0
    dev = torch.device("cuda:0")
    fr = bench.make_batches(dev, NetIf.make(), n=n, rotate=1, rank=0, length=length)[0]
    lay = fr["layout"]
    ring = RingBuffer(128 << 20)
    ring.write_batch(fr["bytes"].cpu().numpy(), lay["offsets_dw"].astype(np.uint64) * 4, lay["lens"])
    used = ring.head - ring.tail
    span = torch.from_numpy(ring.data[:used].copy()).to(dev)
    d_off = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    d_len = torch.empty(n, dtype=torch.int16, device=dev)
    info = torch.zeros(24, dtype=torch.uint8, device=dev)
    wsb = lib.halo_rx_ring_scan_workspace(used, 1514)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    nt = (used // 4 + 4095) // 4096
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        assert lib.halo_rx_ring_scan_device(span.data_ptr(), used, ring.size, 1514, 0, d_off.data_ptr(),
                                            d_len.data_ptr(), info.data_ptr(), ws.data_ptr(), wsb, stream) == 0
    torch.cuda.synchronize()
    tr = d_off.cpu().numpy().view(np.uint64)[: 8 * nt].reshape(nt, 8).astype(np.int64)[:, :6]
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0
    print("tiles", nt, "kernel span (first start -> last end) us", rel[:, 5].max())
    names = ["bytes in", "tables", "guess", "walk", "records+summary"]
    for k, nm in enumerate(names):
        d = rel[:, k + 1] - rel[:, k]
        print(f"{nm:16s} med {np.median(d):.2f}  p10 {np.percentile(d, 10):.2f}  p90 {np.percentile(d, 90):.2f} us")
    life = rel[:, 5] - rel[:, 0]
    print(f"tile lifetime    med {np.median(life):.2f}  p90 {np.percentile(life, 90):.2f} us")
    st = np.sort(rel[:, 0])
    print("starts: 10% / 50% / 90% / last", np.percentile(st, 10), np.percentile(st, 50), np.percentile(st, 90), st[-1])


if __name__ == "__main__":
    main()
