"""Host path timing sweep (tools only): halo_rx_parse_batch_host on registered batches with
zero-copy on / off over several chunk sizes, to see where the time of a host batch goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import contextlib  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from halo_amd import _lib  # noqa: E402
from halo_amd._lib import NetIf  # noqa: E402
from halo_amd.engine import HostBatcher  # noqa: E402


def main():
    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    netif = NetIf.make()
    for name, kw, n in [("64B_1M", dict(length=64), 1 << 20), ("imix_4M", dict(size_mode=1, proto_mode=3), 4 << 20)]:
        fr = bench.make_batches(dev, netif, n=n, rotate=1, rank=0, **kw)[0]
        lay = fr["layout"]

        def own(a):
            b = _lib.host_array(a.shape, a.dtype)
            b[...] = a
            return b

        host = own(fr["bytes"].cpu().numpy())
        offs = own(lay["offsets_dw"].astype(np.uint64) * 4)
        lens = own(np.ascontiguousarray(lay["lens"]))
        out = _lib.host_array(n, _lib.RESULT_DTYPE)
        out.view(np.uint8)[:] = 0
        t0 = time.perf_counter()
        for _ in range(5):
            x = ((offs - offs[0]) >> 2).astype(np.uint32)
            y = lens.copy()
        print(f"{name}: numpy offset conversion {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)
        del x, y
        with contextlib.ExitStack() as regs:
            for a in (host, offs, lens, out):
                regs.enter_context(_lib.registered(a))
            for chunk in (1 << 16, 1 << 18, 1 << 20, 1 << 22):
                if chunk > n:
                    continue
                hb = HostBatcher(0, chunk_frames=chunk)
                for zc in (True, False):
                    hb.set_zero_copy(zc)
                    hb.parse(host, offs, lens, netif, 1, out=out)
                    t0 = time.perf_counter()
                    for _ in range(5):
                        hb.parse(host, offs, lens, netif, 1, out=out)
                    el = (time.perf_counter() - t0) / 5
                    print(f"{name}: chunk {chunk:8d} zero_copy={int(zc)}: {el * 1e3:8.3f} ms  {n / el / 1e6:7.1f} Mpps",
                          flush=True)
                hb.close()
        del fr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
