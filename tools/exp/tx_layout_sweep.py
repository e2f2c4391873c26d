#!/usr/bin/env python3
"""The 1514 B transmit build against its layout (tools only): for each output slot stride, payload
pitch and payload start shift, the build kernel (halo_tx_build_batch_device) and the layout-matched
probe (tools/bench_loop.hip tx_layout_probe_kernel: the same bytes at the same addresses, no build
work), beside the aligned size-matched probe. Says how much of the gap to the size-matched probe is
the layout (slots not a multiple of 64 B, payload bytes 2 B off a dword at the UDP header seam)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    import bench
    from halo_amd import _lib, protocol
    from halo_amd._lib import BUILD_DESC_DTYPE, NetIf

    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda", 0)
    d = bench.Dist()
    n, plen = 1 << 18, 1472
    flen = 14 + 20 + 8 + plen
    netif = NetIf.make(mac="02:00:00:00:00:01", ip="192.168.100.1")
    size_ms = bench.size_matched_probe(dev, n * (40 + plen), n * (1516 + 3), d, nbuf=1, steps=20)
    print(json.dumps({"size_matched_probe_ms": round(size_ms, 5)}), flush=True)
    # (stride, pitch, shift): shift 10 puts payload byte 0 at 42 mod 16, so the build's 16-byte
    # chunks are 16-byte aligned in the payload too
    for stride, pitch, shift in [(1516, 1472, 0), (1536, 1472, 0), (2048, 1472, 0), (1516, 1472, 10),
                                 (1536, 1472, 10), (1536, 1536, 10), (2048, 2048, 10)]:
        desc = np.zeros(n, BUILD_DESC_DTYPE)
        desc["payload_off"] = np.arange(n, dtype=np.uint64) * pitch + shift
        desc["payload_len"] = plen
        desc["proto"] = 17
        rng = np.random.default_rng(0x4255)
        desc["src_port"] = rng.integers(1, 1 << 16, n)
        desc["dst_port"] = rng.integers(1, 1 << 16, n)
        desc["src_ip"] = netif.ip
        desc["dst_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        desc["dst_mac"] = np.frombuffer(bytes.fromhex("aaaaaaaaaaaa"), np.uint8)
        desc_d = torch.from_numpy(desc.view(np.uint8)).to(dev)
        pay_d = torch.randint(0, 256, (n * pitch + shift + 64,), dtype=torch.uint8, device=dev)
        b = protocol.TxBuilder(n, device=dev, ip_id=1)
        frames = torch.empty((n, stride), dtype=torch.uint8, device=dev)
        lens = torch.empty(n, dtype=torch.int16, device=dev)
        rcode = torch.empty(n, dtype=torch.uint8, device=dev)
        _, k = bench.time_torch_loop(lambda: b.build(desc_d, pay_d, netif=netif, out_stride=stride, frames=frames,
                                                     lens=lens, result=rcode, max_payload_hint=plen), 40, 5, d)
        assert int((rcode != 0).sum()) == 0 and int((lens != flen).sum()) == 0
        sink = torch.zeros(16, dtype=torch.int32, device=dev)
        _, kl = bench.time_native(bench.bench_lib().halo_bench_tx_layout_probe, desc_d.data_ptr(),
                                  pay_d.data_ptr() + shift, plen, pitch, frames.data_ptr(), stride, flen,
                                  lens.data_ptr(), rcode.data_ptr(), n, sink.data_ptr(), 0, steps=40, warmup=5, d=d)
        _, ki = bench.time_native(bench.bench_lib().halo_bench_tx_layout_probe, desc_d.data_ptr(),
                                  pay_d.data_ptr() + shift, plen, pitch, frames.data_ptr(), stride, flen,
                                  lens.data_ptr(), rcode.data_ptr(), n, sink.data_ptr(), 1, steps=40, warmup=5, d=d)
        print(json.dumps({"stride": stride, "pitch": pitch, "shift": shift, "build_ms": round(k, 5),
                          "layout_probe_ms": round(kl, 5), "interleaved_probe_ms": round(ki, 5), "build_vs_layout": round(kl / k, 4),
                          "build_vs_size_matched": round(size_ms / k, 4)}), flush=True)
        del desc_d, pay_d, frames, lens, rcode, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
