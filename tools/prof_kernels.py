#!/usr/bin/env python3
"""Launch each hot-path workload a fixed number of times for rocprofv3 (kernel trace / PMC).

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/prof_kernels.py
    rocprofv3 --pmc FETCH_SIZE -d OUT -o run -- python3 tools/prof_kernels.py

Workloads run in a fixed order, each with its own kernel variant, so per-dispatch rows can be
attributed by order (see tools/pmc_summary.py).
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name, synth kwargs, frames, rotating batches, launches, strided length (0 = ragged), flags, hint
WORKLOADS = [
    ("config2", dict(length=64), 1 << 20, 8, 20, 0, 1, 64),
    ("1500B_udp_1M", dict(length=1500), 1 << 20, 2, 10, 0, 1 | 0x8, 1500),  # HALO_RX_UNIFORM_LEN, as bench.py
    ("config4_shard_16M_64B", dict(length=64), 16 << 20, 2, 6, 0, 1, 64),
    ("config3_imix_16M", dict(size_mode=1, proto_mode=3), 16 << 20, 1, 5, 0, 1, 1500),
    ("config5_jumbo_9000B_tcp_4M_ext", dict(length=9000, proto_mode=1, strided=True), 4 << 20, 1, 3, 9000, 3, 0),
    # PacketHandle's LoChan drain (§8a row a12): 1M x 50 B TxIpv4 loopback copies, HALO_RX_L3_START
    ("lo_drain_1M_50B", dict(length=64), 1 << 20, 1, 20, 0, 1 | 0x10, 64),
    # config 2's batches handed over 8 per call (halo_rx_parse_batches_device: one launch per 8M frames)
    ("config2_batch_stream", dict(length=64), 1 << 20, 8, 10, 0, 1, 64),
    # forward / transmit rewrite (§8f row f2): bench.TX_BENCH_STEPS on the config 2 frames
    ("tx_config2", dict(length=64), 1 << 20, 8, 20, 0, 1, 64),
    # flow-key hashing (§8f row f3): NatWanFlowHash + bucket on the parsed config 2 records
    ("flow_hash_config2", dict(length=64), 1 << 20, 1, 20, 0, 1, 64),
    ("flow_hash_config2_compact", dict(length=64), 1 << 20, 1, 20, 0, 1, 64),
    # halo's packet ring (§8f row f1): the record walk over 1M 64 B records (68 MB span)
    ("ring_scan_1M_64B", dict(length=64), 1 << 20, 1, 20, 0, 1, 64),
    ("ring_scan_imix_256k", dict(size_mode=1, proto_mode=3), 1 << 18, 1, 20, 0, 1, 1500),
    # transmit construction (§8f row f2, Build*): bench.tx_build_secondary's two workloads
    ("tx_build_udp_1M_64B", dict(length=64), 1 << 20, 1, 20, 0, 1, 22),
    ("tx_build_udp_256k_1514B", dict(length=64), 1 << 18, 1, 10, 0, 1, 1472),
    # the size-matched probes of the two tx_build lines (every stream_rw_kernel shape, 10 launches
    # each): the same bytes in and out with no build work, for counters next to the build's
    ("probe_tx_build_64B", dict(length=64), 1 << 20, 1, 10, 0, 1, 22),
    ("probe_tx_build_1514B", dict(length=64), 1 << 18, 1, 10, 0, 1, 1472),
]


def main():
    import torch

    import bench
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    only = sys.argv[1:]
    _lib.check("init", _lib.lib.halo_rx_init(0))
    dev = torch.device("cuda:0")
    netif = NetIf.make()
    for name, kw, n, rot, launches, slen, flags, hint in WORKLOADS:
        if only and name not in only:
            continue
        bs = bench.make_batches(dev, netif, n=n, rotate=rot, rank=0, **kw)
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        ops = None
        if name.startswith("tx_"):
            import numpy as np

            ops = torch.from_numpy(bench.tx_ops_for(n).view(np.uint8)).to(dev)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream().cuda_stream
        if name.startswith("ring_scan"):
            import numpy as np

            from halo_amd.ring import RingBuffer

            fr = bs[0]
            lay = fr["layout"]
            ring = RingBuffer(128 << 20)
            ring.write_batch(fr["bytes"].cpu().numpy(), lay["offsets_dw"].astype(np.uint64) * 4, lay["lens"])
            used = ring.head - ring.tail
            span = torch.from_numpy(ring.data[:used].copy()).to(dev)
            d_off = torch.empty(n, dtype=torch.int32, device=dev)
            d_len = torch.empty(n, dtype=torch.int16, device=dev)
            info = torch.zeros(24, dtype=torch.uint8, device=dev)
            wsb = _lib.lib.halo_rx_ring_scan_workspace(used, 1514)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            for i in range(launches):
                _lib.check("ring_scan", _lib.lib.halo_rx_ring_scan_device(
                    span.data_ptr(), used, ring.size, 1514, 0, d_off.data_ptr(), d_len.data_ptr(), info.data_ptr(),
                    ws.data_ptr(), wsb, stream))
            torch.cuda.synchronize()
            print(f"{name}: {launches} walks of {used} bytes", flush=True)
            del bs, out, span, ws
            torch.cuda.empty_cache()
            continue
        if name.startswith("lo_drain"):
            from halo_amd import protocol

            fb = bs[0]["bytes"][:n * 64].view(n, 64)  # uniform 64 B frames, packed
            pk = torch.zeros((n, 52), dtype=torch.uint8, device=dev)
            pk[:, :50] = fb[:, 14:64]  # their IPv4 packets: what Ipv4RouteForward puts in a LoChan,
            offs = torch.arange(n, dtype=torch.int32, device=dev) * 13  # packed at 4-byte aligned starts
            fl = torch.full((n,), 50, dtype=torch.int16, device=dev)
            torch.cuda.synchronize()
            for i in range(launches):
                protocol.parse_ipv4_packets_batch(pk.reshape(-1), offs, fl, netif=netif, max_len_hint=64, out=out)
            torch.cuda.synchronize()
            print(f"{name}: {launches} launches of {n}", flush=True)
            del bs, out, pk
            torch.cuda.empty_cache()
            continue
        if name.startswith("probe_tx_build"):
            del bs, out
            plen = hint
            stride = 64 if plen <= 22 else 1516
            d = bench.Dist()
            k = bench.size_matched_probe(dev, n * (40 + plen), n * (stride + 3), d, nbuf=1, steps=launches)
            print(f"{name}: {launches} launches per shape, {bench.LAST_PROBE_SHAPES} (best {k:.5f} ms)", flush=True)
            torch.cuda.empty_cache()
            continue
        if name.startswith("tx_build"):
            import numpy as np

            from halo_amd import protocol
            from halo_amd._lib import BUILD_DESC_DTYPE

            del bs
            plen = hint
            stride = 64 if plen <= 22 else 1516
            desc = np.zeros(n, BUILD_DESC_DTYPE)
            desc["payload_off"] = np.arange(n, dtype=np.uint64) * plen
            desc["payload_len"], desc["proto"], desc["src_port"], desc["dst_port"] = plen, 17, 1234, 5678
            desc["src_ip"], desc["dst_ip"] = netif.ip, 0x0A000001
            desc_d = torch.from_numpy(desc.view(np.uint8)).to(dev)
            pay = torch.randint(0, 256, (n * plen,), dtype=torch.uint8, device=dev)
            b = protocol.TxBuilder(n, device=dev)
            frames = torch.empty((n, stride), dtype=torch.uint8, device=dev)
            fl = torch.empty(n, dtype=torch.int16, device=dev)
            for i in range(launches):
                b.build(desc_d, pay, netif=netif, out_stride=stride, frames=frames, lens=fl, max_payload_hint=plen)
            torch.cuda.synchronize()
            print(f"{name}: {launches} launches of {n}", flush=True)
            del out, frames, pay, desc_d, b
            torch.cuda.empty_cache()
            continue
        if name == "config2_batch_stream":
            from halo_amd import protocol

            outs = [torch.empty((n, 32), dtype=torch.uint8, device=dev) for _ in bs]
            for i in range(launches):
                protocol.parse_frames_batches([(b["bytes"], b["offsets_dw"], b["lens"], o) for b, o in zip(bs, outs)],
                                              netif=netif, max_len_hint=64)
            torch.cuda.synchronize()
            print(f"{name}: {launches} launches of {len(bs)} x {n} frames", flush=True)
            del bs, out, outs
            torch.cuda.empty_cache()
            continue
        if name.startswith("flow_hash"):
            from halo_amd import protocol

            fr = bs[0]
            compact = name.endswith("_compact")
            if compact:
                out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
            _lib.check("parse", _lib.lib.halo_rx_parse_batch_device(
                fr["bytes"].data_ptr(), fr["offsets_dw"].data_ptr(), fr["lens"].data_ptr(), n,
                1 | (_lib.HALO_RX_RECORD_COMPACT if compact else 0), netif, 64, out.data_ptr(), None, stream))
            h = torch.empty(n, dtype=torch.int64, device=dev)
            bk = torch.empty(n, dtype=torch.int32, device=dev)
            fn = _lib.lib.halo_flow_hash_compact_device if compact else _lib.lib.halo_flow_hash_device
            torch.cuda.synchronize()
            for i in range(launches):
                _lib.check("flow", fn(out.data_ptr(), n, 1, 0, h.data_ptr(), 1 << 20, bk.data_ptr(), stream))
            torch.cuda.synchronize()
            print(f"{name}: {launches} launches of {n} records", flush=True)
            del bs, out
            torch.cuda.empty_cache()
            continue
        for i in range(launches):
            fr = bs[i % len(bs)]
            if ops is not None:
                rc = _lib.lib.halo_tx_fixup_batch_device(fr["bytes"].data_ptr(), fr["offsets_dw"].data_ptr(),
                                                         fr["lens"].data_ptr(), n, ops.data_ptr(), flags, hint,
                                                         out.data_ptr(), stream)
            elif slen:
                rc = _lib.lib.halo_rx_parse_strided_device(fr["bytes"].data_ptr(), slen, None, slen, n, flags, netif,
                                                           out.data_ptr(), None, stream)
            else:
                rc = _lib.lib.halo_rx_parse_batch_device(fr["bytes"].data_ptr(), fr["offsets_dw"].data_ptr(),
                                                         fr["lens"].data_ptr(), n, flags, netif, hint,
                                                         out.data_ptr(), None, stream)
            _lib.check("parse", rc)
        torch.cuda.synchronize()
        print(f"{name}: {launches} launches of {n} frames", flush=True)
        del bs, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
