"""GPU: PacketHandle's LoChan drain (engine/engine.go:353-381) —
halo_rx_parse_batch_device with HALO_RX_L3_START (buffers that start at their IPv4 header),
through the C ABI, bit-exact against the committed fixtures (tests/gen_golden_lo.py) and the
C oracle; the host path and the engine mirror's drain; TxIpv4 loopback copies built on the GPU
(halo_tx_build_batch_device, HALO_TX_BUILD_LOOPBACK) parsed back through the drain."""
from __future__ import annotations

import os

import numpy as np
import pytest

from tests.helpers import assert_records_equal, expected_records, golden_arrays, lo_golden, strip_ethernet

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L3 = 0x10


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def lo():
    return lo_golden(ROOT)


def _to_dev(a, dev, dtype=None):
    import torch

    if dtype is not None:
        a = a.view(dtype)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _parse_l3(dev, data, offs, lens, flags, hint=0, variant=0):
    import torch

    from halo_amd import protocol
    from halo_amd._lib import NetIf

    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_ipv4_packets_batch(_to_dev(data, dev), _to_dev(offs.astype(np.uint32), dev, np.int32),
                                            _to_dev(lens.astype(np.uint16), dev, np.int16), netif=NetIf.make(),
                                            check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2),
                                            max_len_hint=hint, variant=variant, hist=hist)
    torch.cuda.synchronize()
    return protocol.records(out), hist.cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("variant", [1, 4, 8, 16, -1, -2, 0])
def test_lo_fixtures_every_variant(dev, lo, flags, variant):
    from halo_amd._lib import RESULT_DTYPE

    meta, blob = lo
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    got, hist = _parse_l3(dev, data, offs, lens, flags, variant=variant)
    want = expected_records(meta, flags, RESULT_DTYPE, key="packets")
    assert_records_equal(got, want, names, f"GPU L3 flags={flags} G={variant}")
    assert np.array_equal(hist, np.bincount(want["status"], minlength=14))


def test_lo_fixtures_drain_actions(dev, lo):
    """Records from the GPU -> halo_rx_dispatch_loopback == the restated drain (engine_lo)."""
    from halo_amd import ACTION_NAMES
    from halo_amd._lib import NetIf
    from halo_amd.engine import dispatch_loopback

    meta, blob = lo
    data, offs, lens, _ = golden_arrays(meta, blob, key="packets")
    for flags in (0, 1, 3):
        got, _ = _parse_l3(dev, data, offs, lens, flags)
        acts = [ACTION_NAMES[a] for a in dispatch_loopback(got, NetIf.make())]
        assert acts == [e["action"][str(flags)] for e in meta["packets"]]


@pytest.mark.parametrize("variant", [0, 1, 4, -1, -2])
def test_lo_compact_records(dev, lo, variant):
    import torch

    from halo_amd import _lib
    from halo_amd._lib import RECORD16_DTYPE, RESULT_DTYPE, NetIf, compact_of

    meta, blob = lo
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    out = torch.full((len(lens), 16), 0xEE, dtype=torch.uint8, device=dev)
    d, o, ln = _to_dev(data, dev), _to_dev(offs, dev, np.int32), _to_dev(lens, dev, np.int16)
    rc = _lib.lib.halo_rx_parse_batch_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens),
                                             1 | L3 | _lib.HALO_RX_RECORD_COMPACT | _lib.variant_flags(variant),
                                             NetIf.make(), 0, out.data_ptr(), None,
                                             torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(-1).view(RECORD16_DTYPE)
    want = compact_of(expected_records(meta, 1, RESULT_DTYPE, key="packets"))
    bad = np.nonzero(np.any(got.view(np.uint8).reshape(-1, 16) != want.view(np.uint8).reshape(-1, 16), axis=1))[0]
    assert bad.size == 0, [names[i] for i in bad[:5]]


@pytest.fixture(scope="module")
def forwarded(dev, oracle_lib):
    """200k synthetic IMIX frames (1/8 mutated) with their Ethernet header stripped — the copies
    Ipv4RouteForward puts in another NetIf's LoChan (engine/ipv4_engine.go:195-200) — and the
    oracle's records for them."""
    import torch

    from halo_amd import synth
    from halo_amd._lib import NetIf

    n = 200_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=3, first_index=31_000_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    torch.cuda.synchronize()
    data, offs, lens = strip_ethernet(fr["bytes"].cpu().numpy(), lay["offsets_dw"], lay["lens"])
    del fr
    want, whist = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), 1 | L3, offsets_dw=offs, threads=16)
    return data, offs, lens, want, whist


@pytest.mark.parametrize("variant", [0, 1, 4, 8, -1, -2])
def test_lo_forwarded_imix_vs_oracle(dev, forwarded, variant):
    """Every record and the histogram vs the oracle, under each kernel variant."""
    data, offs, lens, want, whist = forwarded
    got, hist = _parse_l3(dev, data, offs, lens, 1, hint=1500, variant=variant)
    assert_records_equal(got, want, None, f"forwarded IMIX L3 G={variant}")
    assert np.array_equal(hist, whist.astype(np.int64))
    st = want["status"]
    assert (st == 0).sum() > len(lens) * 0.8 and (st == 13).sum() > 0  # mostly clean, bit flips caught


def test_lo_host_path_and_engine_drain(dev, lo, oracle_lib):
    """halo_rx_parse_batch_host with HALO_RX_L3_START, and NetIf.lo_drain delivering the local
    UDP / TCP packets of the LoChan to their handlers with packet-relative payloads."""
    from halo_amd import ACTION_NAMES
    from halo_amd._lib import RESULT_DTYPE, NetIf as NetIfAbi
    from halo_amd.engine import HostBatcher, NetIf

    meta, blob = lo
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    hb = HostBatcher(0, chunk_frames=50, chunk_bytes=65536)
    try:
        for flags in (1, 3):
            hist = np.zeros(14, np.uint32)
            got = hb.parse(data, offs.astype(np.uint64) * 4, lens, NetIfAbi.make(), flags | L3, hist)
            want = expected_records(meta, flags, RESULT_DTYPE, key="packets")
            assert_records_equal(got, want, names, f"host path L3 flags={flags}")
            assert np.array_equal(hist, np.bincount(want["status"], minlength=14))
    finally:
        hb.close()

    pkts = [bytes(blob[e["offset"]:e["offset"] + e["len"]]) for e in meta["packets"]]
    got_udp, got_tcp = [], []
    netif = NetIf("eth0", "AA:AA:AA:AA:AA:AA", "192.168.100.100", lambda: None)
    netif.RecvUdp(53, lambda s, p: got_udp.append((s.RemoteIp, s.RemotePort, bytes(p))))
    netif.RecvTcp(22, lambda s, p, seq, ack, fl: got_tcp.append((s.RemotePort, bytes(p), seq, ack, fl)))
    netif.LoChan.extend(pkts)
    res, actions = netif.packet_handle_batch()  # no external frames: the drain still runs
    assert len(res) == 0
    res, actions = netif.lo_drain()
    assert len(actions) == 0 and not netif.LoChan  # drained by packet_handle_batch already
    counts = dict(zip(ACTION_NAMES, netif.action_counts))
    want = [e["action"]["1"] for e in meta["packets"]]
    for a in set(want):
        assert counts[a] == want.count(a), a
    assert (0xC0A86464, 5353, b"loopback udp") in got_udp
    # TCP payload starts at headerLen = 5 bytes into the segment (tcp.go:49,68)
    assert any(p[15:] == b"loopback tcp" and seq == 7 and ack == 9 for _, p, seq, ack, _ in got_tcp)


def test_tx_build_loopback_round_trip(dev):
    """TxIpv4's loopback copies built on the GPU (HALO_TX_BUILD_LOOPBACK, the NetIf's own
    address) drain as local packets with the descriptor's ports and payload."""
    import torch

    from halo_amd import ACTION_NAMES, protocol
    from halo_amd._lib import BUILD_DESC_DTYPE, NetIf
    from halo_amd.engine import dispatch_loopback

    rng = np.random.default_rng(0x10)
    n = 4096
    own = NetIf.make().ip
    plen = rng.integers(0, 1400, n).astype(np.uint16)
    poff = np.zeros(n, np.uint64)
    poff[1:] = np.cumsum(plen[:-1].astype(np.uint64))
    payload = rng.integers(0, 256, int(plen.sum()) + 1, dtype=np.uint8)
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["payload_off"], desc["payload_len"] = poff, plen
    desc["proto"] = rng.choice(np.array([1, 6, 17], np.uint8), n)
    desc["aux"] = np.where(desc["proto"] == 1, 8, 0x18)
    desc["src_port"] = rng.integers(1, 65536, n)
    desc["dst_port"] = rng.integers(1, 65536, n)
    desc["src_ip"] = desc["dst_ip"] = own
    desc["mode"] = protocol.TX_BUILD_LOOPBACK
    b = protocol.TxBuilder(n, device=dev, ip_id=100)
    frames, flen, res = b.build(_to_dev(desc.view(np.uint8), dev), _to_dev(payload, dev), netif=NetIf.make(),
                                out_stride=1516)
    torch.cuda.synchronize()
    flen_h = flen.cpu().numpy().view(np.uint16)
    ok = res.cpu().numpy() == 0
    assert ok.sum() > 0.9 * n
    idx = np.nonzero(ok)[0]
    offs = (idx * (1516 // 4)).astype(np.uint32)
    out = protocol.parse_ipv4_packets_batch(frames.reshape(-1), _to_dev(offs, dev, np.int32),
                                            _to_dev(flen_h[idx], dev, np.int16), netif=NetIf.make(),
                                            max_len_hint=1500)
    torch.cuda.synchronize()
    recs = protocol.records(out)
    acts = [ACTION_NAMES[a] for a in dispatch_loopback(recs, NetIf.make())]
    want = ["LOCAL_ICMP" if p == 1 else "LOCAL_TCP" if p == 6 else "LOCAL_UDP" for p in desc["proto"][idx]]
    assert acts == want
    host = frames.cpu().numpy()
    for k in rng.choice(len(idx), 200, replace=False):
        i = idx[k]
        r = recs[k]
        assert int(r["sport"]) == int(desc["src_port"][i])  # ICMP: the echo id (NatGetSrcDstPort)
        if desc["proto"][i] != 6:  # UDP / ICMP payload at 28; TCP's starts inside its header (tcp.go:68)
            got = host[i, int(r["payload_off"]):int(r["payload_off"]) + int(r["payload_len"])]
            want_p = payload[int(poff[i]):int(poff[i]) + int(plen[i])]
            assert np.array_equal(got, want_p), i
