"""GPU: the single-frame Parse* wrappers (halo_amd.protocol.ParseEthFrm / ParseIpv4Pkt /
ParseUdpPkt / ParseTcpPkt / ParseIcmpPkt) return exactly the reference functions' tuples, error
strings included, on every golden frame, every IPv4 payload and every L4 segment in it (each
segment also through the two other L4 parsers), length edges and random corruptions — checked
against the independent Python restatement (oracle/ref_py.py) with CheckSumEnable on and off."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def frames():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    g = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(g, "frames.json")))
    blob = np.fromfile(os.path.join(g, "frames.bin"), dtype=np.uint8)
    return [blob[e["offset"]:e["offset"] + e["len"]].tobytes() for e in meta["frames"]]


def _text(status, proto):
    from halo_amd import protocol
    from halo_amd._lib import STATUS

    return None if status is None else protocol.error_text(STATUS[status], proto)


@pytest.fixture(params=[True, False], ids=["csum", "nocsum"])
def csum(request):
    from halo_amd import protocol

    old = protocol.CheckSumEnable
    protocol.CheckSumEnable = request.param
    yield request.param
    protocol.CheckSumEnable = old


def test_parse_eth_and_ipv4(frames, csum):
    from halo_amd import protocol
    from oracle import ref_py as R

    c = R.Cfg(csum)
    n_ip = 0
    for f in frames:
        p, d, s, t, err = R.parse_eth_frm(f, c)
        assert protocol.ParseEthFrm(f) == (p, d, s, t, _text(err, None)), f[:16].hex()
        if err or len(f) < 14:
            continue
        pkt = f[14:]
        pay, proto, src, dst, _tl, err = R.parse_ipv4_pkt(pkt, c)
        if err in ("IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN"):
            with pytest.raises(protocol.ReferencePanic):
                protocol.ParseIpv4Pkt(pkt)
            continue
        assert protocol.ParseIpv4Pkt(pkt) == (pay, proto, src, dst, _text(err, None)), pkt[:20].hex()
        n_ip += 1
    assert n_ip > 100


def _segments(frames):
    """(segment, src, dst) of every IPv4 golden frame that passes ParseIpv4Pkt, plus length edges
    and corrupted copies."""
    from oracle import ref_py as R

    segs = []
    c = R.Cfg(False)
    for f in frames:
        if len(f) < 34:
            continue
        pay, proto, src, dst, _tl, err = R.parse_ipv4_pkt(f[14:], c)
        if err is None:
            segs.append((pay, src, dst))
    rng = np.random.default_rng(0x53474D)
    src, dst = bytes([10, 0, 0, 1]), bytes([192, 168, 100, 100])
    for L in list(range(0, 30)) + [1479, 1480, 1481, 1500]:
        segs.append((rng.integers(0, 256, L, dtype=np.uint8).tobytes(), src, dst))
    for k in range(len(segs) // 2):
        s, a, b = segs[k]
        if s:
            m = bytearray(s)
            m[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
            segs.append((bytes(m), a, b))
    return segs


def test_parse_l4(frames, csum):
    from halo_amd import protocol
    from oracle import ref_py as R

    c = R.Cfg(csum)
    ok = {6: 0, 17: 0, 1: 0}
    for seg, src, dst in _segments(frames):
        p, sp, dp, err = R.parse_udp_pkt(seg, src, dst, c)
        assert protocol.ParseUdpPkt(seg, src, dst) == (p, sp, dp, _text(err, 17)), seg[:8].hex()
        p, sp, dp, sq, ak, fl, err = R.parse_tcp_pkt(seg, src, dst, c)
        assert protocol.ParseTcpPkt(seg, src, dst) == (p, sp, dp, sq, ak, fl, _text(err, 6)), seg[:20].hex()
        p, ty, ident, sq, err = R.parse_icmp_pkt(seg, c)
        if err is None:
            ty = int(ty)
        assert protocol.ParseIcmpPkt(seg) == (p, ty, ident, sq, _text(err, 1)), seg[:8].hex()
        for proto, e in ((17, R.parse_udp_pkt(seg, src, dst, c)[-1]), (6, R.parse_tcp_pkt(seg, src, dst, c)[-1]),
                         (1, err)):
            ok[proto] += e is None
    assert all(v > 20 for v in ok.values()), ok
