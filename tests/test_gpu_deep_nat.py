"""GPU: IcmpTtlDeepNat (engine/icmp_engine.go:55-86) — halo_tx_icmp_deep_nat_batch_device through
the C ABI against the committed fixtures (tests/gen_golden_deepnat.py, the Python restatement)
and the C oracle (ora_icmp_quote / ora_icmp_deep_nat), bit-exact: quote records, rewritten frames
and the applied flags; the quote records' NAT_WAN flow keys are NatGetFlowByWan's."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def dn():
    g = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(g, "deep_nat.json")))
    blob = np.fromfile(os.path.join(g, "deep_nat.bin"), dtype=np.uint8)
    expect = np.fromfile(os.path.join(g, "deep_nat_expect.bin"), dtype=np.uint8)
    return meta, blob, expect


def _run(dev, data, offs, lens, en, nat=None):
    import torch

    from halo_amd import protocol

    n = len(lens)
    d = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
    o = torch.from_numpy(np.ascontiguousarray(offs.astype(np.uint32)).view(np.int32)).to(dev)
    ln = torch.from_numpy(np.ascontiguousarray(lens.astype(np.uint16)).view(np.int16)).to(dev)
    q = torch.full((n, 32), 0xEE, dtype=torch.uint8, device=dev)
    a = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    nd = None if nat is None else torch.from_numpy(nat.view(np.uint8)).to(dev)
    protocol.icmp_ttl_deep_nat_batch(d, o, ln, nat=nd, check_sum_enable=bool(en), quote=q, applied=a)
    torch.cuda.synchronize()
    return d.cpu().numpy(), protocol.records(q), a.cpu().numpy()


def _arrays(meta, blob):
    fr = meta["frames"]
    offs = np.array([e["offset"] // 4 for e in fr], np.uint32)
    lens = np.array([e["len"] for e in fr], np.uint16)
    return blob.copy(), offs, lens


@pytest.mark.parametrize("en", [0, 1])
def test_quote_records_vs_oracle_and_fixtures(dev, dn, oracle_lib, en):
    meta, blob, _ = dn
    data, offs, lens = _arrays(meta, blob)
    out, q, a = _run(dev, data, offs, lens, en)
    assert np.array_equal(out, data), "frames must be untouched without NAT results"
    assert np.all(a == 0)
    for k, e in enumerate(meta["frames"]):
        f = blob[e["offset"]:e["offset"] + e["len"]].tobytes()
        want = oracle_lib.icmp_quote(f, en)
        assert q[k].tobytes() == want.tobytes(), e["name"]
        assert int(q[k]["status"]) == e["quote"][str(en)]["status"], e["name"]


@pytest.mark.parametrize("en", [0, 1])
@pytest.mark.parametrize("found", [0, 1])
def test_rewrite_vs_fixtures(dev, dn, en, found):
    from halo_amd._lib import DEEP_NAT_DTYPE

    meta, blob, expect = dn
    data, offs, lens = _arrays(meta, blob)
    nat = np.zeros(len(lens), DEEP_NAT_DTYPE)
    nat["lan_ip"], nat["lan_port"], nat["found"] = meta["lan_ip"], meta["lan_port"], found
    out, _, a = _run(dev, data, offs, lens, en, nat)
    k_ = f"{en}{found}"
    for k, e in enumerate(meta["frames"]):
        o, eo, L = e["offset"], e["expect_offset"][k_], e["len"]
        assert int(a[k]) == e["applied"][k_], e["name"]
        assert out[o:o + L].tobytes() == expect[eo:eo + L].tobytes(), e["name"]


def test_random_ttl_messages_vs_oracle(dev, oracle_lib):
    """20k time-exceeded frames quoting random UDP/TCP/ICMP packets at random quote lengths, a
    quarter corrupted by one bit, random NAT results: every frame and flag vs the oracle."""
    from halo_amd._lib import DEEP_NAT_DTYPE
    from oracle import ref_py as R

    rng = np.random.default_rng(0xD33F)
    frames = []
    for k in range(20_000):
        proto = int(rng.choice([1, 6, 17]))
        pl = bytes(rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8))
        src, dst = bytes(rng.integers(0, 256, 4, dtype=np.uint8)), bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        if proto == 17:
            seg = R.build_udp(pl, int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), src, dst)
        elif proto == 6:
            seg = R.build_tcp(pl, int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), src, dst, 1, 2, 0x10)
        else:
            seg = R.build_icmp(pl, 8, bytes(rng.integers(0, 256, 2, dtype=np.uint8)), 5)
        inner = R.build_ipv4(seg, proto, src, dst)
        q = inner[:int(rng.integers(20, len(inner) + 1))]
        msg = R.build_icmp(q, 11, b"\0\0", 0)
        f = bytearray(R.build_eth(R.build_ipv4(msg, 1, bytes([192, 0, 2, 1]), src), bytes(6), bytes(6), 0x0800))
        if rng.integers(0, 8) == 0:
            f += bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8))  # padding
        if rng.integers(0, 4) == 0:
            bit = int(rng.integers(14 * 8, len(f) * 8))
            f[bit >> 3] ^= 1 << (bit & 7)
        frames.append(bytes(f))
    lens = np.array([len(f) for f in frames], np.uint16)
    sizes = (lens.astype(np.int64) + 3) & ~3
    offs = np.zeros(len(frames), np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    data = np.zeros(int(sizes.sum()) + 16, np.uint8)
    for o, f in zip(offs, frames):
        data[o:o + len(f)] = np.frombuffer(f, np.uint8)
    nat = np.zeros(len(frames), DEEP_NAT_DTYPE)
    nat["lan_ip"] = rng.integers(0, 1 << 32, len(frames), dtype=np.uint64).astype(np.uint32)
    nat["lan_port"] = rng.integers(0, 1 << 16, len(frames))
    nat["found"] = rng.integers(0, 8, len(frames)) != 0
    for en in (0, 1):
        out, q, a = _run(dev, data, offs // 4, lens, en, nat)
        n_applied = 0
        for k, f in enumerate(frames):
            want_q = oracle_lib.icmp_quote(f, en)
            assert q[k].tobytes() == want_q.tobytes(), k
            wf, ok = oracle_lib.icmp_deep_nat(f, int(nat["lan_ip"][k]), int(nat["lan_port"][k]), bool(nat["found"][k]), en)
            assert int(a[k]) == int(ok), k
            assert out[offs[k]:offs[k] + len(f)].tobytes() == wf, k
            n_applied += ok
        assert n_applied > 10_000


def test_quote_flow_key_is_nat_get_flow_by_wan(dev, dn, oracle_lib):
    """hashcode(NAT_WAN) of the GPU quote records == the oracle's hash of a record built from the
    Python restatement's NatGetFlowByWan arguments (remote ip/port, wan ip/port, proto)."""
    import torch

    from halo_amd import hashcode
    from halo_amd._lib import FLOW_NAT_WAN, NAT_SYMMETRIC

    meta, blob, _ = dn
    data, offs, lens = _arrays(meta, blob)
    _, q, _ = _run(dev, data, offs, lens, 1)
    ok = [k for k, e in enumerate(meta["frames"]) if e["quote"]["1"]["args"]]
    recs = torch.from_numpy(q[ok].view(np.uint8).reshape(-1, 32).copy()).to(dev)
    h, _ = hashcode.flow_hash(recs, FLOW_NAT_WAN, NAT_SYMMETRIC)
    want = np.zeros(len(ok), oracle_lib.RESULT_DTYPE)
    for j, k in enumerate(ok):
        proto, remote, rport, wan, wport = meta["frames"][k]["quote"]["1"]["args"]
        want[j]["ip_proto"], want[j]["src_ip"], want[j]["sport"] = proto, remote, rport
        want[j]["dst_ip"], want[j]["dport"] = wan, wport
    wh, _ = oracle_lib.flow_hash_batch(want, FLOW_NAT_WAN, NAT_SYMMETRIC)
    assert np.array_equal(h.cpu().numpy().view(np.uint64), wh)
