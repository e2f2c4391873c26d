"""GPU: the Build* half of SURVEY.md §8f row f2 — halo_tx_build_batch_device against the committed
fixtures (tests/gen_golden_build.py: the Python restatement of BuildUdp/Tcp/IcmpPkt ->
BuildIpv4Pkt -> BuildEthFrm / TxIpv4's LoChan copy) and the C oracle (ora_tx_build_batch),
bit-exact: frame bytes, lengths, result codes and the iphId sequence. Round trip: frames the
GPU builds parse clean on the GPU receive path with the descriptor's fields."""
from __future__ import annotations

import os

import numpy as np
import pytest

from tests.helpers import assert_build_equal, build_golden

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _netif(mac_hex: str):
    from halo_amd._lib import NetIf

    return NetIf.make(mac=":".join(mac_hex[i:i + 2] for i in range(0, 12, 2)), ip="192.168.100.1")


def _run(dev, desc, payload, netif, stride, flags, ip_start, hint=0, fill=0):
    import torch

    from halo_amd.protocol import TxBuilder

    b = TxBuilder(len(desc), device=dev, ip_id=ip_start)
    d = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8)).to(dev)
    pl = torch.from_numpy(np.ascontiguousarray(payload)).to(dev)
    frames = torch.full((len(desc), stride), fill, dtype=torch.uint8, device=dev)
    frames, lens, res = b.build(d, pl, netif=netif, out_stride=stride, frames=frames, check_sum_enable=bool(flags),
                                max_payload_hint=hint)
    torch.cuda.synchronize()
    return frames.cpu().numpy(), lens.cpu().numpy().view(np.uint16), res.cpu().numpy(), b.iph_id


@pytest.mark.parametrize("hint", [0, 10, 500], ids=["G8", "G1", "G4"])
def test_build_golden_fixtures(dev, hint):
    desc, payload, meta, expect = build_golden(ROOT)
    netif = _netif(meta["src_mac"])
    for run in meta["runs"]:
        frames, lens, res, end = _run(dev, desc, payload, netif, 1516, run["flags"], run["ip_id_start"], hint)
        assert_build_equal(frames, lens, res, end, run, expect, f"GPU build flags={run['flags']} hint={hint}")


def test_build_random_batch_vs_oracle(dev, oracle_lib):
    """200k seeded descriptors (every protocol, both modes, payloads of any length up to one past
    the Go limits at any byte alignment, a few unknown protocols), iphId from 0xFF00 so the counter
    wraps: every byte of every slot, the lengths, results and final iphId == the C oracle."""
    from halo_amd._lib import BUILD_DESC_DTYPE

    rng = np.random.default_rng(0x7458)
    n = 200_000
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["proto"] = rng.choice(np.array([17, 6, 1, 17, 6, 99], np.uint8), n)
    lim = np.where(desc["proto"] == 6, 1461, 1473)
    small = rng.random(n) < 0.6
    desc["payload_len"] = np.where(small, rng.integers(0, 64, n), rng.integers(0, 1 << 16, n) % lim)
    offs = np.concatenate([[0], np.cumsum(desc["payload_len"].astype(np.int64) + rng.integers(0, 4, n))[:-1]])
    desc["payload_off"] = offs
    payload = rng.integers(0, 256, int(offs[-1]) + 1500, dtype=np.uint8)
    for f, hi in (("aux", 256), ("src_port", 1 << 16), ("dst_port", 1 << 16)):
        desc[f] = rng.integers(0, hi, n)
    for f in ("src_ip", "dst_ip", "seq", "ack"):
        desc[f] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    desc["dst_mac"] = rng.integers(0, 256, (n, 6))
    desc["mode"] = (rng.random(n) < 0.25).astype(np.uint8)
    mac = bytes.fromhex("020000000001")
    for flags in (1, 0):
        frames, lens, res, end = _run(dev, desc, payload, _netif(mac.hex()), 1516, flags, 0xFF00)
        wf, wl, wr, we = oracle_lib.tx_build_batch(desc, payload, mac, flags, 1516, 0xFF00)
        assert np.array_equal(res, wr) and np.array_equal(lens, wl) and end == we
        bad = np.nonzero(np.any(frames != wf, axis=1))[0]
        assert bad.size == 0, (flags, bad[:5], desc[bad[:2]])


def test_build_slots_ids_and_two_launches(dev, oracle_lib):
    """Frames longer than the slot are refused before Build* (HALO_TX_B_SLOT: no iphId step, the
    slot untouched); two launches on one workspace continue the iphId sequence."""
    import torch

    from halo_amd._lib import BUILD_DESC_DTYPE, TX_B_OK, TX_B_SLOT
    from halo_amd.protocol import TxBuilder

    n = 5000
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["proto"] = 17
    desc["payload_len"] = np.where(np.arange(n) % 7 == 3, 100, 18)  # 132 B frames do not fit 64 B slots
    desc["payload_off"] = np.arange(n) * 3
    desc["src_ip"], desc["dst_ip"] = 0x0A000001, 0x0A000002
    payload = np.arange(3 * n + 200, dtype=np.uint64).astype(np.uint8)
    netif = _netif("020000000001")
    b = TxBuilder(n, device=dev, ip_id=7)
    d = torch.from_numpy(desc.view(np.uint8)).to(dev)
    pl = torch.from_numpy(payload).to(dev)
    ids = []
    for launch in range(2):
        frames = torch.full((n, 64), 0xEE, dtype=torch.uint8, device=dev)
        frames, lens, res = b.build(d, pl, netif=netif, out_stride=64, frames=frames)
        torch.cuda.synchronize()
        f, r = frames.cpu().numpy(), res.cpu().numpy()
        assert np.all((r == TX_B_SLOT) == (np.arange(n) % 7 == 3)) and np.all(r[np.arange(n) % 7 != 3] == TX_B_OK)
        assert np.all(f[r == TX_B_SLOT] == 0xEE)
        ids.append(f[r == TX_B_OK][:, 18].astype(np.int64) * 256 + f[r == TX_B_OK][:, 19])
        wf, wl, wr, we = oracle_lib.tx_build_batch(desc, payload, bytes.fromhex("020000000001"), 1, 64,
                                                   7 + launch * int((r == TX_B_OK).sum()))
        assert np.all(lens.cpu().numpy()[r == TX_B_OK] == 60)
        assert np.array_equal(f[r == TX_B_OK][:, :60], wf[r == TX_B_OK][:, :60])
        assert np.all(f[r == TX_B_OK][:, 60:] == 0xEE)  # slot bytes past the frame's last word untouched
    built = int((np.arange(n) % 7 != 3).sum())
    assert np.array_equal(ids[0], np.arange(8, 8 + built))
    assert np.array_equal(ids[1], np.arange(8 + built, 8 + 2 * built))
    assert b.iph_id == 7 + 2 * built


@pytest.mark.parametrize("hint", [22, 1472])
def test_build_rejections_then_clean_launch(dev, oracle_lib, hint):
    """The finish launch's two paths on one workspace: a batch with rejections spread over many
    tiles (every 97th descriptor an unknown protocol), then a clean batch (the workspace still holds
    the first launch's marks), then the first batch again — frames, lengths, results and the iphId
    sequence equal the oracle's after each launch."""
    import torch

    from halo_amd._lib import BUILD_DESC_DTYPE
    from halo_amd.protocol import TxBuilder

    n = 70_000
    plen = hint
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["proto"] = 17
    desc["payload_len"] = plen
    desc["payload_off"] = np.arange(n, dtype=np.uint64) * plen
    desc["src_ip"], desc["dst_ip"] = 0x0A000001, 0x0A000002
    bad = desc.copy()
    bad["proto"][::97] = 99
    payload = (np.arange(n * plen + 64, dtype=np.uint64) * 7).astype(np.uint8)
    mac = bytes.fromhex("020000000001")
    b = TxBuilder(n, device=dev, ip_id=0xFFF0)
    pl = torch.from_numpy(payload).to(dev)
    want_id = 0xFFF0
    for batch in (bad, desc, bad):
        d = torch.from_numpy(batch.view(np.uint8)).to(dev)
        frames = torch.zeros((n, 1516), dtype=torch.uint8, device=dev)
        frames, lens, res = b.build(d, pl, netif=_netif(mac.hex()), out_stride=1516, frames=frames,
                                    max_payload_hint=hint)
        torch.cuda.synchronize()
        wf, wl, wr, we = oracle_lib.tx_build_batch(batch, payload, mac, 1, 1516, want_id)
        assert np.array_equal(res.cpu().numpy(), wr) and np.array_equal(lens.cpu().numpy().view(np.uint16), wl)
        assert np.array_equal(frames.cpu().numpy(), wf)
        assert b.iph_id == we
        want_id = we


def test_build_then_parse_round_trip(dev):
    """1M 64-byte UDP frames built on the GPU into 64 B slots parse clean on the GPU receive path
    (halo_rx_parse_strided_device) with the descriptors' addresses, ports and payload lengths."""
    import torch

    from halo_amd import protocol
    from halo_amd._lib import BUILD_DESC_DTYPE, NetIf
    from halo_amd.protocol import TxBuilder

    n = 1 << 20
    rng = np.random.default_rng(11)
    desc = np.zeros(n, BUILD_DESC_DTYPE)
    desc["proto"] = 17
    desc["payload_len"] = 22
    desc["payload_off"] = np.arange(n, dtype=np.uint64) * 22
    desc["src_port"] = rng.integers(1, 1 << 16, n)
    desc["dst_port"] = 22222
    desc["src_ip"] = 0x0A000000 | rng.integers(0, 1 << 24, n).astype(np.uint32)
    desc["dst_ip"] = 0xC0A86464
    desc["dst_mac"] = 0xAA
    pl = torch.randint(0, 256, (22 * n + 8,), dtype=torch.uint8, device=dev)
    b = TxBuilder(n, device=dev)
    frames, lens, res = b.build(torch.from_numpy(desc.view(np.uint8)).to(dev), pl, netif=NetIf.make(mac="02:00:00:00:00:01"),
                                out_stride=64, max_payload_hint=22)
    rec = protocol.parse_frames_strided(frames, 64, n, netif=NetIf.make(), lens=lens)
    torch.cuda.synchronize()
    r = protocol.records(rec)
    assert np.all(res.cpu().numpy() == 0) and np.all(lens.cpu().numpy() == 64)
    assert np.all(r["status"] == 0) and np.all(r["flags"] == 5)
    assert np.array_equal(r["src_ip"], desc["src_ip"]) and np.array_equal(r["sport"], desc["src_port"])
    assert np.all(r["payload_len"] == 22) and np.all(r["payload_off"] == 42)
    assert b.iph_id == n & 0xFFFF
