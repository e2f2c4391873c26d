"""GPU: engine.NetIf.packet_handle_batch with drain_every=99 invokes the service handlers and
drains LoChan in exactly the order PacketHandle does (engine/engine.go:339-385: one EthRxFunc poll
per iteration, nil polls counted, the loopback channel drained until empty after every 99th poll),
whatever the batch size; the default (drain after every batch) does not — checked against a
per-frame model of the reference loop built on the Python restatement (oracle/ref_py.py).

The traffic mixes local UDP frames whose handler queues a TxIpv4-style loopback packet into
LoChan (the drained packet reaches a second handler, which may queue another), frames for
other hosts, corrupted frames and nil polls."""
from __future__ import annotations

import collections

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MAC = bytes.fromhex("AAAAAAAAAAAA")
OWN = bytes([192, 168, 100, 100])
PEER = bytes([192, 168, 100, 1])
POLLS = 990  # 10 drains at the reference's cadence


def _frames():
    from oracle import ref_py as R

    rng = np.random.default_rng(0x4341444E)
    sched = []
    for k in range(POLLS - 60):
        if k % 7 == 3:
            sched.append(None)  # EthRxFunc returned nil
            continue
        kind = rng.integers(0, 10)
        pay = b"LO%05d" % k if kind < 4 else b"pk%05d" % k
        dst = OWN if kind < 8 else bytes([10, 0, 0, 9])
        udp = R.build_udp(pay, 5000 + k % 50, 7000, PEER, dst)
        f = bytearray(R.build_eth(R.build_ipv4(udp, 17, PEER, dst, ident=k), MAC, bytes(6), 0x0800))
        if kind == 9:
            f[40] ^= 0x10  # corrupted: DROP_L4 (or FORWARD for the other host)
        sched.append(bytes(f))
    return sched + [None] * 60


def _lo_packet(payload: bytes, dport: int) -> bytes:
    from oracle import ref_py as R

    return R.build_ipv4(R.build_udp(payload, 7000, dport, OWN, OWN), 17, OWN, OWN)


class Handlers:
    """Port 7000: log, and for "LO" payloads queue a loopback packet to port 7001; port 7001: log,
    and for every third packet queue one more (to port 7002) — handlers that feed the drain."""

    def __init__(self, lochan):
        self.log, self.lochan = [], lochan

    def udp(self, port, payload):
        self.log.append((port, bytes(payload)))
        if port == 7000 and payload[:2] == b"LO":
            self.lochan.append(_lo_packet(b"lo" + bytes(payload[2:]), 7001))
        if port == 7001 and int(payload[2:]) % 3 == 0:
            self.lochan.append(_lo_packet(b"l2" + bytes(payload[2:]), 7002))


def _reference_order(sched):
    """PacketHandle, per frame, with the restated parsers: the handler log."""
    from oracle import ref_py as R

    lochan = collections.deque()
    h = Handlers(lochan)
    own_ip = int.from_bytes(OWN, "big")
    c = R.Cfg(True)

    def local_udp(ip_pkt):
        pay, _proto, src, _dst, _tl, err = R.parse_ipv4_pkt(ip_pkt, c)
        up, _sp, dp, err = R.parse_udp_pkt(pay, src, OWN, c)
        assert err is None
        h.udp(dp, up)

    n = 0
    for f in sched:
        if f is not None and R.engine_rx(f, MAC, own_ip) == "LOCAL_UDP":
            local_udp(f[14:])
        n += 1
        if n == 99:
            while lochan:
                p = lochan.popleft()
                if R.engine_lo(p, own_ip) == "LOCAL_UDP":
                    local_udp(p)
            n = 0
    return h.log


def _batched_order(sched, batch, drain_every, cpu_below=0):
    from halo_amd.engine import NetIf

    it = iter(sched)
    polls = [0]

    def rx():
        polls[0] += 1
        return next(it, None)

    netif = NetIf("eth0", "AA:AA:AA:AA:AA:AA", "192.168.100.100", rx, cpu_below=cpu_below)
    h = Handlers(netif.LoChan)
    for port in (7000, 7001, 7002):
        netif.RecvUdp(port, lambda s, p, port=port: h.udp(port, p))
    while polls[0] < POLLS:
        netif.packet_handle_batch(batch=batch, drain_every=drain_every)
    return h.log


@pytest.fixture(scope="module")
def setup():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    sched = _frames()
    return sched, _reference_order(sched)


@pytest.mark.parametrize("batch", [1, 32, 99, 4096])
def test_reference_cadence_reproduces_order(setup, batch):
    sched, want = setup
    assert len(want) > 500 and any(p == 7002 for p, _ in want)
    assert _batched_order(sched, batch, 99) == want


@pytest.mark.parametrize("batch", [32, 4096])
def test_mixed_cpu_gpu_routing_reproduces_order(setup, batch):
    """Batches and drains below 40 frames on the CPU entry point, the rest on the GPU: the same order."""
    sched, want = setup
    assert _batched_order(sched, batch, 99, cpu_below=40) == want


def test_every_batch_drain_differs(setup):
    """Sensitivity: draining after every batch delivers loopback packets earlier than PacketHandle."""
    sched, want = setup
    got = _batched_order(sched, 4096, 0)
    assert sorted(got) == sorted(want) and got != want
