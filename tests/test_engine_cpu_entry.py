"""CPU: engine.NetIf.packet_handle_batch with every batch and LoChan drain on the CPU entry point
(cpu_below above any batch size; halo_rx_parse_batch_cpu, no GPU) invokes the handlers and drains
LoChan in PacketHandle's order at drain_every=99 (engine/engine.go:339-385), against the same
per-frame model of the reference loop as tests/test_gpu_engine_cadence.py, which checks the GPU
and mixed CPU / GPU routings."""
from __future__ import annotations

import pytest

from tests.test_gpu_engine_cadence import _batched_order, _frames, _reference_order

ALL_CPU = 1 << 30


@pytest.fixture(scope="module")
def setup():
    sched = _frames()
    return sched, _reference_order(sched)


@pytest.mark.parametrize("batch", [1, 32, 99, 4096])
def test_cpu_routing_reproduces_reference_order(setup, batch):
    sched, want = setup
    assert len(want) > 500 and any(p == 7002 for p, _ in want)
    assert _batched_order(sched, batch, 99, cpu_below=ALL_CPU) == want


def test_cpu_routing_every_batch_drain_differs(setup):
    sched, want = setup
    got = _batched_order(sched, 4096, 0, cpu_below=ALL_CPU)
    assert sorted(got) == sorted(want) and got != want


def test_cpu_routing_needs_no_device():
    """With every batch below cpu_below no host context (and so no GPU) is ever made."""
    from halo_amd.engine import NetIf

    frames = iter(_frames()[:200])
    netif = NetIf("eth0", "AA:AA:AA:AA:AA:AA", "192.168.100.100", lambda: next(frames, None), cpu_below=ALL_CPU)
    res, acts = netif.packet_handle_batch(batch=4096, drain_every=99)
    assert len(res) > 50 and netif._batcher is None


def test_cpu_routing_empty_frames():
    """EthRxFunc returning empty (non-nil) buffers: ParseEthFrm's length error, dropped (DROP_ETH)."""
    from halo_amd import ACTION
    from halo_amd.engine import NetIf

    frames = iter([b"", b"", None])
    netif = NetIf("eth0", "AA:AA:AA:AA:AA:AA", "192.168.100.100", lambda: next(frames, None), cpu_below=ALL_CPU)
    res, acts = netif.packet_handle_batch(batch=16, drain_every=0)
    assert list(res["status"]) == [1, 1] and list(acts) == [ACTION["DROP_ETH"]] * 2
