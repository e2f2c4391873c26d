"""GPU: the resident consumer behind halo_rx_parse_batch_host (halo_rx_host_ctx_set_resident) — the
latency path of a batched PacketHandle (engine/engine.go:339-385, 99-poll drain cadence :353) and of
the single-frame Parse* wrappers (an Ipv4PktFwdHook, engine/engine.go:132) — and the library's
device drains with resident consumers alive: bit-exact against the C oracle at every
batch size, ragged and uniform layouts, LoChan (L3) batches, registered and pageable record arrays;
drains that stop persistent consumers while another thread polls; a timed-out request retired
before the call returns."""
from __future__ import annotations

import threading
import time

import numpy as np
import pytest

from tests.helpers import assert_records_equal, expected_records, golden_arrays, strip_ethernet

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    yield torch.device("cuda:0")
    assert _lib.registered_count() == 0, _lib.registrations()


def _unaligned(data, offs_dw, lens, shift=1):
    """The frames repacked at odd host offsets (a cgo caller's Go slices have any alignment)."""
    host = np.zeros(int(lens.astype(np.int64).sum()) + 3 * len(lens) + 16, np.uint8)
    hoffs = np.zeros(len(lens), np.uint64)
    pos = shift
    for i in range(len(lens)):
        o, L = int(offs_dw[i]) * 4, int(lens[i])
        host[pos:pos + L] = data[o:o + L]
        hoffs[i] = pos
        pos += L + 3
    return host, hoffs


@pytest.fixture(scope="module")
def fuzz(oracle_lib):
    ni = oracle_lib.NetIf.make()
    data, offs, lens = oracle_lib.fuzz_batch(0x5E5, 20000, ni)
    host, hoffs = _unaligned(data, offs, lens)
    want = {f: oracle_lib.rx_batch(data, lens, ni, f, offsets_dw=offs)[0] for f in (1, 3)}
    return host, hoffs, lens, want


def test_resident_golden_frames(dev, golden):
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.engine import HostBatcher

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    host, hoffs = _unaligned(data, offs, lens)
    hb = HostBatcher(0)
    hb.set_resident(4096)
    try:
        for flags in (0, 1, 2, 3):
            hist = np.zeros(14, np.uint32)
            got = hb.parse(host, hoffs, lens, NetIf.make(), flags, hist)
            want = expected_records(meta, flags, RESULT_DTYPE)
            assert_records_equal(got, want, names, f"resident flags={flags}")
            assert np.array_equal(hist, np.bincount(want["status"], minlength=14))
        st = hb.stats()
        assert st["resident_calls"] == 4 and st["service_launches"] >= 1, st
    finally:
        hb.close()


@pytest.mark.parametrize("registered_out", [False, True], ids=["pageable_out", "registered_out"])
def test_resident_batch_sizes_match_oracle(dev, fuzz, registered_out):
    """Every PacketHandle-sized batch (1 .. 4096 frames, the 99-poll cadence included) = oracle; a
    batch past max_frames (4097) or past the staging bytes takes the chunked path, same records."""
    import contextlib

    from halo_amd import _lib
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.engine import HostBatcher

    host, hoffs, lens, want = fuzz
    hb = HostBatcher(0)
    hb.set_resident(4096, 1 << 20)
    out = _lib.host_array(8192, RESULT_DTYPE)
    try:
        with contextlib.ExitStack() as regs:
            if registered_out:
                regs.enter_context(_lib.registered(out))
            start = 0
            for m in (1, 2, 31, 64, 65, 99, 256, 1000, 4096, 4097, 6000):
                for flags in (1, 3):
                    sl = slice(start, start + m)
                    hist = np.zeros(14, np.uint32)
                    got = hb.parse(host, hoffs[sl], lens[sl], NetIf.make(), flags, hist, out=out)[:m]
                    assert_records_equal(got.copy(), want[flags][sl], None, f"m={m} flags={flags}")
                    assert np.array_equal(hist, np.bincount(want[flags][sl]["status"], minlength=14))
                start = (start + 7919) % (len(lens) - 6000)
        st = hb.stats()
        # 4097 and 6000 exceed max_frames; 1000 / 4096 fuzz frames of up to 9 KB may exceed 1 MiB
        assert st["resident_calls"] >= 10, st
    finally:
        hb.close()


def test_resident_uniform_batches(dev, oracle_lib):
    """Frames of one length travel as the uniform layout (no offset / length arrays): 64 B and
    1500 B synthetic frames, clean and 1/4 mutated, = oracle."""
    from halo_amd import synth
    from halo_amd._lib import NetIf
    from halo_amd.engine import HostBatcher

    hb = HostBatcher(0)
    hb.set_resident(2048, 4 << 20)
    try:
        for length, m in ((64, 99), (64, 2048), (1500, 1), (1500, 700), (60, 33)):
            lay = synth.layout(m, length=length, mutate_shift=2, seed=0x1234 + length)
            data = oracle_lib.synth_batch(lay["seed"], 0, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                          offsets_dw=lay["offsets_dw"])
            host, hoffs = _unaligned(data, lay["offsets_dw"], lay["lens"], shift=2)
            want, _ = oracle_lib.rx_batch(data, lay["lens"], oracle_lib.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
            got = hb.parse(host, hoffs, lay["lens"], NetIf.make(), 1)
            assert_records_equal(got, want, None, f"uniform {length} B x {m}")
            assert (want["status"] != 0).any() or m < 8
        assert hb.stats()["resident_calls"] == 5
    finally:
        hb.close()


def test_resident_lochan_batches(dev, golden, oracle_lib):
    """HALO_RX_L3_START batches (PacketHandle's LoChan drain through a host context) = oracle."""
    from halo_amd._lib import HALO_RX_L3_START, NetIf
    from halo_amd.engine import HostBatcher

    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    pk, poffs, plens = strip_ethernet(data, offs, lens)
    host, hoffs = _unaligned(pk, poffs, plens)
    hb = HostBatcher(0)
    hb.set_resident(4096)
    try:
        for flags in (1, 3):
            want, _ = oracle_lib.rx_batch(pk, plens, oracle_lib.NetIf.make(), flags | HALO_RX_L3_START,
                                          offsets_dw=poffs)
            got = hb.parse(host, hoffs, plens, NetIf.make(), flags | HALO_RX_L3_START)
            assert_records_equal(got, want, None, f"L3 flags={flags}")
        assert hb.stats()["resident_calls"] == 2
    finally:
        hb.close()


def test_resident_timeout_retires_the_request(dev, golden):
    """A forced 1 us timeout: the call fails, and nothing lands in the caller's array after it
    returned (the request was retired: consumer stopped, kernel ended). The next call with the
    default timeout relaunches the consumer and returns the right records."""
    from halo_amd import _lib
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.engine import HostBatcher

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    host, hoffs = _unaligned(data, offs, lens)
    hb = HostBatcher(0)
    hb.set_resident(4096)
    out = np.zeros(len(lens), RESULT_DTYPE)
    try:
        hb.set_service_timeout(1)
        failures = 0
        for _ in range(5):
            out.view(np.uint8)[:] = 0xEE
            try:
                hb.parse(host, hoffs, lens, NetIf.make(), 1, out=out)
            except _lib.HaloError as e:
                assert e.code == _lib.HALO_E_HIP
                failures += 1
                snap = out.copy()
                time.sleep(0.05)
                assert np.array_equal(out.view(np.uint8), snap.view(np.uint8)), "records written after return"
        assert failures >= 1
        hb.set_service_timeout(0)
        got = hb.parse(host, hoffs, lens, NetIf.make(), 1, out=out)
        assert_records_equal(got, expected_records(meta, 1, RESULT_DTYPE), names, "after timeouts")
    finally:
        hb.close()


def test_ring_timeout_retires_the_request(dev, golden, oracle_lib):
    """The same for a HALO_RING_PERSISTENT ring: a failed poll leaves the cursor, the next poll
    returns the same frames, and the failed poll's array is not written after it returned."""
    from halo_amd import _lib
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    ok = [i for i in range(len(lens)) if 42 <= lens[i] <= 1514]
    ring = RingBuffer(1 << 20)
    assert ring.write_batch(data, offs[ok].astype(np.uint64) * 4, lens[ok]) == len(ok)
    cons = RingConsumer(ring, capacity=1514, persistent=True, small_poll=16 << 20)
    try:
        cons.set_service_timeout(1)
        for _ in range(3):
            try:
                cons.poll(NetIf.make())
            except _lib.HaloError as e:
                assert e.code == _lib.HALO_E_HIP
                snap = cons._out.copy()
                time.sleep(0.05)
                assert np.array_equal(cons._out.view(np.uint8), snap.view(np.uint8))
                break
        cons.set_service_timeout(0)
        recs, info, _ = cons.poll(NetIf.make())
        assert info["n_frames"] == len(ok)
        want = expected_records(meta, 1, RESULT_DTYPE)[ok]
        assert_records_equal(recs.copy(), want, [names[i] for i in ok], "poll after a timed-out poll")
        cons.commit()
    finally:
        cons.close()


def test_drains_while_a_persistent_ring_is_polled(dev, oracle_lib):
    """unregistering host memory, attaching and detaching another ring, syncing a route
    table and halo_rx_device_synchronize are device drains. With another thread polling a HALO_RING_PERSISTENT ring non-stop, each
    must finish promptly (the drain stops the resident consumer and keeps polls on launches while it
    waits) and every poll must stay correct."""
    from halo_amd import _lib, synth
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer
    from halo_amd.route import RouteTable

    m = 256
    lay = synth.layout(m, length=64, seed=0xD2A1)
    data = oracle_lib.synth_batch(lay["seed"], 0, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                  offsets_dw=lay["offsets_dw"])
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    want, _ = oracle_lib.rx_batch(data, lay["lens"], oracle_lib.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
    ring = RingBuffer(1 << 22)
    cons = RingConsumer(ring, capacity=1514, persistent=True, small_poll=16 << 20)
    stop = threading.Event()
    errors, polls = [], [0]

    def poller():
        try:
            while not stop.is_set():
                assert ring.write_batch(data, offs, lay["lens"]) == m
                recs, info, _ = cons.poll(NetIf.make())
                assert info["n_frames"] == m
                assert_records_equal(recs.copy(), want, None, "poll during drains")
                cons.commit()
                polls[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = threading.Thread(target=poller)
    th.start()
    durations = {}
    try:
        time.sleep(0.2)
        for rnd in range(3):
            arr = _lib.host_array(1 << 16)
            t0 = time.perf_counter()
            with _lib.registered(arr):
                pass  # unregister = a drain of every device the library used
            durations.setdefault("unregister", []).append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            other = RingConsumer(RingBuffer(1 << 16), capacity=1514, persistent=True)
            other.close()
            durations.setdefault("attach_detach", []).append(time.perf_counter() - t0)
            t = RouteTable(0)
            t.AddRoute(t.entry(0xC0A86400, 0xFFFFFF00, 0, 1))
            t0 = time.perf_counter()
            t.sync()
            t.sync()  # the second sync drains the device before reusing a generation
            durations.setdefault("route_sync", []).append(time.perf_counter() - t0)
            t.close()
            # the exported drain: a caller's device synchronisation that does not wait
            # for the resident consumer another thread keeps busy
            t0 = time.perf_counter()
            _lib.device_synchronize(0)
            durations.setdefault("device_synchronize", []).append(time.perf_counter() - t0)
        time.sleep(0.1)
    finally:
        stop.set()
        th.join(timeout=30)
        st = cons.stats()
        cons.close()
    assert not th.is_alive()
    assert not errors, errors[0]
    assert polls[0] > 10
    worst = {k: max(v) for k, v in durations.items()}
    assert all(v < 1.0 for v in worst.values()), worst
    assert st["service_requests"] > 0, st
