"""GPU: halo's SPSC packet ring as the batch source, bit-exact.

The oracle side is oracle/halo_ring_oracle.c — ReadPacket / the config-1 PacketHandle loop /
the record walk — which tests/test_ring_oracle.py pins against the reference's own
cgo/ring_buffer.h. Here the GPU consumer (halo_rx_ring_poll: raw span DMA, record boundaries
found on the GPU, parse in place) and the device-resident walk (halo_rx_ring_scan_device) must
return exactly the frames, records, positions, stop reason and new tail of that loop: wrap-around,
corrupt and oversize records, max_bytes / max_frames cuts, tile-boundary and dense-record spans.
"""
from __future__ import annotations

import zlib

import numpy as np
import pytest

from tests.helpers import assert_records_equal, golden_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    yield torch.device("cuda:0")
    # every ring and record array these tests registered was unregistered again
    assert _lib.registered_count() == 0, _lib.registrations()


@pytest.fixture(autouse=True)
def _no_registration_outlives_a_test():
    """Each test ends with no live host registration: a registration outliving its test (a
    consumer left attached, an array left registered) is what could leave a stale mapping behind
    for a later pageable copy."""
    import gc

    from halo_amd import _lib

    yield
    gc.collect()  # consumers dropped without close() detach in __del__
    assert _lib.registered_count() == 0, _lib.registrations()


def _seek(ring, pos: int):
    """Move an empty ring's head and tail to stream position `pos`."""
    ring.mem[0:8].view(np.uint64)[0] = pos
    ring.mem[64:72].view(np.uint64)[0] = pos


def _oracle_drain(O, mem, netif, flags, capacity, max_frames=0xFFFFFFFF):
    r2 = O.Ring(mem=mem.copy())
    recs, acts, pos, _ = r2.packet_handle(netif, flags, capacity=capacity, max_frames=max_frames)
    return recs, acts, pos, r2._ct.value


def _span(ring, start, used):
    idx = (start % ring.size + np.arange(used)) % ring.size
    return ring.mem[128:][idx]


SMALL = [0, None, 16 << 20, "persistent"]  # pipelined only / library default / small path for every poll /
SMALL_IDS = ["pipelined", "default", "small16M", "persistent"]  # ... served by the resident consumer kernel


def _small_kw(small_poll):
    """RingConsumer keywords for a SMALL entry ("persistent": HALO_RING_PERSISTENT, every poll small)."""
    if small_poll == "persistent":
        return {"small_poll": 16 << 20, "persistent": True}
    return {"small_poll": small_poll}


@pytest.mark.parametrize("small_poll", SMALL, ids=SMALL_IDS)
@pytest.mark.parametrize("flags", [0, 1, 3])
def test_poll_golden_frames_across_the_wrap(dev, golden, oracle_lib, flags, small_poll):
    from halo_amd._lib import NetIf
    from halo_amd.engine import dispatch
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    ring = RingBuffer(1 << 18)
    _seek(ring, (1 << 40) + (1 << 18) - 2048)  # the batch wraps around the data area's end
    small = (lens > 0) & (lens <= 1514)  # WritePacket refuses empty frames
    n_w = ring.write_batch(data, offs[small].astype(np.uint64) * 4, lens[small])
    assert n_w == int(small.sum())
    want, acts, pos, tail = _oracle_drain(O, ring.mem, O.NetIf.make(), flags, 1514)
    assert len(want) == n_w
    cons = RingConsumer(ring, capacity=1514, **_small_kw(small_poll))
    got, info, gpos = cons.poll(NetIf.make(), check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2),
                                positions=True)
    assert_records_equal(got.copy(), want, [n for n, s in zip(names, small) if s], f"ring flags={flags}")
    assert np.array_equal(gpos, pos)
    assert info["stop"] == "EMPTY" and info["end_bytes"] == tail - ring.tail
    assert np.array_equal(dispatch(got.copy(), NetIf.make()), acts)
    assert ring.tail == (1 << 40) + (1 << 18) - 2048
    cons.commit()
    assert ring.tail == tail
    got2, info2, _ = cons.poll(NetIf.make())
    assert info2["n_frames"] == 0 and info2["stop"] == "EMPTY"
    cons.close()


@pytest.mark.parametrize("small_poll", SMALL, ids=SMALL_IDS)
def test_poll_stops_like_readpacket(dev, golden, oracle_lib, small_poll):
    """An oversize record (> capacity) stops the drain and stays; a corrupt length stops it for
    good; max_frames and max_bytes cut it. Every poll is compared with the oracle loop."""
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    rng = np.random.default_rng(5)
    netif, onetif = NetIf.make(), O.NetIf.make()
    for case in ("capacity", "corrupt", "max_frames", "max_bytes"):
        ring = RingBuffer(1 << 20)
        _seek(ring, int(rng.integers(0, 1 << 30)) * 4)
        sel = rng.permutation(np.nonzero(lens <= 1514)[0])[:120]
        ring.write_batch(data, offs[sel].astype(np.uint64) * 4, lens[sel])
        if case == "capacity":  # a 2000-byte record (ReadPacket leaves it: capacity 1514)
            big = np.zeros(2000, np.uint8)
            ring.write_batch(big, np.zeros(1, np.uint64), np.array([2000], np.uint16))
        if case == "corrupt":  # a record whose length field is 0
            pos = ring.head % ring.size
            ring.mem[128 + (pos + np.arange(8)) % ring.size] = 0
            ring.mem[0:8].view(np.uint64)[0] = ring.head + 8
        ring.write_batch(data, offs[sel].astype(np.uint64) * 4, lens[sel])
        kw = dict(max_frames=50) if case == "max_frames" else dict(max_bytes=6000) if case == "max_bytes" else {}
        cons = RingConsumer(ring, capacity=1514, **_small_kw(small_poll), **kw)
        mem_before = ring.mem.copy()
        got_all = []
        for _ in range(200):
            got, info, _ = cons.poll(netif)
            if info["n_frames"] == 0:
                break
            got_all.append(got.copy())
            cons.commit()
        got_all = np.concatenate(got_all) if got_all else np.zeros(0, got.dtype)
        want, _, _, tail = _oracle_drain(O, mem_before, onetif, 1, 1514)
        assert_records_equal(got_all, want, None, f"ring stop case {case}")
        assert ring.tail == tail, case
        assert info["stop"] == {"capacity": "CAPACITY", "corrupt": "BAD_LEN"}.get(case, "EMPTY"), (case, info)
        cons.close()


def _records_span(rng, lens, corrupt_at=None, corrupt_val=0, garbage=0.0, garbage_bytes=None):
    """A ring span in stream order holding records of `lens` (+ random bytes). `garbage`: the
    fraction of payload dwords replaced by values that pass ReadPacket's length checks (1..1514),
    so walks started off the record chain look valid for a while (record decoys); only within the
    byte range `garbage_bytes` = (lo, hi) when given."""
    lens = np.asarray(lens, np.int64)
    sizes = (4 + lens + 3) & ~3
    starts = np.zeros(len(lens), np.int64)
    starts[1:] = np.cumsum(sizes)[:-1]
    used = int(sizes.sum())
    span = rng.integers(0, 256, used + 16, dtype=np.uint8)
    words = span[:used].view(np.uint32)
    if garbage:
        lo, hi = (0, used) if garbage_bytes is None else garbage_bytes
        win = words[lo // 4:hi // 4]
        decoy = rng.random(win.size) < garbage
        win[decoy] = rng.integers(1, 1515, int(decoy.sum()), dtype=np.uint32)
    words[starts // 4] = lens.astype(np.uint32)
    if corrupt_at is not None:
        words[starts[corrupt_at] // 4] = corrupt_val
    return span, used


SCAN_CASES = [
    # name, lens generator, capacity, max_frames, corrupt (index, value)
    ("empty", lambda r: [], 1514, 0, None),
    ("one", lambda r: [60], 1514, 0, None),
    ("64B_x300k", lambda r: [64] * 300_000, 1514, 0, None),
    ("dense_1to4B", lambda r: r.integers(1, 5, 200_000), 1514, 0, None),
    ("imix", lambda r: r.choice([64, 570, 1500], 100_000, p=[7 / 12, 4 / 12, 1 / 12]), 1514, 0, None),
    ("uniform_to_cap", lambda r: r.integers(1, 1515, 60_000), 1514, 0, None),
    ("jumbo_cap", lambda r: r.integers(1, 9015, 20_000), 9014, 0, None),
    ("max_window", lambda r: r.integers(1, 16377, 8_000), 16376, 0, None),
    ("oversize_mid", lambda r: list(r.integers(1, 1515, 40_000)) + [1515] + [64] * 1000, 1514, 0, None),
    ("bad_len_mid", lambda r: r.integers(1, 1515, 50_000), 1514, 0, (31_337, 0)),
    ("huge_len_mid", lambda r: r.integers(1, 200, 50_000), 1514, 0, (20_001, 0xFFFFFFFF)),
    ("max_frames_cut", lambda r: r.integers(1, 1515, 50_000), 1514, 12_345, None),
    ("max_frames_exact", lambda r: [64] * 5000, 1514, 5000, None),
    ("max_frames_one", lambda r: [64] * 5000, 1514, 1, None),
    # record decoys in the payloads (every / 1 in 100 payload dwords a plausible length)
    ("decoys_all_imix", lambda r: r.choice([64, 570, 1500], 60_000, p=[7 / 12, 4 / 12, 1 / 12]), 1514, 0, None),
    ("decoys_1pct", lambda r: r.integers(1, 1515, 60_000), 1514, 0, None),
    ("decoys_all_dense", lambda r: r.integers(1, 9, 200_000), 1514, 0, None),
    ("decoys_all_bad_len", lambda r: r.integers(1, 1515, 50_000), 1514, 0, (40_000, 0)),
    ("decoys_all_max_frames", lambda r: r.integers(60, 200, 50_000), 1514, 33_333, None),
]
DECOYS = {"decoys_all_imix": 1.0, "decoys_1pct": 0.01, "decoys_all_dense": 1.0, "decoys_all_bad_len": 1.0,
          "decoys_all_max_frames": 1.0}


@pytest.mark.parametrize("name,gen,cap,max_frames,corrupt", SCAN_CASES, ids=[c[0] for c in SCAN_CASES])
def test_scan_device_matches_walk(dev, oracle_lib, name, gen, cap, max_frames, corrupt):
    import torch

    from halo_amd import _lib

    O = oracle_lib
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    lens = gen(rng)
    span, used = _records_span(rng, lens, *(corrupt or (None, 0)), garbage=DECOYS.get(name, 0.0))
    ring_size = 1 << max(12, int(np.ceil(np.log2(max(used, 8)))) + 1)
    for trim in (0, 4, 12) if used > 64 else (0,):  # also spans that end inside a record
        u = max(0, used - trim)
        mf = max_frames or 0xFFFFFFFF
        w_off, w_len, w_stop, w_end, w_ml = O.ring_scan(span, u, ring_size, cap, mf)
        d_span = torch.from_numpy(span).to(dev)
        n_max = max(1, u // 8)
        d_off = torch.zeros(n_max, dtype=torch.int32, device=dev)
        d_len = torch.zeros(n_max, dtype=torch.int16, device=dev)
        info = torch.zeros(24, dtype=torch.uint8, device=dev)
        ws_bytes = _lib.lib.halo_rx_ring_scan_workspace(u, cap)
        ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=dev)
        rc = _lib.lib.halo_rx_ring_scan_device(d_span.data_ptr(), u, ring_size, cap, max_frames, d_off.data_ptr(),
                                               d_len.data_ptr(), info.data_ptr(), ws.data_ptr(), ws_bytes,
                                               torch.cuda.current_stream().cuda_stream)
        _lib.check("halo_rx_ring_scan_device", rc)
        torch.cuda.synchronize()
        inf = info.cpu().numpy().view(_lib.RING_SCAN_DTYPE)[0]
        n = int(inf["n_frames"])
        assert n == len(w_off), (name, trim, n, len(w_off))
        assert (int(inf["stop"]), int(inf["end_bytes"]), int(inf["max_len"])) == (w_stop, w_end, w_ml), (name, trim)
        assert np.array_equal(d_off[:n].cpu().numpy().view(np.uint32), w_off), name
        assert np.array_equal(d_len[:n].cpu().numpy().view(np.uint16), w_len), name


LINK_CHUNK_BYTES = 512 * 16 * 16384  # ring_link_kernel: kLinkThreads x kLinkPer tiles of 16 KB = 128 MiB


@pytest.mark.parametrize("decoys,max_frames", [(False, 0), (True, 0), (True, 2_000_000)],
                         ids=["plain", "decoys_after_boundary", "decoys_max_frames"])
def test_scan_device_beyond_one_link_chunk(dev, oracle_lib, decoys, max_frames):
    """the link kernel passes a whole 8192-tile chunk (128 MiB) with no special tile on its
    summaries alone and enters the next chunk from the last thread's exit — only on spans > 128 MiB.
    2.4M x 64 B records (163 MB); with decoys, every payload dword of the first 64 KB after the chunk
    boundary is a plausible length, so the guesses of the tiles there are wrong and the second chunk
    starts with a second walk from the entry the first chunk handed over. Against the oracle's walk."""
    import torch

    from halo_amd import _lib

    O = oracle_lib
    rng = np.random.default_rng(0x4C494E4B + decoys)
    lens = [64] * 2_400_000
    span, used = _records_span(rng, lens, garbage=1.0 if decoys else 0.0,
                               garbage_bytes=(LINK_CHUNK_BYTES, LINK_CHUNK_BYTES + (64 << 10)))
    assert used > LINK_CHUNK_BYTES + (1 << 20)
    ring_size = 1 << 28
    mf = max_frames or 0xFFFFFFFF
    w_off, w_len, w_stop, w_end, w_ml = O.ring_scan(span, used, ring_size, 1514, mf)
    assert len(w_off) == (max_frames or len(lens))
    d_span = torch.from_numpy(span).to(dev)
    n_max = used // 8
    d_off = torch.zeros(n_max, dtype=torch.int32, device=dev)
    d_len = torch.zeros(n_max, dtype=torch.int16, device=dev)
    info = torch.zeros(24, dtype=torch.uint8, device=dev)
    ws_bytes = _lib.lib.halo_rx_ring_scan_workspace(used, 1514)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    rc = _lib.lib.halo_rx_ring_scan_device(d_span.data_ptr(), used, ring_size, 1514, max_frames, d_off.data_ptr(),
                                           d_len.data_ptr(), info.data_ptr(), ws.data_ptr(), ws_bytes,
                                           torch.cuda.current_stream().cuda_stream)
    _lib.check("halo_rx_ring_scan_device", rc)
    torch.cuda.synchronize()
    inf = info.cpu().numpy().view(_lib.RING_SCAN_DTYPE)[0]
    n = int(inf["n_frames"])
    assert n == len(w_off)
    assert (int(inf["stop"]), int(inf["end_bytes"]), int(inf["max_len"])) == (w_stop, w_end, w_ml)
    assert np.array_equal(d_off[:n].cpu().numpy().view(np.uint32), w_off)
    assert np.array_equal(d_len[:n].cpu().numpy().view(np.uint16), w_len)


@pytest.mark.parametrize("persistent", [False, True], ids=["launch", "persistent"])
def test_small_poll_laps_the_ring(dev, oracle_lib, persistent):
    """The small path reads frames in place in the registered ring: 300 produce/poll/commit rounds
    over a 64 KiB ring (the data area is rewritten ~70 times) with fresh frames each round, a
    record wrapping the end now and then (that poll takes the pipelined path), each poll's records
    == the oracle on exactly the frames written; positions and tail follow ReadPacket."""
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    ring = RingBuffer(1 << 16)
    _seek(ring, (1 << 33) - 100)
    cons = RingConsumer(ring, capacity=1514, persistent=persistent)
    rng = np.random.default_rng(17)
    onetif = O.NetIf.make()
    for it in range(300):
        k = int(rng.integers(1, 24))
        lens = rng.integers(42, 1515, size=k).astype(np.uint16)
        kinds = rng.integers(0, 3, size=k).astype(np.uint8)
        offs = np.concatenate([[0], np.cumsum((lens.astype(np.int64) + 3) & ~3)[:-1]]).astype(np.uint32) // 4
        data = O.synth_batch(it, 0, lens, kinds, onetif, offsets_dw=offs)
        if it % 3 == 1:  # a bit flip somewhere in one frame
            j = int(rng.integers(0, k))
            data[int(offs[j]) * 4 + int(rng.integers(14, int(lens[j])))] ^= 1 << int(rng.integers(0, 8))
        start = ring.head
        assert ring.write_batch(data, offs.astype(np.uint64) * 4, lens) == k
        got, info, pos = cons.poll(NetIf.make(), positions=True)
        want, _ = O.rx_batch(data, lens, onetif, 1, offsets_dw=offs)
        assert info["n_frames"] == k and info["stop"] == "EMPTY", (it, info)
        assert_records_equal(got.copy(), want, None, f"lap round {it}")
        rec = np.concatenate([[0], np.cumsum(4 + ((lens.astype(np.int64) + 3) & ~3))[:-1]])
        assert np.array_equal(pos, start + rec)
        cons.commit()
        assert ring.tail == ring.head
    cons.close()


def test_small_poll_unpinned_out_and_unregistered_ring(dev, golden, oracle_lib):
    """Records into a caller array that is neither pinned nor registered (the small path stages
    them); an unregistered ring has no small path (set_small_poll refuses) and polls pipelined."""
    from halo_amd import _lib
    from halo_amd._lib import RING_SCAN_DTYPE, NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    sel = np.nonzero((lens > 0) & (lens <= 1514))[0][:100]
    for register in (True, False):
        ring = RingBuffer(1 << 18)
        ring.write_batch(data, offs[sel].astype(np.uint64) * 4, lens[sel])
        want, _, _, tail = _oracle_drain(O, ring.mem, O.NetIf.make(), 1, 1514)
        cons = RingConsumer(ring, capacity=1514, register=register)
        if not register:
            assert _lib.lib.halo_rx_ring_set_small_poll(cons._h, 1 << 16) == _lib.HALO_E_INVAL
        out = _lib.host_array(len(sel) + 5, _lib.RESULT_DTYPE)  # registered below: pages of its own
        out.view(np.uint8)[:] = 0xEE
        info = np.zeros(1, RING_SCAN_DTYPE)
        hist = np.zeros(14, np.uint32)
        _lib.check("poll", _lib.lib.halo_rx_ring_poll(cons._h, 1, NetIf.make(), out.ctypes.data, hist.ctypes.data,
                                                      None, info.ctypes.data))
        n = int(info["n_frames"][0])
        assert n == len(sel)
        assert_records_equal(out[:n], want, None, f"unpinned out, registered ring={register}")
        assert np.all(out[n:].view(np.uint8) == 0xEE)
        assert np.array_equal(hist, np.bincount(want["status"], minlength=14))
        cons.commit()
        assert ring.tail == tail
        if register:  # the same array registered for one poll, unregistered for the next
            ring.write_batch(data, offs[sel].astype(np.uint64) * 4, lens[sel])
            _lib.check("register", _lib.lib.halo_rx_host_register(out.ctypes.data, _lib.host_pages(out.nbytes)))
            for k in range(2):
                if k:
                    _lib.check("unregister", _lib.lib.halo_rx_host_unregister(out.ctypes.data))
                    ring.write_batch(data, offs[sel].astype(np.uint64) * 4, lens[sel])
                out.view(np.uint8)[:] = 0xEE
                _lib.check("poll", _lib.lib.halo_rx_ring_poll(cons._h, 1, NetIf.make(), out.ctypes.data, None,
                                                              None, info.ctypes.data))
                assert int(info["n_frames"][0]) == len(sel)
                assert_records_equal(out[:len(sel)], want, None, f"out registered={not k}")
                cons.commit()
        cons.close()


def test_poll_large_imix_ring(dev, oracle_lib):
    """A 256 MiB ring holding ~700k synthetic IMIX frames (1/16 bit-flipped), drained in one poll
    (hundreds of superblocks): records == the per-frame oracle; histogram == records."""
    import torch

    from halo_amd import synth
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    n = 700_000
    lay = synth.layout(n, size_mode=synth.SIZE_IMIX, proto_mode=synth.PROTO_MIX, mutate_shift=4)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    host = fr["bytes"].cpu().numpy()
    ring = RingBuffer(256 << 20)
    _seek(ring, (256 << 20) - 4096)
    assert ring.write_batch(host, lay["offsets_dw"].astype(np.uint64) * 4, lay["lens"]) == n
    cons = RingConsumer(ring, capacity=1514, max_bytes=256 << 20)
    hist = np.zeros(14, np.uint32)
    got, info, _ = cons.poll(NetIf.make(), hist=hist)
    assert info["n_frames"] == n and info["stop"] == "EMPTY"
    want, whist = O.rx_batch(host, lay["lens"], O.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
    assert_records_equal(got.copy(), want, None, "256 MiB IMIX ring")
    assert np.array_equal(hist, whist)
    mutated = (lay["kinds"] & 0x80) != 0
    assert np.all(got["status"][~mutated] == 0) and np.all(got["status"][mutated] != 0)
    cons.commit()
    assert ring.tail == ring.head
    cons.close()
    del fr
    torch.cuda.empty_cache()


def test_wire_rx_batch(dev, golden, oracle_lib):
    """engine.Wire: Tx drops empty and > 1514 B frames; rx_batch returns what Wire.Rx would."""
    from halo_amd._lib import NetIf
    from halo_amd.ring import Wire

    O = oracle_lib
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    w = Wire()
    frames = [data[int(o) * 4:int(o) * 4 + int(ln)].tobytes() for o, ln in zip(offs, lens)]
    for f in frames:
        w.Tx(f)
    kept = [f for f in frames if 0 < len(f) <= 1514]
    recs, got_frames = w.rx_batch(NetIf.make())
    assert got_frames == kept
    want = np.concatenate([O.rx_frame(f, O.NetIf.make(), 1).reshape(1) for f in kept])
    assert recs.tobytes() == want.tobytes()
    w.Destroy()


def test_shard_multi_two_contexts_one_device(dev, oracle_lib):
    """halo_rx_shard_multi with two host contexts (on the one device here): byte-balanced index
    ranges, records in frame order == one context == the oracle."""
    import ctypes

    from halo_amd import _lib, synth
    from halo_amd._lib import NetIf
    from halo_amd.engine import HostBatcher

    O = oracle_lib
    lay = synth.layout(50_000, size_mode=synth.SIZE_IMIX, proto_mode=synth.PROTO_MIX, mutate_shift=3)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    host = fr["bytes"].cpu().numpy()
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    a, b = HostBatcher(0), HostBatcher(0)
    ctxs = (ctypes.c_void_p * 2)(a._ctx, b._ctx)
    out = np.zeros(50_000, _lib.RESULT_DTYPE)
    hist = np.zeros(14, np.uint32)
    first = np.zeros(3, np.uint32)
    rc = _lib.lib.halo_rx_shard_multi(ctxs, 2, host.ctypes.data, offs.ctypes.data, lay["lens"].ctypes.data, 50_000, 1,
                                      NetIf.make(), out.ctypes.data, hist.ctypes.data, first.ctypes.data)
    _lib.check("halo_rx_shard_multi", rc)
    want, whist = O.rx_batch(host, lay["lens"], O.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
    assert_records_equal(out, want, None, "shard_multi")
    assert np.array_equal(hist, whist)
    assert first[0] == 0 and first[2] == 50_000
    half = int(lay["lens"][:first[1]].astype(np.int64).sum())
    total = int(lay["lens"].astype(np.int64).sum())
    assert abs(half - total / 2) <= 1514
    a.close()
    b.close()


def test_registration_registry_refuses_shared_pages(dev):
    """Live registrations never share a page: a second registration or a registered ring attach
    touching a registered page is refused (HALO_E_INVAL), only the base of a live registration can
    be unregistered, and after unregistering the runtime no longer maps the range."""
    import ctypes
    import mmap

    from halo_amd import _lib
    from halo_amd.ring import RingBuffer, RingConsumer

    L, P = _lib.lib, mmap.PAGESIZE
    a = _lib.host_array(8 * P)
    base = a.ctypes.data
    _lib.check("register", L.halo_rx_host_register(base, 4 * P))
    try:
        assert _lib.registrations() == [(base, 4 * P)]
        assert L.halo_rx_host_register(base, 4 * P) == _lib.HALO_E_INVAL          # the same range
        assert L.halo_rx_host_register(base + P, P) == _lib.HALO_E_INVAL          # inside it
        assert L.halo_rx_host_register(base + 3 * P, 2 * P) == _lib.HALO_E_INVAL  # overlapping its end
        # a ring laid out on the registered pages cannot be attached registered
        mem = a[:128 + 4096]
        _lib.check("ring_create", L.halo_ring_create(mem.ctypes.data, mem.nbytes))
        h = ctypes.c_void_p()
        assert L.halo_rx_ring_attach(0, mem.ctypes.data, 0, 1514, 0, 0, _lib.RING_REGISTER,
                                     ctypes.byref(h)) == _lib.HALO_E_INVAL
        # the next page is free: a registration starting there is fine
        _lib.check("register next", L.halo_rx_host_register(base + 4 * P, P))
        assert _lib.registered_count() == 2
        assert L.halo_rx_host_unregister(base + P) == _lib.HALO_E_INVAL           # not a base
        _lib.check("unregister next", L.halo_rx_host_unregister(base + 4 * P))
        assert L.halo_rx_host_unregister(base + 4 * P) == _lib.HALO_E_INVAL       # already gone
    finally:
        _lib.check("unregister", L.halo_rx_host_unregister(base))
    assert _lib.registered_count() == 0
    # a ring consumer's ring and record array are two registrations, removed by close()
    ring = RingBuffer(1 << 16)
    cons = RingConsumer(ring, capacity=1514)
    regs = dict(_lib.registrations())
    assert regs.get(ring.mem.ctypes.data) == _lib.host_pages(ring.mem.nbytes), regs
    assert regs.get(cons._out.ctypes.data) == _lib.host_pages(cons._out.nbytes), regs
    cons.close()
    assert _lib.registered_count() == 0


def test_persistent_consumer_idle_exit_and_relaunch(dev, golden, oracle_lib):
    """HALO_RING_PERSISTENT: the resident consumer exits after 20 ms without a request and the next
    poll relaunches it; polls before and after, and a detach while it is idle or running, all give
    the oracle's records."""
    import time

    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    meta, blob = golden
    fr = [e for e in meta["frames"] if 0 < e["len"] <= 1514]
    offs = np.array([e["offset"] for e in fr], np.uint64)
    lens = np.array([e["len"] for e in fr], np.uint16)
    onetif = O.NetIf.make()
    for detach_idle in (False, True):
        ring = RingBuffer(1 << 20)
        cons = RingConsumer(ring, capacity=1514, persistent=True)
        for rnd in range(4):
            assert ring.write_batch(blob, offs, lens) == len(lens)
            got, info, _ = cons.poll(NetIf.make())
            assert info["n_frames"] == len(lens), (rnd, info)
            want_recs, _, _, _ = _oracle_drain(O, ring.mem, onetif, 1, 1514)
            assert_records_equal(got.copy(), want_recs, None, f"persistent round {rnd}")
            cons.commit()
            time.sleep(0.05 if rnd % 2 == 0 else 0.001)  # > 20 ms: the kernel exits; 1 ms: still resident
        if detach_idle:
            time.sleep(0.05)
        cons.close()


@pytest.mark.parametrize("persistent", [True, False], ids=["persistent", "launch"])
def test_small_polls_of_changing_sizes(dev, oracle_lib, persistent):
    """Small polls (served by the resident consumer, or one launch each) whose sizes cross 64-frame
    window edges and change from poll to poll (1 .. 2600 frames): polls of one frame length
    (64 B: the host walk's same-length run, and the uniform request / strided launch that needs no
    offset arrays) and of mixed 42..64 B lengths, an empty span, a poll cut by max_frames, and
    records into an array that is neither pinned nor registered: every poll's records, positions,
    stop and tail == the oracle."""
    from halo_amd import _lib
    from halo_amd._lib import RING_SCAN_DTYPE, NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    onetif = O.NetIf.make()
    rng = np.random.default_rng(29)
    ring = RingBuffer(1 << 22)
    _seek(ring, (1 << 36) + 4096)
    cons = RingConsumer(ring, capacity=1514, persistent=persistent, max_frames=2000, small_poll=16 << 20)
    plain = np.zeros(cons.max_frames, _lib.RESULT_DTYPE)  # neither pinned nor registered
    before = cons.stats()
    sizes = [1000, 1, 63, 64, 65, 1900, 2, 640, 0, 1000, 129, 2600, 1000, 1000]
    served = 0
    for it, k in enumerate(sizes):
        small = it % 2 == 1  # mixed 42..64 B lengths; even polls: 64 B frames (one same-length run)
        lens = (rng.integers(42, 65, size=k) if small else np.full(k, 64)).astype(np.uint16)
        kinds = rng.integers(0, 3, size=k).astype(np.uint8)
        offs = np.concatenate([[0], np.cumsum((lens.astype(np.int64) + 3) & ~3)[:-1]]).astype(np.uint32) // 4
        data = O.synth_batch(1000 + it, 0, lens, kinds, onetif, offsets_dw=offs) if k else np.zeros(4, np.uint8)
        if k and it % 3 == 2:  # a bit flip in one frame
            j = int(rng.integers(0, k))
            data[int(offs[j]) * 4 + int(rng.integers(14, int(lens[j])))] ^= 1 << int(rng.integers(0, 8))
        start = ring.head
        if k:
            assert ring.write_batch(data, offs.astype(np.uint64) * 4, lens) == k
        want_n = min(k, cons.max_frames)
        want, _ = O.rx_batch(data, lens[:want_n], onetif, 1, offsets_dw=offs[:want_n]) if want_n else (None, None)
        served += 0 < min(k, cons.max_frames)
        if it in (5, 6):  # records into plain memory: the library stages them
            info = np.zeros(1, RING_SCAN_DTYPE)
            pos = np.zeros(cons.max_frames, np.uint64)
            _lib.check("poll", _lib.lib.halo_rx_ring_poll(cons._h, 1, NetIf.make(), plain.ctypes.data, None,
                                                          pos.ctypes.data, info.ctypes.data))
            n, stop = int(info["n_frames"][0]), int(info["stop"][0])
            got, pos = plain[:n], pos[:n]
        else:
            got, d, pos = cons.poll(NetIf.make(), positions=True)
            n, stop = d["n_frames"], {"EMPTY": 0, "MAX": 4}.get(d["stop"], -1)
        assert n == want_n, (it, k, n)
        assert stop == (4 if k > cons.max_frames else 0), (it, stop)
        if n:
            assert_records_equal(got.copy(), want, None, f"poll {it} ({k} frames)")
            rec = np.concatenate([[0], np.cumsum(4 + ((lens[:n].astype(np.int64) + 3) & ~3))[:-1]])
            assert np.array_equal(pos, start + rec)
        cons.commit()
        if k > cons.max_frames:  # the rest in the next poll
            got, d, _ = cons.poll(NetIf.make())
            rest, _ = O.rx_batch(data, lens[want_n:], onetif, 1, offsets_dw=offs[want_n:])
            assert d["n_frames"] == k - want_n
            assert_records_equal(got.copy(), rest, None, f"poll {it} rest")
            cons.commit()
        assert ring.tail == ring.head
    st = cons.stats()
    got_small = st["small_polls"] - before["small_polls"]
    assert got_small >= served > 10  # every poll with frames took the small path
    if persistent:
        assert st["service_requests"] - before["service_requests"] >= served
    cons.close()


def test_persistent_consumer_after_small_poll_growth(dev, oracle_lib):
    """growing the small-poll arrays (halo_rx_ring_set_small_poll above the 4 MiB
    default on a ring large enough for them to grow) frees the pinned offset / length arrays the
    resident consumer was created over. The consumer must relaunch over the new ones: ragged polls
    (42..64 B, read through the arrays) before and after two growths, each == the oracle."""
    from halo_amd import _lib
    from halo_amd._lib import NetIf
    from halo_amd.ring import RingBuffer, RingConsumer

    O = oracle_lib
    onetif = O.NetIf.make()
    rng = np.random.default_rng(31)
    ring = RingBuffer(1 << 24)
    cons = RingConsumer(ring, capacity=1514, persistent=True)
    assert cons.max_frames > (4 << 20) // 8  # room for the arrays to grow past the default's
    for it, small_poll in enumerate([None, 8 << 20, 16 << 20]):
        if small_poll is not None:
            _lib.check("halo_rx_ring_set_small_poll", _lib.lib.halo_rx_ring_set_small_poll(cons._h, small_poll))
        for rep in range(2):
            k = int(rng.integers(500, 3000))
            lens = rng.integers(42, 65, size=k).astype(np.uint16)
            kinds = rng.integers(0, 3, size=k).astype(np.uint8)
            offs = np.concatenate([[0], np.cumsum((lens.astype(np.int64) + 3) & ~3)[:-1]]).astype(np.uint32) // 4
            data = O.synth_batch(7000 + 10 * it + rep, 0, lens, kinds, onetif, offsets_dw=offs)
            assert ring.write_batch(data, offs.astype(np.uint64) * 4, lens) == k
            want, _ = O.rx_batch(data, lens, onetif, 1, offsets_dw=offs)
            got, d, _ = cons.poll(NetIf.make())
            assert d["n_frames"] == k
            assert_records_equal(got.copy(), want, None, f"growth {it} poll {rep}")
            cons.commit()
    st = cons.stats()
    assert st["service_requests"] >= 6 and st["small_polls"] >= 6, st
    cons.close()
