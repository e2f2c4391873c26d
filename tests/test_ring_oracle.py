"""CPU: halo's SPSC packet ring (BASELINE config 1).

Pins oracle/halo_ring_oracle.c (the C restatement of mem/ring_buffer.go) against the
REFERENCE's own C ring, cgo/ring_buffer.h, compiled from where it lies into oracle/_ref/
(`make -C oracle ref`; skipped where /root/reference is absent): identical ring memory, return
values and frames over random write/read sequences with wrap-around, corrupt and oversize
records. Then the oracle's other ring functions (the batch walk, the config-1 PacketHandle loop)
are checked against that pinned read loop, and the product's producer (halo_ring_write_batch)
and attach validation run without a GPU.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = "/root/reference"
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_ring.so")


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(os.path.join(REF_DIR, "cgo", "ring_buffer.h")):
        pytest.skip("reference sources absent (GPU box): the ring is pinned in the build container")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    L = ctypes.CDLL(REF_LIB)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.ref_ring_create.restype = vp
    L.ref_ring_create.argtypes = [vp, u64]
    L.ref_ring_mapping.restype = vp
    L.ref_ring_mapping.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
    L.ref_producer_new.restype = vp
    L.ref_producer_new.argtypes = [vp, ctypes.c_int64]
    L.ref_consumer_new.restype = vp
    L.ref_consumer_new.argtypes = [vp, ctypes.c_int64]
    L.ref_free.restype = None
    L.ref_free.argtypes = [vp]
    L.ref_write.restype = ctypes.c_int
    L.ref_write.argtypes = [vp, vp, u32]
    L.ref_read.restype = ctypes.c_int
    L.ref_read.argtypes = [vp, vp, u32, ctypes.POINTER(u32)]
    return L


def _same_ring(a: np.ndarray, b: np.ndarray):
    """Ring memories equal except the stored buffer pointer (bytes 88..95: each its own address)."""
    assert np.array_equal(a[:88], b[:88]), "headers differ"
    assert np.array_equal(a[96:], b[96:]), "headers / data differ"


def _frame(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("data_size,seed", [(64, 1), (256, 2), (4096, 3), (4096, 4), (1 << 16, 5)])
def test_restatement_matches_reference_ring(oracle_lib, ref, data_size, seed):
    O = oracle_lib
    rng = np.random.default_rng(seed)
    ref_mem = O.aligned_zeros(128 + data_size)
    assert ref.ref_ring_create(ref_mem.ctypes.data, ref_mem.nbytes)
    ora = O.Ring(data_size)
    _same_ring(ref_mem, ora.mem)
    prod = ref.ref_producer_new(ref_mem.ctypes.data, 0)
    cons = ref.ref_consumer_new(ref_mem.ctypes.data, 0)
    assert prod and cons
    try:
        for step in range(3000):
            if rng.random() < 0.55:
                kind = rng.random()
                ln = (0 if kind < 0.03 else int(rng.integers(data_size // 2 + 1, data_size + 9)) if kind < 0.08
                      else int(rng.integers(1, max(2, min(1600, data_size // 2 + 1)))))
                f = _frame(rng, ln)
                b = np.frombuffer(f + b"\0", np.uint8)
                got = ora.write(f)
                want = bool(ref.ref_write(prod, b.ctypes.data, ln))
                assert got == want, (step, "write", ln)
            else:
                cap = int(rng.choice([0, 1, 7, 64, 1514, data_size]))
                buf = np.zeros(max(1, cap), np.uint8)
                ln = ctypes.c_uint32()
                want = bool(ref.ref_read(cons, buf.ctypes.data, cap, ctypes.byref(ln)))
                got, frame, gl = ora.read(cap)
                assert got == want and gl == ln.value, (step, "read", cap, gl, ln.value)
                if got:
                    assert frame == buf[:ln.value].tobytes()
            _same_ring(ref_mem, ora.mem)
    finally:
        ref.ref_free(prod)
        ref.ref_free(cons)


def test_product_producer_matches_reference(ref):
    """halo_ring_create + halo_ring_write_batch (the product's producer side) write the same
    ring memory as the reference's ring_buffer_create + ring_buffer_producer_write_packet, and
    the reference's own mapping check accepts the product's ring."""
    from halo_amd.ring import RingBuffer

    rng = np.random.default_rng(7)
    size = 1 << 14
    prod_ring = RingBuffer(size)
    from oracle.oracle import aligned_zeros

    ref_mem = aligned_zeros(128 + size)
    assert ref.ref_ring_create(ref_mem.ctypes.data, ref_mem.nbytes)
    _same_ring(ref_mem, prod_ring.mem)
    off = ctypes.c_int64(99)
    assert ref.ref_ring_mapping(prod_ring.mem.ctypes.data, ctypes.byref(off)) and off.value == 0
    p = ref.ref_producer_new(ref_mem.ctypes.data, 0)
    c = ref.ref_consumer_new(ref_mem.ctypes.data, 0)
    try:
        for rnd in range(40):
            lens = rng.integers(0, 1600, int(rng.integers(1, 30))).astype(np.uint16)
            lens[rng.random(lens.shape[0]) < 0.05] = 0
            offs = np.zeros(lens.shape[0], np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
            data = rng.integers(0, 256, int(lens.astype(np.int64).sum()) + 1, dtype=np.uint8)
            acc = np.zeros(lens.shape[0], np.uint8)
            n = prod_ring.write_batch(data, offs, lens, accepted=acc)
            want = [bool(ref.ref_write(p, data.ctypes.data + int(o), int(ln))) for o, ln in zip(offs, lens)]
            assert list(acc.astype(bool)) == want and n == sum(want)
            _same_ring(ref_mem, prod_ring.mem)
            # consume a random number of records on both rings (reference consumer on both)
            c2 = ref.ref_consumer_new(prod_ring.mem.ctypes.data, 0)
            buf = np.zeros(2048, np.uint8)
            ln = ctypes.c_uint32()
            for _ in range(int(rng.integers(0, 40))):
                a = ref.ref_read(c, buf.ctypes.data, 2048, ctypes.byref(ln))
                b = ref.ref_read(c2, buf.ctypes.data, 2048, ctypes.byref(ln))
                assert a == b
            ref.ref_free(c2)
            _same_ring(ref_mem, prod_ring.mem)
    finally:
        ref.ref_free(p)
        ref.ref_free(c)


def _fill_ring_states(O, rng, data_size, n_frames, corrupt=False):
    """A ring moved to a random stream position, then filled with random records (optionally a
    corrupt length field somewhere)."""
    ring = O.Ring(data_size)
    ring.set_cursors(int(rng.integers(0, 1 << 40)) * 4)
    frames = []
    for k in range(n_frames):
        ln = int(rng.choice([1, 2, 3, 5, 42, 60, 64, 570, 1500, 1514, 1515, 2000, 9000]))
        if ln > data_size // 2:
            ln = int(rng.integers(1, data_size // 2 + 1))
        f = _frame(rng, ln)
        if not ring.write(f):
            break
        frames.append(f)
    if corrupt and frames:
        ring.write_raw(int(rng.choice([0, data_size // 2 + 4, 0xFFFFFFFF])), b"\xee" * 8)
    return ring, frames


def _unwrapped(ring, used):
    start = ring.tail % ring.size
    idx = (start + np.arange(used)) % ring.size
    return ring.mem[128:][idx]


@pytest.mark.parametrize("seed", range(6))
def test_ring_scan_matches_read_loop(oracle_lib, seed):
    """ora_ring_scan (the walk the GPU restates) == repeated ora_ring_read (pinned above)."""
    O = oracle_lib
    rng = np.random.default_rng(100 + seed)
    data_size = [1 << 12, 1 << 14, 1 << 16][seed % 3]
    ring, frames = _fill_ring_states(O, rng, data_size, 400, corrupt=seed % 2 == 1)
    used = ring.head - ring.tail
    span = _unwrapped(ring, used)
    for cap in (1514, 64, 16376):
        for max_frames in (0xFFFFFFFF, 3, len(frames)):
            off, lens, stop, end, ml = O.ring_scan(span, used, ring.size, cap, max_frames)
            r2 = O.Ring(mem=ring.mem.copy())
            want_pos, want_len = [], []
            while len(want_len) < max_frames:
                before = r2._ct.value
                ok, f, ln = r2.read(cap)
                if not ok:
                    break
                want_pos.append(before - ring.tail)
                want_len.append(ln)
            assert list(lens) == want_len
            assert list((off.astype(np.int64) - 1) * 4) == want_pos
            assert end == r2._ct.value - ring.tail
            assert ml == (max(want_len) if want_len else 0)
            another = r2.read(cap)[0]  # would ReadPacket have returned one more frame?
            assert (stop == O.RING_STOP["MAX"]) == (len(want_len) == max_frames and another)
            if stop == O.RING_STOP["EMPTY"]:
                assert end == used and not another


def test_packet_handle_over_ring_equals_per_frame_parse(oracle_lib, golden):
    """Config 1's loop (ReadPacket -> RxEthernet over a Wire-sized ring) == the per-frame oracle."""
    from tests.helpers import golden_arrays

    O = oracle_lib
    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    ring = O.Ring(8 << 20)
    ring.set_cursors((8 << 20) - 1024)  # the frames wrap around the end of the data area
    accepted = []
    for o, ln in zip(offs, lens):
        accepted.append(ring.write(data[int(o) * 4:int(o) * 4 + int(ln)].tobytes()))
    netif = O.NetIf.make()
    for flags in (0, 1, 3):
        r2 = O.Ring(mem=ring.mem.copy())
        recs, acts, pos, (fb, fo) = r2.packet_handle(netif, flags, capacity=1514, frames=True)
        keep = np.array([a and 0 < ln <= 1514 for a, ln in zip(accepted, lens)])
        # ReadPacket stops at the first record longer than the buffer and leaves it there
        first_big = next((i for i, ln in enumerate(lens) if accepted[i] and ln > 1514), len(lens))
        sel = [i for i in range(first_big) if keep[i]]
        assert len(recs) == len(sel)
        want, _ = O.rx_batch(data, lens[sel], netif, flags, offsets_dw=offs[sel])
        assert recs.tobytes() == want.tobytes()
        assert np.array_equal(acts, O.engine_batch(data, lens[sel], netif, flags, offsets_dw=offs[sel]))


def test_ring_attach_validation_without_gpu():
    """halo_rx_ring_attach checks the header like ring_buffer_mapping before touching a device."""
    import torch

    from halo_amd import _lib
    from halo_amd.ring import RingBuffer

    L = _lib.lib
    h = ctypes.c_void_p()
    rb = RingBuffer(1 << 12)

    def attach(mem, offset=0, cap=0):
        return L.halo_rx_ring_attach(0, mem.ctypes.data, offset, cap, 0, 0, 0, ctypes.byref(h))

    def corrupted(byte, value):
        m = rb.mem
        old = int(m[byte])
        m[byte] = value
        rc = attach(m)
        m[byte] = old
        return rc

    assert corrupted(8, 2) == -1        # layout version
    assert corrupted(30, 0) == -1       # 0xAA fill
    assert corrupted(100, 0) == -1      # 0xFF fill
    assert corrupted(72, 7) == -1       # size not a power of two
    assert corrupted(80, 0) == -1       # mask != size - 1
    assert attach(rb.mem, offset=64) == -1  # mapping offset mismatch
    assert attach(rb.mem, cap=20000) == -1  # capacity beyond the tile window
    rb.mem[0:8].view(np.uint64)[0] = (1 << 12) + 8  # head - tail > size
    assert attach(rb.mem) == -1
    rb.mem[0:8].view(np.uint64)[0] = 0
    if not torch.cuda.is_available():
        assert attach(rb.mem) == _lib.HALO_E_NODEV
    # the device-side walk validates its arguments first too
    info = np.zeros(1, _lib.RING_SCAN_DTYPE)
    assert L.halo_rx_ring_scan_device(None, 6, 1 << 12, 0, 0, None, None, info.ctypes.data, None, 0, None) == -1
    assert L.halo_rx_ring_scan_device(None, 8, 12, 0, 0, None, None, info.ctypes.data, None, 0, None) == -1
    assert L.halo_rx_ring_scan_workspace(1 << 20, 1514) > 0
    assert L.halo_rx_ring_scan_workspace(1 << 20, 20000) == 0


def test_shard_multi_validation_without_gpu():
    from halo_amd import _lib

    L, n = _lib.lib, _lib.NetIf.make()
    out = np.zeros(4, _lib.RESULT_DTYPE)
    assert L.halo_rx_shard_multi(None, 1, None, None, None, 0, 1, n, out.ctypes.data, None, None) == -1
    ctxs = (ctypes.c_void_p * 2)(None, None)
    assert L.halo_rx_shard_multi(ctxs, 2, None, None, None, 0, 1, n, out.ctypes.data, None, None) == -1
    assert L.halo_rx_shard_multi(ctxs, 0, None, None, None, 0, 1, n, out.ctypes.data, None, None) == -1
