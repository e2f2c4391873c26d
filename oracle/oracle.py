"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (halo_rx_oracle.c).

The C restatement of protocol.Parse* / GetCheckSum / engine.RxEthernet->RxIpv4->Rx* (see
the file header of halo_rx_oracle.c for the reference lines it follows). Used as the
parity checker in tests/ and smoke(), and timed as bench.py's cpu_baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

RESULT_DTYPE = np.dtype([
    ("status", "u1"), ("flags", "u1"), ("ethertype", "<u2"),
    ("ip_proto", "u1"), ("l4_aux", "u1"), ("ip_total_len", "<u2"),
    ("src_ip", "<u4"), ("dst_ip", "<u4"),
    ("sport", "<u2"), ("dport", "<u2"),
    ("payload_off", "<u2"), ("payload_len", "<u2"),
    ("l4_seq", "<u4"), ("l4_ack", "<u4"),
])
STATUS_COUNT = 14
TX_OP_DTYPE = np.dtype([("steps", "u1"), ("pad", "u1"), ("dst_port", "<u2"), ("dst_ip", "<u4"),
                        ("src_port", "<u2"), ("pad2", "<u2"), ("src_ip", "<u4")])


class NetIf(ctypes.Structure):
    _fields_ = [("mac", ctypes.c_uint8 * 6), ("pad", ctypes.c_uint8 * 2), ("ip", ctypes.c_uint32),
                ("nat_enable", ctypes.c_uint32)]

    @classmethod
    def make(cls, mac="AA:AA:AA:AA:AA:AA", ip="192.168.100.100", nat_enable=False):
        n = cls()
        for i, p in enumerate(mac.split(":")[:6]):
            n.mac[i] = int(p, 16)
        a = [int(x) for x in ip.split(".")]
        n.ip = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]
        n.nat_enable = int(nat_enable)
        return n


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("halo_rx_oracle.c", "halo_tx_oracle.c", "halo_xxh3_oracle.c",
                                            "halo_route_oracle.c", "halo_ring_oracle.c")]
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(map(os.path.getmtime, srcs)):
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "liboracle.so"], check=True)
    if os.path.exists("/root/reference/cgo/ring_buffer.h"):
        # the reference's own C ring, compiled from where it lies (build container only; the
        # GPU box has no /root/reference and uses the prebuilt oracle/_ref files if any)
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.ora_get_checksum.restype = ctypes.c_uint16
        L.ora_get_checksum.argtypes = [vp, ctypes.c_size_t]
        L.ora_rx_frame.restype = None
        L.ora_rx_frame.argtypes = [vp, u32, u32, ctypes.POINTER(NetIf), vp]
        L.ora_engine_rx.restype = ctypes.c_int
        L.ora_engine_rx.argtypes = [vp, u32, u32, ctypes.POINTER(NetIf)]
        L.ora_rx_batch.restype = ctypes.c_int
        L.ora_rx_batch.argtypes = [vp, vp, vp, u64, u32, u32, u32, ctypes.POINTER(NetIf), vp, vp, ctypes.c_int]
        L.ora_rx_batch_reps.restype = ctypes.c_int
        L.ora_rx_batch_reps.argtypes = [vp, vp, vp, u64, u32, u32, u32, ctypes.POINTER(NetIf), vp, vp, ctypes.c_int, u32]
        L.ora_engine_lo.restype = ctypes.c_int
        L.ora_engine_lo.argtypes = [vp, u32, u32, ctypes.POINTER(NetIf)]
        L.ora_engine_batch.restype = None
        L.ora_engine_batch.argtypes = [vp, vp, vp, u64, u32, u32, u32, ctypes.POINTER(NetIf), vp]
        L.ora_synth_kind.restype = None
        L.ora_synth_kind.argtypes = [u64, u64, u32, u32, u32, u32, vp, vp]
        L.ora_synth_frame.restype = None
        L.ora_synth_frame.argtypes = [u64, u64, u32, ctypes.c_uint8, ctypes.POINTER(NetIf), vp]
        L.ora_tx_frame.restype = ctypes.c_uint8
        L.ora_tx_frame.argtypes = [vp, u32, vp, u32]
        L.ora_xxh3_64.restype = ctypes.c_uint64
        L.ora_xxh3_64.argtypes = [vp, ctypes.c_size_t]
        L.ora_xxh3_batch.restype = None
        L.ora_xxh3_batch.argtypes = [vp, vp, vp, u32, vp]
        L.ora_flow_hash_batch.restype = None
        L.ora_flow_hash_batch.argtypes = [vp, u32, u32, u32, vp, u32, vp]
        L.ora_route_create.restype = vp
        L.ora_route_create.argtypes = []
        L.ora_route_destroy.restype = None
        L.ora_route_destroy.argtypes = [vp]
        L.ora_route_update.restype = u32
        L.ora_route_update.argtypes = [vp, vp, vp]
        L.ora_route_find.restype = u32
        L.ora_route_find.argtypes = [vp, u32]
        L.ora_route_find_batch.restype = None
        L.ora_route_find_batch.argtypes = [vp, vp, u32, vp]
        L.ora_tx_batch.restype = ctypes.c_int
        L.ora_tx_batch.argtypes = [vp, vp, vp, u32, vp, u32, vp, ctypes.c_int]
        L.ora_icmp_quote.restype = None
        L.ora_icmp_quote.argtypes = [vp, u32, u32, vp]
        L.ora_icmp_deep_nat.restype = ctypes.c_int
        L.ora_icmp_deep_nat.argtypes = [vp, u32, u32, u32, ctypes.c_uint16, ctypes.c_int]
        L.ora_tx_build_batch.restype = ctypes.c_int
        L.ora_tx_build_batch.argtypes = [vp, u32, vp, u32, vp, vp, u32, vp, vp, ctypes.POINTER(ctypes.c_uint16)]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.ora_ring_create.restype = ctypes.c_int
        L.ora_ring_create.argtypes = [vp, u64]
        L.ora_ring_cursor.restype = None
        L.ora_ring_cursor.argtypes = [vp, ctypes.c_int, u64p, u64p]
        L.ora_ring_write.restype = ctypes.c_int
        L.ora_ring_write.argtypes = [vp, u64p, u64p, vp, u32]
        L.ora_ring_read.restype = ctypes.c_int
        L.ora_ring_read.argtypes = [vp, u64p, u64p, vp, u32, u32p]
        L.ora_ring_packet_handle.restype = u32
        L.ora_ring_packet_handle.argtypes = [vp, u64p, u64p, u32, u32, u32, ctypes.POINTER(NetIf), vp, vp, vp, vp,
                                             vp]
        L.ora_ring_scan.restype = u32
        L.ora_ring_scan.argtypes = [vp, u64, u64, u32, u32, vp, vp, u32p, u64p, u32p]
        L.ora_fuzz_layout.restype = u64
        L.ora_fuzz_layout.argtypes = [u64, u32, vp, vp]
        L.ora_fuzz_fill.restype = None
        L.ora_fuzz_fill.argtypes = [u64, u32, vp, vp, ctypes.POINTER(NetIf), vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def get_checksum(data: bytes) -> int:
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    return lib().ora_get_checksum(_p(b) if len(b) else None, len(b))


def rx_frame(frame: bytes, netif: NetIf, flags: int = 1) -> np.ndarray:
    b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8)
    out = np.zeros(1, dtype=RESULT_DTYPE)
    lib().ora_rx_frame(_p(b), len(frame), flags, netif, _p(out))
    return out[0]


def engine_rx(frame: bytes, netif: NetIf, flags: int = 1) -> int:
    b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8)
    return lib().ora_engine_rx(_p(b), len(frame), flags, netif)


def engine_lo(packet: bytes, netif: NetIf, flags: int = 1) -> int:
    """PacketHandle's LoChan drain decision for one packet (ora_engine_lo)."""
    b = np.frombuffer(bytes(packet) + b"\0", dtype=np.uint8)
    return lib().ora_engine_lo(_p(b), len(packet), flags, netif)


def rx_batch(data: np.ndarray, lens: np.ndarray, netif: NetIf, flags: int = 1, offsets_dw=None, stride: int = 0,
             length: int = 0, threads: int = 1, reps: int = 1, out=None):
    """Returns (records, status histogram). `reps`: every thread parses its shard that many times
    (timing: one thread start per measurement). `out`: a RESULT_DTYPE array of n records to reuse
    (timing: no fresh allocation per call)."""
    n = int(lens.shape[0]) if lens is not None else int(data.shape[0] // stride)
    if out is None:
        out = np.zeros(n, dtype=RESULT_DTYPE)
    assert out.dtype == RESULT_DTYPE and out.shape[0] >= n and out.flags.c_contiguous
    hist = np.zeros(STATUS_COUNT, dtype=np.uint32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    lens_c = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    offs_c = None if offsets_dw is None else np.ascontiguousarray(offsets_dw, dtype=np.uint32)
    rc = lib().ora_rx_batch_reps(_p(data), _p(offs_c), _p(lens_c), stride, length, n, flags, netif, _p(out),
                                 _p(hist), threads, reps)
    assert rc == 0
    return out, hist


def engine_batch(data, lens, netif, flags=1, offsets_dw=None, stride=0, length=0) -> np.ndarray:
    n = int(lens.shape[0])
    acts = np.zeros(n, dtype=np.uint8)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    lens_c = np.ascontiguousarray(lens, dtype=np.uint16)
    offs_c = None if offsets_dw is None else np.ascontiguousarray(offsets_dw, dtype=np.uint32)
    lib().ora_engine_batch(_p(data), _p(offs_c), _p(lens_c), stride, length, n, flags, netif, _p(acts))
    return acts


def synth_kind(seed, index, size_mode=0, length=64, proto_mode=0, mutate_shift=0):
    L = np.zeros(1, np.uint16)
    k = np.zeros(1, np.uint8)
    lib().ora_synth_kind(seed, index, size_mode, length, proto_mode, mutate_shift, _p(L), _p(k))
    return int(L[0]), int(k[0])


def synth_frame(seed: int, index: int, length: int, kind: int, netif: NetIf) -> bytes:
    f = np.zeros(length, dtype=np.uint8)
    lib().ora_synth_frame(seed, index, length, kind, netif, _p(f))
    return f.tobytes()


def synth_batch(seed, first_index, lens, kinds, netif, offsets_dw=None, stride=0, fill=0) -> np.ndarray:
    """Host twin of halo_synth_frames_device: the same bytes laid out the same way."""
    n = len(lens)
    if offsets_dw is not None:
        total = (int(offsets_dw[-1]) * 4 + ((int(lens[-1]) + 3) & ~3)) if n else 0
    else:
        total = stride * n
    buf = np.full(max(16, (total + 15) & ~15), fill, dtype=np.uint8)
    for k in range(n):
        start = int(offsets_dw[k]) * 4 if offsets_dw is not None else k * stride
        L = int(lens[k])
        buf[start:start + L] = np.frombuffer(synth_frame(seed, first_index + k, L, int(kinds[k]), netif), np.uint8)
    return buf


def tx_frame(frame: bytes, op: np.void, flags: int = 1):
    """Returns (rewritten frame bytes, HALO_TX_R_* byte)."""
    b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8).copy()
    o = np.array([op], dtype=TX_OP_DTYPE)
    r = lib().ora_tx_frame(_p(b), len(frame), _p(o), flags)
    return b[:len(frame)].tobytes(), int(r)


def tx_batch(data: np.ndarray, offsets_dw: np.ndarray, lens: np.ndarray, ops: np.ndarray, flags: int = 1,
             threads: int = 1):
    """Rewrites a COPY of `data`; returns (new data, result bytes)."""
    out = np.array(data, dtype=np.uint8, copy=True)
    n = int(lens.shape[0])
    res = np.zeros(n, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets_dw, dtype=np.uint32)
    lens_c = np.ascontiguousarray(lens, dtype=np.uint16)
    ops_c = np.ascontiguousarray(ops, dtype=TX_OP_DTYPE)
    assert lib().ora_tx_batch(_p(out), _p(offs), _p(lens_c), n, _p(ops_c), flags, _p(res), threads) == 0
    return out, res


# halo_tx_build_desc_t (40 B), include/halo_rx.h
BUILD_DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("payload_len", "<u2"), ("proto", "u1"), ("aux", "u1"),
                             ("src_port", "<u2"), ("dst_port", "<u2"), ("src_ip", "<u4"), ("dst_ip", "<u4"),
                             ("seq", "<u4"), ("ack", "<u4"), ("dst_mac", "u1", (6,)), ("mode", "u1"),
                             ("pad", "u1")])
assert BUILD_DESC_DTYPE.itemsize == 40


def tx_build_batch(desc: np.ndarray, payload: np.ndarray, src_mac: bytes, flags: int = 1, out_stride: int = 1516,
                   ip_id: int = 0):
    """The Build* chain over a descriptor batch (ora_tx_build_batch): (frames [n, out_stride] with
    untouched slot bytes 0, lens, results, new iphId)."""
    desc = np.ascontiguousarray(desc, dtype=BUILD_DESC_DTYPE)
    n = int(desc.shape[0])
    pay = np.ascontiguousarray(payload, dtype=np.uint8)
    frames = np.zeros((max(n, 1), out_stride), dtype=np.uint8)
    lens = np.zeros(max(n, 1), dtype=np.uint16)
    res = np.zeros(max(n, 1), dtype=np.uint8)
    mac = np.frombuffer(bytes(src_mac), dtype=np.uint8).copy()
    iph = ctypes.c_uint16(ip_id)
    assert lib().ora_tx_build_batch(_p(desc), n, _p(pay), flags, _p(mac), _p(frames), out_stride, _p(lens), _p(res),
                                    ctypes.byref(iph)) == 0
    return frames[:n], lens[:n], res[:n], int(iph.value)


def icmp_quote(frame: bytes, flags: int = 1) -> np.ndarray:
    """IcmpTtlDeepNat's checks up to its NAT lookup, as a record (ora_icmp_quote)."""
    b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8)
    out = np.zeros(1, dtype=RESULT_DTYPE)
    lib().ora_icmp_quote(_p(b), len(frame), flags, _p(out))
    return out[0]


def icmp_deep_nat(frame: bytes, lan_ip: int, lan_port: int, found: bool, flags: int = 1):
    """IcmpTtlDeepNat on a copy of the frame: (rewritten frame bytes, isIcmpTtl)."""
    b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8).copy()
    ok = lib().ora_icmp_deep_nat(_p(b), len(frame), flags, lan_ip, lan_port, int(found))
    return b[:len(frame)].tobytes(), bool(ok)


def xxh3_64(data: bytes) -> int:
    b = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    return int(lib().ora_xxh3_64(_p(b), len(data)))


def xxh3_batch(data: np.ndarray, offsets: np.ndarray, lens: np.ndarray) -> np.ndarray:
    n = int(lens.shape[0])
    out = np.zeros(n, dtype=np.uint64)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    lib().ora_xxh3_batch(_p(data), _p(np.ascontiguousarray(offsets, np.uint64)),
                         _p(np.ascontiguousarray(lens, np.uint32)), n, _p(out))
    return out


def flow_hash_batch(records: np.ndarray, kind: int, nat_type: int, bucket_count: int = 0):
    """(hash u64[n], bucket u32[n] or None) for halo_rx_result_t records."""
    recs = np.ascontiguousarray(records).view(RESULT_DTYPE)
    n = recs.shape[0]
    h = np.zeros(n, dtype=np.uint64)
    b = np.zeros(n, dtype=np.uint32) if bucket_count else None
    lib().ora_flow_hash_batch(_p(recs), n, kind, nat_type, _p(h), bucket_count, _p(b))
    return h, b


ROUTE_DTYPE = np.dtype([("dst_ip", "<u4"), ("network_mask", "<u4"), ("next_hop", "<u4"), ("netif", "<u4")])


class RouteTable:
    """The C restatement of engine.RouteTable (oracle/halo_route_oracle.c)."""

    def __init__(self):
        self._t = lib().ora_route_create()

    def __del__(self):
        if getattr(self, "_t", None):
            lib().ora_route_destroy(self._t)
            self._t = None

    def update(self, old, new=None) -> int:
        o = np.array([tuple(old)], ROUTE_DTYPE)
        n = None if new is None else np.array([tuple(new)], ROUTE_DTYPE)
        return int(lib().ora_route_update(self._t, _p(o), _p(n)))

    def add(self, r) -> int:
        return self.update(r, r)

    def delete(self, r) -> None:
        self.update(r, None)

    def find(self, ip: int) -> int:
        return int(lib().ora_route_find(self._t, ip))

    def find_batch(self, ips: np.ndarray) -> np.ndarray:
        ips = np.ascontiguousarray(ips, np.uint32)
        out = np.zeros(ips.shape[0], np.uint32)
        lib().ora_route_find_batch(self._t, _p(ips), ips.shape[0], _p(out))
        return out


# ---- halo's SPSC packet ring (oracle/halo_ring_oracle.c) ---------------------------------------
RING_HEADER = 128
RING_STOP = {"EMPTY": 0, "BAD_LEN": 1, "PARTIAL": 2, "CAPACITY": 3, "MAX": 4, "BAD_CURSOR": 5}


def aligned_zeros(nbytes: int, align: int = 64) -> np.ndarray:
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


class Ring:
    """A RingBuffer (mem/ring_buffer.go:18-26) in host memory owned by this object, with one
    producer and one consumer cursor (WritePacket / ReadPacket restated in C)."""

    def __init__(self, data_size: int = 8 << 20, mem: np.ndarray | None = None):
        self.mem = aligned_zeros(RING_HEADER + data_size) if mem is None else mem
        self.size = self.mem.nbytes - RING_HEADER
        if mem is None:
            assert lib().ora_ring_create(_p(self.mem), self.mem.nbytes) == 0
        self._ph, self._pt = ctypes.c_uint64(), ctypes.c_uint64()
        self._ct, self._ch = ctypes.c_uint64(), ctypes.c_uint64()
        lib().ora_ring_cursor(_p(self.mem), 0, ctypes.byref(self._ph), ctypes.byref(self._pt))
        lib().ora_ring_cursor(_p(self.mem), 1, ctypes.byref(self._ct), ctypes.byref(self._ch))

    @property
    def head(self) -> int:
        return int(self.mem[0:8].view(np.uint64)[0])

    @property
    def tail(self) -> int:
        return int(self.mem[64:72].view(np.uint64)[0])

    def set_cursors(self, pos: int):
        """An empty ring whose head and tail both sit at stream position `pos` (a restarted
        producer/consumer pair that already moved pos bytes through)."""
        self.mem[0:8].view(np.uint64)[0] = pos
        self.mem[64:72].view(np.uint64)[0] = pos
        self._ph.value = self._pt.value = self._ct.value = self._ch.value = pos

    def write(self, frame: bytes) -> bool:
        b = np.frombuffer(bytes(frame) + b"\0", dtype=np.uint8)
        return bool(lib().ora_ring_write(_p(self.mem), ctypes.byref(self._ph), ctypes.byref(self._pt), _p(b),
                                         len(frame)))

    def write_raw(self, length_field: int, payload: bytes = b"") -> None:
        """A record whose length field is `length_field` whatever the payload (corrupt records),
        then head advanced by the record size the field implies, capped at the ring size."""
        pos = self.head & (self.size - 1)
        self.mem[RING_HEADER + pos:RING_HEADER + pos + 4] = np.frombuffer(
            np.uint32(length_field).tobytes(), np.uint8)
        for k, byte in enumerate(payload):
            self.mem[RING_HEADER + (pos + 4 + k) % self.size] = byte
        adv = min(((4 + length_field + 3) & ~3), self.size - (self.head - self.tail))
        self.mem[0:8].view(np.uint64)[0] = self.head + adv
        self._ph.value = self.head

    def read(self, capacity: int = 1514):
        """(ok, frame bytes or None, length)"""
        buf = np.zeros(max(1, capacity), np.uint8)
        ln = ctypes.c_uint32()
        ok = lib().ora_ring_read(_p(self.mem), ctypes.byref(self._ct), ctypes.byref(self._ch), _p(buf), capacity,
                                 ctypes.byref(ln))
        return bool(ok), (buf[:ln.value].tobytes() if ok else None), int(ln.value)

    def packet_handle(self, netif: NetIf, flags: int = 1, capacity: int = 1514, max_frames: int = 0xFFFFFFFF,
                      actions: bool = True, frames: bool = False):
        """BASELINE config 1's loop (ora_ring_packet_handle): (records, actions, positions, frames)."""
        n_max = min(max_frames, self.size // 8)
        out = np.zeros(n_max, RESULT_DTYPE)
        act = np.zeros(n_max, np.uint8) if actions else None
        pos = np.zeros(n_max, np.uint64)
        fb = np.zeros(self.size + 16, np.uint8) if frames else None
        fo = np.zeros(n_max, np.uint32) if frames else None
        n = lib().ora_ring_packet_handle(_p(self.mem), ctypes.byref(self._ct), ctypes.byref(self._ch), capacity,
                                         n_max, flags, netif, _p(out), _p(act), _p(pos), _p(fb), _p(fo))
        return out[:n], (act[:n] if actions else None), pos[:n], ((fb, fo[:n]) if frames else None)


def ring_scan(span: np.ndarray, used: int, ring_size: int, capacity: int = 1514, max_frames: int = 0xFFFFFFFF):
    """ora_ring_scan: (off_dw, lens, stop, end_bytes, max_len)."""
    n_max = max(1, used // 8)
    off = np.zeros(n_max, np.uint32)
    lens = np.zeros(n_max, np.uint16)
    stop, ml = ctypes.c_uint32(), ctypes.c_uint32()
    end = ctypes.c_uint64()
    span = np.ascontiguousarray(span, np.uint8)
    n = lib().ora_ring_scan(_p(span), used, ring_size, capacity, max_frames, _p(off), _p(lens), ctypes.byref(stop),
                            ctypes.byref(end), ctypes.byref(ml))
    return off[:n], lens[:n], int(stop.value), int(end.value), int(ml.value)


def fuzz_batch(seed: int, n: int, netif: NetIf):
    """(data, offsets_dw, lens) of n structured-fuzz frames (halo_fuzz.c), 4-byte aligned."""
    lens = np.zeros(n, np.uint16)
    offs = np.zeros(n, np.uint32)
    total_dw = lib().ora_fuzz_layout(seed, n, _p(lens), _p(offs))
    data = np.zeros(max(16, 4 * total_dw), np.uint8)
    lib().ora_fuzz_fill(seed, n, _p(lens), _p(offs), netif, _p(data))
    return data, offs, lens
