"""halo's SPSC packet ring as the receive source of GPU batches.

The reference moves received frames from the DPDK lcore to Go through ``mem.RingBuffer``
(mem/ring_buffer.go:18-352, the Go twin of cgo/ring_buffer.h), and ``engine.Wire``
(engine/engine.go:507-559) is the same ring used as an in-memory link. Its consumer reads one
record per ``ReadPacket`` call into a 1514-byte buffer and ``PacketHandle`` parses it.

* ``RingBuffer`` — ``RingBufferCreate`` over host memory this object owns, and a batch producer
  (``WritePacket`` per frame: ``halo_ring_write_batch``).
* ``RingConsumer`` — ``NewRingBufferConsumer`` + batched ``ReadPacket``: ``poll`` parses every
  frame between the consumer's cursor and the producer's head on the GPU
  (``halo_rx_ring_poll``: raw DMA of the span, record boundaries found on the GPU, parse in
  place, one record per frame), ``commit`` releases them (``tail`` store-release).
* ``Wire`` — ``engine.NewWire`` (an 8 MiB ring) with ``Tx`` and a GPU ``rx_batch``.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import (RESULT_DTYPE, RING_HEADER, RING_PERSISTENT, RING_REGISTER, RING_SCAN_DTYPE, RING_STATS_DTYPE,
                   RING_STOP_NAMES, NetIf)
from .protocol import flags_word

WIRE_MAX_PACKET_SIZE = 1514  # engine/engine.go:507
MAX_PACKET_SIZE = 1514       # dpdk/dpdk.go:20 (EthQueueRxPkt's receive buffer)


class RingBuffer:
    """A RingBuffer (128-byte header + ``data_size``-byte power-of-two data area) in host memory."""

    def __init__(self, data_size: int = 8 << 20):
        self.mem = _lib.host_array(RING_HEADER + data_size)  # pages of its own: it may be registered
        _lib.check("halo_ring_create", _lib.lib.halo_ring_create(self.mem.ctypes.data, self.mem.nbytes))
        self.size = data_size

    @property
    def head(self) -> int:
        return int(self.mem[0:8].view(np.uint64)[0])

    @property
    def tail(self) -> int:
        return int(self.mem[64:72].view(np.uint64)[0])

    @property
    def data(self) -> np.ndarray:
        return self.mem[RING_HEADER:]

    def write_batch(self, data: np.ndarray, offsets: np.ndarray, lens: np.ndarray,
                    accepted: Optional[np.ndarray] = None) -> int:
        """WritePacket for every frame data[offsets[i]:offsets[i]+lens[i]]; refused frames are
        dropped (accepted[i] = 0). Returns the number written."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        written = ctypes.c_uint32()
        rc = _lib.lib.halo_ring_write_batch(self.mem.ctypes.data, _lib.ptr(data), _lib.ptr(offsets), _lib.ptr(lens),
                                            lens.shape[0], _lib.ptr(accepted), ctypes.byref(written))
        _lib.check("halo_ring_write_batch", rc)
        return int(written.value)

    def write(self, frames) -> int:
        frames = [bytes(f) for f in frames]
        if not frames:
            return 0
        lens = np.fromiter((len(f) for f in frames), dtype=np.uint16, count=len(frames))
        offs = np.zeros(len(frames), dtype=np.uint64)
        np.cumsum(lens[:-1], out=offs[1:])
        return self.write_batch(np.frombuffer(b"".join(frames) + b"\0", np.uint8), offs, lens)

    def length_at(self, position: int) -> int:
        """The u32 length field of the record at stream position `position`."""
        p = position % self.size  # records are 4-byte aligned: the field never wraps
        return int(self.data[p:p + 4].view(np.uint32)[0])

    def frame_at(self, position: int, length: int) -> bytes:
        """The frame whose record sits at stream position `position` (unwrapped)."""
        start = (position + 4) % self.size
        idx = (start + np.arange(length)) % self.size
        return self.data[idx].tobytes()


class RingConsumer:
    """The GPU consumer of one ring (halo_rx_ring_attach). ``capacity`` is ReadPacket's
    ``len(data)`` (1514 in the DPDK driver and Wire). ``small_poll``: spans up to this many bytes
    take the one-launch small path (None: the library default; 0: always the pipelined path).
    ``persistent``: small polls are served by a resident consumer kernel (HALO_RING_PERSISTENT):
    no launch and no stream synchronisation per poll."""

    def __init__(self, ring: RingBuffer, device: int = 0, capacity: int = MAX_PACKET_SIZE, max_bytes: int = 0,
                 max_frames: int = 0, register: bool = True, small_poll: int | None = None, persistent: bool = False):
        self.ring = ring
        self._out_registered = False
        h = ctypes.c_void_p()
        flags = (RING_REGISTER if register else 0) | (RING_PERSISTENT if persistent else 0)
        rc = _lib.lib.halo_rx_ring_attach(device, ring.mem.ctypes.data, 0, capacity, max_bytes, max_frames, flags,
                                          ctypes.byref(h))
        _lib.check("halo_rx_ring_attach", rc)
        self._h = h
        if small_poll is not None:
            _lib.check("halo_rx_ring_set_small_poll", _lib.lib.halo_rx_ring_set_small_poll(h, small_poll))
        cap = max_bytes or min(ring.size, 256 << 20)
        self.max_frames = min(max_frames or (1 << 32) - 1, min(cap, ring.size) // 8)
        self._out = _lib.host_array(self.max_frames, RESULT_DTYPE)  # registered below: pages of its own
        # the records come back by DMA straight into this array: pin it too
        self._out_registered = register and _lib.lib.halo_rx_host_register(
            self._out.ctypes.data, _lib.host_pages(self._out.nbytes)) == 0

    def close(self):
        """Detach from the ring and unregister the record array. Raises HaloError if either
        registration could not be removed: the memory then stays mapped for the device, so the
        consumer keeps references to both arrays instead of letting them be freed."""
        if getattr(self, "_h", None):
            rc = _lib.lib.halo_rx_ring_detach(self._h)
            self._h = None
            rc2 = _lib.HALO_OK
            if self._out_registered:
                rc2 = _lib.lib.halo_rx_host_unregister(self._out.ctypes.data)
                self._out_registered = False
            if rc != _lib.HALO_OK or rc2 != _lib.HALO_OK:
                _lib._leaked.append((self.ring, self._out))  # still registered: never free them
                _lib.check("halo_rx_ring_detach" if rc != _lib.HALO_OK else "halo_rx_host_unregister",
                           rc if rc != _lib.HALO_OK else rc2)

    def __del__(self):
        self.close()

    def poll(self, netif: NetIf, check_sum_enable: bool = True, jumbo: bool = False, hist=None,
             positions: bool = False):
        """Parse the next frames. Returns (records view, info dict, positions or None); the records
        view is reused by the next poll."""
        info = np.zeros(1, dtype=RING_SCAN_DTYPE)
        pos = np.zeros(self.max_frames, dtype=np.uint64) if positions else None
        rc = _lib.lib.halo_rx_ring_poll(self._h, flags_word(check_sum_enable, jumbo), netif, self._out.ctypes.data,
                                        _lib.ptr(hist), _lib.ptr(pos), info.ctypes.data)
        _lib.check("halo_rx_ring_poll", rc)
        n = int(info["n_frames"][0])
        d = {"n_frames": n, "stop": RING_STOP_NAMES[int(info["stop"][0])], "end_bytes": int(info["end_bytes"][0]),
             "max_len": int(info["max_len"][0])}
        return self._out[:n], d, (pos[:n] if positions else None)

    def commit(self):
        _lib.check("halo_rx_ring_commit", _lib.lib.halo_rx_ring_commit(self._h))

    def set_service_timeout(self, us: int):
        """Bound on one resident request's wait (0 = the default 2 s; fault injection)."""
        _lib.check("halo_rx_ring_set_service_timeout", _lib.lib.halo_rx_ring_set_service_timeout(self._h, us))

    def stats(self) -> dict:
        """halo_rx_ring_get_stats: poll counters and where the small polls' time went."""
        st = np.zeros(1, RING_STATS_DTYPE)
        _lib.check("halo_rx_ring_get_stats", _lib.lib.halo_rx_ring_get_stats(self._h, st.ctypes.data))
        return {k: int(st[k][0]) for k in RING_STATS_DTYPE.names}


class Wire:
    """engine.Wire (engine/engine.go:507-559): a ring with an 8 MiB data area as a virtual link."""

    def __init__(self, device: int = 0, data_size: int = 8 << 20, persistent: bool = False):
        self.ring = RingBuffer(data_size)
        self.consumer = RingConsumer(self.ring, device=device, capacity=WIRE_MAX_PACKET_SIZE, persistent=persistent)

    def Tx(self, pkt: bytes) -> None:  # engine/engine.go:548-553
        if len(pkt) == 0 or len(pkt) > WIRE_MAX_PACKET_SIZE:
            return
        self.ring.write([pkt])

    def rx_batch(self, netif: NetIf, check_sum_enable: bool = True):
        """Every frame Wire.Rx would return until it returns nil, parsed: (records, frames)."""
        recs, info, pos = self.consumer.poll(netif, check_sum_enable, positions=True)
        frames = [self.ring.frame_at(int(p), self.ring.length_at(int(p))) for p in pos]
        out = recs.copy()
        self.consumer.commit()
        return out, frames

    def Destroy(self):
        self.consumer.close()
