"""Batched mirror of halo's receive engine (engine/engine.go:339-385 and its callees).

The reference's ``NetIf.PacketHandle`` pulls one frame per iteration from
``NetIfConfig.EthRxFunc`` (engine/engine.go:76,348) and runs ``RxEthernet`` -> ``RxIpv4``
-> ``Rx{Udp,Tcp,Icmp}`` on it. ``NetIf.packet_handle_batch`` drains up to ``batch`` frames
from the same kind of ``eth_rx_func`` (a callable returning ``bytes`` or ``None``), parses
and verifies the whole batch on the GPU through ``halo_rx_parse_batch_host`` (pinned
staging, double-buffered H2D -> kernel -> D2H), maps every record to the reference
engine's decision with ``halo_rx_dispatch`` and invokes the registered UDP / TCP service
handlers in frame order, with the same session and payload arguments as
engine/udp_engine.go:16-20 and engine/tcp_engine.go:79-88. It drains the NetIf's ``LoChan``
(bare IPv4 packets: TxIpv4's loopback copies, Ipv4RouteForward's copies for another NetIf's
address) the way PacketHandle does (engine/engine.go:353-381): a HALO_RX_L3_START batch parse,
``halo_rx_dispatch_loopback``, then the same handlers, until the channel is empty — after every
batch by default, or, with ``drain_every=99``, at PacketHandle's own cadence of one drain per 99
polls (a batch then ends at that poll), which reproduces the reference's order of handler calls
and drains exactly.
"""
from __future__ import annotations

import collections
import ctypes
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import _lib
from ._lib import ACTION, ACTION_NAMES, RESULT_DTYPE, NetIf as NetIfAbi
from .protocol import flags_word


def dispatch(results: np.ndarray, netif: NetIfAbi) -> np.ndarray:
    """Reference engine decision per record (halo_rx_dispatch), as uint8 action codes."""
    results = np.ascontiguousarray(results).view(RESULT_DTYPE).reshape(-1)
    actions = np.empty(results.shape[0], dtype=np.uint8)
    rc = _lib.lib.halo_rx_dispatch(_lib.ptr(results), results.shape[0], netif, _lib.ptr(actions), None)
    _lib.check("halo_rx_dispatch", rc)
    return actions


def dispatch_loopback(results: np.ndarray, netif: NetIfAbi) -> np.ndarray:
    """PacketHandle's LoChan drain decision per record (halo_rx_dispatch_loopback)."""
    results = np.ascontiguousarray(results).view(RESULT_DTYPE).reshape(-1)
    actions = np.empty(results.shape[0], dtype=np.uint8)
    rc = _lib.lib.halo_rx_dispatch_loopback(_lib.ptr(results), results.shape[0], netif, _lib.ptr(actions), None)
    _lib.check("halo_rx_dispatch_loopback", rc)
    return actions


@dataclass
class UdpSession:  # engine/udp_engine.go:47-50
    RemoteIp: int
    RemotePort: int


@dataclass
class TcpSession:  # engine/tcp_engine.go:103-106
    RemoteIp: int
    RemotePort: int


class HostBatcher:
    """Owns a halo_rx_host_ctx (pinned staging + two streams) on one device."""

    def __init__(self, device: int = 0, chunk_frames: int = 0, chunk_bytes: int = 0):
        h = ctypes.c_void_p()
        _lib.check("halo_rx_host_ctx_create",
                   _lib.lib.halo_rx_host_ctx_create(device, chunk_frames, chunk_bytes, ctypes.byref(h)))
        self._ctx = h

    def set_zero_copy(self, enable: bool):
        """Registered batches parsed in place over PCIe (default) or DMA'd in chunks."""
        _lib.check("halo_rx_host_ctx_set_zero_copy", _lib.lib.halo_rx_host_ctx_set_zero_copy(self._ctx, int(enable)))

    def set_resident(self, max_frames: int, max_bytes: int = 0):
        """Batches of up to ``max_frames`` frames (and ``max_bytes`` of staging; 0 = the library's
        default) go to a resident consumer kernel: no launch or stream synchronisation per call
        (halo_rx_host_ctx_set_resident). 0 turns it off."""
        _lib.check("halo_rx_host_ctx_set_resident",
                   _lib.lib.halo_rx_host_ctx_set_resident(self._ctx, max_frames, max_bytes))

    def set_service_timeout(self, us: int):
        """Bound on one resident request's wait (0 = the default 2 s; fault injection)."""
        _lib.check("halo_rx_host_ctx_set_service_timeout",
                   _lib.lib.halo_rx_host_ctx_set_service_timeout(self._ctx, us))

    def stats(self) -> dict:
        """halo_rx_host_ctx_get_stats: call counts and where the resident path's time went."""
        st = np.zeros(1, _lib.HOST_STATS_DTYPE)
        _lib.check("halo_rx_host_ctx_get_stats", _lib.lib.halo_rx_host_ctx_get_stats(self._ctx, st.ctypes.data))
        return {k: int(st[k][0]) for k in _lib.HOST_STATS_DTYPE.names}

    def close(self):
        if self._ctx:
            _lib.lib.halo_rx_host_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def parse(self, data: np.ndarray, offsets: np.ndarray, lens: np.ndarray, netif: NetIfAbi, flags: int,
              hist: Optional[np.ndarray] = None, out: Optional[np.ndarray] = None) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        n = lens.shape[0]
        if out is None:
            out = np.empty(n, dtype=RESULT_DTYPE)
        assert out.dtype == RESULT_DTYPE and out.shape[0] >= n and out.flags.c_contiguous
        if hist is not None:
            assert hist.dtype == np.uint32 and hist.flags.c_contiguous
        rc = _lib.lib.halo_rx_parse_batch_host(self._ctx, _lib.ptr(data), _lib.ptr(offsets), _lib.ptr(lens), n,
                                               flags, netif, _lib.ptr(out), _lib.ptr(hist))
        _lib.check("halo_rx_parse_batch_host", rc)
        return out


@dataclass
class NetIf:
    """engine.NetIf / NetIfConfig (engine/engine.go:65-121), receive side only."""

    Name: str
    MacAddr: str
    IpAddr: str
    EthRxFunc: Callable[[], Optional[bytes]]
    NatEnable: bool = False
    CheckSumEnable: bool = True  # protocol.CheckSumEnable for this interface's batches
    UdpServiceMap: dict = field(default_factory=dict)
    TcpServiceMap: dict = field(default_factory=dict)
    LoChan: collections.deque = field(default_factory=collections.deque)  # NetIf.LoChan (engine/engine.go:106, cap 1024 :209)
    device: int = 0
    # batches of up to this many frames go to the host context's resident consumer (no launch per
    # batch: PacketHandle-sized batches, e.g. drain_every=99, are latency-bound); 0 = launches only
    resident_frames: int = 4096
    # batches (and LoChan drains) of fewer frames go to the CPU entry point (halo_amd.cpu,
    # include/halo_rx_cpu.h: the same records on the calling core, ~9 ns per frame against ~8 us per
    # GPU round trip; crossover ~3,800 frames); 0 = every batch on the GPU
    cpu_below: int = 0

    def __post_init__(self):
        self.abi = NetIfAbi.make(self.MacAddr, self.IpAddr, self.NatEnable)
        self._batcher: Optional[HostBatcher] = None
        self.action_counts = np.zeros(len(ACTION_NAMES), dtype=np.int64)
        self._polls = 0  # EthRxFunc polls since the last LoChan drain: PacketHandle's n

    def RecvUdp(self, port: int, handle: Callable):  # engine/udp_engine.go:56-58
        self.UdpServiceMap[port] = handle

    def RecvTcp(self, port: int, handle: Callable):  # engine/tcp_engine.go:112-114
        self.TcpServiceMap[port] = handle

    def packet_handle_batch(self, batch: int = 4096, drain_every: int = 0):
        """One batched iteration of PacketHandle: poll, parse (on the GPU, or on the CPU entry point
        for a batch below ``cpu_below`` frames), dispatch, deliver; then drain LoChan when it is due.

        drain_every = 0: a batch ends at ``batch`` frames or at the first poll that returns None,
        and LoChan is drained after every batch. drain_every = 99: PacketHandle's cadence
        (engine/engine.go:353, ``n == 100-1``) — polls are counted across calls (None polls
        included), a batch also ends at the poll that makes the count 99, and the drain runs
        there, so handlers and drains run in the reference's order.
        Returns (results, actions) for the frames polled this iteration."""
        frames = []
        while len(frames) < batch:
            f = self.EthRxFunc()
            self._polls += 1
            if f is not None:
                frames.append(bytes(f))
            if drain_every and self._polls >= drain_every:
                break
            if f is None and not drain_every:
                break
        res, actions = np.empty(0, RESULT_DTYPE), np.empty(0, np.uint8)
        if frames:
            lens = np.fromiter((len(f) for f in frames), dtype=np.uint16, count=len(frames))
            offsets = np.zeros(len(frames), dtype=np.uint64)
            np.cumsum(lens[:-1], out=offsets[1:])
            data = np.frombuffer(b"".join(frames), dtype=np.uint8)
            res = self._parse(data, offsets, lens, l3=False)
            actions = dispatch(res, self.abi)
            self._deliver(frames, res, actions)
        if not drain_every or self._polls >= drain_every:
            self.lo_drain()
            self._polls = 0
        return res, actions

    def lo_drain(self, max_batch: int = 4096):
        """PacketHandle's loopback drain (engine/engine.go:353-381): until LoChan is empty, parse
        what is queued (ParseIpv4Pkt, own-address filter, local RxIcmp / RxUdp / RxTcp) as one GPU
        batch of at most ``max_batch`` packets and deliver it in order; packets the handlers queue
        meanwhile are drained by the same call, as the reference's select loop drains them.
        Returns (results, actions) for every packet drained."""
        all_res, all_act = [], []
        while self.LoChan:
            pkts = []
            while self.LoChan and len(pkts) < max_batch:
                pkts.append(bytes(self.LoChan.popleft()))
            lens = np.fromiter((len(p) for p in pkts), dtype=np.uint16, count=len(pkts))
            sizes = (lens.astype(np.uint64) + 3) & ~np.uint64(3)  # 4-byte aligned starts, like ring records
            offsets = np.zeros(len(pkts), dtype=np.uint64)
            np.cumsum(sizes[:-1], out=offsets[1:])
            data = np.zeros(int(sizes.sum()) + 4, dtype=np.uint8)
            for o, p in zip(offsets, pkts):
                data[int(o):int(o) + len(p)] = np.frombuffer(p, dtype=np.uint8)
            res = self._parse(data, offsets, lens, l3=True)
            actions = dispatch_loopback(res, self.abi)
            self._deliver(pkts, res, actions)
            all_res.append(res)
            all_act.append(actions)
        if not all_res:
            return np.empty(0, RESULT_DTYPE), np.empty(0, np.uint8)
        return np.concatenate(all_res), np.concatenate(all_act)

    def _parse(self, data, offsets, lens, *, l3: bool) -> np.ndarray:
        """One batch's records: on the CPU entry point below ``cpu_below`` frames, else on the GPU."""
        if lens.shape[0] < self.cpu_below:
            from . import cpu

            return cpu.parse_frames_cpu(data, offsets, lens, netif=self.abi, check_sum_enable=self.CheckSumEnable,
                                        l3_start=l3)
        return self._host().parse(data, offsets, lens, self.abi, flags_word(self.CheckSumEnable, l3_start=l3))

    def _host(self) -> HostBatcher:
        if self._batcher is None:
            self._batcher = HostBatcher(self.device)
            if self.resident_frames:
                self._batcher.set_resident(self.resident_frames)
        return self._batcher

    def _deliver(self, bufs, res, actions):
        """Invoke the UDP / TCP service handlers for the LOCAL_UDP / LOCAL_TCP records, in order."""
        np.add.at(self.action_counts, actions, 1)
        for i in np.nonzero((actions == ACTION["LOCAL_UDP"]) | (actions == ACTION["LOCAL_TCP"]))[0]:
            r = res[i]
            payload = bufs[i][int(r["payload_off"]):int(r["payload_off"]) + int(r["payload_len"])]
            if actions[i] == ACTION["LOCAL_UDP"]:
                h = self.UdpServiceMap.get(int(r["dport"]))
                if h is not None:
                    h(UdpSession(int(r["src_ip"]), int(r["sport"])), payload)
            else:
                h = self.TcpServiceMap.get(int(r["dport"]))
                if h is not None:
                    h(TcpSession(int(r["src_ip"]), int(r["sport"])), payload, int(r["l4_seq"]),
                      int(r["l4_ack"]), int(r["l4_aux"]))
