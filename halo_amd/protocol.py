"""Batch mirror of halo's ``protocol`` package on the receive path.

The reference parses one frame per call (``protocol.ParseEthFrm`` -> ``ParseIpv4Pkt`` ->
``ParseUdpPkt`` / ``ParseTcpPkt`` / ``ParseIcmpPkt``, gated by the package global
``protocol.CheckSumEnable``). Here one call parses a whole device-resident batch through the
C ABI (``halo_rx_parse_batch_device``); the per-frame Go return values become one 32-byte
``halo_rx_result_t`` record per frame (see ``include/halo_rx.h`` for the field contract).

Names and constants follow the reference so code reads like its own:
``check_sum_enable`` is ``CheckSumEnable`` (protocol/utils.go:8), the EtherType / IP
protocol / ICMP constants are those of protocol/ethernet.go:16-22, protocol/ipv4.go:27-32,
protocol/icmp.go:25-30 and protocol/tcp.go:26-33, and ``ERROR_TEXT`` maps each status to the
error string the reference returns for it.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import HALO_RX_CSUM_ENABLE, HALO_RX_JUMBO_EXT, RESULT_DTYPE, STATUS, STATUS_NAMES, NetIf

# protocol/ethernet.go:16-22
IEEE_802_3 = 0x05DC
ETH_PROTO_IPV4 = 0x0800
ETH_PROTO_ARP = 0x0806
ETH_PROTO_IPV6 = 0x86DD
ETH_PROTO_UNKNOWN = 0xFFFF
BROADCAST_MAC_ADDR = b"\xff" * 6
# protocol/ipv4.go:27-32
IPH_PROTO_ICMP = 0x01
IPH_PROTO_TCP = 0x06
IPH_PROTO_UDP = 0x11
IPH_PROTO_UNKNOWN = 0xFF
# protocol/icmp.go:25-30
ICMP_REQUEST = 0x08
ICMP_REPLY = 0x00
ICMP_TTL = 0x0B
ICMP_UNKNOWN = 0xFF
# protocol/tcp.go:26-33
TCP_FLAGS_URG = 0x20
TCP_FLAGS_ACK = 0x10
TCP_FLAGS_PSH = 0x08
TCP_FLAGS_RST = 0x04
TCP_FLAGS_SYN = 0x02
TCP_FLAGS_FIN = 0x01

# status -> the error the reference returns at that check (None: no error / build-defined). The
# L4 length check has one text per protocol: L4_LEN_TEXT[ip_proto] (error_text picks it).
ERROR_TEXT = {
    "OK": None,
    "ETH_LEN": "ethernet frame len must >= 42 and <= 1514 bytes",   # ethernet.go:32
    "ETH_TYPE": "unknown ethernet protocol",                        # ethernet.go:49
    "IP_LEN": "ip packet len must >= 20 and <= 1500 bytes",         # ipv4.go:50
    "IP_VER": "not support type of ip packet",                      # ipv4.go:53
    "IP_FRAG": "not support ip frg",                                # ipv4.go:60
    "IP_PROTO": "unknown ip protocol",                              # ipv4.go:71
    "IP_HDR_CKSUM": "header check sum error",                       # ipv4.go:76
    "IP_TOTLEN_UNDERFLOW": None,  # Go: slice-bounds panic (ipv4.go:84)
    "IP_TOTLEN_OVERRUN": None,    # Go: stale bytes or slice-bounds panic (ipv4.go:84)
    "L4_LEN": None,               # per protocol: L4_LEN_TEXT
    "ICMP_TYPE": "not support type of icmp packet",                 # icmp.go:46
    "ICMP_CODE": "not support type of icmp packet",                 # icmp.go:50
    "L4_CKSUM": "check sum error",                                  # udp.go:43 / tcp.go:64 / icmp.go:54
}
L4_LEN_TEXT = {
    IPH_PROTO_UDP: "udp packet len must >= 8 and <= 1480 bytes",    # udp.go:23
    IPH_PROTO_TCP: "tcp packet len must >= 20 and <= 1480 bytes",   # tcp.go:38
    IPH_PROTO_ICMP: "icmp packet len must >= 8 and <= 1480 bytes",  # icmp.go:35
}


def error_text(status: int, ip_proto: int = IPH_PROTO_UNKNOWN):
    """The error string the reference function that failed returns for a record's status (None for
    OK and for the build-defined totalLen statuses, where Go panics). L4_LEN is told apart by the
    record's ip_proto, which ParseIpv4Pkt set before the L4 parser ran."""
    name = STATUS_NAMES[status]
    if name == "L4_LEN":
        return L4_LEN_TEXT[ip_proto]
    return ERROR_TEXT[name]


def flags_word(check_sum_enable: bool = True, jumbo: bool = False, variant: int = 0, uniform_len: bool = False,
               l3_start: bool = False) -> int:
    """The ABI ``flags`` word that replaces the ``CheckSumEnable`` package global (plus the
    per-call kernel variant, lanes per frame with -1 = mix, the uniform-length hint and the
    LoChan layout: buffers that start at their IPv4 header)."""
    return ((HALO_RX_CSUM_ENABLE if check_sum_enable else 0) | (HALO_RX_JUMBO_EXT if jumbo else 0)
            | _lib.variant_flags(variant) | (_lib.HALO_RX_UNIFORM_LEN if uniform_len else 0)
            | (_lib.HALO_RX_L3_START if l3_start else 0))


def _stream_handle(stream):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _check_out(out, n: int):
    import torch

    assert out.dtype == torch.uint8 and out.is_cuda and out.numel() >= 32 * n, "out: cuda uint8[n*32]"


def parse_frames_batch(frames, offsets_dw, lens, *, netif: NetIf, check_sum_enable: bool = True,
                       jumbo: bool = False, max_len_hint: int = 0, uniform_len: bool = False, variant: int = 0,
                       out=None, hist=None, stream=None, l3_start: bool = False):
    """Parse + verify a ragged, device-resident batch (ParseEthFrm..ParseIcmpPkt per frame).

    frames: cuda uint8 tensor; offsets_dw: cuda int32 tensor (frame i at 4*offsets_dw[i]);
    lens: cuda int16 tensor (u16 lengths). Returns the cuda uint8 [n, 32] result tensor.
    ``hist`` (cuda int32[14]) is incremented per status. Asynchronous on ``stream``.
    ``uniform_len``: every frame is ``max_len_hint`` bytes; ``variant``: force lanes per frame
    (1/4/8/16, -1 = mix) for this call — speed only, records are identical. ``l3_start``:
    the buffers are LoChan packets starting at their IPv4 header (parse_ipv4_packets_batch).
    """
    import torch

    n = int(lens.numel())
    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=frames.device)
    _check_out(out, n)
    rc = _lib.lib.halo_rx_parse_batch_device(
        _lib.ptr(frames), _lib.ptr(offsets_dw), _lib.ptr(lens), n,
        flags_word(check_sum_enable, jumbo, variant, uniform_len, l3_start), netif, max_len_hint, _lib.ptr(out),
        _lib.ptr(hist),
        _stream_handle(stream))
    _lib.check("halo_rx_parse_batch_device", rc)
    return out


def parse_frames_batches(batches, *, netif: NetIf, check_sum_enable: bool = True, jumbo: bool = False,
                         max_len_hint: int = 0, variant: int = 0, compact: bool = False, l3_start: bool = False,
                         hist=None, stream=None):
    """Several ragged device-resident batches in one call (halo_rx_parse_batches_device): each of
    ``batches`` is (frames, offsets_dw, lens, out) with the tensors of parse_frames_batch; frames of
    at most 64 B (max_len_hint <= 64 or variant 1) run as one launch. Returns the outs."""
    import ctypes

    k = len(batches)
    descs = (_lib.BatchDesc * max(k, 1))()
    for j, (fr, offs, ln, out) in enumerate(batches):
        n = int(ln.numel())
        assert out.is_cuda and out.numel() * out.element_size() >= (16 if compact else 32) * n, "out too small"
        descs[j] = _lib.BatchDesc(_lib.ptr(fr), _lib.ptr(offs), _lib.ptr(ln), _lib.ptr(out), n, 0)
    fl = flags_word(check_sum_enable, jumbo, variant, False, l3_start) | (_lib.HALO_RX_RECORD_COMPACT if compact else 0)
    rc = _lib.lib.halo_rx_parse_batches_device(ctypes.cast(descs, ctypes.c_void_p), k, fl, netif, max_len_hint,
                                               _lib.ptr(hist), _stream_handle(stream))
    _lib.check("halo_rx_parse_batches_device", rc)
    return [b[3] for b in batches]


def parse_ipv4_packets_batch(packets, offsets_dw, lens, *, netif: NetIf, **kw):
    """ParseIpv4Pkt + local L4 parse of a batch of LoChan packets (buffers that start at their
    IPv4 header: engine/engine.go:353-381), HALO_RX_L3_START. Same arguments and record as
    parse_frames_batch; map the records to the drain's decisions with
    engine.dispatch_loopback."""
    return parse_frames_batch(packets, offsets_dw, lens, netif=netif, l3_start=True, **kw)


def parse_frames_strided(frames, stride: int, n: int, *, netif: NetIf, length: int = 0, lens=None,
                         check_sum_enable: bool = True, jumbo: bool = False, out=None, hist=None,
                         stream=None):
    """Same as parse_frames_batch for frames at i*stride (uniform ``length`` or ``lens``)."""
    import torch

    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=frames.device)
    _check_out(out, n)
    rc = _lib.lib.halo_rx_parse_strided_device(
        _lib.ptr(frames), stride, _lib.ptr(lens), length, n, flags_word(check_sum_enable, jumbo), netif,
        _lib.ptr(out), _lib.ptr(hist), _stream_handle(stream))
    _lib.check("halo_rx_parse_strided_device", rc)
    return out


def records(out) -> np.ndarray:
    """View a result buffer (cuda or host, uint8 [n,32]) as a numpy structured array."""
    a = out.cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)
    return np.ascontiguousarray(a).reshape(-1).view(RESULT_DTYPE)


def status_name(code: int) -> str:
    return STATUS_NAMES[code] if 0 <= code < len(STATUS_NAMES) else "UNKNOWN"




# ---- forward / transmit direction -------------------------------------
# Step bits of halo_tx_op_t.steps: NatChangeDst, HandleIpv4PktTtl, NatChangeSrc, the ReCalc*
# pair for the packet's protocol, and eth_tx's DPDK software checksum fill, applied in the order
# Ipv4RouteForward applies them (engine/ipv4_engine.go:108-269).
from ._lib import (TX_DPDK_FILL, TX_NAT_DST, TX_NAT_SRC, TX_OP_DTYPE, TX_R_OVERRUN,  # noqa: E402
                   TX_R_SKIPPED, TX_R_TTL_ALIVE, TX_RECALC, TX_TTL)




def tx_ops(n: int, steps: int = 0, dst_ip: int = 0, dst_port: int = 0, src_ip: int = 0, src_port: int = 0):
    """A host halo_tx_op_t array (numpy) with every field broadcast; edit per frame as needed."""
    ops = np.zeros(n, dtype=TX_OP_DTYPE)
    ops["steps"], ops["dst_ip"], ops["dst_port"], ops["src_ip"], ops["src_port"] = (
        steps, dst_ip, dst_port, src_ip, src_port)
    return ops


def tx_fixup_batch(frames, offsets_dw, lens, ops, *, check_sum_enable: bool = True, max_len_hint: int = 0,
                   result=None, stream=None):
    """Rewrite a device-resident ragged batch in place (halo_tx_fixup_batch_device).

    frames: cuda uint8 tensor (modified); offsets_dw / lens as parse_frames_batch; ops: cuda
    uint8 tensor of n*16 bytes holding halo_tx_op_t records (``torch.from_numpy(tx_ops(...)
    .view(np.uint8)).cuda()``). ``result`` (cuda uint8[n], optional) receives HALO_TX_R_* per
    frame. Asynchronous on ``stream``; returns ``result``.
    """
    n = int(lens.numel())
    assert ops.is_cuda and ops.numel() >= 16 * n, "ops: cuda uint8[n*16]"
    if result is not None:
        assert result.is_cuda and result.numel() >= n
    rc = _lib.lib.halo_tx_fixup_batch_device(
        _lib.ptr(frames), _lib.ptr(offsets_dw), _lib.ptr(lens), n, _lib.ptr(ops),
        HALO_RX_CSUM_ENABLE if check_sum_enable else 0, max_len_hint, _lib.ptr(result), _stream_handle(stream))
    _lib.check("halo_tx_fixup_batch_device", rc)
    return result


# ---- transmit construction (the Build* half) ---------------------------------
from ._lib import BUILD_DESC_DTYPE, TX_BUILD_ETH, TX_BUILD_LOOPBACK  # noqa: E402,F401


class TxBuilder:
    """Batched NetIf.TxUdp / TxTcp / TxIcmp -> TxIpv4 -> TxEthernet on the GPU
    (halo_tx_build_batch_device). Owns the device workspace and the iphId counter
    (protocol.iphId, protocol/ipv4.go:33), which advances by one per packet built, in order."""

    def __init__(self, max_frames: int, device=None, ip_id: int = 0):
        import torch

        self.device = device or torch.device("cuda", torch.cuda.current_device())
        ws = int(_lib.lib.halo_tx_build_workspace(max_frames))
        self.max_frames = max_frames
        self.ws = torch.empty(ws, dtype=torch.uint8, device=self.device)  # scratch, no initialisation needed
        self.ip_id = torch.from_numpy(np.array([ip_id & 0xFFFF], np.uint16).view(np.int16)).to(self.device)

    def SetIpHeaderId(self, value: int) -> None:
        """protocol.SetRandIpHeaderId's effect with a given value."""
        self.ip_id.fill_(int(np.array(value & 0xFFFF, np.uint16).view(np.int16)))

    @property
    def iph_id(self) -> int:
        return int(self.ip_id.cpu().numpy().view(np.uint16)[0])

    def build(self, desc, payload, *, netif: NetIf, out_stride: int, frames=None, lens=None, result=None,
              check_sum_enable: bool = True, max_payload_hint: int = 0, stream=None):
        """desc: cuda uint8 tensor of n * 40 bytes (halo_tx_build_desc_t); payload: cuda uint8.
        Returns (frames [n, out_stride] uint8, lens int16 [n], result uint8 [n]); asynchronous."""
        import torch

        n = desc.numel() // BUILD_DESC_DTYPE.itemsize
        assert n <= self.max_frames
        if frames is None:
            frames = torch.zeros((n, out_stride), dtype=torch.uint8, device=desc.device)
        if lens is None:
            lens = torch.zeros(n, dtype=torch.int16, device=desc.device)
        if result is None:
            result = torch.zeros(n, dtype=torch.uint8, device=desc.device)
        rc = _lib.lib.halo_tx_build_batch_device(
            _lib.ptr(desc), n, _lib.ptr(payload), HALO_RX_CSUM_ENABLE if check_sum_enable else 0, netif,
            max_payload_hint, _lib.ptr(frames), out_stride, _lib.ptr(lens), _lib.ptr(result), _lib.ptr(self.ip_id),
            _lib.ptr(self.ws), self.ws.numel(), _stream_handle(stream))
        _lib.check("halo_tx_build_batch_device", rc)
        return frames, lens, result


# ---- IcmpTtlDeepNat (engine/icmp_engine.go:55-86) -----------------------------------------------
from ._lib import DEEP_NAT_DTYPE  # noqa: E402,F401


def icmp_ttl_deep_nat_batch(frames, offsets_dw, lens, *, nat=None, check_sum_enable: bool = True, quote=None,
                            applied=None, stream=None):
    """IcmpTtlDeepNat over a device-resident ragged batch (halo_tx_icmp_deep_nat_batch_device).

    nat None: only the checks — ``quote`` (cuda uint8 [n, 32], halo_rx_result_t) receives per
    frame the NatGetFlowByWan arguments (hash them with flow_hash kind NAT_WAN). nat: cuda uint8
    tensor of n * 8 bytes (DEEP_NAT_DTYPE records: the lookups' LanHost and found) — frames
    rewritten in place, ``applied`` (cuda uint8 [n]) = IcmpTtlDeepNat's bool. Asynchronous."""
    n = int(lens.numel())
    rc = _lib.lib.halo_tx_icmp_deep_nat_batch_device(
        _lib.ptr(frames), _lib.ptr(offsets_dw), _lib.ptr(lens), n, _lib.ptr(nat),
        HALO_RX_CSUM_ENABLE if check_sum_enable else 0, _lib.ptr(quote), _lib.ptr(applied), _stream_handle(stream))
    _lib.check("halo_tx_icmp_deep_nat_batch_device", rc)
    return quote, applied


# ---- single-frame Parse* with the reference's signatures ------------------------------------------
# For callers that hold one frame or packet at a time — an Ipv4PktFwdHook (engine/engine.go:132,
# example/example.go:162-168) or code ported from the reference — each wrapper returns exactly the
# tuple its Go function returns, with `err` the reference's error string (None on success). The
# frame goes through the GPU like a batch of one (halo_rx_parse_batch_host, a per-process host
# context whose resident consumer serves it: one request, no launch) unless SINGLE_FRAME_CPU is set,
# which sends it to the CPU entry point instead (halo_amd.cpu, include/halo_rx_cpu.h: the same record
# on the calling core, no GPU round trip). Batches of frames belong on parse_frames_batch / engine.
CheckSumEnable = True  # protocol.CheckSumEnable (protocol/utils.go:8) for the wrappers below
DEVICE = 0             # the device the wrappers' host context uses
SINGLE_FRAME_CPU = False  # the caller's choice, read at every call (go/gpurx SingleFrameCPU)


class ReferencePanic(RuntimeError):
    """The Go function panics on this input: ParseIpv4Pkt with totalLen < 20 or > len(pkt) slices
    pkt[20:totalLen] out of bounds (protocol/ipv4.go:84). Batches report these as the build-defined
    statuses IP_TOTLEN_UNDERFLOW / IP_TOTLEN_OVERRUN."""


_ctx = {}


def _parse_one(buf: bytes, l3: bool) -> np.void:
    """One Ethernet frame (or, l3, one bare IPv4 packet) parsed on the GPU (on the CPU entry point
    with SINGLE_FRAME_CPU): its halo_rx_result_t.
    Lengths past 65535 are passed as 65535 (any length over the reference's caps gets the same
    ETH_LEN / IP_LEN verdict)."""
    import ctypes

    if SINGLE_FRAME_CPU:
        from . import cpu

        n = min(len(buf), 0xFFFF)
        data = np.frombuffer(bytes(buf[:n]), np.uint8) if n else np.zeros(4, np.uint8)
        return cpu.parse_frames_cpu(data, np.zeros(1, np.uint64), np.array([n], np.uint16), netif=NetIf.make(),
                                    check_sum_enable=CheckSumEnable, l3_start=l3)[0]
    if DEVICE not in _ctx:
        h = ctypes.c_void_p()
        _lib.check("halo_rx_host_ctx_create", _lib.lib.halo_rx_host_ctx_create(DEVICE, 64, 1 << 16, ctypes.byref(h)))
        # one frame per call: the resident consumer serves it (no launch or synchronisation per frame)
        _lib.check("halo_rx_host_ctx_set_resident", _lib.lib.halo_rx_host_ctx_set_resident(h, 64, 1 << 16))
        _ctx[DEVICE] = h
    n = min(len(buf), 0xFFFF)
    data = np.zeros(max(4, n), np.uint8)
    data[:n] = np.frombuffer(bytes(buf[:n]), np.uint8)
    offs = np.zeros(1, np.uint64)
    lens = np.array([n], np.uint16)
    out = np.zeros(1, RESULT_DTYPE)
    rc = _lib.lib.halo_rx_parse_batch_host(_ctx[DEVICE], _lib.ptr(data), _lib.ptr(offs), _lib.ptr(lens), 1,
                                           flags_word(CheckSumEnable, l3_start=l3), NetIf.make(), _lib.ptr(out), None)
    _lib.check("halo_rx_parse_batch_host", rc)
    return out[0]


def _ip_wrap(seg: bytes, proto: int, src: bytes, dst: bytes) -> bytes:
    """seg behind a minimal valid IPv4 header (0x45, DF, the given protocol and addresses, header
    checksum filled), so the L3 parse hands exactly `seg` to the L4 parser: pkt[20:totalLen] = seg,
    and the pseudo header carries src / dst. Only its verdicts for seg are read back."""
    tl = 20 + len(seg)
    h = bytearray(20)
    h[0], h[6], h[8], h[9] = 0x45, 0x40, 64, proto
    h[2:4] = (tl & 0xFFFF).to_bytes(2, "big")
    h[12:16], h[16:20] = src, dst
    s = sum(int.from_bytes(h[k:k + 2], "big") for k in range(0, 20, 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    h[10:12] = (~s & 0xFFFF).to_bytes(2, "big")
    return bytes(h) + bytes(seg)


def _addr4(a) -> bytes:
    a = bytes(a)
    if len(a) != 4:
        raise ValueError("srcAddr / dstAddr must be 4-byte IPv4 addresses")
    return a


def ParseEthFrm(frm):
    """protocol.ParseEthFrm (protocol/ethernet.go:29-55): (payload, dstMac, srcMac, ethProto, err)."""
    r = _parse_one(frm, False)
    if STATUS_NAMES[r["status"]] in ("ETH_LEN", "ETH_TYPE"):
        return None, None, None, ETH_PROTO_UNKNOWN, error_text(int(r["status"]))
    frm = bytes(frm)
    return frm[14:], frm[0:6], frm[6:12], int(r["ethertype"]), None


def ParseIpv4Pkt(pkt):
    """protocol.ParseIpv4Pkt (protocol/ipv4.go:48-86): (payload, ipHeadProto, srcAddr, dstAddr, err).
    Raises ReferencePanic where the Go slice expression panics."""
    r = _parse_one(pkt, True)
    name = STATUS_NAMES[r["status"]]
    if name in ("IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN"):
        raise ReferencePanic(f"ParseIpv4Pkt: totalLen {int(r['ip_total_len'])} outside [20, {len(pkt)}]")
    if name in ("IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM"):
        return None, IPH_PROTO_UNKNOWN, None, None, error_text(int(r["status"]))
    pkt = bytes(pkt)
    return pkt[20:int(r["ip_total_len"])], int(r["ip_proto"]), pkt[12:16], pkt[16:20], None


def _l4(seg, proto: int, src, dst):
    """The record of seg's L4 parse, and the error text for it (None when it passed)."""
    r = _parse_one(_ip_wrap(bytes(seg), proto, _addr4(src), _addr4(dst)), True)
    name = STATUS_NAMES[r["status"]]
    if name in ("IP_LEN", "L4_LEN"):  # IP_LEN: 20 + len(seg) > 1500, i.e. len(seg) > 1480
        return r, L4_LEN_TEXT[proto]
    return r, (None if name == "OK" else error_text(int(r["status"]), proto))


def ParseUdpPkt(pkt, srcAddr, dstAddr):
    """protocol.ParseUdpPkt (protocol/udp.go:21-49): (payload, srcPort, dstPort, err)."""
    r, err = _l4(pkt, IPH_PROTO_UDP, srcAddr, dstAddr)
    if err:
        return None, 0, 0, err
    return bytes(pkt)[8:], int(r["sport"]), int(r["dport"]), None


def ParseTcpPkt(pkt, srcAddr, dstAddr):
    """protocol.ParseTcpPkt (protocol/tcp.go:36-70): (payload, srcPort, dstPort, seqNum, ackNum, flags,
    err); the payload starts at the data-offset nibble used as BYTES, as tcp.go:49,68 does."""
    r, err = _l4(pkt, IPH_PROTO_TCP, srcAddr, dstAddr)
    if err:
        return None, 0, 0, 0, 0, 0, err
    off = int(r["payload_off"]) - 20  # record offsets are in the wrapped packet's coordinates
    return (bytes(pkt)[off:], int(r["sport"]), int(r["dport"]), int(r["l4_seq"]), int(r["l4_ack"]),
            int(r["l4_aux"]), None)


def ParseIcmpPkt(pkt):
    """protocol.ParseIcmpPkt (protocol/icmp.go:33-63): (payload, icmpType, icmpId, icmpSeq, err).
    The checksum is always verified, as the reference does."""
    r, err = _l4(pkt, IPH_PROTO_ICMP, b"\0\0\0\0", b"\0\0\0\0")
    if err:
        return None, ICMP_UNKNOWN, None, 0, err
    seq = int(r["l4_seq"])
    return bytes(pkt)[8:], int(r["l4_aux"]), (seq >> 16).to_bytes(2, "big"), seq & 0xFFFF, None


__all__ = [name for name in dir() if not name.startswith("_")] + ["STATUS"]
