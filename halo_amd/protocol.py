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

# status -> the error the reference returns at that check (None: no error / build-defined)
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
    "L4_LEN": "udp/tcp/icmp packet len out of range",               # udp.go:23 / tcp.go:38 / icmp.go:35
    "ICMP_TYPE": "not support type of icmp packet",                 # icmp.go:46
    "ICMP_CODE": "not support type of icmp packet",                 # icmp.go:50
    "L4_CKSUM": "check sum error",                                  # udp.go:43 / tcp.go:55 / icmp.go:54
}


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


__all__ = [name for name in dir() if not name.startswith("_")] + ["STATUS"]


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
