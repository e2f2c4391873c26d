"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of halo's forward/transmit rewrite (§8f f2).

Written independently of oracle/halo_tx_oracle.c, on ``bytearray`` packets, from the Go source
(paths under /root/reference). Runs only in the build container, to generate the committed
fixtures tests/golden/tx_* (tests/gen_golden.py) and to cross-check the C restatement.

  handle_ipv4_pkt_ttl   protocol/ipv4.go:134-145
  recalc_ipv4           protocol/ipv4.go:148-161
  recalc_icmp           protocol/ipv4.go:164-174
  recalc_tcp / _udp     protocol/ipv4.go:177-200, :203-226
  nat_change_src / _dst protocol/ipv4.go:249-275, :277-302
  tx_frame step order   engine/ipv4_engine.go:108-269 (Ipv4RouteForward: DNAT, TTL, SNAT)
  dpdk_tx_fill          cgo/dpdk.c:333-365 (offloads off) over DPDK 20.11.10's rte_ipv4_cksum /
                        rte_ipv4_udptcp_cksum. DPDK sums little-endian host words and stores the
                        result as a host u16; this restatement uses the byte-order independence of
                        the one's-complement sum instead (sum big-endian words, store big-endian),
                        so it is a different derivation of the same bytes.
"""
from __future__ import annotations

from .ref_py import get_checksum

NAT_DST, TTL, NAT_SRC, RECALC, DPDK_FILL = 0x01, 0x02, 0x04, 0x08, 0x10
R_TTL_ALIVE, R_SKIPPED, R_OVERRUN = 0x01, 0x02, 0x04


def _put16(b: bytearray, at: int, v: int):
    b[at] = (v >> 8) & 0xFF
    b[at + 1] = v & 0xFF


def recalc_ipv4(pkt: bytearray, en: bool) -> bool:
    """Returns True when the length guard returned early."""
    if len(pkt) < 20:
        return True
    _put16(pkt, 10, 0)
    if en:
        _put16(pkt, 10, get_checksum(bytes(pkt[:20])))
    return False


def recalc_icmp(pkt: bytearray) -> bool:
    if len(pkt) < 24:
        return True
    _put16(pkt, 22, 0)
    _put16(pkt, 22, get_checksum(bytes(pkt[20:])))
    return False


def _recalc_l4(pkt: bytearray, en: bool, guard: int, at: int, proto: int) -> bool:
    if len(pkt) < guard:
        return True
    _put16(pkt, at, 0)
    if not en:
        return False
    total_len = (pkt[2] << 8) | pkt[3]
    fake = bytes(pkt[12:16]) + bytes(pkt[16:20]) + bytes([0, proto]) + ((total_len - 20) & 0xFFFF).to_bytes(2, "big")
    _put16(pkt, at, get_checksum(fake + bytes(pkt[20:])))
    return False


def recalc_tcp(pkt: bytearray, en: bool) -> bool:
    return _recalc_l4(pkt, en, 38, 36, 6)


def recalc_udp(pkt: bytearray, en: bool) -> bool:
    return _recalc_l4(pkt, en, 28, 26, 17)


def handle_ipv4_pkt_ttl(pkt: bytearray, en: bool):
    """Returns (alive, skipped)."""
    if len(pkt) < 9:
        return False, True
    if pkt[8] <= 1:
        return False, False
    pkt[8] -= 1
    return True, recalc_ipv4(pkt, en)


def _nat(pkt: bytearray, ip: int, port: int, en: bool, addr_at: int, port_at: int) -> bool:
    if len(pkt) < 26:
        return True
    pkt[addr_at:addr_at + 4] = ip.to_bytes(4, "big")
    skipped = recalc_ipv4(pkt, en)
    proto = pkt[9]
    if proto == 1:
        _put16(pkt, 24, port)
        skipped |= recalc_icmp(pkt)
    elif proto == 6:
        _put16(pkt, port_at, port)
        skipped |= recalc_tcp(pkt, en)
    elif proto == 17:
        _put16(pkt, port_at, port)
        skipped |= recalc_udp(pkt, en)
    return skipped


def nat_change_src(pkt: bytearray, ip: int, port: int, en: bool) -> bool:
    return _nat(pkt, ip, port, en, 12, 20)


def nat_change_dst(pkt: bytearray, ip: int, port: int, en: bool) -> bool:
    return _nat(pkt, ip, port, en, 16, 22)


def _ones_sum_be(b: bytes) -> int:
    if len(b) & 1:
        b = b + b"\0"
    s = sum(int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def dpdk_tx_fill(frame: bytearray) -> int:
    """cgo/dpdk.c:333-365; returns R_OVERRUN or 0. Build-defined where DPDK would touch bytes
    beyond the frame: that checksum stays zero and R_OVERRUN is reported."""
    L = len(frame)
    if L < 14 or frame[12:14] != b"\x08\x00":
        return 0
    if L < 34:
        return R_OVERRUN
    rc = 0
    _put16(frame, 24, 0)
    hlen = (frame[14] & 0xF) * 4
    if 14 + hlen <= L:
        _put16(frame, 24, (~_ones_sum_be(bytes(frame[14:14 + hlen]))) & 0xFFFF)
    else:
        rc |= R_OVERRUN
    proto = frame[23]
    at = {17: 14 + 20 + 6, 6: 14 + 20 + 16}.get(proto)
    if at is None:
        return rc
    if at + 2 > L:
        return rc | R_OVERRUN
    _put16(frame, at, 0)
    l3 = (frame[16] << 8) | frame[17]
    if l3 < hlen:
        return rc
    l4 = l3 - hlen
    if 34 + l4 > L:
        return rc | R_OVERRUN
    pseudo = bytes(frame[26:34]) + bytes([0, proto]) + l4.to_bytes(2, "big")
    s = _ones_sum_be(pseudo) + _ones_sum_be(bytes(frame[34:34 + l4]))
    s = (s & 0xFFFF) + (s >> 16)
    c = (~s) & 0xFFFF
    if c == 0 and proto == 17:
        c = 0xFFFF
    _put16(frame, at, c)
    return rc


def tx_frame(frame: bytearray, steps: int, dst_ip=0, dst_port=0, src_ip=0, src_port=0, check_sum_enable=True) -> int:
    """Applies `steps` to `frame` in place; returns the HALO_TX_R_* byte."""
    en = check_sum_enable
    if len(frame) < 14:
        return R_SKIPPED if steps & (NAT_DST | TTL | NAT_SRC | RECALC) else 0
    pkt = frame[14:]  # a copy; written back below (Go's pkt aliases the frame)
    skipped = False
    r = 0
    if steps & NAT_DST:
        skipped |= nat_change_dst(pkt, dst_ip, dst_port, en)
    if steps & TTL:
        alive, sk = handle_ipv4_pkt_ttl(pkt, en)
        skipped |= sk
        if not alive:
            frame[14:] = pkt
            return R_SKIPPED if skipped else 0
        r |= R_TTL_ALIVE
    if steps & NAT_SRC:
        skipped |= nat_change_src(pkt, src_ip, src_port, en)
    if steps & RECALC:
        skipped |= recalc_ipv4(pkt, en)
        if len(pkt) >= 10:
            if pkt[9] == 1:
                skipped |= recalc_icmp(pkt)
            elif pkt[9] == 6:
                skipped |= recalc_tcp(pkt, en)
            elif pkt[9] == 17:
                skipped |= recalc_udp(pkt, en)
    frame[14:] = pkt
    if skipped:
        r |= R_SKIPPED
    if steps & DPDK_FILL:
        r |= dpdk_tx_fill(frame)
    return r


# ---- the Build* half of row f2 (locally originated packets), restated from the Go source -------
#   BuildUdpPkt protocol/udp.go:52-91, BuildTcpPkt tcp.go:73-123, BuildIcmpPkt icmp.go:66-89,
#   BuildIpv4Pkt ipv4.go:89-131 (iphId ipv4.go:33, `iphId++` before use), BuildEthFrm
#   ethernet.go:58-82; drivers NetIf.Tx{Udp,Tcp,Icmp} -> TxIpv4 (engine/ipv4_engine.go:50-99,
#   the LoChan copy at :72-79) -> TxEthernet (engine/ethernet_engine.go:34-50).
B_OK, B_PAYLOAD_LEN, B_PROTO, B_SLOT = 0, 1, 2, 3
MODE_ETH, MODE_LOOPBACK = 0, 1


class BuildError(Exception):
    pass


def go_build_udp(payload: bytes, src_port: int, dst_port: int, src: bytes, dst: bytes, en: bool) -> bytearray:
    if len(payload) > 1472:
        raise BuildError("payload len must <= 1472")
    udp_len = (len(payload) + 8) & 0xFFFF
    pkt = bytearray()
    pkt += src_port.to_bytes(2, "big") + dst_port.to_bytes(2, "big") + udp_len.to_bytes(2, "big") + b"\x00\x00"
    pkt += payload
    if en:
        fake = bytes(src) + bytes(dst) + b"\x00\x11" + udp_len.to_bytes(2, "big")
        _put16(pkt, 6, get_checksum(fake + bytes(pkt)))
    else:
        _put16(pkt, 6, 0)
    return pkt


def go_build_tcp(payload: bytes, src_port: int, dst_port: int, src: bytes, dst: bytes, seq: int, ack: int,
                 flags: int, en: bool) -> bytearray:
    if len(payload) > 1460:
        raise BuildError("payload len must <= 1460")
    pkt = bytearray()
    pkt += src_port.to_bytes(2, "big") + dst_port.to_bytes(2, "big")
    pkt += seq.to_bytes(4, "big") + ack.to_bytes(4, "big")
    pkt += bytes([0x50, flags, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00])
    pkt += payload
    if en:
        total = 20 + len(payload)
        fake = bytes(src) + bytes(dst) + b"\x00\x06" + (total & 0xFFFF).to_bytes(2, "big")
        _put16(pkt, 16, get_checksum(fake + bytes(pkt)))
    else:
        _put16(pkt, 16, 0)
    return pkt


def go_build_icmp(payload: bytes, icmp_type: int, icmp_id: bytes, seq: int) -> bytearray:
    if len(payload) > 1472:
        raise BuildError("payload len must <= 1472")
    pkt = bytearray([icmp_type, 0x00, 0x00, 0x00]) + bytearray(icmp_id) + bytearray(seq.to_bytes(2, "big"))
    pkt += payload
    _put16(pkt, 2, get_checksum(bytes(pkt)))  # CheckSumEnable is not consulted (icmp.go:84-87)
    return pkt


class IphId:
    """protocol.iphId: the package-global IPv4 identification counter."""

    def __init__(self, value: int = 0):
        self.value = value & 0xFFFF


def go_build_ipv4(payload: bytes, proto: int, src: bytes, dst: bytes, iph: IphId, en: bool) -> bytearray:
    if len(payload) > 1480:
        raise BuildError("payload len must <= 1480 bytes")
    pkt = bytearray([0x45, 0x00]) + bytearray(((len(payload) + 20) & 0xFFFF).to_bytes(2, "big"))
    iph.value = (iph.value + 1) & 0xFFFF
    pkt += iph.value.to_bytes(2, "big") + b"\x00\x00" + bytes([0x80, proto, 0x00, 0x00]) + bytes(src) + bytes(dst)
    _put16(pkt, 10, get_checksum(bytes(pkt)) if en else 0)
    return pkt + bytearray(payload)


def go_build_eth(payload: bytes, dst_mac: bytes, src_mac: bytes, eth_proto: int) -> bytearray:
    if len(payload) > 1500:
        raise BuildError("payload len must <= 1500 bytes")
    frm = bytearray(dst_mac) + bytearray(src_mac) + bytearray(eth_proto.to_bytes(2, "big")) + bytearray(payload)
    return frm + bytearray(max(0, 60 - len(frm)))


def tx_build(desc: dict, payload: bytes, src_mac: bytes, iph: IphId, check_sum_enable=True):
    """One halo_tx_build_desc_t through Tx* -> TxIpv4 -> TxEthernet / LoChan: (result, frame)."""
    en = bool(check_sum_enable)
    src = desc["src_ip"].to_bytes(4, "big")
    dst = desc["dst_ip"].to_bytes(4, "big")
    proto = desc["proto"]
    try:
        if proto == 0x11:
            l4 = go_build_udp(payload, desc["src_port"], desc["dst_port"], src, dst, en)
        elif proto == 0x06:
            l4 = go_build_tcp(payload, desc["src_port"], desc["dst_port"], src, dst, desc["seq"], desc["ack"],
                              desc["aux"], en)
        elif proto == 0x01:
            l4 = go_build_icmp(payload, desc["aux"], desc["src_port"].to_bytes(2, "big"), desc["dst_port"])
        else:
            return B_PROTO, b""
    except BuildError:
        return B_PAYLOAD_LEN, b""
    ip = go_build_ipv4(bytes(l4), proto, src, dst, iph, en)
    if desc["mode"] == MODE_LOOPBACK:
        return B_OK, bytes(ip)
    return B_OK, bytes(go_build_eth(bytes(ip), bytes(desc["dst_mac"]), src_mac, 0x0800))


def tx_build_len(desc: dict) -> int:
    """The frame length the Build* chain produces for a descriptor (no bytes needed)."""
    l4 = (20 if desc["proto"] == 0x06 else 8) + desc["payload_len"]
    return 20 + l4 if desc["mode"] == MODE_LOOPBACK else max(60, 34 + l4)


# ---- IcmpTtlDeepNat (engine/icmp_engine.go:55-86): the NAT rewrite of the packet an ICMP
#      time-exceeded message quotes, applied by Ipv4RouteForward before its own DNAT
#      (engine/ipv4_engine.go:111-130). The NAT table lookup (NatGetFlowByWan) is the caller's.
def icmp_quote(eth_payload: bytes, check_sum_enable=True):
    """The checks of IcmpTtlDeepNat up to its flow lookup. Returns (status name, lookup args) with
    lookup args = (proto, remote ip, remote port, wan ip, wan port) as NatGetFlowByWan takes them,
    or None when the function returns early. Status: "OK", the rx status of ParseIpv4Pkt /
    ParseIcmpPkt when they fail, "IP_PROTO" when the packet is not ICMP, "ICMP_TYPE" when the type
    is not ICMP_TTL, "L4_LEN" when the quote is shorter than 28 bytes."""
    from . import ref_py as R

    c = R.Cfg(check_sum_enable, False)
    ipv4_payload, proto, _src, _dst, _tl, err = R.parse_ipv4_pkt(bytes(eth_payload), c)
    if err:
        return err, None
    if proto != 0x01:
        return "IP_PROTO", None
    icmp_payload, icmp_type, _id, _seq, err = R.parse_icmp_pkt(ipv4_payload, c)
    if err:
        return err, None
    if icmp_type != 0x0B:
        return "ICMP_TYPE", None
    if len(icmp_payload) < 28:
        return "L4_LEN", None
    wan_port, remote_port = R.nat_get_src_dst_port(icmp_payload)
    return "OK", (icmp_payload[9], R.ip_addr_to_u(icmp_payload[16:20]), remote_port,
                  R.ip_addr_to_u(icmp_payload[12:16]), wan_port)


def icmp_ttl_deep_nat(eth_payload: bytearray, lan_ip: int, lan_port: int, found: bool,
                      check_sum_enable=True) -> bool:
    """IcmpTtlDeepNat on eth_payload in place, natFlow = (lan_ip, lan_port) when found.
    Returns isIcmpTtl."""
    st, args = icmp_quote(bytes(eth_payload), check_sum_enable)
    if st != "OK" or not found:
        return False
    total_len = (eth_payload[2] << 8) | eth_payload[3]
    # icmpPayload = ipv4Payload[8:] = eth_payload[28:totalLen], a slice aliasing eth_payload
    inner = bytearray(eth_payload[28:total_len])
    nat_change_src(inner, lan_ip, lan_port, check_sum_enable)
    eth_payload[28:total_len] = inner
    nat_change_dst(eth_payload, lan_ip, 0, check_sum_enable)  # the whole (untrimmed) slice
    return True
