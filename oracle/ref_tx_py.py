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
