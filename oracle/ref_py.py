"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of halo's rx parse path.

Written independently of oracle/halo_rx_oracle.c, function by function from the Go source
(paths under /root/reference). It runs only in the build container, to produce the committed
golden fixtures (tests/gen_golden.py) and to cross-check the C restatement on small batches.
Go slices are Python bytes; a Go `error` is returned as a status name.

  get_checksum        protocol/utils.go:11-31
  ip_addr_to_u        protocol/utils.go:34-44
  parse_eth_frm       protocol/ethernet.go:29-55
  parse_ipv4_pkt      protocol/ipv4.go:48-86
  parse_udp_pkt       protocol/udp.go:21-49
  parse_tcp_pkt       protocol/tcp.go:36-70
  parse_icmp_pkt      protocol/icmp.go:33-63
  nat_get_src_dst_port protocol/ipv4.go:229-246
  rx_ethernet/rx_ipv4 engine/ethernet_engine.go:13-31, engine/ipv4_engine.go:18-47
  rx_lo_packet/engine_lo  PacketHandle's LoChan drain, engine/engine.go:353-381
"""
from __future__ import annotations

STATUS = ["OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
          "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM"]
ACTIONS = ["DROP_ETH", "IGNORE_MAC", "ARP", "IGNORE_TYPE", "DROP_IP", "BCAST_UDP", "DROP_BCAST_UDP",
           "IGNORE_BCAST", "FORWARD", "LOCAL_ICMP", "LOCAL_UDP", "LOCAL_TCP", "DROP_L4", "LO_NOT_OWN"]


class Cfg:
    def __init__(self, check_sum_enable=True, jumbo=False):
        self.check_sum_enable = check_sum_enable
        self.eth_max, self.ip_max, self.l4_max = (9014, 9000, 8980) if jumbo else (1514, 1500, 1480)


def get_checksum(data: bytes) -> int:
    s = 0
    length = len(data)
    index = 0
    while length > 1:
        s += (data[index] << 8) + data[index + 1]
        s &= 0xFFFFFFFF  # uint32 arithmetic
        index += 2
        length -= 2
    if length > 0:
        s += data[index] << 8
        s &= 0xFFFFFFFF
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ip_addr_to_u(a) -> int:
    if a is None or len(a) != 4:
        return 0
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


def be16(b: bytes) -> int:
    return (b[0] << 8) | b[1]


def parse_eth_frm(frm: bytes, c: Cfg):
    if len(frm) < 42 or len(frm) > c.eth_max:
        return None, None, None, 0xFFFF, "ETH_LEN"
    t = be16(frm[12:14])
    if t not in (0x05DC, 0x0800, 0x0806, 0x86DD):
        return None, None, None, 0xFFFF, "ETH_TYPE"
    return frm[14:], frm[0:6], frm[6:12], t, None


def parse_ipv4_pkt(pkt: bytes, c: Cfg):
    """Returns (payload, proto, src, dst, totalLen, err). totalLen outside [20, len(pkt)]
    is the build-defined TOTLEN_* status (Go panics or reads stale bytes, ipv4.go:84)."""
    if len(pkt) < 20 or len(pkt) > c.ip_max:
        return None, 0xFF, None, None, 0, "IP_LEN"
    if pkt[0] != 0x45:
        return None, 0xFF, None, None, 0, "IP_VER"
    total_len = be16(pkt[2:4])
    if (pkt[6] != 0x40 and pkt[6] != 0x00) or pkt[7] != 0x00:
        return None, 0xFF, None, None, 0, "IP_FRAG"
    if pkt[9] not in (0x01, 0x06, 0x11):
        return None, 0xFF, None, None, 0, "IP_PROTO"
    if c.check_sum_enable and get_checksum(pkt[0:20]) != 0:
        return None, 0xFF, None, None, 0, "IP_HDR_CKSUM"
    if total_len < 20:
        return None, 0xFF, None, None, 0, "IP_TOTLEN_UNDERFLOW"
    if total_len > len(pkt):
        return None, 0xFF, None, None, 0, "IP_TOTLEN_OVERRUN"
    return pkt[20:total_len], pkt[9], pkt[12:16], pkt[16:20], total_len, None


def parse_udp_pkt(pkt: bytes, src: bytes, dst: bytes, c: Cfg):
    if len(pkt) < 8 or len(pkt) > c.l4_max:
        return None, 0, 0, "L4_LEN"
    sport, dport, total_len = be16(pkt[0:2]), be16(pkt[2:4]), be16(pkt[4:6])
    if c.check_sum_enable:
        fake = bytes(src) + bytes(dst) + bytes([0x00, 0x11, total_len >> 8, total_len & 0xFF])
        if get_checksum(fake + pkt) != 0:
            return None, 0, 0, "L4_CKSUM"
    return pkt[8:], sport, dport, None


def parse_tcp_pkt(pkt: bytes, src: bytes, dst: bytes, c: Cfg):
    if len(pkt) < 20 or len(pkt) > c.l4_max:
        return None, 0, 0, 0, 0, 0, "L4_LEN"
    sport, dport = be16(pkt[0:2]), be16(pkt[2:4])
    seq = int.from_bytes(pkt[4:8], "big")
    ack = int.from_bytes(pkt[8:12], "big")
    header_len = pkt[12] >> 4  # words, used as bytes (tcp.go:49,68)
    flags = pkt[13]
    if c.check_sum_enable:
        tl = len(pkt)
        fake = bytes(src) + bytes(dst) + bytes([0x00, 0x06, (tl >> 8) & 0xFF, tl & 0xFF])
        if get_checksum(fake + pkt) != 0:
            return None, 0, 0, 0, 0, 0, "L4_CKSUM"
    return pkt[header_len:], sport, dport, seq, ack, flags, None


def parse_icmp_pkt(pkt: bytes, c: Cfg):
    if len(pkt) < 8 or len(pkt) > c.l4_max:
        return None, 0xFF, None, 0, "L4_LEN"
    if pkt[0] not in (0x08, 0x00, 0x0B):
        return None, 0xFF, None, 0, "ICMP_TYPE"
    if pkt[1] != 0x00:
        return None, 0xFF, None, 0, "ICMP_CODE"
    if get_checksum(pkt) != 0:  # always (icmp.go:53)
        return None, 0xFF, None, 0, "L4_CKSUM"
    return pkt[8:], pkt[0], pkt[4:6], be16(pkt[6:8]), None


def nat_get_src_dst_port(pkt: bytes):
    if len(pkt) < 26:
        return 0, 0
    if pkt[9] == 0x01:
        return be16(pkt[24:26]), be16(pkt[24:26])
    if pkt[9] in (0x06, 0x11):
        return be16(pkt[20:22]), be16(pkt[22:24])
    return 0, 0


def rx_frame(frame: bytes, mac: bytes, own_ip: int, check_sum_enable=True, jumbo=False) -> dict:
    """The halo_rx_result_t record for one frame (field contract in include/halo_rx.h)."""
    c = Cfg(check_sum_enable, jumbo)
    r = dict(status="OK", flags=0, ethertype=0xFFFF, ip_proto=0xFF, l4_aux=0, ip_total_len=0, src_ip=0, dst_ip=0,
             sport=0, dport=0, payload_off=0, payload_len=0, l4_seq=0, l4_ack=0)
    eth_payload, dst_mac, _src_mac, et, err = parse_eth_frm(frame, c)
    r["ethertype"] = et
    if err:
        r["status"] = err
        return r
    if dst_mac == mac or dst_mac == b"\xff" * 6:
        r["flags"] |= 1
    r["payload_off"], r["payload_len"] = 14, len(eth_payload)
    if et != 0x0800:
        return r
    ip_payload, proto, src, dst, total_len, err = parse_ipv4_pkt(eth_payload, c)
    if err:
        r["status"] = err
        return r
    r.update(ip_proto=proto, ip_total_len=total_len, src_ip=ip_addr_to_u(src), dst_ip=ip_addr_to_u(dst))
    if dst[3] == 255:
        r["flags"] |= 2
    if r["dst_ip"] == own_ip:
        r["flags"] |= 4
    r["sport"], r["dport"] = nat_get_src_dst_port(eth_payload)
    r["payload_off"], r["payload_len"] = 34, len(ip_payload)
    if proto == 0x11:
        pay, _sp, _dp, err = parse_udp_pkt(ip_payload, src, dst, c)
        off = 8
    elif proto == 0x06:
        pay, _sp, _dp, seq, ack, fl, err = parse_tcp_pkt(ip_payload, src, dst, c)
        if not err:
            r.update(l4_aux=fl, l4_seq=seq, l4_ack=ack)
        off = None if err else ip_payload[12] >> 4
    else:
        pay, typ, icmp_id, icmp_seq, err = parse_icmp_pkt(ip_payload, c)
        if not err:
            r.update(l4_aux=typ, l4_seq=(be16(icmp_id) << 16) | icmp_seq)
        off = 8
    if err:
        r["status"] = err
        return r
    r["payload_off"], r["payload_len"] = 34 + off, len(pay)
    return r


def engine_rx(frame: bytes, mac: bytes, own_ip: int, nat_enable=False, check_sum_enable=True, jumbo=False) -> str:
    """The reference engine's action for one frame (RxEthernet -> RxIpv4 -> Rx*)."""
    c = Cfg(check_sum_enable, jumbo)
    eth_payload, dst_mac, _s, et, err = parse_eth_frm(frame, c)
    if err:
        return "DROP_ETH"
    if not (dst_mac == mac or dst_mac == b"\xff" * 6):
        return "IGNORE_MAC"
    if et == 0x0806:
        return "ARP"
    if et != 0x0800:
        return "IGNORE_TYPE"
    ip_payload, proto, src, dst, _tl, err = parse_ipv4_pkt(eth_payload, c)
    if err:
        return "DROP_IP"
    if dst[3] == 255:
        if proto != 0x11:
            return "IGNORE_BCAST"
        return "DROP_BCAST_UDP" if parse_udp_pkt(ip_payload, src, dst, c)[3] else "BCAST_UDP"
    own = own_ip.to_bytes(4, "big")
    if dst != own or nat_enable:
        return "FORWARD"
    if proto == 0x01:
        return "DROP_L4" if parse_icmp_pkt(ip_payload, c)[4] else "LOCAL_ICMP"
    if proto == 0x11:
        return "DROP_L4" if parse_udp_pkt(ip_payload, src, own, c)[3] else "LOCAL_UDP"
    return "DROP_L4" if parse_tcp_pkt(ip_payload, src, own, c)[6] else "LOCAL_TCP"


def rx_lo_packet(pkt: bytes, own_ip: int, check_sum_enable=True, jumbo=False) -> dict:
    """The record for one LoChan packet (HALO_RX_L3_START, include/halo_rx.h): the chain of
    rx_frame without its Ethernet layer. engine/engine.go:361 hands the packet straight to
    ParseIpv4Pkt; the channel carries IPv4 only, so the record's EtherType is 0x0800."""
    c = Cfg(check_sum_enable, jumbo)
    r = dict(status="OK", flags=0, ethertype=0x0800, ip_proto=0xFF, l4_aux=0, ip_total_len=0, src_ip=0, dst_ip=0,
             sport=0, dport=0, payload_off=0, payload_len=0, l4_seq=0, l4_ack=0)
    ip_payload, proto, src, dst, total_len, err = parse_ipv4_pkt(pkt, c)
    if err:
        r["status"] = err
        return r
    r.update(ip_proto=proto, ip_total_len=total_len, src_ip=ip_addr_to_u(src), dst_ip=ip_addr_to_u(dst))
    if dst[3] == 255:
        r["flags"] |= 2
    if r["dst_ip"] == own_ip:
        r["flags"] |= 4
    r["sport"], r["dport"] = nat_get_src_dst_port(pkt)
    r["payload_off"], r["payload_len"] = 20, len(ip_payload)
    if proto == 0x11:
        pay, _sp, _dp, err = parse_udp_pkt(ip_payload, src, dst, c)
        off = 8
    elif proto == 0x06:
        pay, _sp, _dp, seq, ack, fl, err = parse_tcp_pkt(ip_payload, src, dst, c)
        if not err:
            r.update(l4_aux=fl, l4_seq=seq, l4_ack=ack)
        off = None if err else ip_payload[12] >> 4
    else:
        pay, typ, icmp_id, icmp_seq, err = parse_icmp_pkt(ip_payload, c)
        if not err:
            r.update(l4_aux=typ, l4_seq=(be16(icmp_id) << 16) | icmp_seq)
        off = 8
    if err:
        r["status"] = err
        return r
    r["payload_off"], r["payload_len"] = 20 + off, len(pay)
    return r


def engine_lo(pkt: bytes, own_ip: int, check_sum_enable=True, jumbo=False) -> str:
    """What PacketHandle's LoChan drain does with one packet (engine/engine.go:360-377)."""
    c = Cfg(check_sum_enable, jumbo)
    ip_payload, proto, src, dst, _tl, err = parse_ipv4_pkt(pkt, c)
    if err:
        return "DROP_IP"  # logged, continue
    own = own_ip.to_bytes(4, "big")
    if dst != own:
        return "LO_NOT_OWN"  # bytes.Equal(ipv4DstAddr, i.IpAddr) fails: continue
    if proto == 0x01:  # i.RxIcmp
        return "DROP_L4" if parse_icmp_pkt(ip_payload, c)[4] else "LOCAL_ICMP"
    if proto == 0x11:  # i.RxUdp: pseudo dst = i.IpAddr (udp_engine.go:11)
        return "DROP_L4" if parse_udp_pkt(ip_payload, src, own, c)[3] else "LOCAL_UDP"
    return "DROP_L4" if parse_tcp_pkt(ip_payload, src, own, c)[6] else "LOCAL_TCP"


# ---- frame builders for fixtures (BuildEthFrm / BuildIpv4Pkt / BuildUdpPkt / BuildTcpPkt /
#      BuildIcmpPkt: protocol/ethernet.go:58-82, ipv4.go:89-131, udp.go:52-91, tcp.go:73-123,
#      icmp.go:66-89), with every field overridable so fixtures can break one check at a time.
def build_udp(payload: bytes, sport: int, dport: int, src: bytes, dst: bytes, udp_len=None, csum=None) -> bytes:
    ln = len(payload) + 8 if udp_len is None else udp_len
    seg = bytearray(sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + ln.to_bytes(2, "big") + b"\0\0" + payload)
    fake = src + dst + bytes([0, 0x11]) + ln.to_bytes(2, "big")
    s = get_checksum(fake + bytes(seg)) if csum is None else csum
    seg[6:8] = s.to_bytes(2, "big")
    return bytes(seg)


def build_tcp(payload: bytes, sport: int, dport: int, src: bytes, dst: bytes, seq: int, ack: int, flags: int,
              off_byte=0x50, csum=None) -> bytes:
    seg = bytearray(sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + seq.to_bytes(4, "big") +
                    ack.to_bytes(4, "big") + bytes([off_byte, flags, 0x01, 0x00, 0, 0, 0, 0]) + payload)
    fake = src + dst + bytes([0, 0x06]) + len(seg).to_bytes(2, "big")
    s = get_checksum(fake + bytes(seg)) if csum is None else csum
    seg[16:18] = s.to_bytes(2, "big")
    return bytes(seg)


def build_icmp(payload: bytes, typ: int, icmp_id: bytes, seq: int, code=0, csum=None) -> bytes:
    seg = bytearray(bytes([typ, code, 0, 0]) + icmp_id + seq.to_bytes(2, "big") + payload)
    s = get_checksum(bytes(seg)) if csum is None else csum
    seg[2:4] = s.to_bytes(2, "big")
    return bytes(seg)


def build_ipv4(payload: bytes, proto: int, src: bytes, dst: bytes, ident=1, ttl=0x80, frag=b"\0\0",
               ver_ihl=0x45, total_len=None, csum=None) -> bytes:
    tl = len(payload) + 20 if total_len is None else total_len
    hdr = bytearray(bytes([ver_ihl, 0]) + tl.to_bytes(2, "big") + ident.to_bytes(2, "big") + frag +
                    bytes([ttl, proto, 0, 0]) + src + dst)
    s = get_checksum(bytes(hdr)) if csum is None else csum
    hdr[10:12] = s.to_bytes(2, "big")
    return bytes(hdr) + payload


def build_eth(payload: bytes, dst: bytes, src: bytes, proto: int, pad=True) -> bytes:
    f = dst + src + proto.to_bytes(2, "big") + payload
    if pad and len(f) < 60:
        f += b"\0" * (60 - len(f))
    return f
