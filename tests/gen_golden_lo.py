"""Generate the LoChan (loopback drain) fixtures tests/golden/lo_packets.{bin,json} (build container).

PacketHandle drains a NetIf's LoChan every 99 polls (engine/engine.go:353-381): each entry is
a bare IPv4 packet — TxIpv4's loopback copy of a packet it built for its own address
(engine/ipv4_engine.go:72-79: exactly totalLen bytes) or Ipv4RouteForward's copy of a received
frame's Ethernet payload for another NetIf's address (:195-200: Ethernet padding included).
Expected records and drain decisions come from oracle/ref_py.py (rx_lo_packet / engine_lo),
under the four flags words; the C oracle and the GPU (HALO_RX_L3_START) are tested against them.

    python tests/gen_golden_lo.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_py as R  # noqa: E402
from tests import gen_golden as G  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
FLAGS = (0, 1, 2, 3)
OTHER = bytes([192, 168, 100, 7])


def ip_udp(payload=bytes(range(22)), src=G.PEER, dst=G.OWN, **ip_kw):
    return R.build_ipv4(R.build_udp(payload, 12345, 22222, src, dst), 0x11, src, dst, **ip_kw)


def cases():
    c = []
    # every golden Ethernet frame's payload, as Ipv4RouteForward copies it (padding included)
    blob = open(os.path.join(OUT, "frames.bin"), "rb").read()
    for e in json.load(open(os.path.join(OUT, "frames.json")))["frames"]:
        f = blob[e["offset"]:e["offset"] + e["len"]]
        if len(f) >= 14 and f[12:14] == b"\x08\x00":
            c.append(("fwd_" + e["name"], f[14:]))
    # ParseIpv4Pkt's own length check (ipv4.go:49), unreachable behind ParseEthFrm, reachable here
    c.append(("lo_len_0", b""))
    c.append(("lo_len_19", ip_udp()[:19]))
    c.append(("lo_len_20_hdr_only", R.build_ipv4(b"", 0x11, G.PEER, G.OWN)))
    c.append(("lo_len_1500", ip_udp(payload=bytes(random.Random(11).randrange(256) for _ in range(1472)))))
    c.append(("lo_len_1501", ip_udp(payload=bytes(random.Random(12).randrange(256) for _ in range(1473)))))
    c.append(("lo_len_9000", ip_udp(payload=bytes(random.Random(13).randrange(256) for _ in range(8972)))))
    c.append(("lo_len_9001", ip_udp(payload=bytes(random.Random(14).randrange(256) for _ in range(8973)))))
    # NatGetSrcDstPort below 26 bytes (ipv4.go:230) and the L4 length checks around it
    for ln in range(20, 30):
        for proto in (0x01, 0x06, 0x11):
            p = bytearray(R.build_ipv4(bytes(range(0x40, 0x40 + ln - 20)), proto, G.PEER, G.OWN))
            c.append((f"lo_short_{ln}_p{proto}", bytes(p)))
    # TxIpv4's loopback copies: built for the own address (and a few that the drain skips)
    for proto, seg in ((0x11, R.build_udp(b"loopback udp", 5353, 53, G.OWN, G.OWN)),
                       (0x06, R.build_tcp(b"loopback tcp", 40001, 22, G.OWN, G.OWN, 7, 9, 0x18)),
                       (0x01, R.build_icmp(b"ping self", 8, b"\x00\x01", 1))):
        c.append((f"tx_loop_p{proto}", R.build_ipv4(seg, proto, G.OWN, G.OWN, ident=77)))
        c.append((f"tx_loop_other_p{proto}", R.build_ipv4(seg, proto, G.OWN, OTHER, ident=78)))
        c.append((f"tx_loop_bcast_p{proto}", R.build_ipv4(seg, proto, G.OWN, bytes([192, 168, 100, 255]))))
    c.append(("lo_udp_bad_csum_own", R.build_ipv4(R.build_udp(b"x" * 9, 1, 2, G.PEER, G.OWN, csum=0x1111), 0x11,
                                                  G.PEER, G.OWN)))
    c.append(("lo_udp_bad_csum_other", R.build_ipv4(R.build_udp(b"x" * 9, 1, 2, G.PEER, OTHER, csum=0x1111), 0x11,
                                                    G.PEER, OTHER)))
    c.append(("lo_icmp_bad_csum", R.build_ipv4(R.build_icmp(b"abc", 0, b"\x00\x02", 3, csum=5), 0x01, G.PEER, G.OWN)))
    c.append(("lo_tcp_quirk_offset", R.build_ipv4(R.build_tcp(b"data" * 5, 1, 2, G.PEER, G.OWN, 1, 2, 0x10,
                                                              off_byte=0xF0), 0x06, G.PEER, G.OWN)))
    c.append(("lo_padding_garbage", ip_udp(payload=b"\x01\x02") + b"\xde\xad\xbe\xef\x99"))
    c.append(("lo_totlen_overrun", ip_udp(total_len=51)))
    c.append(("lo_totlen_underflow", ip_udp(total_len=12)))
    c.append(("lo_ver_46", ip_udp(ver_ihl=0x46)))
    c.append(("lo_frag", ip_udp(frag=b"\x20\x00")))
    c.append(("lo_proto_2", R.build_ipv4(bytes(12), 0x02, G.PEER, G.OWN)))
    c.append(("lo_hdr_csum_bad", ip_udp(csum=0x0101)))
    # seeded random packets with single-bit flips
    rnd = random.Random(0x4C4F)
    for k in range(120):
        kind = rnd.choice(["udp", "tcp", "icmp"])
        size = rnd.choice([20, 28, 36, 50, 51, 52, 53, 100, 556, 1486, 1500])
        dst = rnd.choice([G.OWN, G.OWN, G.OWN, OTHER])
        if kind == "udp":
            p = R.build_ipv4(R.build_udp(bytes(rnd.randrange(256) for _ in range(max(0, size - 28))),
                                         rnd.randrange(1, 65536), rnd.randrange(1, 65536), G.PEER, dst),
                             0x11, G.PEER, dst, ident=rnd.randrange(65536))
        elif kind == "tcp":
            p = R.build_ipv4(R.build_tcp(bytes(rnd.randrange(256) for _ in range(max(0, size - 40))),
                                         rnd.randrange(65536), rnd.randrange(65536), G.PEER, dst,
                                         rnd.randrange(1 << 32), rnd.randrange(1 << 32), rnd.randrange(256)),
                             0x06, G.PEER, dst)
        else:
            p = R.build_ipv4(R.build_icmp(bytes(rnd.randrange(256) for _ in range(max(0, size - 28))),
                                          rnd.choice([0, 8, 11]), bytes([rnd.randrange(256), rnd.randrange(256)]),
                                          rnd.randrange(65536)), 0x01, G.PEER, dst)
        name = f"lo_rand_{k:03d}_{kind}_{len(p)}"
        if k % 3 == 0:
            bit = rnd.randrange(0, len(p) * 8)
            b = bytearray(p)
            b[bit >> 3] ^= 1 << (bit & 7)
            p, name = bytes(b), name + f"_flip{bit}"
        c.append((name, p))
    return c


def main():
    blob = bytearray()
    entries = []
    for name, p in cases():
        off = len(blob)
        blob += p
        blob += b"\0" * ((-len(blob)) % 4)
        exp, act = {}, {}
        for fl in FLAGS:
            r = R.rx_lo_packet(p, G.OWN_U, check_sum_enable=bool(fl & 1), jumbo=bool(fl & 2))
            r["status"] = R.STATUS.index(r["status"])
            exp[str(fl)] = r
            act[str(fl)] = R.engine_lo(p, G.OWN_U, check_sum_enable=bool(fl & 1), jumbo=bool(fl & 2))
        entries.append({"name": name, "offset": off, "len": len(p), "expect": exp, "action": act})
    with open(os.path.join(OUT, "lo_packets.bin"), "wb") as fh:
        fh.write(bytes(blob))
    with open(os.path.join(OUT, "lo_packets.json"), "w") as fh:
        json.dump({"netif": {"mac": G.MAC.hex(), "ip": G.OWN_U}, "packets": entries}, fh, indent=0,
                  separators=(",", ":"))
    print(f"{len(entries)} packets, {len(blob)} bytes -> {OUT}")


if __name__ == "__main__":
    main()
