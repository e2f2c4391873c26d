"""Generate the committed golden fixtures in tests/golden/ (run in the build container).

Expected outputs come from oracle/ref_py.py (the pure-Python restatement of the Go path);
the C oracle and the GPU kernels are then tested against these files. Frames: one or more
per status code and per reference quirk, then seeded random and bit-flipped
frames. Every frame is evaluated under all four `flags` combinations.

    python tests/gen_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_py as R  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
MAC = bytes.fromhex("aaaaaaaaaaaa")
OWN = bytes([192, 168, 100, 100])
OWN_U = R.ip_addr_to_u(OWN)
PEER = bytes([192, 168, 100, 1])
SRC_MAC = bytes.fromhex("020000000001")
FLAGS = (0, 1, 2, 3)  # bit0 CheckSumEnable, bit1 jumbo extension


def udp_frame(payload=bytes(range(22)), dst_ip=OWN, dst_mac=MAC, src=PEER, sport=12345, dport=22222, **kw):
    ip_kw = {k[3:]: v for k, v in kw.items() if k.startswith("ip_")}
    udp_kw = {k[4:]: v for k, v in kw.items() if k.startswith("udp_")}
    seg = R.build_udp(payload, sport, dport, src, dst_ip, **udp_kw)
    return R.build_eth(R.build_ipv4(seg, 0x11, src, dst_ip, **ip_kw), dst_mac, SRC_MAC, 0x0800)


def tcp_frame(payload=b"hello tcp payload!", dst_ip=OWN, flags=0x18, **kw):
    ip_kw = {k[3:]: v for k, v in kw.items() if k.startswith("ip_")}
    tcp_kw = {k[4:]: v for k, v in kw.items() if k.startswith("tcp_")}
    seg = R.build_tcp(payload, 40000, 80, PEER, dst_ip, 1234567890, 987654321, flags, **tcp_kw)
    return R.build_eth(R.build_ipv4(seg, 0x06, PEER, dst_ip, **ip_kw), MAC, SRC_MAC, 0x0800)


def icmp_frame(payload=b"abcdefghijklmnopqrstuvwabcdefghi", typ=8, code=0, dst_ip=OWN, **kw):
    ip_kw = {k[3:]: v for k, v in kw.items() if k.startswith("ip_")}
    icmp_kw = {k[5:]: v for k, v in kw.items() if k.startswith("icmp_")}
    seg = R.build_icmp(payload, typ, b"\x12\x34", 7, code=code, **icmp_kw)
    return R.build_eth(R.build_ipv4(seg, 0x01, PEER, dst_ip, **ip_kw), MAC, SRC_MAC, 0x0800)


def with_bytes(frame: bytes, at: int, new: bytes) -> bytes:
    return frame[:at] + new + frame[at + len(new):]


def cases():
    c = []
    canon = bytes.fromhex(
        "aaaaaaaaaaaa020000000001080045000032000100008011f103c0a86401c0a86464303956ce001ec07a"
        "000102030405060708090a0b0c0d0e0f101112131415")
    c.append(("kat_canonical_64B_udp", canon))
    c.append(("udp_builder_64B", udp_frame()))
    # ---- ETH_LEN / ETH_TYPE / non-IPv4 EtherTypes (ethernet.go:31-50)
    c.append(("eth_len_0", b""))
    c.append(("eth_len_41", udp_frame()[:41]))
    c.append(("eth_len_42_min", udp_frame(payload=b"")[:42]))
    c.append(("eth_len_1515", udp_frame(payload=bytes(1473))))
    c.append(("eth_type_unknown", with_bytes(udp_frame(), 12, b"\x12\x34")))
    c.append(("eth_type_vlan", with_bytes(udp_frame(), 12, b"\x81\x00")))
    c.append(("eth_type_8023_other_len", with_bytes(udp_frame(), 12, b"\x05\xdd")))
    c.append(("eth_type_8023", with_bytes(udp_frame(), 12, b"\x05\xdc")))
    c.append(("eth_type_ipv6", with_bytes(udp_frame(), 12, b"\x86\xdd")))
    arp = R.build_eth(bytes.fromhex("0001080006040001") + SRC_MAC + PEER + bytes(6) + OWN, b"\xff" * 6, SRC_MAC, 0x0806)
    c.append(("arp_request_bcast", arp))
    c.append(("arp_unicast_other_mac", with_bytes(arp, 0, bytes.fromhex("bbbbbbbbbbbb"))))
    # ---- MAC filter (ethernet_engine.go:22)
    c.append(("mac_other", udp_frame(dst_mac=bytes.fromhex("aaaaaaaaaaab"))))
    c.append(("mac_broadcast", udp_frame(dst_mac=b"\xff" * 6)))
    # ---- IPv4 checks (ipv4.go:48-86)
    c.append(("ip_ver_options", udp_frame(ip_ver_ihl=0x46)))
    c.append(("ip_ver_6", udp_frame(ip_ver_ihl=0x65)))
    c.append(("ip_frag_mf", udp_frame(ip_frag=b"\x20\x00")))
    c.append(("ip_frag_offset", udp_frame(ip_frag=b"\x00\x01")))
    c.append(("ip_frag_df_offset", udp_frame(ip_frag=b"\x40\x01")))
    c.append(("ip_df_ok", udp_frame(ip_frag=b"\x40\x00")))
    c.append(("ip_proto_igmp", R.build_eth(R.build_ipv4(bytes(30), 0x02, PEER, OWN), MAC, SRC_MAC, 0x0800)))
    c.append(("ip_proto_ipv6encap", R.build_eth(R.build_ipv4(bytes(30), 0x29, PEER, OWN), MAC, SRC_MAC, 0x0800)))
    c.append(("ip_hdr_cksum_bad", udp_frame(ip_csum=0x1234)))
    c.append(("ip_hdr_cksum_zero", udp_frame(ip_csum=0)))
    c.append(("ip_totlen_underflow_19", udp_frame(ip_total_len=19)))
    c.append(("ip_totlen_underflow_0", udp_frame(ip_total_len=0)))
    c.append(("ip_totlen_overrun", udp_frame(ip_total_len=51)))
    c.append(("ip_totlen_overrun_max", udp_frame(ip_total_len=0xFFFF)))
    c.append(("ip_totlen_20_udp", udp_frame(ip_total_len=20)))
    c.append(("ip_padding_trimmed_60B", udp_frame(payload=b"\x01\x02")))
    c.append(("ip_padding_trimmed_garbage", with_bytes(udp_frame(payload=b"\x01\x02"), 44, b"\xde\xad\xbe\xef")))
    # ---- UDP (udp.go:21-49)
    c.append(("udp_len_7", udp_frame(ip_total_len=27)))
    c.append(("udp_empty_payload", udp_frame(payload=b"")))
    c.append(("udp_odd_payload", udp_frame(payload=bytes(range(23)))))
    c.append(("udp_odd_payload_133", udp_frame(payload=bytes(random.Random(5).randrange(256) for _ in range(133)))))
    c.append(("udp_csum_zero_not_special", udp_frame(udp_csum=0)))
    c.append(("udp_csum_bad", udp_frame(udp_csum=0xBEEF)))
    c.append(("udp_len_field_small", udp_frame(udp_udp_len=12)))   # pseudo uses the header field
    c.append(("udp_len_field_large", udp_frame(udp_udp_len=400)))
    c.append(("udp_bcast_dst", udp_frame(dst_ip=bytes([192, 168, 100, 255]))))
    c.append(("udp_bcast_dst_badcsum", udp_frame(dst_ip=bytes([192, 168, 100, 255]), udp_csum=1)))
    c.append(("udp_limited_bcast", udp_frame(dst_ip=b"\xff" * 4, dst_mac=b"\xff" * 6)))
    c.append(("udp_forward_other_ip", udp_frame(dst_ip=bytes([10, 0, 0, 1]))))
    c.append(("udp_forward_other_ip_badcsum", udp_frame(dst_ip=bytes([10, 0, 0, 1]), udp_csum=7)))
    c.append(("udp_max_1514", udp_frame(payload=bytes(random.Random(1).randrange(256) for _ in range(1472)))))
    # ---- TCP (tcp.go:36-70)
    c.append(("tcp_ok", tcp_frame()))
    c.append(("tcp_syn", tcp_frame(flags=0x02)))
    c.append(("tcp_empty", tcp_frame(payload=b"")))
    c.append(("tcp_len_19", tcp_frame(payload=b"", ip_total_len=39)))
    c.append(("tcp_offset_quirk_options", tcp_frame(tcp_off_byte=0x80)))
    c.append(("tcp_offset_zero", tcp_frame(tcp_off_byte=0x00)))
    c.append(("tcp_csum_bad", tcp_frame(tcp_csum=0)))
    c.append(("tcp_odd", tcp_frame(payload=b"odd")))
    c.append(("tcp_bcast_ignored", tcp_frame(dst_ip=bytes([192, 168, 100, 255]))))
    c.append(("tcp_max_1514", tcp_frame(payload=bytes(random.Random(2).randrange(256) for _ in range(1460)))))
    # ---- ICMP (icmp.go:33-63; checksum ALWAYS verified)
    c.append(("icmp_echo_request", icmp_frame()))
    c.append(("icmp_echo_reply", icmp_frame(typ=0)))
    c.append(("icmp_ttl_exceeded", icmp_frame(typ=11)))
    c.append(("icmp_type_unreach", icmp_frame(typ=3)))
    c.append(("icmp_code_1", icmp_frame(code=1)))
    c.append(("icmp_csum_bad", icmp_frame(icmp_csum=0x4242)))
    c.append(("icmp_len_7", icmp_frame(payload=b"", ip_total_len=27)))
    c.append(("icmp_odd", icmp_frame(payload=b"xyz")))
    c.append(("icmp_forward", icmp_frame(dst_ip=bytes([8, 8, 8, 8]))))
    # ---- jumbo (9000-byte L2 buffer: ETH_LEN in the reference, OK in the extension)
    rj = random.Random(3)
    c.append(("jumbo_tcp_9000", tcp_frame(payload=bytes(rj.randrange(256) for _ in range(8946)))))
    c.append(("jumbo_udp_9014", udp_frame(payload=bytes(rj.randrange(256) for _ in range(8972)))))
    c.append(("jumbo_udp_9015", udp_frame(payload=bytes(rj.randrange(256) for _ in range(8973)))))
    c.append(("jumbo_icmp_odd", icmp_frame(payload=bytes(rj.randrange(256) for _ in range(4001)))))
    # ---- seeded random frames and single-bit flips
    rnd = random.Random(0x48414C4F)
    for k in range(240):
        kind = rnd.choice(["udp", "tcp", "icmp"])
        size = rnd.choice([60, 64, 65, 66, 67, 128, 333, 570, 1024, 1500, 1514])
        if kind == "udp":
            f = udp_frame(payload=bytes(rnd.randrange(256) for _ in range(max(0, size - 42))),
                          sport=rnd.randrange(1, 65536), dport=rnd.randrange(1, 65536))
        elif kind == "tcp":
            f = tcp_frame(payload=bytes(rnd.randrange(256) for _ in range(max(0, size - 54))),
                          flags=rnd.randrange(256))
        else:
            f = icmp_frame(payload=bytes(rnd.randrange(256) for _ in range(max(0, size - 42))),
                           typ=rnd.choice([0, 8, 11]))
        name = f"rand_{k:03d}_{kind}_{len(f)}"
        if k % 3 == 0:
            bit = rnd.randrange(14 * 8, len(f) * 8)
            b = bytearray(f)
            b[bit >> 3] ^= 1 << (bit & 7)
            f, name = bytes(b), name + f"_flip{bit}"
        c.append((name, f))
    return c


def main():
    os.makedirs(OUT, exist_ok=True)
    blob = bytearray()
    entries = []
    for name, f in cases():
        off = len(blob)
        blob += f
        blob += b"\0" * ((-len(blob)) % 4)
        exp = {}
        act = {}
        for fl in FLAGS:
            r = R.rx_frame(f, MAC, OWN_U, check_sum_enable=bool(fl & 1), jumbo=bool(fl & 2))
            r["status"] = R.STATUS.index(r["status"])
            exp[str(fl)] = r
            for nat in (0, 1):
                act[f"{fl}{nat}"] = R.engine_rx(f, MAC, OWN_U, nat_enable=bool(nat),
                                                check_sum_enable=bool(fl & 1), jumbo=bool(fl & 2))
        entries.append({"name": name, "offset": off, "len": len(f), "expect": exp, "action": act})
    with open(os.path.join(OUT, "frames.bin"), "wb") as fh:
        fh.write(bytes(blob))
    with open(os.path.join(OUT, "frames.json"), "w") as fh:
        json.dump({"netif": {"mac": MAC.hex(), "ip": OWN_U}, "frames": entries}, fh, indent=0,
                  separators=(",", ":"))
    kat = {
        "rfc1071_sec3": {"data": "0001f203f4f5f6f7", "checksum": R.get_checksum(bytes.fromhex("0001f203f4f5f6f7"))},
        "ipv4_header_valid": {"data": "450000730000400040 11b861c0a80001c0a800c7".replace(" ", ""),
                              "checksum": R.get_checksum(bytes.fromhex("45000073000040004011b861c0a80001c0a800c7"))},
        "canonical_64B_udp_ip_hdr": {"ip_csum": 0xF103, "udp_csum": 0xC07A},
    }
    with open(os.path.join(OUT, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    print(f"{len(entries)} frames, {len(blob)} bytes -> {OUT}")


if __name__ == "__main__":
    main()
