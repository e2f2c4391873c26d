"""Generate the IcmpTtlDeepNat fixtures tests/golden/deep_nat.{json,bin} (build container).

engine/icmp_engine.go:55-86 on the Ethernet payload of ICMP time-exceeded frames a router
would receive for NATed flows: quoting UDP / TCP / ICMP packets with quotes of 28 bytes (the
RFC 792 minimum: TCP's ReCalcTcpCheckSum guard of 38 bytes skips it), 36, 48, 68 and whole
packets; Ethernet padding with garbage; and every early return (not ICMP, not ICMP_TTL, a code,
an outer checksum error, a quote of 27 bytes, no NAT flow). Expected values from the Python
restatement oracle/ref_tx_py.py (icmp_quote / icmp_ttl_deep_nat), under CheckSumEnable off/on.

    python tests/gen_golden_deepnat.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_py as R  # noqa: E402
from oracle import ref_tx_py as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
ROUTER_MAC, WAN_MAC = bytes.fromhex("aaaaaaaaaaaa"), bytes.fromhex("020000000009")
WAN = bytes([203, 0, 113, 5])        # the router's public address (the quoted packet's NATed source)
REMOTE = bytes([198, 51, 100, 77])   # the far end (the quoted packet's destination)
HOP = bytes([192, 0, 2, 1])          # the router on the path that sent the time-exceeded message
LAN_IP, LAN_PORT = 0xC0A80A17, 50123  # 192.168.10.23:50123, the NAT flow's LAN host


def quoted(proto: int, payload: bytes, sport=40000, dport=53, ttl=1) -> bytes:
    if proto == 0x11:
        seg = R.build_udp(payload, sport, dport, WAN, REMOTE)
    elif proto == 0x06:
        seg = R.build_tcp(payload, sport, dport, WAN, REMOTE, 0x01020304, 0x0A0B0C0D, 0x18)
    else:
        seg = R.build_icmp(payload, 8, sport.to_bytes(2, "big"), 9)
    return R.build_ipv4(seg, proto, WAN, REMOTE, ttl=ttl)


def ttl_frame(quote: bytes, typ=11, code=0, pad=b"", icmp_csum=None, ip_csum=None, outer_proto=0x01) -> bytes:
    msg = R.build_icmp(quote, typ, b"\0\0", 0, code=code, csum=icmp_csum)
    pkt = R.build_ipv4(msg, outer_proto, HOP, WAN, csum=ip_csum)
    return R.build_eth(pkt, ROUTER_MAC, WAN_MAC, 0x0800, pad=False) + pad


def cases():
    c = []
    rnd = random.Random(0xDEE9)
    for proto in (0x11, 0x06, 0x01):
        for plen in (0, 8, 20, 40, 120, 500):
            full = quoted(proto, bytes(rnd.randrange(256) for _ in range(plen)), sport=rnd.randrange(1, 65536))
            for qlen in (28, 36, 40, 48, 68, len(full)):
                if qlen <= len(full):
                    c.append((f"p{proto}_pl{plen}_q{qlen}", ttl_frame(full[:qlen])))
    base = quoted(0x11, b"hello", sport=33333)
    c.append(("padding_garbage", ttl_frame(base[:28], pad=b"\xde\xad\xbe\xef")))
    c.append(("padding_zero_to_60", ttl_frame(base[:12], pad=bytes(4))))  # quote 12 B: returns early
    c.append(("quote_27", ttl_frame(base[:27])))
    c.append(("quote_odd_29", ttl_frame(base[:29])))
    c.append(("echo_request_not_ttl", ttl_frame(base[:28], typ=8)))
    c.append(("unreachable_type_3", ttl_frame(base[:28], typ=3)))
    c.append(("ttl_code_1", ttl_frame(base[:28], code=1)))
    c.append(("icmp_csum_bad", ttl_frame(base[:28], icmp_csum=0x1234)))
    c.append(("ip_csum_bad", ttl_frame(base[:28], ip_csum=0x4321)))
    c.append(("not_icmp_udp", ttl_frame(base[:28], outer_proto=0x11)))
    c.append(("inner_proto_47", ttl_frame(R.build_ipv4(bytes(16), 47, WAN, REMOTE))))
    c.append(("inner_short_hdr_len_ok", ttl_frame(quoted(0x06, bytes(100))[:38])))
    return c


def main():
    blob, expect = bytearray(), bytearray()
    entries = []
    for name, f in cases():
        off, eoff = len(blob), len(expect)
        blob += f + b"\0" * ((-len(f)) % 4)
        e = {"name": name, "offset": off, "len": len(f), "quote": {}, "applied": {}, "expect_offset": {}}
        for en in (0, 1):
            st, args = T.icmp_quote(f[14:], bool(en))
            e["quote"][str(en)] = {"status": R.STATUS.index(st) if st in R.STATUS else st,
                                   "args": list(args) if args else None}
            for found in (0, 1):
                eth = bytearray(f[14:])
                ok = T.icmp_ttl_deep_nat(eth, LAN_IP, LAN_PORT, bool(found), bool(en))
                out = f[:14] + bytes(eth)
                e["applied"][f"{en}{found}"] = int(ok)
                e["expect_offset"][f"{en}{found}"] = len(expect)
                expect += out + b"\0" * ((-len(out)) % 4)
        del eoff
        entries.append(e)
    with open(os.path.join(OUT, "deep_nat.bin"), "wb") as fh:
        fh.write(bytes(blob))
    with open(os.path.join(OUT, "deep_nat_expect.bin"), "wb") as fh:
        fh.write(bytes(expect))
    with open(os.path.join(OUT, "deep_nat.json"), "w") as fh:
        json.dump({"lan_ip": LAN_IP, "lan_port": LAN_PORT, "frames": entries}, fh, indent=0, separators=(",", ":"))
    print(f"{len(entries)} frames -> {OUT}")


if __name__ == "__main__":
    main()
