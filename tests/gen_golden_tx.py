"""Generate the committed forward/transmit (§8f row f2) fixtures in tests/golden/ (build container).

Expected outputs come from oracle/ref_tx_py.py (the pure-Python restatement of NatChangeDst /
HandleIpv4PktTtl / NatChangeSrc / ReCalc* and of eth_tx's DPDK software fill); the C oracle and
the GPU kernel are tested against these files.

Frames: every rx golden frame (tests/gen_golden.py), plus TX-specific ones — TTL 0/1/2/255,
IHL != 5, total-length underflow / overrun / padding, every truncation of a UDP, TCP and ICMP
frame from 0 to 60 bytes, non-IPv4 EtherTypes, and UDP / TCP packets whose fresh checksum is
zero (DPDK sends UDP's as 0xFFFF). Each frame gets seven step sets (the two Ipv4RouteForward
directions, everything, RECALC, DPDK_FILL, TTL alone and one seeded random set) with seeded
NAT addresses and ports, under CheckSumEnable false and true.

Files: tx_frames.bin (input frames, 4-byte aligned), tx.json (frames, entries: frame index,
op, result byte per flag), tx_expect.bin (per entry and flag 0 then 1: the first min(len, 52)
bytes of the rewritten frame, zero padded to 52 — no step touches a byte past 51).

    python tests/gen_golden_tx.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import ref_py as R  # noqa: E402
from oracle import ref_tx_py as T  # noqa: E402
import gen_golden as G  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
HDR = 52
COMBOS = (
    T.NAT_DST | T.TTL,                             # WAN -> LAN forward (DNAT, TTL)
    T.TTL | T.NAT_SRC,                             # LAN -> WAN forward (TTL, SNAT)
    T.NAT_DST | T.TTL | T.NAT_SRC | T.DPDK_FILL,   # everything, then eth_tx
    T.RECALC,
    T.DPDK_FILL,
    T.TTL,
)


def zero_sum_udp(proto_tcp=False):
    """A UDP (or TCP) frame whose recomputed checksum is 0x0000 (sum 0xFFFF)."""
    base = G.tcp_frame(payload=b"\0\0" + bytes(range(30))) if proto_tcp else G.udp_frame(payload=b"\0\0" + bytes(30))
    b = bytearray(base)
    T.tx_frame(b, T.RECALC)  # fresh checksum c; making it 0 means adding ~c... solve for the filler word
    at = 14 + 20 + (20 if proto_tcp else 8)
    c = (b[at - (4 if proto_tcp else 2)] << 8) | b[at - (3 if proto_tcp else 1)]
    f = bytearray(base)
    f[at:at + 2] = c.to_bytes(2, "big")  # adds c to the sum: ~(S + c) = ~0xFFFF = 0
    chk = bytearray(f)
    T.tx_frame(chk, T.RECALC)
    field = 14 + 20 + (16 if proto_tcp else 6)
    assert chk[field:field + 2] == b"\0\0", chk[field:field + 2].hex()
    return bytes(f)


def tx_cases():
    c = list(G.cases())
    for ttl in (0, 1, 2, 255):
        c.append((f"tx_ttl_{ttl}_udp", G.udp_frame(ip_ttl=ttl)))
    c.append(("tx_ttl_1_icmp", G.icmp_frame(ip_ttl=1)))
    c.append(("tx_ttl_2_tcp", G.tcp_frame(ip_ttl=2)))
    for vi in (0x40, 0x44, 0x46, 0x4F):
        c.append((f"tx_ihl_{vi & 15}_udp", G.udp_frame(ip_ver_ihl=vi, payload=bytes(range(40)))))
    c.append(("tx_ihl_15_short_frame", G.udp_frame(ip_ver_ihl=0x4F, payload=b"")))
    for tl in (0, 19, 20, 21, 28, 29, 200, 0xFFFF):
        c.append((f"tx_totlen_{tl}_udp", G.udp_frame(ip_total_len=tl)))
        c.append((f"tx_totlen_{tl}_tcp", G.tcp_frame(ip_total_len=tl)))
    c.append(("tx_padding_udp", G.udp_frame(payload=b"\x01")))
    c.append(("tx_padding_garbage_tcp", G.with_bytes(G.tcp_frame(payload=b""), 55, b"\xde\xad\xbe")))
    long_udp = G.udp_frame(payload=bytes(range(60)))
    long_tcp = G.tcp_frame(payload=bytes(range(60)))
    long_icmp = G.icmp_frame(payload=bytes(range(60)))
    for L in range(0, 61):
        c.append((f"tx_trunc_udp_{L}", long_udp[:L]))
        if L in (14, 23, 24, 33, 34, 37, 38, 39, 41, 42, 49, 50, 51, 52, 53):
            c.append((f"tx_trunc_tcp_{L}", long_tcp[:L]))
            c.append((f"tx_trunc_icmp_{L}", long_icmp[:L]))
    c.append(("tx_ethertype_arp_like", G.with_bytes(long_udp, 12, b"\x08\x06")))
    c.append(("tx_ethertype_vlan", G.with_bytes(long_udp, 12, b"\x81\x00")))
    c.append(("tx_proto_igmp", R.build_eth(R.build_ipv4(bytes(40), 0x02, G.PEER, G.OWN), G.MAC, G.SRC_MAC, 0x0800)))
    c.append(("tx_udp_zero_sum", zero_sum_udp(False)))
    c.append(("tx_tcp_zero_sum", zero_sum_udp(True)))
    c.append(("tx_all_ff_udp", G.udp_frame(payload=b"\xff" * 40)))
    return c


def main():
    rnd = random.Random(0x54584658)
    blob = bytearray()
    frames, entries = [], []
    expect = bytearray()
    for k, (name, f) in enumerate(tx_cases()):
        off = len(blob)
        blob += f
        blob += b"\0" * ((-len(blob)) % 4)
        frames.append({"name": name, "offset": off, "len": len(f)})
        big = len(f) > 4000
        combos = COMBOS[2:4] if big else COMBOS + (rnd.randrange(32),)
        for steps in combos:
            op = [steps, rnd.getrandbits(32), rnd.randrange(65536), rnd.getrandbits(32), rnd.randrange(65536)]
            res = {}
            for en in (0, 1):
                b = bytearray(f)
                res[str(en)] = T.tx_frame(b, op[0], dst_ip=op[1], dst_port=op[2], src_ip=op[3], src_port=op[4],
                                          check_sum_enable=bool(en))
                assert b[HDR:] == f[HDR:], name  # nothing past byte 51 changes
                expect += bytes(b[:HDR]) + b"\0" * (HDR - min(len(b), HDR))
            entries.append({"frame": k, "op": op, "result": res})
    with open(os.path.join(OUT, "tx_frames.bin"), "wb") as fh:
        fh.write(bytes(blob))
    with open(os.path.join(OUT, "tx_expect.bin"), "wb") as fh:
        fh.write(bytes(expect))
    with open(os.path.join(OUT, "tx.json"), "w") as fh:
        json.dump({"hdr_bytes": HDR, "frames": frames, "entries": entries}, fh, indent=0, separators=(",", ":"))
    print(f"{len(frames)} frames, {len(entries)} entries, {len(blob)} + {len(expect)} bytes -> {OUT}")


if __name__ == "__main__":
    main()
