"""Generate the committed Build* (§8f row f2, transmit construction) fixtures in tests/golden/.

Expected outputs come from oracle/ref_tx_py.py's pure-Python restatement of BuildUdpPkt /
BuildTcpPkt / BuildIcmpPkt -> BuildIpv4Pkt (iphId) -> BuildEthFrm and of TxIpv4's LoChan copy;
the C oracle (ora_tx_build_batch) and the GPU kernel (halo_tx_build_batch_device) are tested
against these files.

Descriptors: the canonical 64 B UDP frame of SURVEY.md §8a (its known bytes are asserted here),
every payload length around the 60-byte padding boundary and the Go limits (UDP/ICMP 1472,
TCP 1460, one byte over each), odd lengths, every ICMP type the reference sends, unknown IP
protocols, broadcast MACs, loopback (IPv4-only) mode, and 240 seeded random descriptors with
payloads at any byte alignment. Two runs: CheckSumEnable true with iphId starting at 0, and
false starting at 0xFFF0 (the 16-bit counter wraps inside the batch).

Files: tx_build_payload.bin (payload bytes), tx_build.json (descriptors, per run: start id, end
id, lens, results, offsets into the expect blob), tx_build_expect.bin (built frames back to back).

    python tests/gen_golden_build.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_tx_py as T  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SRC_MAC = bytes.fromhex("020000000001")
OWN_IP = 0xC0A86401      # 192.168.100.1 (the canonical frame's source)
PEER_IP = 0xC0A86464     # 192.168.100.100
KAT = ("aaaaaaaaaaaa020000000001080045000032000100008011f103c0a86401c0a86464303956ce001ec07a"
       "000102030405060708090a0b0c0d0e0f101112131415")


def main():
    rng = random.Random(0x4255494C)
    payload = bytearray()
    descs = []

    def add(plen, proto, mode=0, aux=0, sport=12345, dport=22222, src=OWN_IP, dst=PEER_IP, seq=0, ack=0,
            mac=b"\xaa" * 6, data=None, align=None):
        if align is not None:
            while len(payload) % 4 != align:
                payload.append(rng.randrange(256))
        off = len(payload)
        payload.extend(data if data is not None else bytes(rng.randrange(256) for _ in range(plen)))
        descs.append(dict(payload_off=off, payload_len=plen, proto=proto, aux=aux, src_port=sport, dst_port=dport,
                          src_ip=src, dst_ip=dst, seq=seq, ack=ack, dst_mac=list(mac), mode=mode))

    add(22, 0x11, data=bytes(range(22)), align=0)                       # the canonical frame (id 1)
    for plen in (0, 1, 2, 3, 17, 18, 19, 22, 23, 100, 501, 1471, 1472, 1473, 2000):
        add(plen, 0x11, align=plen % 4)
    for plen in (0, 1, 5, 6, 7, 535, 536, 1459, 1460, 1461):
        add(plen, 0x06, aux=0x18, seq=0x01020304, ack=0xA0B0C0D0, sport=80, dport=51000, align=(plen + 1) % 4)
    for t in (8, 0, 11):
        for plen in (0, 5, 18, 56, 1472, 1473):
            add(plen, 0x01, aux=t, sport=0xBEEF, dport=t * 7 + plen, align=(plen + 2) % 4)
    for proto in (0x00, 0x02, 0x29, 0x3A, 0xFF):
        add(30, proto)
    add(40, 0x11, mac=b"\xff" * 6, dst=0xC0A864FF)                       # broadcast (TxIpv4 dst[3]==255)
    for plen, proto in ((0, 0x11), (22, 0x11), (1472, 0x11), (7, 0x06), (1460, 0x06), (56, 0x01), (1473, 0x11)):
        add(plen, proto, mode=1, dst=OWN_IP, aux=8 if proto == 1 else 0x10)  # loopback: TxIpv4's LoChan copy
    for _ in range(240):
        proto = rng.choice([0x11, 0x11, 0x06, 0x06, 0x01, 0x07])
        lim = 1460 if proto == 0x06 else 1472
        plen = rng.choice([rng.randrange(0, 64), rng.randrange(0, 600), rng.randrange(0, lim + 1),
                           rng.randrange(lim - 3, lim + 3)])
        add(plen, proto, mode=rng.choice([0, 0, 0, 1]), aux=rng.choice([8, 0, 11]) if proto == 1 else rng.randrange(256),
            sport=rng.randrange(65536), dport=rng.randrange(65536), src=rng.randrange(1 << 32),
            dst=rng.randrange(1 << 32), seq=rng.randrange(1 << 32), ack=rng.randrange(1 << 32),
            mac=bytes(rng.randrange(256) for _ in range(6)), align=rng.randrange(4))
    payload.extend(b"\0" * 8)

    expect = bytearray()
    runs = []
    for csum, start in ((True, 0), (False, 0xFFF0)):
        iph = T.IphId(start)
        lens, results, offs = [], [], []
        for d in descs:
            p = bytes(payload[d["payload_off"]:d["payload_off"] + d["payload_len"]])
            r, f = T.tx_build(dict(d, dst_mac=bytes(d["dst_mac"])), p, SRC_MAC, iph, csum)
            assert r != T.B_OK or len(f) == T.tx_build_len(d)
            offs.append(len(expect))
            expect.extend(f)
            lens.append(len(f))
            results.append(r)
        runs.append(dict(flags=1 if csum else 0, ip_id_start=start, ip_id_end=iph.value, lens=lens, results=results,
                         expect_offsets=offs))
    first = bytes(expect[runs[0]["expect_offsets"][0]:runs[0]["expect_offsets"][0] + runs[0]["lens"][0]])
    assert first.hex() == KAT, first.hex()
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "tx_build_payload.bin"), "wb") as fh:
        fh.write(bytes(payload))
    with open(os.path.join(OUT, "tx_build_expect.bin"), "wb") as fh:
        fh.write(bytes(expect))
    with open(os.path.join(OUT, "tx_build.json"), "w") as fh:
        json.dump(dict(src_mac=SRC_MAC.hex(), descs=descs, runs=runs), fh, separators=(",", ":"))
    print(f"{len(descs)} descriptors, {len(payload)} payload bytes, {len(expect)} expected bytes")


if __name__ == "__main__":
    main()
