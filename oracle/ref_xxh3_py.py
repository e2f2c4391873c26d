"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of hashcode/xxh3.go (§8f row f3).

Independent of oracle/halo_xxh3_oracle.c: written from the Go source with Python integers
(explicit 64-bit masking) and ``int.from_bytes`` for the little-endian reads. Used to
cross-check the C restatement and to generate tests/golden/flow_hash.json.

  xxh3_64                hashcode/xxh3.go:43-56 (hashSmall :59-91, hashMedium :94-113,
                         hashLarge :116-129, hashLong :132-209)
  nat_flow_key           engine/ipv4_engine.go:451-459 / :471-479 with the key normalisation of
                         NatGetFlowByHash :524-551 / NatGetFlowByWan :554-581
"""
from __future__ import annotations

M64 = (1 << 64) - 1

SECRET = bytes.fromhex(
    "b8fe6c3923a44bbe7c01812cf721ad1cded46de9839097db7240a4a4b7b3671f"
    "cb79e64eccc0e578825ad07dccff7221b8084674f743248ee03590e6813a264c"
    "3c2852bb91c300cb88d0658b1b532ea371644897a20df94e3819ef46a9deacd8"
    "a8fa763fe39c343ff9dcbbc7c70b4f1d8a51e04bcdb45931c89f7ec9d9787364"
    "eac5ac8334d3ebc3c581a0fffa1363eb170ddd51b7f0da49d316552629d4689e"
    "2b16be587d47a1fc8ff8b8d17ad031ce45cb3a8f95160428afd7fbcabb4b407e")
P32 = (2654435761, 2246822519, 3266489917)
P64 = (11400714785074694791, 14029467366897019727, 1609587929392839161, 9650029242287828579,
       2870177450012600261)


def _r64(b, o):
    return int.from_bytes(b[o:o + 8], "little")


def _r32(b, o):
    return int.from_bytes(b[o:o + 4], "little")


def _mulfold(a, b):
    p = a * b
    return (p & M64) ^ (p >> 64)


def _aval(v):
    v ^= v >> 37
    v = (v * 0x165667919E3779F9) & M64
    return v ^ (v >> 32)


def _aval_small(v):
    v ^= v >> 33
    v = (v * P64[1]) & M64
    v ^= v >> 29
    v = (v * P64[2]) & M64
    return v ^ (v >> 32)


def _rotl(v, r):
    return ((v << r) | (v >> (64 - r))) & M64


def _mix16(d, do, so):
    return _mulfold(_r64(d, do) ^ _r64(SECRET, so), _r64(d, do + 8) ^ _r64(SECRET, so + 8))


def xxh3_64(data: bytes) -> int:
    d = bytes(data)
    n = len(d)
    if n == 0:
        return 0x2D06800538D394C2
    if n <= 3:
        c1, c2, c3 = d[0], d[n >> 1], d[n - 1]  # the canonical 1..3 byte combine (== xxh3.go:71-80)
        comb = (c1 << 16) | (c2 << 24) | c3 | (n << 8)
        return _aval_small(comb ^ (_r32(SECRET, 0) ^ _r32(SECRET, 4)))
    if n <= 8:
        v = (_r32(d, n - 4) + (_r32(d, 0) << 32)) ^ (_r64(SECRET, 8) ^ _r64(SECRET, 16))
        v ^= _rotl(v, 49) ^ _rotl(v, 24)
        v = (v * 0x9FB21C651E98DF25) & M64
        v ^= ((v >> 35) + n) & M64
        v = (v * 0x9FB21C651E98DF25) & M64
        return v ^ (v >> 28)
    if n <= 16:
        lo = _r64(d, 0) ^ (_r64(SECRET, 24) ^ _r64(SECRET, 32))
        hi = _r64(d, n - 8) ^ (_r64(SECRET, 40) ^ _r64(SECRET, 48))
        swapped = int.from_bytes(lo.to_bytes(8, "little"), "big")
        return _aval((n + swapped + hi + _mulfold(lo, hi)) & M64)
    acc = (n * P64[0]) & M64
    if n <= 128:
        pairs = [(0, 0, n - 16, 16)]
        if n > 32:
            pairs.append((16, 32, n - 32, 48))
        if n > 64:
            pairs.append((32, 64, n - 48, 80))
        if n > 96:
            pairs.append((48, 96, n - 64, 112))
        for a, sa, b, sb in pairs:
            acc = (acc + _mix16(d, a, sa) + _mix16(d, b, sb)) & M64
        return _aval(acc)
    if n <= 240:
        for o in range(0, 128, 16):
            acc = (acc + _mix16(d, o, o)) & M64
        acc = _aval(acc)
        for o in range(128, n & ~15, 16):
            acc = (acc + _mix16(d, o, o - 125)) & M64
        return _aval((acc + _mix16(d, n - 16, 119)) & M64)
    accs = [P32[2], P64[0], P64[1], P64[2], P64[3], P32[1], P64[4], P32[0]]

    def stripe(off, soff):
        for j in range(8):
            v = _r64(d, off + 8 * j)
            k = v ^ _r64(SECRET, soff + 8 * j)
            accs[j ^ 1] = (accs[j ^ 1] + v) & M64
            accs[j] = (accs[j] + (k & 0xFFFFFFFF) * (k >> 32)) & M64

    nblocks = (n - 1) // 1024
    for blk in range(nblocks):
        for s in range(16):
            stripe(blk * 1024 + 64 * s, 8 * s)
        for j in range(8):
            a = accs[j]
            a ^= a >> 47
            a ^= _r64(SECRET, 128 + 8 * j)
            accs[j] = (a * P32[0]) & M64
    base = nblocks * 1024
    for s in range((n - 1 - base) // 64):
        stripe(base + 64 * s, 8 * s)
    stripe(n - 64, 121)
    r = (n * P64[0]) & M64
    for i in range(4):
        r = (r + _mulfold(accs[2 * i] ^ _r64(SECRET, 11 + 16 * i), accs[2 * i + 1] ^ _r64(SECRET, 19 + 16 * i))) & M64
    return _aval(r)


def nat_flow_key(rec: dict, kind: int, nat_type: int) -> bytes:
    """kind 0: NatFlowHash as NatGetFlowByHash(dst, dport, src, sport) builds it; 1: NatWanFlowHash as
    NatGetFlowByWan(src, sport, dst, dport). nat_type 0 = NatTypeSymmetric."""
    if kind == 1:
        remote, rport, local, lport = rec["src_ip"], rec["sport"], rec["dst_ip"], rec["dport"]
    else:
        remote, rport, local, lport = rec["dst_ip"], rec["dport"], rec["src_ip"], rec["sport"]
    if nat_type != 0:
        remote, rport = 0, 0
    if rec["ip_proto"] == 1:
        rport = 0
    return (int(remote).to_bytes(4, "little") + int(rport).to_bytes(2, "little") + int(local).to_bytes(4, "little")
            + int(lport).to_bytes(2, "little") + bytes([int(rec["ip_proto"])]))
