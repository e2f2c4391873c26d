"""Generate tests/golden/xxh3_canonical.npz: XXH3-64 values computed by the canonical xxHash library
(python-xxhash 3.8.1 over libxxhash 0.8.2, ``xxhash.xxh3_64``, seed 0, default secret) — an oracle
independent of this repository's restatements for §8f row f3.

The reference's hashcode/xxh3.go:1 declares itself a port of github.com/zeebo/xxh3, which implements
XXH3_64bits with the default secret; GetHashCodeXXH3 (hashcode/xxh3.go:43-88) is that function with
seed 0. So the canonical library's value is the reference's value.

* strings: every length 0..4096, plus 300 seeded random lengths in 4097..9000, each cut from
  tests/golden/hash_stream.bin (32 KiB, committed by gen_golden_hash.py) at a seeded unaligned
  offset;
* NAT flow keys: the 13-byte keys of the rx golden frames' records (tests/golden/frames.*, flags 1),
  both key kinds (NatFlowHash / NatWanFlowHash) and both NAT types, laid out as
  engine/ipv4_engine.go:442-479 builds them (remote ip, remote port, local ip, local port, proto,
  little-endian), hashed by the canonical library.

    python tests/gen_golden_xxh3_canonical.py
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden")


def nat_key(rec: dict, kind: int, nat_type: int) -> bytes:
    """NatGetFlowByHash (kind 0: dst, dport, src, sport) / NatGetFlowByWan (kind 1: src, sport, dst,
    dport) key bytes; NatTypeSymmetric (0) keeps the remote end, other types zero it; ICMP has no
    remote port (engine/ipv4_engine.go:442-479)."""
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


def main():
    import xxhash

    assert xxhash.VERSION == "3.8.1", xxhash.VERSION
    stream = np.fromfile(os.path.join(OUT, "hash_stream.bin"), dtype=np.uint8).tobytes()
    rnd = random.Random(0xC0FFEE)
    lens = list(range(0, 4097)) + sorted(rnd.randrange(4097, 9001) for _ in range(300))
    offs = [rnd.randrange(0, len(stream) - n + 1) for n in lens]
    hashes = [xxhash.xxh3_64_intdigest(stream[o:o + n]) for o, n in zip(offs, lens)]
    meta = json.load(open(os.path.join(OUT, "frames.json")))
    f_frame, f_kind, f_nat, f_key, f_hash = [], [], [], [], []
    for i, e in enumerate(meta["frames"]):
        r = e["expect"]["1"]
        for kind in (0, 1):
            for nt in (0, 1):
                k = nat_key(r, kind, nt)
                f_frame.append(i)
                f_kind.append(kind)
                f_nat.append(nt)
                f_key.append(np.frombuffer(k, np.uint8))
                f_hash.append(xxhash.xxh3_64_intdigest(k))
    np.savez_compressed(
        os.path.join(OUT, "xxh3_canonical.npz"),
        str_off=np.array(offs, np.uint32), str_len=np.array(lens, np.uint32), str_hash=np.array(hashes, np.uint64),
        flow_frame=np.array(f_frame, np.uint32), flow_kind=np.array(f_kind, np.uint8),
        flow_nat=np.array(f_nat, np.uint8), flow_key=np.stack(f_key), flow_hash=np.array(f_hash, np.uint64))
    print(f"{len(lens)} strings, {len(f_hash)} flow keys -> {OUT}/xxh3_canonical.npz")


if __name__ == "__main__":
    main()
