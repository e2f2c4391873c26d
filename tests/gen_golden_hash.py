"""Generate the committed XXH3 / flow-key fixtures (§8f row f3): tests/golden/flow_hash.json.

Expected values come from oracle/ref_xxh3_py.py (pure-Python restatement of hashcode/xxh3.go),
which tests/test_flow_hash_oracle.py first pins to the published XXH3-64 sanity vectors.
Strings: every length 0..260 and a set of long ones (block / stripe boundaries) cut from a
seeded byte stream at odd offsets. Flow keys: the records the rx restatement produces for the
rx golden frames (tests/golden/frames.*), both key kinds, both NAT types, with buckets for
two table sizes.

    python tests/gen_golden_hash.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_xxh3_py as X  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
LONG = (240, 241, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 1087, 1088, 1089, 2047, 2048, 2049, 2240,
        2367, 3072, 4095, 4096, 4097, 9000)
BUCKETS = (1024, 1000003)


def main():
    rnd = random.Random(0x58584833)
    stream = bytes(rnd.randrange(256) for _ in range(1 << 15))
    strings = []
    pos = 1
    for n in list(range(0, 261)) + list(LONG):
        strings.append({"offset": pos, "len": n, "hash": f"{X.xxh3_64(stream[pos:pos + n]):016x}"})
        pos = (pos + n + rnd.randrange(1, 8)) % ((1 << 15) - 10000)
    meta = json.load(open(os.path.join(OUT, "frames.json")))
    recs = []
    for e in meta["frames"]:
        r = e["expect"]["1"]
        recs.append({k: r[k] for k in ("status", "ip_proto", "src_ip", "dst_ip", "sport", "dport")})
    flows = []
    for i, r in enumerate(recs):
        for kind in (0, 1):
            for nt in (0, 1):
                h = X.xxh3_64(X.nat_flow_key(r, kind, nt))
                flows.append({"frame": i, "kind": kind, "nat_type": nt, "hash": f"{h:016x}",
                              "bucket": [h % b for b in BUCKETS]})
    with open(os.path.join(OUT, "hash_stream.bin"), "wb") as fh:
        fh.write(stream)
    with open(os.path.join(OUT, "flow_hash.json"), "w") as fh:
        json.dump({"buckets": BUCKETS, "strings": strings, "flows": flows}, fh, indent=0, separators=(",", ":"))
    print(f"{len(strings)} strings, {len(flows)} flow keys -> {OUT}")


if __name__ == "__main__":
    main()
