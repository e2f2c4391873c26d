"""CPU: the flow-hash restatements (§8f row f3). XXH3-64 (hashcode/xxh3.go) is pinned to the
published XXH3-64 sanity vectors (xxHash's sanity buffer, seed 0 — the algorithm the reference
ports from github.com/zeebo/xxh3 v1.1.0); the C oracle and the independent Python restatement
agree with them, with each other on every length class, and with the committed fixtures."""
from __future__ import annotations

import json
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# XXH3_64bits(sanity_buffer, len), seed 0 — the published known answers
SANITY = {0: 0x2D06800538D394C2, 1: 0xC44BDFF4074EECDB, 6: 0x27B56A84CD2D7325, 12: 0xA713DAF0DFBB77E7,
          24: 0xA3FE70BF9D3510EB, 48: 0x397DA259ECBA1F11, 80: 0xBCDEFBBB2C47C90A, 195: 0xCD94217EE362EC3A,
          403: 0xCDEB804D65C6DEA4, 512: 0x617E49599013CB6B, 2048: 0xDD59E2C3A5F038E0,
          2240: 0x6E73A90539CF2948, 2367: 0xCB37AEB9E5D361ED}


def sanity_buffer(n):
    """xxHash's test buffer: byte i = top byte of PRIME32 * PRIME64^i (mod 2^64)."""
    out, g = bytearray(n), 2654435761
    for i in range(n):
        out[i] = g >> 56
        g = (g * 11400714785074694797) & ((1 << 64) - 1)
    return bytes(out)


def test_xxh3_published_sanity_vectors(oracle_lib):
    from oracle import ref_xxh3_py as X

    buf = sanity_buffer(2367)
    for n, want in SANITY.items():
        assert oracle_lib.xxh3_64(buf[:n]) == want, n
        assert X.xxh3_64(buf[:n]) == want, n
    assert oracle_lib.xxh3_64(b"abc") == X.xxh3_64(b"abc")


def test_c_and_python_xxh3_agree_every_length_class(oracle_lib):
    from oracle import ref_xxh3_py as X

    rnd = random.Random(3)
    lens = list(range(0, 300)) + [rnd.randrange(300, 9100) for _ in range(60)] + [1024, 1025, 2048, 4096, 8192]
    for n in lens:
        b = bytes(rnd.randrange(256) for _ in range(n))
        assert oracle_lib.xxh3_64(b) == X.xxh3_64(b), n


def _fixture():
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "flow_hash.json")))
    stream = np.fromfile(os.path.join(ROOT, "tests", "golden", "hash_stream.bin"), dtype=np.uint8)
    return meta, stream


def test_c_oracle_matches_hash_fixtures(oracle_lib):
    meta, stream = _fixture()
    offs = np.array([s["offset"] for s in meta["strings"]], np.uint64)
    lens = np.array([s["len"] for s in meta["strings"]], np.uint32)
    got = oracle_lib.xxh3_batch(stream, offs, lens)
    want = np.array([int(s["hash"], 16) for s in meta["strings"]], np.uint64)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("nat_type", [0, 1])
def test_c_oracle_flow_keys_match_fixtures(oracle_lib, golden, kind, nat_type):
    from tests.helpers import golden_arrays

    meta, stream = _fixture()
    gmeta, blob = golden
    data, offs, lens, _ = golden_arrays(gmeta, blob)
    recs, _ = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), 1, offsets_dw=offs)
    for nb_i, nb in enumerate(meta["buckets"]):
        h, b = oracle_lib.flow_hash_batch(recs, kind, nat_type, nb)
        want = [f for f in meta["flows"] if f["kind"] == kind and f["nat_type"] == nat_type]
        assert len(want) == len(recs)
        assert [f"{int(x):016x}" for x in h] == [f["hash"] for f in want]
        assert list(map(int, b)) == [f["bucket"][nb_i] for f in want]


def _canonical():
    """tests/golden/xxh3_canonical.npz: values from the canonical xxHash library (gen_golden_xxh3_canonical.py)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "xxh3_canonical.npz"))
    stream = np.fromfile(os.path.join(ROOT, "tests", "golden", "hash_stream.bin"), dtype=np.uint8)
    return z, stream


def test_c_oracle_equals_canonical_xxhash_every_length_0_to_4096_and_long(oracle_lib):
    """the C oracle == canonical libxxhash on every length 0..4096 and 300 random
    lengths up to 9000 (unaligned offsets)."""
    z, stream = _canonical()
    got = oracle_lib.xxh3_batch(stream, z["str_off"].astype(np.uint64), z["str_len"])
    bad = np.nonzero(got != z["str_hash"])[0]
    assert bad.size == 0, [int(z["str_len"][i]) for i in bad[:8]]
    assert set(range(4097)) <= set(z["str_len"].tolist()) and int(z["str_len"].max()) <= 9000


def test_python_restatement_equals_canonical_xxhash_sample():
    from oracle import ref_xxh3_py as X

    z, stream = _canonical()
    b = stream.tobytes()
    for i in list(range(0, 300)) + list(range(300, len(z["str_len"]), 97)):
        o, n = int(z["str_off"][i]), int(z["str_len"][i])
        assert X.xxh3_64(b[o:o + n]) == int(z["str_hash"][i]), n


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("nat_type", [0, 1])
def test_c_oracle_nat_keys_equal_canonical_xxhash(oracle_lib, golden, kind, nat_type):
    """The 13-byte NAT keys of the golden frames' records: the key bytes the oracle hashes and the
    canonical library's hash of them."""
    from oracle import ref_xxh3_py as X
    from tests.helpers import golden_arrays

    z, _ = _canonical()
    sel = (z["flow_kind"] == kind) & (z["flow_nat"] == nat_type)
    gmeta, blob = golden
    data, offs, lens, _ = golden_arrays(gmeta, blob)
    recs, _ = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), 1, offsets_dw=offs)
    assert int(sel.sum()) == len(recs)
    h, _ = oracle_lib.flow_hash_batch(recs, kind, nat_type, 1024)
    assert np.array_equal(np.asarray(h, np.uint64), z["flow_hash"][sel])
    for r, key in zip(recs[:64], z["flow_key"][sel][:64]):
        rec = {k: int(r[k]) for k in ("ip_proto", "src_ip", "dst_ip", "sport", "dport")}
        assert X.nat_flow_key(rec, kind, nat_type) == key.tobytes()
