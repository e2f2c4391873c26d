"""CPU: pin the oracle (C restatement) against known answers and the golden fixtures,
and cross-check it against the independent pure-Python restatement."""
from __future__ import annotations

import json
import os
import random

import numpy as np
import pytest

from oracle import ref_py as R
from tests.helpers import STATUS_NAMES, assert_records_equal, expected_records, golden_arrays

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAC = bytes.fromhex("aaaaaaaaaaaa")
OWN = 0xC0A86464  # 192.168.100.100 (example/example.go:768-773)
CANON = bytes.fromhex(
    "aaaaaaaaaaaa020000000001080045000032000100008011f103c0a86401c0a86464303956ce001ec07a"
    "000102030405060708090a0b0c0d0e0f101112131415")


def test_known_answers(oracle_lib):
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    # RFC 1071 §3: the words 0001 f203 f4f5 f6f7 sum to ddf2 -> checksum 220d
    assert oracle_lib.get_checksum(bytes.fromhex("0001f203f4f5f6f7")) == 0x220D
    assert R.get_checksum(bytes.fromhex("0001f203f4f5f6f7")) == 0x220D
    assert kat["rfc1071_sec3"]["checksum"] == 0x220D
    hdr = bytes.fromhex("45000073000040004011b861c0a80001c0a800c7")
    assert oracle_lib.get_checksum(hdr) == 0 and R.get_checksum(hdr) == 0
    # canonical 64 B UDP frame of SURVEY.md §8a: IP csum f103, UDP csum c07a, both verify
    assert CANON[24:26] == b"\xf1\x03" and CANON[40:42] == b"\xc0\x7a"
    assert oracle_lib.get_checksum(CANON[14:34]) == 0
    n = oracle_lib.NetIf.make()
    r = oracle_lib.rx_frame(CANON, n, 1)
    assert r["status"] == 0 and r["sport"] == 12345 and r["dport"] == 22222
    assert r["src_ip"] == 0xC0A86401 and r["dst_ip"] == OWN and r["payload_off"] == 42 and r["payload_len"] == 22


def test_checksum_edge_cases(oracle_lib):
    for data in [b"", b"\x01", b"\xff\xff", b"\x00\x00", b"\xff", bytes(range(255)), b"\xff" * 9001]:
        assert oracle_lib.get_checksum(data) == R.get_checksum(data)
    assert oracle_lib.get_checksum(b"") == 0xFFFF       # ^0
    assert oracle_lib.get_checksum(b"\x01") == 0xFEFF    # odd trailing byte is the HIGH byte
    rnd = random.Random(7)
    for _ in range(300):
        data = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 200)))
        assert oracle_lib.get_checksum(data) == R.get_checksum(data)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_oracle_matches_golden(golden, oracle_lib, flags):
    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    n = oracle_lib.NetIf.make()
    got, hist = oracle_lib.rx_batch(data, lens, n, flags, offsets_dw=offs)
    want = expected_records(meta, flags, oracle_lib.RESULT_DTYPE)
    assert_records_equal(got, want, names, f"C oracle vs golden flags={flags}")
    assert hist.sum() == len(names)
    assert np.array_equal(hist, np.bincount(want["status"], minlength=14))


def test_golden_is_reproducible(golden):
    """The committed expectations still follow from ref_py (fixtures did not drift)."""
    meta, blob = golden
    for e in meta["frames"]:
        f = bytes(blob[e["offset"]:e["offset"] + e["len"]])
        for fl in ("1", "2"):
            r = R.rx_frame(f, MAC, OWN, check_sum_enable=fl == "1", jumbo=fl == "2")
            r["status"] = STATUS_NAMES.index(r["status"])
            assert r == e["expect"][fl], e["name"]


def test_engine_actions_match_golden(golden, oracle_lib):
    meta, blob = golden
    for nat in (0, 1):
        n = oracle_lib.NetIf.make(nat_enable=bool(nat))
        for e in meta["frames"]:
            f = bytes(blob[e["offset"]:e["offset"] + e["len"]])
            for fl in (0, 1, 2, 3):
                a = oracle_lib.engine_rx(f, n, fl)
                assert R.ACTIONS[a] == e["action"][f"{fl}{nat}"], (e["name"], fl, nat)


def test_every_reachable_status_has_a_fixture(golden):
    meta, _ = golden
    seen = {e["expect"][fl]["status"] for e in meta["frames"] for fl in ("0", "1", "2", "3")}
    # IP_LEN (ipv4.go:49) is unreachable behind ParseEthFrm's own length check: every frame
    # that passes ethernet.go:31 leaves an IPv4 packet of 28..1500 (jumbo: ..9000) bytes.
    assert seen == set(range(14)) - {3}


def _random_frame(rnd: random.Random) -> bytes:
    src, dst = bytes([10, 1, 2, 3]), (OWN.to_bytes(4, "big") if rnd.random() < 0.7 else bytes([10, 9, 9, 255]))
    kind = rnd.randrange(3)
    pay = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 200)))
    if kind == 0:
        seg = R.build_udp(pay, rnd.randrange(65536), rnd.randrange(65536), src, dst)
        proto = 0x11
    elif kind == 1:
        seg = R.build_tcp(pay, 1, 2, src, dst, rnd.getrandbits(32), rnd.getrandbits(32), rnd.randrange(256),
                          off_byte=rnd.randrange(256))
        proto = 0x06
    else:
        seg = R.build_icmp(pay, rnd.choice([0, 8, 11, 3]), b"\x00\x01", rnd.randrange(65536))
        proto = 0x01
    f = bytearray(R.build_eth(R.build_ipv4(seg, proto, src, dst, ident=rnd.randrange(65536)),
                              MAC if rnd.random() < 0.9 else b"\x01" * 6, b"\x02" * 6, 0x0800))
    for _ in range(rnd.choice([0, 0, 1, 2])):  # bit flips anywhere, headers included
        bit = rnd.randrange(len(f) * 8)
        f[bit >> 3] ^= 1 << (bit & 7)
    if rnd.random() < 0.05:
        f = f[:rnd.randrange(len(f) + 1)]
    return bytes(f)


def test_c_oracle_vs_python_restatement_random(oracle_lib):
    rnd = random.Random(1234)
    for nat in (False, True):
        n = oracle_lib.NetIf.make(nat_enable=nat)
        for _ in range(400):
            f = _random_frame(rnd)
            for fl in (0, 1):
                want = R.rx_frame(f, MAC, OWN, check_sum_enable=bool(fl))
                got = oracle_lib.rx_frame(f, n, fl)
                for k, v in want.items():
                    gv = int(got[k])
                    assert gv == (STATUS_NAMES.index(v) if k == "status" else v), (k, f.hex(), fl)
                a = oracle_lib.engine_rx(f, n, fl)
                assert R.ACTIONS[a] == R.engine_rx(f, MAC, OWN, nat_enable=nat, check_sum_enable=bool(fl))


@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_batch_layouts(golden, oracle_lib, threads):
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    n = oracle_lib.NetIf.make()
    want, _ = oracle_lib.rx_batch(data, lens, n, 1, offsets_dw=offs)
    got, _ = oracle_lib.rx_batch(data, lens, n, 1, offsets_dw=offs, threads=threads)
    assert_records_equal(got, want, what="threads")
    stride = int(((lens.max() + 3) // 4) * 4)
    strided = np.zeros(stride * len(lens), np.uint8)
    for i in range(len(lens)):
        o, L = int(offs[i]) * 4, int(lens[i])
        strided[i * stride:i * stride + L] = data[o:o + L]
    got2, _ = oracle_lib.rx_batch(strided, lens, n, 1, stride=stride, threads=threads)
    assert_records_equal(got2, want, what="strided")
