"""CPU: IcmpTtlDeepNat (engine/icmp_engine.go:55-86, the f2 family of SURVEY.md §8f) — the C
restatement (oracle/halo_tx_oracle.c ora_icmp_quote / ora_icmp_deep_nat) against the committed
fixtures from the independent Python restatement (tests/gen_golden_deepnat.py), and the rewritten
frames against the reference's own receive checks."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dn():
    g = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(g, "deep_nat.json")))
    blob = np.fromfile(os.path.join(g, "deep_nat.bin"), dtype=np.uint8)
    expect = np.fromfile(os.path.join(g, "deep_nat_expect.bin"), dtype=np.uint8)
    return meta, blob, expect


@pytest.mark.parametrize("en", [0, 1])
def test_quote_matches_fixtures(oracle_lib, dn, en):
    meta, blob, _ = dn
    for e in meta["frames"]:
        f = blob[e["offset"]:e["offset"] + e["len"]].tobytes()
        q = oracle_lib.icmp_quote(f, en)
        want = e["quote"][str(en)]
        assert int(q["status"]) == want["status"], e["name"]
        if want["args"]:
            proto, remote, rport, wan, wport = want["args"]
            got = (int(q["ip_proto"]), int(q["src_ip"]), int(q["sport"]), int(q["dst_ip"]), int(q["dport"]))
            assert got == (proto, remote, rport, wan, wport), e["name"]


@pytest.mark.parametrize("en", [0, 1])
@pytest.mark.parametrize("found", [0, 1])
def test_deep_nat_matches_fixtures(oracle_lib, dn, en, found):
    meta, blob, expect = dn
    for e in meta["frames"]:
        f = blob[e["offset"]:e["offset"] + e["len"]].tobytes()
        out, ok = oracle_lib.icmp_deep_nat(f, meta["lan_ip"], meta["lan_port"], bool(found), en)
        k = f"{en}{found}"
        assert int(ok) == e["applied"][k], e["name"]
        o = e["expect_offset"][k]
        assert out == expect[o:o + e["len"]].tobytes(), e["name"]


def test_fixture_coverage(dn):
    meta, _, _ = dn
    st = {e["quote"]["1"]["status"] for e in meta["frames"]}
    assert {0, 6, 7, 10, 11, 12, 13} <= st  # applied, not ICMP, IP checksum, short quote, type, code, ICMP cksum
    assert sum(e["applied"]["11"] for e in meta["frames"]) >= 80


def test_rewritten_outer_packet_verifies(oracle_lib, dn):
    """After the rewrite the outer packet passes ParseIpv4Pkt + ParseIcmpPkt again (its checksums
    were recomputed over the modified quote), addressed to the LAN host."""
    meta, blob, expect = dn
    own = oracle_lib.NetIf.make(ip="192.168.10.23")
    for e in meta["frames"]:
        if not e["applied"]["11"]:
            continue
        o = e["expect_offset"]["11"]
        pkt = expect[o + 14:o + e["len"]].tobytes()
        r = oracle_lib.rx_frame(pkt, own, 1 | 0x10)
        if e["name"] == "padding_garbage":
            # the quirk: ReCalcIcmpCheckSum sums the UNTRIMMED Ethernet payload (ipv4.go:164-174 on
            # NatChangeDst's ethPayload), padding included, so the receiver's check fails
            assert int(r["status"]) == 13, e["name"]
            continue
        assert int(r["status"]) == 0 and int(r["dst_ip"]) == meta["lan_ip"], e["name"]
