"""CPU: the forward/transmit restatements (§8f row f2) — the C oracle (oracle/halo_tx_oracle.c)
against the committed fixtures made by the independent Python restatement, the two against
each other on fuzzed frames, and the properties that pin them to the reference's intent."""
from __future__ import annotations

import os
import random

import numpy as np
import pytest

from tests.helpers import assert_tx_equal, tx_batch_arrays, tx_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("flag", [0, 1])
def test_c_oracle_matches_tx_fixtures(oracle_lib, flag):
    meta, blob, exp = tx_golden(ROOT)
    data, offs, lens, ops, originals = tx_batch_arrays(meta, blob, oracle_lib.TX_OP_DTYPE)
    out, res = oracle_lib.tx_batch(data, offs, lens, ops, flags=flag, threads=4)
    assert_tx_equal(out, offs, lens, res, meta, exp, flag, what="C oracle vs fixtures")
    for k in range(len(lens)):  # nothing past the header region is touched
        o, L = int(offs[k]) * 4, int(lens[k])
        assert np.array_equal(out[o + 52:o + L], originals[k][52:])


def _fuzz_frames(n, seed):
    from oracle import ref_py as R

    rnd = random.Random(seed)
    for _ in range(n):
        proto = rnd.choice([1, 6, 17, 17, 2])
        pay = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 7, 26, 100, 333])))
        src, dst = bytes(rnd.randrange(256) for _ in range(4)), bytes(rnd.randrange(256) for _ in range(4))
        if proto == 17:
            seg = R.build_udp(pay, rnd.randrange(65536), rnd.randrange(65536), src, dst)
        elif proto == 6:
            seg = R.build_tcp(pay, rnd.randrange(65536), rnd.randrange(65536), src, dst, rnd.getrandbits(32),
                              rnd.getrandbits(32), rnd.randrange(256))
        elif proto == 1:
            seg = R.build_icmp(pay, rnd.choice([0, 8, 11]), bytes([rnd.randrange(256), rnd.randrange(256)]), 1)
        else:
            seg = pay
        ip = bytearray(R.build_ipv4(seg, proto, src, dst, ttl=rnd.choice([0, 1, 2, 64, 255])))
        if rnd.random() < 0.2:
            ip[0] = rnd.choice([0x44, 0x46, 0x4F, 0x45])
        if rnd.random() < 0.2:
            ip[2:4] = rnd.randrange(65536).to_bytes(2, "big")
        f = bytearray(R.build_eth(bytes(ip), b"\xaa" * 6, b"\x02" * 6, 0x0800))
        if rnd.random() < 0.1:
            f = f[:rnd.randrange(len(f) + 1)]
        if rnd.random() < 0.05:
            f[12:14] = b"\x86\xdd"
        yield bytes(f), rnd.randrange(32), [rnd.getrandbits(32), rnd.randrange(65536), rnd.getrandbits(32),
                                            rnd.randrange(65536)]


def test_c_oracle_matches_python_restatement_fuzz(oracle_lib):
    from oracle import ref_tx_py as T

    for f, steps, (dip, dpt, sip, spt) in _fuzz_frames(1500, 77):
        op = np.zeros(1, oracle_lib.TX_OP_DTYPE)[0]
        op["steps"], op["dst_ip"], op["dst_port"], op["src_ip"], op["src_port"] = steps, dip, dpt, sip, spt
        for en in (0, 1):
            got, r = oracle_lib.tx_frame(f, op, flags=en)
            b = bytearray(f)
            want_r = T.tx_frame(b, steps, dip, dpt, sip, spt, check_sum_enable=bool(en))
            assert (got, r) == (bytes(b), want_r), (f.hex(), steps, en)


def test_rewritten_frames_verify_clean(oracle_lib, golden):
    """NAT + TTL on well-formed frames yields frames the rx path verifies as OK — except the
    reference's own inconsistencies, which are reproduced, not fixed: ReCalcUdp/TcpCheckSum sum
    pkt[20:] INCLUDING Ethernet padding and take the pseudo length from totalLen-20
    (protocol/ipv4.go:189-196, :215-222), while ParseIpv4Pkt trims to totalLen (:84) and
    ParseUdpPkt uses the UDP length field (udp.go:30-40). A NATed frame with non-zero padding or
    a UDP length field != totalLen-20 therefore fails the reference's own receive check."""
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    n = oracle_lib.NetIf.make()
    before, _ = oracle_lib.rx_batch(data, lens, n, 1, offsets_dw=offs)
    ok = (before["status"] == 0) & (before["ip_proto"] != 0xFF)
    ops = np.zeros(len(lens), oracle_lib.TX_OP_DTYPE)
    ops["steps"] = 0x01 | 0x02 | 0x04
    ops["dst_ip"], ops["dst_port"], ops["src_ip"], ops["src_port"] = 0x0A000001, 8080, 0xC0A80001, 40000
    new, res = oracle_lib.tx_batch(data, offs, lens, ops, flags=1)
    after, _ = oracle_lib.rx_batch(new, lens, n, 1, offsets_dw=offs)
    alive = (res & 0x01) != 0
    quirk = np.array([nm in ("ip_padding_trimmed_garbage", "udp_len_field_small", "udp_len_field_large")
                      for nm in names])
    assert np.all(after["status"][ok & alive & quirk] == 13)  # L4_CKSUM, as the reference would
    sel = ok & alive & ~quirk
    assert sel.sum() > 150
    assert np.all(after["status"][sel] == 0), [names[i] for i in np.nonzero(sel & (after["status"] != 0))[0][:5]]
    assert np.all(after["dst_ip"][sel] == 0x0A000001) and np.all(after["src_ip"][sel] == 0xC0A80001)
    udp_tcp = sel & (after["ip_proto"] != 1)
    assert np.all(after["dport"][udp_tcp] == 8080) and np.all(after["sport"][udp_tcp] == 40000)
    icmp = sel & (after["ip_proto"] == 1)
    assert icmp.sum() > 5 and np.all(after["sport"][icmp] == 40000)  # SNAT ran last on the echo id


def test_dpdk_fill_equals_go_recalc_on_well_formed(oracle_lib):
    """eth_tx's DPDK fill and ReCalc* agree on IHL-5, untrimmed, UDP/TCP packets (the arithmetic
    is the same RFC 1071 sum); they differ only where a UDP checksum computes to zero."""
    from oracle import ref_tx_py as T

    rnd = random.Random(9)
    for f, _, _ in _fuzz_frames(600, 5):
        if len(f) < 54 or f[12:14] != b"\x08\x00" or f[14] != 0x45 or f[23] not in (6, 17):
            continue
        if ((f[16] << 8) | f[17]) != len(f) - 14:
            continue
        a, _ = oracle_lib.tx_frame(f, np.array([(T.RECALC, 0, 0, 0, 0, 0, 0)], oracle_lib.TX_OP_DTYPE)[0], 1)
        b, _ = oracle_lib.tx_frame(f, np.array([(T.DPDK_FILL, 0, 0, 0, 0, 0, 0)], oracle_lib.TX_OP_DTYPE)[0], 1)
        at = 40 if f[23] == 17 else 50
        if a != b:
            assert f[23] == 17 and a[at:at + 2] == b"\0\0" and b[at:at + 2] == b"\xff\xff"
            assert a[:at] == b[:at] and a[at + 2:] == b[at + 2:]
        rnd.random()


def test_dpdk_fill_known_answer(golden):
    """Zeroing both checksums of the canonical 64-byte UDP frame and running the DPDK fill gives
    back its known checksums (IP 0xF103, UDP 0xC07A)."""
    from oracle import oracle as O

    kat = bytes.fromhex(
        "aaaaaaaaaaaa020000000001080045000032000100008011f103c0a86401c0a86464303956ce001ec07a"
        "000102030405060708090a0b0c0d0e0f101112131415")
    z = bytearray(kat)
    z[24:26] = b"\0\0"
    z[40:42] = b"\0\0"
    got, r = O.tx_frame(bytes(z), np.array([(0x10, 0, 0, 0, 0, 0, 0)], O.TX_OP_DTYPE)[0], 0)
    assert got == kat and r == 0
    got, r = O.tx_frame(bytes(z), np.array([(0x08, 0, 0, 0, 0, 0, 0)], O.TX_OP_DTYPE)[0], 1)
    assert got == kat and r == 0


# ---- the Build* half of row f2 -----------------------------------------------------------------
def test_build_oracle_matches_fixtures():
    """ora_tx_build_batch (C) == the Python restatement's fixtures, both runs (CheckSumEnable
    true from iphId 0, false from 0xFFF0 across the wrap); the first frame is the canonical one."""
    from tests.helpers import assert_build_equal, build_golden
    from oracle import oracle as O

    desc, payload, meta, expect = build_golden(ROOT)
    mac = bytes.fromhex(meta["src_mac"])
    for run in meta["runs"]:
        frames, lens, res, end = O.tx_build_batch(desc, payload, mac, run["flags"], 1516, run["ip_id_start"])
        assert_build_equal(frames, lens, res, end, run, expect, f"C oracle flags={run['flags']}")
    assert set(meta["runs"][0]["results"]) == {0, 1, 2}


def test_built_frames_parse_clean():
    """Every Ethernet frame the Build* chain makes with CheckSumEnable passes the receive chain
    (ParseEthFrm -> ParseIpv4Pkt -> ParseUdp/Tcp/IcmpPkt) with its fields intact: the transmit
    and receive restatements agree on the same arithmetic."""
    from tests.helpers import build_golden
    from oracle import oracle as O

    desc, payload, meta, expect = build_golden(ROOT)
    run = meta["runs"][0]
    netif = O.NetIf.make(mac="AA:AA:AA:AA:AA:AA", ip="192.168.100.100")
    checked = 0
    for i, d in enumerate(desc):
        if run["results"][i] != 0 or d["mode"] != 0 or run["lens"][i] > 1514:
            continue
        o, ln = run["expect_offsets"][i], run["lens"][i]
        r = O.rx_frame(bytes(expect[o:o + ln]), netif, 1)
        assert r["status"] == 0, (i, int(r["status"]))
        assert int(r["ip_proto"]) == int(d["proto"]) and int(r["src_ip"]) == int(d["src_ip"])
        assert int(r["dst_ip"]) == int(d["dst_ip"])
        if d["proto"] != 1:
            assert (int(r["sport"]), int(r["dport"])) == (int(d["src_port"]), int(d["dst_port"]))
        checked += 1
    assert checked > 150
