"""CPU: PacketHandle's LoChan drain (engine/engine.go:353-381).

The C oracle's HALO_RX_L3_START mode and ora_engine_lo against the committed fixtures
(tests/gen_golden_lo.py, expected values from the independent Python restatement
oracle/ref_py.py), the two restatements against each other on the structured fuzz corpus with
its Ethernet headers stripped, and the product's host-side drain decision
(halo_rx_dispatch_loopback) over those records. No GPU: the library's argument checks for the
flag run before any HIP call.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from tests.helpers import assert_records_equal, expected_records, golden_arrays, lo_golden, strip_ethernet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L3 = 0x10


@pytest.fixture(scope="module")
def lo():
    return lo_golden(ROOT)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_oracle_l3_records_match_fixtures(oracle_lib, lo, flags):
    meta, blob = lo
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    got, hist = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), flags | L3, offsets_dw=offs)
    want = expected_records(meta, flags, oracle_lib.RESULT_DTYPE, key="packets")
    assert_records_equal(got, want, names, f"C oracle L3 flags={flags}")
    assert np.array_equal(hist, np.bincount(want["status"], minlength=14))


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_oracle_engine_lo_matches_fixtures(oracle_lib, lo, flags):
    from oracle import ref_py as R

    meta, blob = lo
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    acts = oracle_lib.engine_batch(data, lens, oracle_lib.NetIf.make(), flags | L3, offsets_dw=offs)
    want = [e["action"][str(flags)] for e in meta["packets"]]
    bad = [(names[i], R.ACTIONS[a], w) for i, (a, w) in enumerate(zip(acts, want)) if R.ACTIONS[a] != w]
    assert not bad, bad[:5]


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_dispatch_loopback_matches_fixtures(lo, flags):
    """The product's record-based drain decision == the restated drain, on every fixture."""
    from halo_amd import ACTION_NAMES
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.engine import dispatch_loopback

    meta, _ = lo
    recs = expected_records(meta, flags, RESULT_DTYPE, key="packets")
    acts = dispatch_loopback(recs, NetIf.make())
    want = [e["action"][str(flags)] for e in meta["packets"]]
    got = [ACTION_NAMES[a] for a in acts]
    bad = [(meta["packets"][i]["name"], g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:5]


def test_fixtures_cover_the_drain():
    """Every drain outcome and every status the L3 chain can produce has a fixture."""
    meta, _ = lo_golden(ROOT)
    acts = {e["action"][fl] for e in meta["packets"] for fl in "0123"}
    assert acts == {"DROP_IP", "LO_NOT_OWN", "LOCAL_ICMP", "LOCAL_UDP", "LOCAL_TCP", "DROP_L4"}
    st = {e["expect"][fl]["status"] for e in meta["packets"] for fl in "0123"}
    assert st == set(range(14)) - {1, 2}  # everything but the Ethernet statuses
    # NatGetSrcDstPort below 26 bytes: ports 0 even where the header has them
    short = [e for e in meta["packets"] if e["len"] < 26 and e["len"] >= 24]
    assert short and all(e["expect"]["1"]["sport"] == 0 for e in short)


def test_oracle_l3_equals_python_restatement_on_fuzz(oracle_lib):
    """Structured fuzz frames with their Ethernet header stripped: C == Python, record by record."""
    from oracle import ref_py as R

    data, offs, lens = oracle_lib.fuzz_batch(0xF00D, 3000, oracle_lib.NetIf.make())
    pdata, poffs, plens = strip_ethernet(data, offs, lens)
    own = oracle_lib.NetIf.make().ip
    for flags in (1, 2):
        got, _ = oracle_lib.rx_batch(pdata, plens, oracle_lib.NetIf.make(), flags | L3, offsets_dw=poffs)
        acts = oracle_lib.engine_batch(pdata, plens, oracle_lib.NetIf.make(), flags | L3, offsets_dw=poffs)
        for i in range(len(plens)):
            o, L = int(poffs[i]) * 4, int(plens[i])
            p = bytes(pdata[o:o + L])
            r = R.rx_lo_packet(p, own, check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2))
            r["status"] = R.STATUS.index(r["status"])
            for f, v in r.items():
                assert int(got[i][f]) == v, (i, f, int(got[i][f]), v)
            assert R.ACTIONS[acts[i]] == R.engine_lo(p, own, check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2))


def test_l3_flag_refused_where_unsupported():
    """Fused passes, strided layouts and the ring poll take Ethernet frames only."""
    import ctypes

    from halo_amd import _lib
    from halo_amd._lib import NetIf

    L = _lib.lib
    dummy = ctypes.c_void_p(16)
    rc = L.halo_rx_parse_strided_device(dummy, 64, None, 64, 4, 1 | L3, NetIf.make(), dummy, None, None)
    assert rc == _lib.HALO_E_INVAL
    rc = L.halo_rx_parse_flow_batch_device(dummy, dummy, dummy, 4, 1 | L3, NetIf.make(), 0, dummy, None, 0, 0,
                                           ctypes.c_void_p(64), 0, None, None)
    assert rc == _lib.HALO_E_INVAL
