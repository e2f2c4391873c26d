"""Structured fuzz corpus (oracle/halo_fuzz.c) on the CPU: it reaches every reachable status
under every flags word and every engine action, and the host dispatcher (halo_rx_dispatch,
product host code) maps the oracle's records to the reference engine's actions.

The same corpus drives tests/test_gpu_fuzz.py, where the HIP kernels are held to the oracle.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import STATUS_NAMES

SEED = 0xF022


@pytest.fixture(scope="module")
def corpus(oracle_lib):
    ni = oracle_lib.NetIf.make()
    return ni, oracle_lib.fuzz_batch(SEED, 60_000, ni)


def test_fuzz_is_deterministic(oracle_lib):
    ni = oracle_lib.NetIf.make()
    a = oracle_lib.fuzz_batch(11, 3000, ni)
    b = oracle_lib.fuzz_batch(11, 3000, ni)
    c = oracle_lib.fuzz_batch(12, 3000, ni)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not np.array_equal(a[0], c[0])
    data, offs, lens = a
    assert np.all(offs[1:].astype(np.int64) * 4 - offs[:-1].astype(np.int64) * 4 == (lens[:-1].astype(np.int64) + 3) & ~3)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_fuzz_reaches_every_reachable_status(corpus, oracle_lib, flags):
    ni, (data, offs, lens) = corpus
    _, hist = oracle_lib.rx_batch(data, lens, ni, flags, offsets_dw=offs, threads=4)
    missing = [STATUS_NAMES[s] for s in range(14) if hist[s] == 0 and STATUS_NAMES[s] != "IP_LEN"]
    if not flags & 1:
        missing.remove("IP_HDR_CKSUM")  # checksums off: no checksum verdicts
    assert not missing, missing
    assert hist[3] == 0  # IP_LEN unreachable behind ParseEthFrm (tests/test_oracle.py)
    assert hist.sum() == len(lens)


def test_fuzz_reaches_every_action_and_host_dispatch_agrees(corpus, oracle_lib):
    from halo_amd import engine
    from halo_amd._lib import NetIf

    ni, (data, offs, lens) = corpus
    for flags in (1, 3):
        recs, _ = oracle_lib.rx_batch(data, lens, ni, flags, offsets_dw=offs, threads=4)
        want = oracle_lib.engine_batch(data, lens, ni, flags, offsets_dw=offs)
        assert np.all(np.bincount(want, minlength=13) > 0)
        got = engine.dispatch(recs, NetIf.make())
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (flags, bad[:5], got[bad[:5]], want[bad[:5]])
