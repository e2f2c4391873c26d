"""GPU parity on the structured fuzz corpus (oracle/halo_fuzz.c): 512k frames of every size
class (0..41, 42..1514, 1515..9100 B) with header-targeted mutations, packed ragged at 4-byte
boundaries. Every kernel variant, every flags word, full and compact records: bit-exact against
the C oracle; status histograms and the engine actions of the records (halo_rx_dispatch) equal
the oracle's.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_records_equal

pytestmark = pytest.mark.gpu

SEED = 0xF0221
N = 1 << 19
N_VARIANT = 1 << 17


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def corpus(dev, oracle_lib):
    import torch

    ni = oracle_lib.NetIf.make()
    data, offs, lens = oracle_lib.fuzz_batch(SEED, N, ni)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.view(np.int16)).to(dev)
    want = {f: oracle_lib.rx_batch(data, lens, ni, f, offsets_dw=offs, threads=8) for f in (0, 1, 2, 3)}
    return (data, offs, lens), (d, o, ln), want


def _parse(dev, d, o, ln, n, flags, compact=False):
    import torch

    from halo_amd import _lib
    from halo_amd._lib import NetIf

    width = 16 if compact else 32
    out = torch.full((n, width), 0xEE, dtype=torch.uint8, device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    rc = _lib.lib.halo_rx_parse_batch_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), n,
                                             flags | (_lib.HALO_RX_RECORD_COMPACT if compact else 0),
                                             NetIf.make(), 0, out.data_ptr(), hist.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream)
    _lib.check("halo_rx_parse_batch_device", rc)
    torch.cuda.synchronize()
    return out.cpu().numpy(), hist.cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_fuzz_auto_variant_bit_exact(dev, corpus, flags):
    from halo_amd import engine
    from halo_amd._lib import RESULT_DTYPE, NetIf

    _, (d, o, ln), want = corpus
    wrec, whist = want[flags]
    got, hist = _parse(dev, d, o, ln, N, flags)
    got = got.reshape(-1).view(RESULT_DTYPE)
    assert_records_equal(got, wrec, None, f"fuzz flags={flags}")
    assert np.array_equal(hist, whist.astype(np.int64))
    assert np.array_equal(engine.dispatch(got, NetIf.make()), engine.dispatch(wrec, NetIf.make()))


@pytest.mark.parametrize("variant", [1, 4, 8, 16, -1, -2])
def test_fuzz_every_variant_full_and_compact(dev, corpus, variant):
    from halo_amd import _lib
    from halo_amd._lib import RECORD16_DTYPE, RESULT_DTYPE, compact_of

    _, (d, o, ln), want = corpus
    vf = _lib.variant_flags(variant)
    for flags in (1, 3):
        wrec = want[flags][0][:N_VARIANT]
        got, hist = _parse(dev, d, o, ln, N_VARIANT, flags | vf)
        assert_records_equal(got.reshape(-1).view(RESULT_DTYPE), wrec, None, f"fuzz G={variant} flags={flags}")
        assert np.array_equal(hist, np.bincount(wrec["status"], minlength=14))
        got16, _ = _parse(dev, d, o, ln, N_VARIANT, flags | vf, compact=True)
        w16 = compact_of(wrec)
        bad = np.nonzero(np.any(got16.reshape(-1, 16) != w16.view(np.uint8).reshape(-1, 16), axis=1))[0]
        assert bad.size == 0, (variant, flags, bad[:5])
        assert got16.reshape(-1).view(RECORD16_DTYPE).shape[0] == N_VARIANT
