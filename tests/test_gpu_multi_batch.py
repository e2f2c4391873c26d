"""GPU: several device-resident batches in one call (halo_rx_parse_batches_device) — the batch
stream of the reference's poll loop (engine/engine.go:344-351) handed over K batches at a time.
Every batch's records are bit-exact against the C oracle (and identical to K separate
halo_rx_parse_batch_device calls); the histogram counts all batches; empty batches are skipped;
frames over 64 B take one launch per batch; compact records and LoChan (L3) batches too."""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_records_equal, strip_ethernet

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _batch(dev, oracle_lib, n, seed, length=64, size_mode=0, proto_mode=0, mutate_shift=3):
    import torch

    from halo_amd import synth
    from halo_amd._lib import NetIf

    lay = synth.layout(n, length=length, size_mode=size_mode, proto_mode=proto_mode, mutate_shift=mutate_shift,
                       seed=seed)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0x5A)
    host = fr["bytes"].cpu().numpy()
    want = {f: oracle_lib.rx_batch(host, lay["lens"], oracle_lib.NetIf.make(), f, offsets_dw=lay["offsets_dw"])[0]
            for f in (0, 1, 3)}
    out = torch.empty((max(n, 1), 32), dtype=torch.uint8, device=dev)
    return fr, lay, want, out, host


@pytest.mark.parametrize("flags", [0, 1, 3])
def test_multi_batch_64B_one_launch(dev, oracle_lib, flags):
    import torch

    from halo_amd import protocol
    from halo_amd._lib import NetIf

    sizes = [100_000, 0, 1, 63, 64, 65, 4097, 250_000]
    bs = [_batch(dev, oracle_lib, n, 0x3000 + k) for k, n in enumerate(sizes)]
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    protocol.parse_frames_batches([(b[0]["bytes"], b[0]["offsets_dw"], b[0]["lens"], b[3]) for b in bs],
                                  netif=NetIf.make(), check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2),
                                  max_len_hint=64, hist=hist)
    total = np.zeros(14, np.int64)
    for n, b in zip(sizes, bs):
        if not n:
            continue
        got = protocol.records(b[3][:n])
        assert_records_equal(got, b[2][flags], None, f"batch of {n}")
        total += np.bincount(b[2][flags]["status"], minlength=14)
    assert np.array_equal(hist.cpu().numpy(), total)
    assert total[1:].sum() > 0  # mutated frames fail somewhere


def test_multi_batch_compact_and_32_batches(dev, oracle_lib):
    import torch

    from halo_amd import _lib, protocol
    from halo_amd._lib import NetIf

    bs = [_batch(dev, oracle_lib, 1000 + 37 * k, 0x4000 + k) for k in range(32)]
    outs = [torch.empty((b[1]["n"], 16), dtype=torch.uint8, device=dev) for b in bs]
    protocol.parse_frames_batches([(b[0]["bytes"], b[0]["offsets_dw"], b[0]["lens"], o) for b, o in zip(bs, outs)],
                                  netif=NetIf.make(), max_len_hint=64, compact=True)
    for b, o in zip(bs, outs):
        got = o.cpu().numpy().reshape(-1).view(_lib.RECORD16_DTYPE)
        want = _lib.compact_of(b[2][1])
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    with pytest.raises(_lib.HaloError):  # at most 32 batches per call
        protocol.parse_frames_batches([(b[0]["bytes"], b[0]["offsets_dw"], b[0]["lens"], b[3]) for b in bs + bs[:1]],
                                      netif=NetIf.make(), max_len_hint=64)


def test_multi_batch_larger_frames_per_batch_launches(dev, oracle_lib):
    """IMIX batches (frames up to 1500 B): one launch per batch, same records."""
    import torch

    from halo_amd import protocol
    from halo_amd._lib import NetIf

    bs = [_batch(dev, oracle_lib, n, 0x5000 + n, size_mode=1, proto_mode=3) for n in (20_000, 7, 30_001)]
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    protocol.parse_frames_batches([(b[0]["bytes"], b[0]["offsets_dw"], b[0]["lens"], b[3]) for b in bs],
                                  netif=NetIf.make(), max_len_hint=1500, hist=hist)
    total = np.zeros(14, np.int64)
    for b in bs:
        n = b[1]["n"]
        assert_records_equal(protocol.records(b[3][:n]), b[2][1], None, f"IMIX batch of {n}")
        total += np.bincount(b[2][1]["status"], minlength=14)
    assert np.array_equal(hist.cpu().numpy(), total)
    # and the lane kernel forced on the same large frames (one launch) gives the same records
    for b in bs:
        b[3].zero_()
    protocol.parse_frames_batches([(b[0]["bytes"], b[0]["offsets_dw"], b[0]["lens"], b[3]) for b in bs],
                                  netif=NetIf.make(), variant=1)
    for b in bs:
        n = b[1]["n"]
        assert_records_equal(protocol.records(b[3][:n]), b[2][1], None, f"IMIX lane batch of {n}")


def test_multi_batch_lochan(dev, golden, oracle_lib):
    import torch

    from halo_amd import protocol
    from halo_amd._lib import HALO_RX_L3_START, NetIf
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    pk, poffs, plens = strip_ethernet(data, offs, lens)
    want, _ = oracle_lib.rx_batch(pk, plens, oracle_lib.NetIf.make(), 1 | HALO_RX_L3_START, offsets_dw=poffs)
    d = torch.from_numpy(pk).to(dev)
    o = torch.from_numpy(poffs.view(np.int32)).to(dev)
    ln = torch.from_numpy(plens.view(np.int16)).to(dev)
    outs = [torch.empty((len(plens), 32), dtype=torch.uint8, device=dev) for _ in range(3)]
    protocol.parse_frames_batches([(d, o, ln, x) for x in outs], netif=NetIf.make(), variant=1, l3_start=True)
    for x in outs:
        assert_records_equal(protocol.records(x), want, None, "L3 multi")
