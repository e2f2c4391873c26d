"""GPU parity for §8f row f2 (forward / transmit rewrite): halo_tx_fixup_batch_device against
the committed fixtures and the C oracle, bit-exact over the WHOLE byte buffer (frames, gap
bytes and tail), for every lanes-per-frame width, plus full-size synthetic batches and the
rx round trip (rewritten frames verify on the GPU receive path)."""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_tx_equal, tx_batch_arrays, tx_golden

pytestmark = pytest.mark.gpu

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _run(dev, data, offs, lens, ops, flag, hint, with_result=True):
    import torch

    from halo_amd import protocol

    d = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
    o = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev)
    op = torch.from_numpy(np.ascontiguousarray(ops).view(np.uint8)).to(dev)
    res = torch.full((max(1, len(lens)),), 0xEE, dtype=torch.uint8, device=dev) if with_result else None
    protocol.tx_fixup_batch(d, o, ln, op, check_sum_enable=bool(flag), max_len_hint=hint, result=res)
    torch.cuda.synchronize()
    return d.cpu().numpy(), (res.cpu().numpy()[:len(lens)] if with_result else None)


# hint -> lanes per frame: 64 -> 1, 1000 -> 4, 4000 -> 8, 0 / 9014 -> 16
@pytest.mark.parametrize("flag", [0, 1])
@pytest.mark.parametrize("hint", [64, 1000, 4000, 0])
def test_tx_fixtures_every_group_width(dev, oracle_lib, flag, hint):
    from halo_amd._lib import TX_OP_DTYPE

    meta, blob, exp = tx_golden(ROOT)
    data, offs, lens, ops, _ = tx_batch_arrays(meta, blob, TX_OP_DTYPE)
    got, res = _run(dev, data, offs, lens, ops, flag, hint)
    assert_tx_equal(got, offs, lens, res, meta, exp, flag, what=f"GPU tx flag={flag} hint={hint}")
    want, wres = oracle_lib.tx_batch(data, offs, lens, ops, flags=flag, threads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} buffer bytes differ from the oracle (first {bad[:8]})"
    assert np.array_equal(res, wres)


def test_tx_gap_bytes_untouched_and_no_result(dev, oracle_lib):
    """Gap bytes between frames hold garbage; they must come back unchanged (whole-buffer
    compare), and a null result pointer is allowed."""
    from halo_amd._lib import TX_OP_DTYPE

    meta, blob, _ = tx_golden(ROOT)
    data, offs, lens, ops, _ = tx_batch_arrays(meta, blob, TX_OP_DTYPE)
    rng = np.random.default_rng(11)
    mask = np.ones(data.shape[0], bool)
    for o, L in zip(offs.astype(np.int64) * 4, lens.astype(np.int64)):
        mask[o:o + L] = False
    data = data.copy()
    data[mask] = rng.integers(0, 256, mask.sum(), dtype=np.uint8)
    got, _ = _run(dev, data, offs, lens, ops, 1, 0, with_result=False)
    want, _ = oracle_lib.tx_batch(data, offs, lens, ops, flags=1)
    assert np.array_equal(got, want)
    assert np.array_equal(got[mask], data[mask])


def test_tx_empty_batch_and_validation(dev):
    from halo_amd import _lib

    L = _lib.lib
    assert L.halo_tx_fixup_batch_device(None, None, None, 0, None, 1, 0, None, None) == 0
    import torch

    b = torch.zeros(64, dtype=torch.uint8, device=dev)
    assert L.halo_tx_fixup_batch_device(b.data_ptr(), b.data_ptr(), b.data_ptr(), 1, b.data_ptr() + 4, 1, 0, None,
                                        None) == _lib.HALO_E_INVAL  # ops not 16-byte aligned
    assert L.halo_tx_fixup_batch_device(b.data_ptr(), b.data_ptr(), b.data_ptr(), 1, b.data_ptr(), 2, 0, None,
                                        None) == _lib.HALO_E_INVAL  # unknown flag bit


def _random_ops(n, seed):
    from halo_amd import protocol

    rng = np.random.default_rng(seed)
    ops = protocol.tx_ops(n)
    ops["steps"] = rng.integers(0, 32, n, dtype=np.uint8)
    ops["dst_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ops["src_ip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ops["dst_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
    ops["src_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
    return ops


@pytest.mark.parametrize("size_mode,proto_mode,length,hint", [(0, 0, 64, 64), (1, 3, 0, 1514), (0, 3, 9000, 9014),
                                                              (1, 3, 0, 64)])
def test_tx_synth_batches_vs_oracle(dev, oracle_lib, size_mode, proto_mode, length, hint):
    """Full-buffer bit-exact compare on synthetic traffic (64 B UDP, IMIX mix, jumbo) with random
    step sets and addresses; hint 64 on IMIX runs lane-per-frame over frames up to 1514 B."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 200_000 if length != 9000 else 20_000
    lay = synth.layout(n, length=length or 64, size_mode=size_mode, proto_mode=proto_mode, mutate_shift=4,
                       first_index=777_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0x5A)
    before = fr["bytes"].cpu().numpy()
    ops = _random_ops(n, 5)
    for flag in (0, 1):
        d = fr["bytes"].clone()
        res = torch.empty(n, dtype=torch.uint8, device=dev)
        protocol.tx_fixup_batch(d, fr["offsets_dw"], fr["lens"], torch.from_numpy(ops.view(np.uint8)).to(dev),
                                check_sum_enable=bool(flag), max_len_hint=hint, result=res)
        torch.cuda.synchronize()
        want, wres = oracle_lib.tx_batch(before, lay["offsets_dw"], lay["lens"], ops, flags=flag, threads=16)
        got = d.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"flag={flag}: {bad.size} bytes differ (first {bad[:8]})"
        assert np.array_equal(res.cpu().numpy(), wres)


def test_tx_config2_full_size_round_trip(dev, oracle_lib):
    """BASELINE config 2 at full size (1M x 64 B UDP): DNAT + TTL + SNAT on the GPU, then the GPU
    receive path verifies every clean rewritten frame and sees the new addresses and ports
    (frames with TTL <= 1 keep their source: the chain stops at HandleIpv4PktTtl); bytes equal
    the oracle's."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 1 << 20
    lay = synth.layout(n, length=64, mutate_shift=6)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    before = fr["bytes"].cpu().numpy()
    ops = protocol.tx_ops(n, protocol.TX_NAT_DST | protocol.TX_TTL | protocol.TX_NAT_SRC, dst_ip=0x0A000002,
                          dst_port=8080, src_ip=0xC6336401, src_port=50000)
    res = torch.empty(n, dtype=torch.uint8, device=dev)
    protocol.tx_fixup_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], torch.from_numpy(ops.view(np.uint8)).to(dev),
                            max_len_hint=64, result=res)
    torch.cuda.synchronize()
    r = res.cpu().numpy()
    ttl = before[lay["offsets_dw"].astype(np.int64) * 4 + 22]
    alive = ttl > 1  # HandleIpv4PktTtl: TTL <= 1 takes the TTL-exceeded branch, SNAT not applied
    assert 0 < (~alive).sum() < n // 50
    assert np.all(r[alive] == protocol.TX_R_TTL_ALIVE) and np.all(r[~alive] == 0)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(), max_len_hint=64)
    recs = protocol.records(out)
    mutated = (lay["kinds"] & 0x80) != 0
    # both checksums are recomputed over whatever the frame holds, so clean frames verify (and so
    # do mutated ones whose flip no parse check catches)
    assert np.all(recs["status"][~mutated] == 0)
    ok = recs[~mutated & alive]
    assert np.all(ok["dst_ip"] == 0x0A000002) and np.all(ok["src_ip"] == 0xC6336401)
    assert np.all(ok["dport"] == 8080) and np.all(ok["sport"] == 50000)
    dead = recs[~mutated & ~alive]
    assert np.all(dead["dst_ip"] == 0x0A000002) and np.all(dead["src_ip"] != 0xC6336401)
    want, _ = oracle_lib.tx_batch(before, lay["offsets_dw"], lay["lens"], ops, flags=1, threads=16)
    assert np.array_equal(fr["bytes"].cpu().numpy(), want)
