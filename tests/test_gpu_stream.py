"""GPU: the byte-stream kernel (HALO_RX_VARIANT_STREAM, rx_parse.hip rx_stream_kernel) on the
layouts its window logic distinguishes, every record bit-exact against the C oracle:
dense in index order (one coalesced pass per window), frames shuffled inside their window
(out-of-order segments, still dense), frames shuffled across the whole buffer and frames with
big gaps (windows not dense: each lane sums its own segment), a data pointer off any 128-byte
line, and windows with no checksummed segment at all."""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_records_equal

pytestmark = pytest.mark.gpu
STREAM = -2


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def frames(dev):
    """40k IMIX frames (mixed protocols, 1/8 mutated) as a list of byte strings."""
    from halo_amd import synth
    from halo_amd._lib import NetIf

    n = 40_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=3, first_index=123_456)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0x5A)
    blob = fr["bytes"].cpu().numpy()
    offs = lay["offsets_dw"].astype(np.int64) * 4
    return [blob[o:o + int(L)].tobytes() for o, L in zip(offs, lay["lens"])]


def _pack(frames, order, gaps, lead=0):
    """frames[order[k]] placed in order k, each at a dword boundary after gaps[k] extra dwords;
    returns (buffer, offsets_dw indexed by frame, lens)."""
    n = len(frames)
    lens = np.array([len(f) for f in frames], np.uint16)
    offs = np.zeros(n, np.int64)
    pos = lead
    for k, f in enumerate(order):
        pos += 4 * int(gaps[k])
        offs[f] = pos
        pos += (int(lens[f]) + 3) & ~3
    data = np.full(pos + 64, 0xA5, np.uint8)
    for f in range(n):
        data[offs[f]:offs[f] + lens[f]] = np.frombuffer(frames[f], np.uint8)
    return data, offs, lens


def _check(dev, oracle_lib, data, offs, lens, flags, lead=0, what=""):
    import torch

    from halo_amd import _lib, protocol
    from halo_amd._lib import NetIf, RECORD16_DTYPE, compact_of

    buf = torch.from_numpy(data).to(dev)
    view = buf[lead:]  # the data pointer the kernel sees: `lead` bytes into the allocation
    rel = (offs - lead) // 4
    o = torch.from_numpy(rel.astype(np.uint32).view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.view(np.int16)).to(dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(view, o, ln, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                                      jumbo=bool(flags & 2), hist=hist, variant=STREAM)
    out16 = torch.empty((len(lens), 16), dtype=torch.uint8, device=dev)
    fw = protocol.flags_word(bool(flags & 1), bool(flags & 2), STREAM) | _lib.HALO_RX_RECORD_COMPACT
    _lib.check("parse16", _lib.lib.halo_rx_parse_batch_device(_lib.ptr(view), _lib.ptr(o), _lib.ptr(ln), len(lens), fw,
                                                              NetIf.make(), 0, _lib.ptr(out16), None, None))
    torch.cuda.synchronize()
    want, _ = oracle_lib.rx_batch(data[lead:], lens, oracle_lib.NetIf.make(), flags, offsets_dw=rel.astype(np.uint32),
                                  threads=8)
    assert_records_equal(protocol.records(out), want, None, f"stream {what} flags={flags}")
    assert np.array_equal(hist.cpu().numpy(), np.bincount(want["status"], minlength=14))
    got16 = out16.cpu().numpy().view(np.uint8).reshape(-1, 16)
    assert np.array_equal(got16, compact_of(want).view(np.uint8).reshape(-1, 16)), what
    assert got16.shape[0] == len(lens) and RECORD16_DTYPE.itemsize == 16
    return want


@pytest.mark.parametrize("flags", [1, 3, 0])
def test_dense_in_order(dev, oracle_lib, frames, flags):
    n = len(frames)
    data, offs, lens = _pack(frames, np.arange(n), np.zeros(n, np.int64))
    want = _check(dev, oracle_lib, data, offs, lens, flags, what="dense")
    assert (want["status"] == 0).sum() > n // 2


def test_shuffled_inside_windows(dev, oracle_lib, frames):
    """Memory order permuted inside each run of 64 frames: segments out of order, still dense."""
    n = len(frames)
    rng = np.random.default_rng(7)
    order = np.concatenate([w + rng.permutation(min(64, n - w)) for w in range(0, n, 64)])
    data, offs, lens = _pack(frames, order, rng.integers(0, 3, n))
    _check(dev, oracle_lib, data, offs, lens, 1, what="window-shuffled")


def test_shuffled_whole_buffer_and_gaps(dev, oracle_lib, frames):
    """Frames in random memory order over the whole buffer, then frames 4-16 KB apart: windows
    that are not dense (each lane sums its own segment)."""
    n = len(frames) // 4
    sub = frames[:n]
    rng = np.random.default_rng(8)
    data, offs, lens = _pack(sub, rng.permutation(n), np.zeros(n, np.int64))
    _check(dev, oracle_lib, data, offs, lens, 1, what="shuffled")
    data, offs, lens = _pack(sub, np.arange(n), rng.integers(1024, 4096, n))
    _check(dev, oracle_lib, data, offs, lens, 1, what="gapped")


@pytest.mark.parametrize("lead", [4, 60, 124])
def test_data_pointer_off_line(dev, oracle_lib, frames, lead):
    """The data pointer `lead` bytes past a 128-byte boundary, the first frame at offset 0."""
    sub = frames[:5000]
    n = len(sub)
    data, offs, lens = _pack(sub, np.arange(n), np.zeros(n, np.int64), lead=lead)
    _check(dev, oracle_lib, data, offs, lens, 1, lead=lead, what=f"lead={lead}")


def test_windows_without_segments(dev, oracle_lib, frames):
    """600 runts (0-13 B: nothing readable) among good frames, checksums on and off (off: only
    the ICMP frames have a segment to sum, so some windows have none)."""
    n = 3000
    rng = np.random.default_rng(9)
    sub = list(frames[:n])
    for k in rng.choice(n, 600, replace=False):
        sub[k] = sub[k][:int(rng.integers(0, 14))]
    data, offs, lens = _pack(sub, np.arange(n), np.zeros(n, np.int64))
    _check(dev, oracle_lib, data, offs, lens, 1, what="runts")
    _check(dev, oracle_lib, data, offs, lens, 0, what="runts flags=0")


@pytest.mark.parametrize("flags", [1, 0])
def test_dense_windows_with_page_holes(dev, oracle_lib, frames, flags):
    """The read contract (include/halo_rx.h): windows that pass the 2x density test but hold a
    hole of >= 16 KB (whole 4 KB pages with no frame byte) in the middle of every 64-frame window.
    The stream kernel must sum those windows frame by frame (window_pages_covered) and read no
    block in the hole; records bit-exact against the oracle. Holes of one page at every other
    window, and of less than a page (still streamed), are mixed in."""
    n = 12_800
    sub = frames[:n]
    gaps = np.zeros(n, np.int64)
    gaps[32::64] = 4096 + 1024          # 20 KB inside every window
    gaps[96::128] = 1024 + 3            # ~4 KB: at most one empty page at those windows
    gaps[16::64] = 300                  # 1.2 KB: no empty page
    data, offs, lens = _pack(sub, np.arange(n), gaps)
    # the density test alone would stream these windows: span <= 2 x frame bytes + 8 KB
    w0 = offs[:64]
    span = int((w0 + lens[:64]).max() - w0.min())
    assert span <= 2 * int(lens[:64].astype(np.int64).sum()) + 8192 and span > 16384
    _check(dev, oracle_lib, data, offs, lens, flags, what="page holes")
