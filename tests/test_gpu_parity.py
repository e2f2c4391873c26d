"""GPU parity: the HIP path (through the C ABI) against the oracle, bit-exact.

Small cases compare every record with the committed golden fixtures and with the C oracle
on identical frames; BASELINE.json's full sizes are checked through size-independent
properties (every clean frame verifies, every bit-flipped frame is rejected, the status
histogram equals the per-record statuses) plus an oracle comparison on a sample.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_records_equal, expected_records, golden_arrays

pytestmark = pytest.mark.gpu

SEED = 0x48414C4F


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _to_dev(a, dev, dtype=None):
    import torch

    if dtype is not None:
        a = a.view(dtype)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _parse_ragged(dev, data, offs_dw, lens, flags, hint=0, netif=None, variant=0):
    import torch

    from halo_amd import protocol
    from halo_amd._lib import NetIf

    netif = netif or NetIf.make()
    d = _to_dev(data, dev)
    o = _to_dev(offs_dw.astype(np.uint32), dev, np.int32)
    ln = _to_dev(lens.astype(np.uint16), dev, np.int16)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(d, o, ln, netif=netif, check_sum_enable=bool(flags & 1),
                                      jumbo=bool(flags & 2), max_len_hint=hint, hist=hist, variant=variant)
    torch.cuda.synchronize()
    return protocol.records(out), hist.cpu().numpy().astype(np.int64)


@pytest.fixture
def lanes_per_frame(request):
    """The kernel variant (G lanes per frame, -1 = mix, 0 = automatic) a test forces per call."""
    return request.param


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("lanes_per_frame", [1, 4, 8, 16, -1, -2], indirect=True)
def test_golden_ragged_all_group_widths(dev, golden, flags, lanes_per_frame):
    from halo_amd._lib import RESULT_DTYPE

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    got, hist = _parse_ragged(dev, data, offs, lens, flags, 0, variant=lanes_per_frame)
    want = expected_records(meta, flags, RESULT_DTYPE)
    assert_records_equal(got, want, names, f"GPU ragged flags={flags} G={lanes_per_frame}")
    assert np.array_equal(hist, np.bincount(want["status"], minlength=14))


@pytest.mark.parametrize("hint", [0, 64, 128, 256, 512, 1514, 9014])
def test_golden_ragged_auto_variant(dev, golden, hint):
    from halo_amd._lib import RESULT_DTYPE

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    got, _ = _parse_ragged(dev, data, offs, lens, 3, hint)
    assert_records_equal(got, expected_records(meta, 3, RESULT_DTYPE), names, f"GPU ragged hint={hint}")


@pytest.mark.parametrize("lanes_per_frame", [1, 4, 8, 16, -1, -2], indirect=True)
def test_random_imix_every_group_width(dev, oracle_lib, lanes_per_frame):
    """30k IMIX frames, mixed protocols, 1/4 mutated: each kernel variant vs the oracle."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 30_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=2, first_index=77_000_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0x3C)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      variant=lanes_per_frame)
    torch.cuda.synchronize()
    want, _ = oracle_lib.rx_batch(fr["bytes"].cpu().numpy(), lay["lens"], oracle_lib.NetIf.make(), 1,
                                  offsets_dw=lay["offsets_dw"], threads=8)
    assert_records_equal(protocol.records(out), want, None, f"IMIX G={lanes_per_frame}")


@pytest.mark.parametrize("lanes_per_frame", [0, 1, 4, 8, 16, -1, -2], indirect=True)
def test_golden_compact_records(dev, golden, lanes_per_frame):
    """HALO_RX_RECORD_COMPACT: 16-byte records == the compact form of the expected records."""
    import torch

    from halo_amd import _lib
    from halo_amd._lib import RECORD16_DTYPE, RESULT_DTYPE, NetIf, compact_of

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    d = _to_dev(data, dev)
    o = _to_dev(offs.astype(np.uint32), dev, np.int32)
    ln = _to_dev(lens.astype(np.uint16), dev, np.int16)
    for flags in (1, 3):
        out = torch.full((len(lens), 16), 0xEE, dtype=torch.uint8, device=dev)
        rc = _lib.lib.halo_rx_parse_batch_device(d.data_ptr(), o.data_ptr(), ln.data_ptr(), len(lens),
                                                 flags | _lib.HALO_RX_RECORD_COMPACT | _lib.variant_flags(lanes_per_frame),
                                                 NetIf.make(), 0,
                                                 out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(-1).view(RECORD16_DTYPE)
        want = compact_of(expected_records(meta, flags, RESULT_DTYPE))
        bad = np.nonzero(got.view(np.uint8).reshape(-1, 16) != want.view(np.uint8).reshape(-1, 16))[0]
        assert bad.size == 0, [names[i] for i in np.unique(bad)[:5]]


def test_golden_gap_bytes_are_ignored(dev, golden):
    """Bytes between frames (4-byte padding) and after the batch are garbage: no effect."""
    from halo_amd._lib import RESULT_DTYPE

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    dirty = np.full(data.shape[0] + 64, 0xA7, np.uint8)
    for i in range(len(lens)):
        o, L = int(offs[i]) * 4, int(lens[i])
        dirty[o:o + L] = data[o:o + L]
    got, _ = _parse_ragged(dev, dirty, offs, lens, 1, 0)
    assert_records_equal(got, expected_records(meta, 1, RESULT_DTYPE), names, "gap garbage")


@pytest.mark.parametrize("uniform", [False, True])
def test_golden_strided(dev, golden, uniform):
    import torch

    from halo_amd import protocol
    from halo_amd._lib import RESULT_DTYPE, NetIf

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    idx = np.nonzero(lens == 64)[0] if uniform else np.arange(len(lens))
    stride = 64 if uniform else 9016
    buf = np.full(stride * len(idx), 0x5A, np.uint8)
    for j, i in enumerate(idx):
        o, L = int(offs[i]) * 4, int(lens[i])
        buf[j * stride:j * stride + L] = data[o:o + L]
    want = expected_records(meta, 3, RESULT_DTYPE)[idx]
    d = _to_dev(buf, dev)
    ln = None if uniform else _to_dev(lens[idx].astype(np.uint16), dev, np.int16)
    out = protocol.parse_frames_strided(d, stride, len(idx), netif=NetIf.make(), length=64 if uniform else 0,
                                        lens=ln, check_sum_enable=True, jumbo=True)
    torch.cuda.synchronize()
    assert_records_equal(protocol.records(out), want, [names[i] for i in idx], "strided")


def test_empty_batch_is_noop(dev):
    import torch

    from halo_amd import _lib
    from halo_amd._lib import NetIf

    out = torch.zeros(32, dtype=torch.uint8, device=dev)
    rc = _lib.lib.halo_rx_parse_batch_device(None, None, None, 0, 1, NetIf.make(), 0, out.data_ptr(), None, None)
    assert rc == 0
    assert int(out.sum()) == 0


@pytest.mark.parametrize("size_mode,proto_mode,length", [(0, 0, 64), (0, 1, 1514), (0, 2, 333), (1, 3, 0),
                                                        (0, 1, 9000)])
def test_synth_device_matches_host_twin(dev, oracle_lib, size_mode, proto_mode, length):
    import torch

    from halo_amd import synth
    from halo_amd._lib import NetIf

    n = 1500
    lay = synth.layout(n, length=length or 64, size_mode=size_mode, proto_mode=proto_mode, mutate_shift=3,
                       first_index=12345)
    frames = synth.frames_device(lay, NetIf.make(), device=dev, fill=0xA5)
    torch.cuda.synchronize()
    got = frames["bytes"].cpu().numpy()
    want = oracle_lib.synth_batch(SEED, 12345, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                  offsets_dw=lay["offsets_dw"], fill=0xA5)
    assert got.shape == want.shape
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def _sample_check(dev, oracle_lib, frames, lay, recs, flags, idx, stride=0):
    """Oracle on the frames `idx` copied back from the device; recs[k] is frame idx[k]'s record."""
    data = frames["bytes"]
    lens = lay["lens"]
    chunks, offs = [], []
    pos = 0
    for i in idx:
        start = i * stride if stride else int(lay["offsets_dw"][i]) * 4
        L = int(lens[i])
        chunks.append(data[start:start + ((L + 3) & ~3)])
        offs.append(pos // 4)
        pos += (L + 3) & ~3
    import torch

    host = torch.cat(chunks).cpu().numpy()
    want, _ = oracle_lib.rx_batch(host, lens[idx], oracle_lib.NetIf.make(), flags,
                                  offsets_dw=np.array(offs, np.uint32), threads=8)
    assert_records_equal(recs, want, [str(i) for i in idx], "sample vs oracle")


@pytest.mark.parametrize("flags", [0, 1])
def test_random_imix_batch_vs_oracle(dev, oracle_lib, flags):
    """200k IMIX frames, UDP/TCP/ICMP mix, 1/8 mutated: every record bit-exact vs oracle."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 200_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=3, first_index=5_000_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      check_sum_enable=bool(flags), max_len_hint=1500, hist=hist)
    torch.cuda.synchronize()
    got = protocol.records(out)
    host = fr["bytes"].cpu().numpy()
    want, whist = oracle_lib.rx_batch(host, lay["lens"], oracle_lib.NetIf.make(), flags,
                                      offsets_dw=lay["offsets_dw"], threads=16)
    assert_records_equal(got, want, None, f"IMIX flags={flags}")
    assert np.array_equal(hist.cpu().numpy(), whist.astype(np.int32))
    if flags:
        mutated = (lay["kinds"] & 0x80) != 0
        assert np.all(got["status"][~mutated] == 0) and np.all(got["status"][mutated] != 0)


@pytest.mark.parametrize("hint", [0, 64, 1514])
def test_config2_full_size_1M_64B(dev, oracle_lib, hint):
    """BASELINE config 2 at full size: 1M x 64 B UDP; 1/64 mutated."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 1 << 20
    lay = synth.layout(n, length=64, mutate_shift=6)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      max_len_hint=hint, hist=hist)
    torch.cuda.synchronize()
    recs = protocol.records(out)
    mutated = (lay["kinds"] & 0x80) != 0
    h = hist.cpu().numpy()
    assert h[0] == (~mutated).sum() and h.sum() == n
    assert np.array_equal(np.bincount(recs["status"], minlength=14), h)
    assert np.all(recs["status"][~mutated] == 0) and np.all(recs["status"][mutated] != 0)
    ok = recs[~mutated]
    assert np.all(ok["dst_ip"] == 0xC0A86464) and np.all(ok["payload_len"] == 22) and np.all(ok["flags"] == 5)
    host = fr["bytes"].cpu().numpy()
    want, _ = oracle_lib.rx_batch(host, lay["lens"], oracle_lib.NetIf.make(), 1, offsets_dw=lay["offsets_dw"],
                                  threads=16)
    assert_records_equal(recs, want, None, "config2 full")


def test_config3_full_size_16M_imix(dev, oracle_lib):
    """BASELINE config 3 at full size: 16M IMIX TCP/UDP/ICMP (6 GB), 1/64 mutated, through the
    automatic variant (the byte-stream kernel). Whole batch vs the oracle (16 threads), histogram
    == records == the oracle's, every clean frame OK and every mutated one rejected."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 16 << 20
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=6)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      max_len_hint=1500, hist=hist)
    torch.cuda.synchronize()
    recs = protocol.records(out)
    del out
    mutated = (lay["kinds"] & 0x80) != 0
    h = hist.cpu().numpy().astype(np.int64)
    assert h.sum() == n and h[0] == (~mutated).sum()
    assert np.array_equal(np.bincount(recs["status"], minlength=14), h)
    assert np.all(recs["status"][~mutated] == 0) and np.all(recs["status"][mutated] != 0)
    host = fr["bytes"].cpu().numpy()
    del fr
    want, whist = oracle_lib.rx_batch(host, lay["lens"], oracle_lib.NetIf.make(), 1,
                                      offsets_dw=lay["offsets_dw"], threads=16)
    assert np.array_equal(h, whist.astype(np.int64))
    assert_records_equal(recs, want, None, "config3 16M IMIX whole batch")


def test_config4_shard_16M_64B_whole_batch(dev, oracle_lib):
    """BASELINE config 4: one GPU's shard — the last of eight, 16M x 64 B UDP at first_index
    7 * 16M — through halo_rx_parse_batch_device. 16M frames take the lane kernel's grid-stride
    loop over several passes (its grid covers 4M frames per pass). Whole batch vs the oracle,
    histogram == records == the oracle's, every clean frame OK and every mutated one rejected."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 16 << 20
    first = 7 * n
    lay = synth.layout(n, length=64, mutate_shift=6, first_index=first)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      max_len_hint=64, hist=hist)
    torch.cuda.synchronize()
    recs = protocol.records(out)
    del out
    h = hist.cpu().numpy().astype(np.int64)
    mutated = (lay["kinds"] & 0x80) != 0
    assert 0 < mutated.sum() < n // 32
    assert h.sum() == n and h[0] == (~mutated).sum()
    assert np.array_equal(np.bincount(recs["status"], minlength=14), h)
    assert np.all(recs["status"][~mutated] == 0) and np.all(recs["status"][mutated] != 0)
    host = fr["bytes"].cpu().numpy()
    del fr
    want, whist = oracle_lib.rx_batch(host, lay["lens"], oracle_lib.NetIf.make(), 1,
                                      offsets_dw=lay["offsets_dw"], threads=16)
    assert np.array_equal(h, whist.astype(np.int64))
    assert_records_equal(recs, want, None, "config4 shard 7 of 8 (16M x 64 B)")


@pytest.mark.parametrize("variant", [1, 4, 16, -1, -2])
def test_histogram_tree_across_grid_sizes_and_launches(dev, variant):
    """The status histogram's two-level tree (flush_hist: 1024 level-1 slots, 32 level-2 slots, the
    last block to arrive moves a slot up): grids below, at and above 1024 and 32 x 1024 blocks,
    three launches in a row into one histogram on one stream (the slots and arrival counters must
    be left zero by every launch), and a histogram-less launch in between. Histogram == 3 x the
    records' statuses."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    # (1M frames = 16384 lane blocks: the largest grid halved with a histogram; one group more is not)
    for n, length in [(7, 64), (64 * 1024 + 1, 64), (40000, 200), (1 << 20, 64), ((1 << 20) + 64, 64), (1 << 21, 64)]:
        lay = synth.layout(n, length=length, mutate_shift=3)
        fr = synth.frames_device(lay, NetIf.make(), device=dev)
        hist = torch.zeros(14, dtype=torch.int32, device=dev)
        for rep in range(3):
            out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                              max_len_hint=length, hist=hist, variant=variant)
            if rep == 1:
                protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                            max_len_hint=length, variant=variant)
        torch.cuda.synchronize()
        want = 3 * np.bincount(protocol.records(out)["status"], minlength=14)
        assert np.array_equal(hist.cpu().numpy().astype(np.int64), want), (n, length, variant)
        assert want[1:].sum() > 0 or n < 64


def _hist_batches(dev, specs):
    """Device batches for the histogram concurrency tests: (frames, expected histogram per parse)."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    out = []
    for n, length in specs:
        lay = synth.layout(n, length=length, mutate_shift=3)
        fr = synth.frames_device(lay, NetIf.make(), device=dev)
        rec = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                          max_len_hint=length)
        torch.cuda.synchronize()
        want = np.bincount(protocol.records(rec)["status"], minlength=14)
        assert want[1:].sum() > 0
        out.append((fr, length, want))
    return out


def test_histogram_tree_two_threads_on_per_thread_stream(dev):
    """hipStreamPerThread is ONE handle value for a different stream on every host
    thread, so two threads' histogram-on parses run at once under the same handle. The trees belong
    to HSA queues (claimed on the device from the dispatch packet's queue, used only under the
    packet's barrier bit), so two threads x 150 parses each, every thread into its own histogram,
    must count exactly 150 x the records' statuses."""
    import ctypes
    import threading

    import torch

    from halo_amd import _lib
    from halo_amd._lib import NetIf

    per_thread = ctypes.c_void_p(2)  # hipStreamPerThread
    hip_sync = _lib.lib.hipStreamSynchronize  # the HIP runtime libhalo_rx.so is linked against
    hip_sync.restype, hip_sync.argtypes = ctypes.c_int, [ctypes.c_void_p]
    batches = _hist_batches(dev, [(1 << 18, 64), (70001, 200)])
    reps = 150
    hists = [torch.zeros(14, dtype=torch.int32, device=dev) for _ in batches]
    outs = [torch.empty((fr["lens"].numel(), 32), dtype=torch.uint8, device=dev) for fr, _, _ in batches]
    netif = NetIf.make()
    errors = []

    def run(k):
        try:
            fr, length, _ = batches[k]
            for _ in range(reps):
                rc = _lib.lib.halo_rx_parse_batch_device(
                    _lib.ptr(fr["bytes"]), _lib.ptr(fr["offsets_dw"]), _lib.ptr(fr["lens"]), fr["lens"].numel(), 1,
                    netif, length, _lib.ptr(outs[k]), _lib.ptr(hists[k]), per_thread)
                _lib.check("halo_rx_parse_batch_device", rc)
            # the thread's own stream: a device-wide sync after the thread has exited does not wait
            # for its per-thread stream (seen on ROCm 7: counts still rising after it)
            assert hip_sync(per_thread) == 0
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(batches))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    _lib.device_synchronize(0)
    assert not errors, errors
    for k, (_, _, want) in enumerate(batches):
        assert np.array_equal(hists[k].cpu().numpy().astype(np.int64), reps * want), k


def test_histogram_tree_graph_replayed_on_two_streams(dev):
    """a histogram-on parse captured in a hipGraph (no allocation inside the capture:
    halo_rx_init made the trees) and replayed on two streams at once, several times — both replays of
    one graph share their arguments, so only the per-queue trees keep them apart. Histogram ==
    2 x replays x the records' statuses; afterwards an ordinary launch still counts exactly."""
    import torch

    from halo_amd import protocol
    from halo_amd._lib import NetIf

    [(fr, length, want)] = _hist_batches(dev, [(1 << 20, 64)])
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    out = torch.empty((fr["lens"].numel(), 32), dtype=torch.uint8, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                    max_len_hint=length, hist=hist, out=out)
    torch.cuda.synchronize()
    hist.zero_()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    reps = 20
    for _ in range(reps):
        with torch.cuda.stream(s1):
            g.replay()
        with torch.cuda.stream(s2):
            g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), 2 * reps * want)
    hist.zero_()
    protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                max_len_hint=length, hist=hist, out=out)
    torch.cuda.synchronize()
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), want)
    del g


def test_config5_full_size_4M_9000B(dev, oracle_lib):
    """BASELINE config 5 at full size: 4M x 9000 B TCP, strided, 37.7 GB in one call (frame
    addresses past 2^32 and 2^35). Reference verdict (caps kept): ETH_LEN for every frame. Jumbo
    extension: every clean frame OK, every mutated one rejected, histogram == records, and 4096
    frames sampled across the whole batch (first, last, spread) bit-exact vs the oracle."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 4 << 20
    lay = synth.layout(n, length=9000, proto_mode=1, mutate_shift=6, ragged=False, first_index=3 << 22)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, stride=9000)
    mutated = (lay["kinds"] & 0x80) != 0
    for flags in (1, 3):
        hist = torch.zeros(14, dtype=torch.int32, device=dev)
        out = protocol.parse_frames_strided(fr["bytes"], 9000, n, netif=NetIf.make(), length=9000,
                                            check_sum_enable=True, jumbo=bool(flags & 2), hist=hist)
        torch.cuda.synchronize()
        h = hist.cpu().numpy().astype(np.int64)
        st = out[:, 0].cpu().numpy()
        assert np.array_equal(np.bincount(st, minlength=14), h)
        if flags == 1:
            assert h[1] == n  # ETH_LEN: len > 1514 (protocol/ethernet.go:31)
        else:
            assert h[0] == (~mutated).sum() and h.sum() == n
            assert np.all(st[~mutated] == 0) and np.all(st[mutated] != 0)
            idx = np.unique(np.concatenate([np.arange(1024), np.arange(n - 1024, n),
                                            np.random.default_rng(5).choice(n, 2048, replace=False)]))
            recs = protocol.records(out[torch.from_numpy(idx).to(dev)])
            _sample_check(dev, oracle_lib, fr, lay, recs, flags, idx, stride=9000)
        del out
    del fr
    torch.cuda.empty_cache()


@pytest.mark.parametrize("length", [570, 1500])
def test_uniform_ragged_batch_uniform_len_flag(dev, oracle_lib, length):
    """A ragged batch of one frame length flagged HALO_RX_UNIFORM_LEN takes the uniform-length
    kernel table (570 B: 4 lanes, 1500 B: 8 lanes per frame) instead of the mix kernel: records
    bit-exact vs the oracle and identical to the automatic (mix) choice."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 200_000
    lay = synth.layout(n, length=length, proto_mode=3, mutate_shift=4, first_index=31_000_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    outs = []
    for uniform in (True, False):
        hist = torch.zeros(14, dtype=torch.int32, device=dev)
        out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                          max_len_hint=length, uniform_len=uniform, hist=hist)
        torch.cuda.synchronize()
        outs.append((protocol.records(out), hist.cpu().numpy().astype(np.int64)))
    want, whist = oracle_lib.rx_batch(fr["bytes"].cpu().numpy(), lay["lens"], oracle_lib.NetIf.make(), 1,
                                      offsets_dw=lay["offsets_dw"], threads=16)
    for recs, h in outs:
        assert_records_equal(recs, want, None, f"{length} B uniform")
        assert np.array_equal(h, whist.astype(np.int64))


def test_config5_jumbo_9000B(dev, oracle_lib):
    """BASELINE config 5 shape (9000 B TCP, strided) on 1M frames: the reference verdict is
    ETH_LEN for every frame; the jumbo extension verifies every clean frame."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 1 << 20
    lay = synth.layout(n, length=9000, proto_mode=1, mutate_shift=6, ragged=False)
    fr = synth.frames_device(lay, NetIf.make(), device=dev, stride=9000)
    for flags in (1, 3):
        hist = torch.zeros(14, dtype=torch.int32, device=dev)
        out = protocol.parse_frames_strided(fr["bytes"], 9000, n, netif=NetIf.make(), length=9000,
                                            check_sum_enable=True, jumbo=bool(flags & 2), hist=hist)
        torch.cuda.synchronize()
        h = hist.cpu().numpy()
        mutated = (lay["kinds"] & 0x80) != 0
        if flags == 1:
            assert h[1] == n
        else:
            assert h[0] == (~mutated).sum() and h.sum() == n
            st = out[:, 0].cpu().numpy()
            assert np.all(st[mutated] != 0)
            _sample_check(dev, oracle_lib, fr, lay, protocol.records(out[:3000]), 3, np.arange(3000), stride=9000)
    del fr


def test_shard_is_slice_of_global_stream(dev, oracle_lib):
    """Config 4 sharding: rank r's frames are global frames [r*n, (r+1)*n) (no exchange)."""
    import torch

    from halo_amd import synth
    from halo_amd._lib import NetIf

    n = 4096
    for rank in (0, 3, 7):
        lay = synth.layout(n, length=64, first_index=rank * (16 << 20))
        fr = synth.frames_device(lay, NetIf.make(), device=dev, fill=0)
        torch.cuda.synchronize()
        got = fr["bytes"].cpu().numpy()
        for k in (0, 1, n - 1):
            want = oracle_lib.synth_frame(SEED, rank * (16 << 20) + k, 64, 0, oracle_lib.NetIf.make())
            assert got[k * 64:(k + 1) * 64].tobytes() == want


def test_host_path_double_buffered(dev, golden, oracle_lib):
    """halo_rx_parse_batch_host: unaligned host offsets, tiny chunks (many round trips)."""
    from halo_amd._lib import RESULT_DTYPE, NetIf
    from halo_amd.engine import HostBatcher

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    # repack with odd (unaligned) host offsets
    host = np.zeros(int(lens.astype(np.int64).sum()) + 3 * len(lens) + 16, np.uint8)
    hoffs = np.zeros(len(lens), np.uint64)
    pos = 1
    for i in range(len(lens)):
        o, L = int(offs[i]) * 4, int(lens[i])
        host[pos:pos + L] = data[o:o + L]
        hoffs[i] = pos
        pos += L + 3
    for chunk_frames in (7, 1 << 18):
        hb = HostBatcher(0, chunk_frames=chunk_frames, chunk_bytes=65536)
        for flags in (1, 3):
            hist = np.zeros(14, np.uint32)
            got = hb.parse(host, hoffs, lens, NetIf.make(), flags, hist)
            want = expected_records(meta, flags, RESULT_DTYPE)
            assert_records_equal(got, want, names, f"host path chunk={chunk_frames} flags={flags}")
            assert np.array_equal(hist, np.bincount(want["status"], minlength=14))
        hb.close()


def test_host_path_direct_dma_registered(dev, oracle_lib):
    """Packed host batch (ascending 4-byte-aligned offsets): the direct-DMA mode, with the
    buffer registered and not, in chunks much smaller than the batch."""
    from halo_amd import _lib, synth
    from halo_amd._lib import NetIf
    from halo_amd.engine import HostBatcher

    lay = synth.layout(40_000, size_mode=1, proto_mode=3, mutate_shift=3, first_index=9_000_000)
    data = oracle_lib.synth_batch(synth.SEED, 9_000_000, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                  offsets_dw=lay["offsets_dw"], fill=0x77)
    offs = lay["offsets_dw"].astype(np.uint64) * 4
    reg = _lib.host_array(data.shape, data.dtype)  # registered below: pages of its own
    reg[...] = data
    data = reg
    want, whist = oracle_lib.rx_batch(data, lay["lens"], oracle_lib.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
    hb = HostBatcher(0, chunk_frames=3000, chunk_bytes=1 << 20)
    import contextlib

    out = _lib.host_array(len(lay["lens"]), _lib.RESULT_DTYPE)
    try:
        # registered frames: zero-copy (parsed in place over PCIe) and, forced, the DMA path;
        # records into a registered array (written by the kernel over PCIe) or a pageable one
        for registered, zero_copy, out_reg in [(False, True, False), (True, False, False), (True, True, False),
                                               (True, True, True), (False, True, True)]:
            hb.set_zero_copy(zero_copy)
            hist = np.zeros(14, np.uint32)
            out.view(np.uint8)[:] = 0xEE
            with contextlib.ExitStack() as regs:
                if registered:
                    regs.enter_context(_lib.registered(data))
                if out_reg:
                    regs.enter_context(_lib.registered(out))
                got = hb.parse(data, offs, lay["lens"], NetIf.make(), 1, hist, out=out if out_reg else None)
            assert_records_equal(got, want, None,
                                 f"host direct registered={registered} zero_copy={zero_copy} out_registered={out_reg}")
            assert np.array_equal(hist, whist)
    finally:
        hb.close()
    assert _lib.registered_count() == 0, _lib.registrations()


def test_host_path_zero_copy_any_order(dev, oracle_lib):
    """Zero-copy takes frames in any order inside one registration (span = min..max of the
    chunk); a chunk whose offsets are not 4-byte aligned relative to each other, or whose span
    starts off a dword, is refused and goes the DMA / repack way. Records identical to the
    oracle in every case."""
    from halo_amd import _lib, synth
    from halo_amd._lib import NetIf
    from halo_amd.engine import HostBatcher

    n = 20_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=4, first_index=123_456)
    data = oracle_lib.synth_batch(synth.SEED, 123_456, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                  offsets_dw=lay["offsets_dw"], fill=0x5A)
    perm = np.random.default_rng(7).permutation(n)
    lens = np.ascontiguousarray(lay["lens"][perm])
    base_offs = lay["offsets_dw"][perm].astype(np.uint64) * 4
    want, whist = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), 1,
                                      offsets_dw=np.ascontiguousarray(lay["offsets_dw"][perm]))
    size = data.shape[0]
    reg = _lib.host_array(2 * size + 4096, np.uint8)
    hb = HostBatcher(0, chunk_frames=4096, chunk_bytes=1 << 20)
    try:
        cases = []
        # shuffled, aligned: zero-copy; shifted by one byte: relative alignment kept, span off a dword
        for shift in (0, 1):
            cases.append((f"shuffled shift={shift}", shift, base_offs + shift, None))
        # one frame per chunk relocated to a 2 mod 4 offset: that chunk is repacked by the CPU
        offs = base_offs.copy()
        moved = np.arange(0, n, 4096)
        cases.append(("one misaligned frame per chunk", 0, offs, moved))
        for label, shift, offs, moved in cases:
            reg[:] = 0
            reg[shift:shift + size] = data
            offs = offs.copy()
            if moved is not None:
                pos = size + 2
                for i in moved:
                    o, L = int(offs[i]), int(lens[i])
                    reg[pos:pos + L] = reg[o:o + L]
                    offs[i] = pos
                    pos += L + 4
            hist = np.zeros(14, np.uint32)
            with _lib.registered(reg):
                got = hb.parse(reg, offs, lens, NetIf.make(), 1, hist)
            assert_records_equal(got, want, None, f"zero-copy {label}")
            assert np.array_equal(hist, whist)
    finally:
        hb.close()
    assert _lib.registered_count() == 0, _lib.registrations()


def test_host_path_zero_copy_gpu_metadata(dev, oracle_lib):
    """Frames, offsets and lengths all registered: the GPU converts the caller's u64 offsets
    itself (zc_meta_kernel) and parses in place; with a frame outside the frames' registration
    that chunk is flagged and re-parsed on the DMA path, its first counts dropped from the
    histogram. Records and histograms identical to the oracle in every case."""
    import contextlib

    from halo_amd import _lib, synth
    from halo_amd._lib import NetIf
    from halo_amd.engine import HostBatcher

    n = 30_000
    lay = synth.layout(n, size_mode=1, proto_mode=3, mutate_shift=3, first_index=777_000)
    data = oracle_lib.synth_batch(synth.SEED, 777_000, lay["lens"], lay["kinds"], oracle_lib.NetIf.make(),
                                  offsets_dw=lay["offsets_dw"], fill=0x33)
    want, whist = oracle_lib.rx_batch(data, lay["lens"], oracle_lib.NetIf.make(), 1, offsets_dw=lay["offsets_dw"])
    frames = _lib.host_array(data.shape, np.uint8)
    frames[...] = data
    offs = _lib.host_array(n, np.uint64)
    lens = _lib.host_array(n, np.uint16)
    lens[...] = lay["lens"]
    out = _lib.host_array(n, _lib.RESULT_DTYPE)
    # a copy of frame 5000 and 21000 in pageable memory, outside every registration
    outside = {i: np.array(data[int(lay["offsets_dw"][i]) * 4:int(lay["offsets_dw"][i]) * 4 + int(lay["lens"][i])])
               for i in (5000, 21000)}
    hb = HostBatcher(0, chunk_frames=4096, chunk_bytes=1 << 20)
    try:
        for label, out_reg, move in [("all registered", True, False), ("records pageable", False, False),
                                     ("two frames outside", True, True)]:
            offs[...] = lay["offsets_dw"].astype(np.uint64) * 4
            if move:
                base = frames.ctypes.data
                for i, buf in outside.items():
                    offs[i] = np.uint64((buf.ctypes.data - base) % (1 << 64))
            out.view(np.uint8)[:] = 0xEE
            hist = np.zeros(14, np.uint32)
            with contextlib.ExitStack() as regs:
                for arr in (frames, offs, lens) + ((out,) if out_reg else ()):
                    regs.enter_context(_lib.registered(arr))
                got = hb.parse(frames, offs, lens, NetIf.make(), 1, hist, out=out if out_reg else None)
            assert_records_equal(got, want, None, f"zero-copy GPU metadata: {label}")
            assert np.array_equal(hist, whist), label
    finally:
        hb.close()
    assert _lib.registered_count() == 0, _lib.registrations()


def test_netif_packet_handle_batch(dev, golden, oracle_lib):
    """Batched PacketHandle: same actions as the reference engine, handlers get payloads."""
    from halo_amd import ACTION_NAMES
    from halo_amd.engine import NetIf

    meta, blob = golden
    frames = [bytes(blob[e["offset"]:e["offset"] + e["len"]]) for e in meta["frames"]]
    it = iter(frames)
    got_udp, got_tcp = [], []
    netif = NetIf("eth0", "AA:AA:AA:AA:AA:AA", "192.168.100.100", lambda: next(it, None))
    netif.RecvUdp(22222, lambda s, p: got_udp.append((s.RemoteIp, s.RemotePort, bytes(p))))
    netif.RecvTcp(80, lambda s, p, seq, ack, fl: got_tcp.append((s.RemotePort, bytes(p), seq, ack, fl)))
    res, actions = netif.packet_handle_batch(batch=100000)
    assert len(actions) == len(frames)
    want = [e["action"]["10"] for e in meta["frames"]]
    assert [ACTION_NAMES[a] for a in actions] == want
    assert (0xC0A86401, 12345, bytes(range(22))) in got_udp
    # TCP payload starts at segment byte headerLen = 5 (tcp.go:49,68 quirk): 15 header bytes first
    assert any(len(p) == 33 and p[15:] == b"hello tcp payload!" for _, p, _, _, _ in got_tcp)


def _dense_repack(src: np.ndarray, src_offs_dw: np.ndarray, lens: np.ndarray, lead_dw: int):
    """Frames src[4*src_offs_dw[i] : +lens[i]] packed back to back at 4-byte-aligned starts, the first
    `lead_dw` dwords into the buffer (so a 64-frame window's span starts off a 16-byte boundary)."""
    sizes = (lens.astype(np.int64) + 3) & ~3
    offs = np.zeros(len(lens), dtype=np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    offs += 4 * lead_dw
    out = np.full(int(offs[-1] + sizes[-1]) + 64, 0x5A, dtype=np.uint8)
    for i in range(len(lens)):
        s, L, o = int(src_offs_dw[i]) * 4, int(lens[i]), int(offs[i])  # Python ints (NEP 50: no u16 wrap)
        out[o:o + L] = src[s:s + L]
    return out, (offs // 4).astype(np.uint32)


@pytest.mark.parametrize("case", ["64B_aligned", "64B_lead1", "64B_lead3", "ragged_1to64", "mixed_long",
                                  "swapped", "partial_tail"])
def test_lane_coalesced_windows(dev, oracle_lib, case):
    """Lane-kernel windows of 64 frames of <= 64 B packed back to back (spans starting off a 16-byte
    boundary, ragged 1..64 B lengths), windows with a longer frame, records out of memory order and
    a partial last window: bit-exact vs the oracle, histogram = records, under the lane variant and
    the automatic one (hint 64). Written for the coalesced round 0 tried in round 6 (DESIGN §15.4,
    commit 0b3928e), kept as coverage of the per-lane path's layouts."""
    from halo_amd import synth
    from halo_amd._lib import NetIf

    rng = np.random.default_rng(zlib_crc(case))
    n = 64 * 700 + (17 if case == "partial_tail" else 0)
    long_ = case == "mixed_long"
    lay = synth.layout(n, length=128 if long_ else 64, mutate_shift=3, first_index=5_000_000)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    src = fr["bytes"].cpu().numpy()
    lens = lay["lens"].astype(np.int64).copy()
    if case == "ragged_1to64":
        lens = rng.integers(1, 65, n)
    elif long_:  # 64 B frames, and in one window in five a frame of 65..128 B
        lens[:] = 64
        for w in range(0, n // 64, 5):
            lens[64 * w + int(rng.integers(0, 64))] = int(rng.integers(65, 129))
    lead = {"64B_lead1": 1, "64B_lead3": 3}.get(case, 0)
    data, offs = _dense_repack(src, lay["offsets_dw"], lens.astype(np.uint16), lead)
    if case == "swapped":  # frames in memory order, but two records of every other window swapped
        for w in range(0, n // 64, 2):
            a, b = 64 * w + 5, 64 * w + 40
            offs[a], offs[b] = offs[b], offs[a]
            lens[a], lens[b] = lens[b], lens[a]
    lens16 = lens.astype(np.uint16)
    want, whist = oracle_lib.rx_batch(data, lens16, oracle_lib.NetIf.make(), 1, offsets_dw=offs, threads=8)
    for variant, hint in ((1, 0), (0, 64)):
        got, hist = _parse_ragged(dev, data, offs, lens16, 1, hint=hint, variant=variant)
        assert_records_equal(got, want, None, f"coalesced windows {case} variant={variant}")
        assert np.array_equal(hist, whist.astype(np.int64))
    assert whist[1:].sum() > 0


def zlib_crc(s: str) -> int:
    import zlib

    return zlib.crc32(s.encode())
