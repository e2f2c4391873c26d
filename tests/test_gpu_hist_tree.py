"""The status histogram's edge paths: the fallback a launch
takes when its HSA queue finds no tree key, more distinct queues than the old 16 keys, a capture
before halo_rx_init, and halo_rx_release followed by captured-graph replays and eager calls. Every
count is exact: histogram == reps x the bincount of the records' statuses. The histogram replaces
the reference's per-frame counters' role at engine/ethernet_engine.go:19 and ipv4_engine.go:21."""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = 64  # kHistTrees (halo_common.h)


@pytest.fixture(scope="module")
def dev():
    import torch

    from halo_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def batch(dev):
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    n = 1 << 20
    lay = synth.layout(n, length=64, mutate_shift=3)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(), max_len_hint=64)
    torch.cuda.synchronize()
    want = np.bincount(protocol.records(out)["status"], minlength=14).astype(np.int64)
    assert want[1:].sum() > 0
    return fr, n, want


def _keys(op, arg=0):
    from halo_amd import _lib

    rc = _lib.lib.halo_rx_debug_hist_keys(0, op, arg)
    assert rc >= 0, rc
    return rc


def _launch(fr, n, out, hist, stream_handle):
    from halo_amd import _lib
    from halo_amd._lib import NetIf

    rc = _lib.lib.halo_rx_parse_batch_device(_lib.ptr(fr["bytes"]), _lib.ptr(fr["offsets_dw"]), _lib.ptr(fr["lens"]),
                                             n, 1, NetIf.make(), 64, _lib.ptr(out), _lib.ptr(hist),
                                             ctypes.c_void_p(stream_handle))
    _lib.check("halo_rx_parse_batch_device", rc)


def _timed(fr, n, out, hist, reps):
    import torch

    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        _launch(fr, n, out, hist, s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us per launch


def test_forced_fallback_is_exact_and_reset_restores_trees(dev, batch):
    """Poisoned keys: every launch counts straight into the caller's counters (the fallback). Exact;
    its cost beside the tree's is printed. Reset: the trees come back."""
    import torch

    fr, n, want = batch
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    hist = torch.zeros(14, dtype=torch.int32, device=dev)
    _keys(3)
    _timed(fr, n, out, hist, 3)
    us_tree = _timed(fr, n, out, hist, 20)
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), 23 * want)
    assert _keys(0) >= 1
    _keys(1)  # poison
    assert _keys(0) == 0
    hist.zero_()
    us_fallback = _timed(fr, n, out, hist, 20)
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), 20 * want)
    _keys(3)
    assert _keys(0) == 0
    hist.zero_()
    _timed(fr, n, out, hist, 5)
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), 5 * want)
    assert _keys(0) >= 1
    print(f"\n[hist] 1M x 64 B histogram-on launch: tree {us_tree:.1f} us, fallback {us_fallback:.1f} us "
          f"({us_fallback / us_tree:.1f}x)")


def _cu_masked_streams(count):
    """`count` streams created with a CU mask (each gets an HSA queue of its own): all CUs but one,
    a different one per stream."""
    import torch

    from halo_amd import _lib

    create = _lib.lib.hipExtStreamCreateWithCUMask
    create.restype, create.argtypes = ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                     ctypes.POINTER(ctypes.c_uint32)]
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    streams = []
    for k in range(count):
        mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
        if ncu % 32:
            mask[words - 1] = (1 << (ncu % 32)) - 1
        cu = (7 * k + 3) % ncu
        mask[cu // 32] &= ~(1 << (cu % 32)) & 0xFFFFFFFF
        h = ctypes.c_void_p()
        assert create(ctypes.byref(h), words, mask) == 0
        streams.append(h.value)
    return streams


def _sync_destroy(streams):
    from halo_amd import _lib

    sync, destroy = _lib.lib.hipStreamSynchronize, _lib.lib.hipStreamDestroy
    sync.restype, sync.argtypes = ctypes.c_int, [ctypes.c_void_p]
    destroy.restype, destroy.argtypes = ctypes.c_int, [ctypes.c_void_p]
    for h in streams:
        assert sync(h) == 0
    for h in streams:
        assert destroy(h) == 0


@pytest.mark.parametrize("queues", [20])
def test_more_queues_than_the_old_sixteen_keys(dev, batch, queues):
    """20 CU-masked streams (20 HSA queues) with histogram-on parses interleaved over them, each
    stream into its own histogram: every count exact, and more than 16 queues hold a tree."""
    import torch

    fr, n, want = batch
    _keys(3)
    streams = _cu_masked_streams(queues)
    try:
        outs = [torch.empty((n, 32), dtype=torch.uint8, device=dev) for _ in streams]
        hists = [torch.zeros(14, dtype=torch.int32, device=dev) for _ in streams]
        torch.cuda.synchronize()
        reps = 4
        for _ in range(reps):
            for k, h in enumerate(streams):
                _launch(fr, n, outs[k], hists[k], h)
    finally:
        _sync_destroy(streams)
    torch.cuda.synchronize()
    for k in range(queues):
        assert np.array_equal(hists[k].cpu().numpy().astype(np.int64), reps * want), k
    assert _keys(0) > 16
    _keys(3)


def test_queues_beyond_the_free_keys_fall_back_exactly(dev, batch):
    """All keys but 2 occupied, then 6 CU-masked queues: 2 get trees, 4 take the fallback, all
    concurrently; every stream's histogram exact."""
    import torch

    fr, n, want = batch
    _keys(2, 2)
    assert _keys(0) == KEYS - 2
    streams = _cu_masked_streams(6)
    try:
        outs = [torch.empty((n, 32), dtype=torch.uint8, device=dev) for _ in streams]
        hists = [torch.zeros(14, dtype=torch.int32, device=dev) for _ in streams]
        torch.cuda.synchronize()
        reps = 5
        for _ in range(reps):
            for k, h in enumerate(streams):
                _launch(fr, n, outs[k], hists[k], h)
    finally:
        _sync_destroy(streams)
    torch.cuda.synchronize()
    for k in range(len(hists)):
        assert np.array_equal(hists[k].cpu().numpy().astype(np.int64), reps * want), k
    assert _keys(0) == KEYS
    _keys(3)
    assert _keys(0) == 0


def test_capture_before_init_then_release(dev):
    """In a fresh process (the trees are made once per process): a histogram-on parse captured before
    halo_rx_init returns HALO_E_NOMEM; after init a captured graph counts exactly; after
    halo_rx_release (keys back, trees kept) the same graph and an eager call still count exactly."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_capture_before_init.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    res = json.loads(p.stdout.strip().splitlines()[-1])
    print(f"\n[hist] capture-before-init child ({time.time() - t0:.1f}s): {res}")
    assert res["rc_capture_before_init"] == -5  # HALO_E_NOMEM
    assert res["hist_after_refused"] == 0
    assert res["rc_init"] == 0 and res["rc_capture_after_init"] == 0
    assert res["replay3_exact"]
    assert res["rc_release"] == 0 and res["claimed_after_release"] == 0
    assert res["replay_after_release_exact"] and res["eager_after_release_exact"]
    assert res["claimed_end"] >= 1
