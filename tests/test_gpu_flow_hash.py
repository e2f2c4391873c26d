"""GPU parity for §8f row f3: halo_xxh3_64_batch_device and halo_flow_hash_device against the
committed fixtures and the C oracle (itself pinned to the published XXH3-64 vectors), bit-exact."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _xxh3_dev(dev, data, offs, lens):
    import torch

    from halo_amd import hashcode

    d = torch.from_numpy(np.ascontiguousarray(data, np.uint8)).to(dev)
    o = torch.from_numpy(np.ascontiguousarray(offs, np.uint64).view(np.int64)).to(dev)
    ln = torch.from_numpy(np.ascontiguousarray(lens, np.uint32).view(np.int32)).to(dev)
    h = hashcode.GetHashCodeXXH3(d, o, ln)
    torch.cuda.synchronize()
    return h.cpu().numpy().view(np.uint64)


def test_xxh3_fixture_strings(dev):
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "flow_hash.json")))
    stream = np.fromfile(os.path.join(ROOT, "tests", "golden", "hash_stream.bin"), dtype=np.uint8)
    offs = np.array([s["offset"] for s in meta["strings"]], np.uint64)
    lens = np.array([s["len"] for s in meta["strings"]], np.uint32)
    got = _xxh3_dev(dev, stream, offs, lens)
    want = np.array([int(s["hash"], 16) for s in meta["strings"]], np.uint64)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(offs[i])) for i in bad[:8]]


@pytest.mark.parametrize("mix", ["short", "long", "ragged", "kcp"])
def test_xxh3_random_batches_vs_oracle(dev, oracle_lib, mix):
    """Unaligned byte offsets; short-only, long-only, every class mixed, KCP-segment sizes."""
    rng = np.random.default_rng({"short": 1, "long": 2, "ragged": 3, "kcp": 4}[mix])
    n = 20_000
    if mix == "short":
        lens = rng.integers(0, 241, n)
    elif mix == "long":
        lens = rng.integers(241, 5000, n)
    elif mix == "ragged":
        lens = np.where(rng.random(n) < 0.2, rng.integers(241, 9001, n), rng.integers(0, 241, n))
    else:
        lens = rng.integers(24, 1400, n)  # KCP segments (protocol/kcp, ByteCheckModeXXH3)
    lens = lens.astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    gaps = rng.integers(0, 7, n)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1].astype(np.uint64))
    offs += 3
    data = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]) + 8, dtype=np.uint8)
    got = _xxh3_dev(dev, data, offs, lens)
    want = oracle_lib.xxh3_batch(data, offs, lens)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(offs[i])) for i in bad[:8]]


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("nat_type", [0, 1, 7])
def test_flow_hash_golden_and_imix_records(dev, oracle_lib, golden, kind, nat_type):
    """NAT flow keys from GPU-parsed records (golden frames + 200k IMIX) vs the oracle."""
    import torch

    from halo_amd import hashcode, protocol, synth
    from halo_amd._lib import NetIf
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    out_g = protocol.parse_frames_batch(torch.from_numpy(data).to(dev),
                                        torch.from_numpy(offs.view(np.int32)).to(dev),
                                        torch.from_numpy(lens.view(np.int16)).to(dev), netif=NetIf.make())
    lay = synth.layout(200_000, size_mode=1, proto_mode=3, mutate_shift=5, first_index=31337)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    out_i = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                        max_len_hint=1500)
    for out in (out_g, out_i):
        for buckets in (0, 1024, 1000003):
            h, b = hashcode.flow_hash(out, kind, nat_type, buckets)
            torch.cuda.synchronize()
            recs = protocol.records(out)
            wh, wb = oracle_lib.flow_hash_batch(recs, kind, nat_type, buckets)
            assert np.array_equal(h.cpu().numpy().view(np.uint64), wh)
            if buckets:
                assert np.array_equal(b.cpu().numpy().view(np.uint32), wb)


@pytest.mark.parametrize("kind", [0, 1])
def test_flow_hash_compact_records(dev, oracle_lib, kind):
    """halo_flow_hash_compact_device over HALO_RX_RECORD_COMPACT parse output = the full records'
    hashes and buckets (oracle)."""
    import torch

    from halo_amd import hashcode, protocol, synth
    from halo_amd._lib import HALO_RX_RECORD_COMPACT, NetIf

    lay = synth.layout(100_000, size_mode=1, proto_mode=3, mutate_shift=4, first_index=777)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    full = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                       max_len_hint=1500)
    comp = torch.empty((lay["n"], 16), dtype=torch.uint8, device=dev)
    rc = protocol._lib.lib.halo_rx_parse_batch_device(
        fr["bytes"].data_ptr(), fr["offsets_dw"].data_ptr(), fr["lens"].data_ptr(), lay["n"],
        1 | HALO_RX_RECORD_COMPACT, NetIf.make(), 1500, comp.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    for nat_type in (0, 1):
        for buckets in (0, 1 << 20):
            hf, bf = hashcode.flow_hash(full, kind, nat_type, buckets)
            hc, bc = hashcode.flow_hash(comp, kind, nat_type, buckets)
            wh, wb = oracle_lib.flow_hash_batch(protocol.records(full), kind, nat_type, buckets)
            assert np.array_equal(hc.cpu().numpy().view(np.uint64), wh)
            assert np.array_equal(hf.cpu().numpy().view(np.uint64), wh)
            if buckets:
                assert np.array_equal(bc.cpu().numpy().view(np.uint32), wb)


def test_flow_hash_validation(dev):
    from halo_amd import _lib

    L = _lib.lib
    assert L.halo_flow_hash_device(None, 0, 0, 0, None, 0, None, None) == 0
    assert L.halo_flow_hash_device(None, 0, 2, 0, None, 0, None, None) == _lib.HALO_E_INVAL  # unknown kind
    import torch

    r = torch.zeros(64, dtype=torch.uint8, device=dev)
    h = torch.zeros(2, dtype=torch.int64, device=dev)
    assert L.halo_flow_hash_device(r.data_ptr(), 2, 0, 0, h.data_ptr(), 0, h.data_ptr(), None) == _lib.HALO_E_INVAL


@pytest.mark.parametrize("variant", [0, 1, 4, 8, 16, -1, -2])
def test_fused_parse_flow_hash(dev, oracle_lib, golden, variant):
    """halo_rx_parse_flow_batch_device: the same records as the plain parse (full and compact),
    and the flow hashes / buckets the oracle computes from those records — golden frames, a
    structured-fuzz corpus and IMIX, every kernel variant."""
    import torch

    from halo_amd import _lib, protocol, synth
    from halo_amd._lib import NetIf
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    fdata, foffs, flens = oracle_lib.fuzz_batch(0xF10, 50_000, oracle_lib.NetIf.make())
    lay = synth.layout(100_000, size_mode=1, proto_mode=3, mutate_shift=5, first_index=4242)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    batches = [(torch.from_numpy(d).to(dev), torch.from_numpy(o.view(np.int32)).to(dev),
                torch.from_numpy(ln.view(np.int16)).to(dev), hint)
               for d, o, ln, hint in ((data, offs, lens, 0), (fdata, foffs, flens, 0))]
    batches.append((fr["bytes"], fr["offsets_dw"], fr["lens"], 1500))
    stream = torch.cuda.current_stream().cuda_stream
    vf = _lib.variant_flags(variant)
    for d, o, ln, hint in batches:
        n = int(ln.numel())
        for compact in (False, True):
            flags = 1 | vf | (_lib.HALO_RX_RECORD_COMPACT if compact else 0)
            width = 16 if compact else 32
            ref = torch.empty((n, width), dtype=torch.uint8, device=dev)
            _lib.check("parse", _lib.lib.halo_rx_parse_batch_device(
                d.data_ptr(), o.data_ptr(), ln.data_ptr(), n, flags, NetIf.make(), hint, ref.data_ptr(), None,
                stream))
            full = protocol.parse_frames_batch(d, o, ln, netif=NetIf.make(), max_len_hint=hint)
            for kind, nat, buckets in ((1, 0, 1 << 20), (0, 1, 0), (0, 0, 1000003)):
                got = torch.full((n, width), 0xEE, dtype=torch.uint8, device=dev)
                h = torch.zeros(n, dtype=torch.int64, device=dev)
                b = torch.zeros(n, dtype=torch.int32, device=dev)
                _lib.check("fused", _lib.lib.halo_rx_parse_flow_batch_device(
                    d.data_ptr(), o.data_ptr(), ln.data_ptr(), n, flags, NetIf.make(), hint, got.data_ptr(),
                    None, kind, nat, h.data_ptr(), buckets, b.data_ptr() if buckets else None, stream))
                torch.cuda.synchronize()
                assert torch.equal(got, ref), (variant, compact, kind)
                wh, wb = oracle_lib.flow_hash_batch(protocol.records(full), kind, nat, buckets)
                assert np.array_equal(h.cpu().numpy().view(np.uint64), wh), (variant, compact, kind, nat)
                if buckets:
                    assert np.array_equal(b.cpu().numpy().view(np.uint32), wb)


def test_xxh3_canonical_every_length(dev):
    """halo_xxh3_64_batch_device == the canonical xxHash library (committed values,
    tests/gen_golden_xxh3_canonical.py) on every length 0..4096 and 300 lengths up to 9000."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "xxh3_canonical.npz"))
    stream = np.fromfile(os.path.join(ROOT, "tests", "golden", "hash_stream.bin"), dtype=np.uint8)
    got = _xxh3_dev(dev, stream, z["str_off"].astype(np.uint64), z["str_len"])
    bad = np.nonzero(got != z["str_hash"])[0]
    assert bad.size == 0, [int(z["str_len"][i]) for i in bad[:8]]


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("nat_type", [0, 1])
def test_flow_hash_golden_records_equal_canonical(dev, golden, kind, nat_type):
    """NAT flow keys of the GPU-parsed golden frames, hashed on the GPU (standalone and fused into
    the parse) == the canonical library's XXH3 of the 13-byte keys."""
    import torch

    from halo_amd import _lib, hashcode, protocol
    from halo_amd._lib import NetIf
    from tests.helpers import golden_arrays

    z = np.load(os.path.join(ROOT, "tests", "golden", "xxh3_canonical.npz"))
    want = z["flow_hash"][(z["flow_kind"] == kind) & (z["flow_nat"] == nat_type)]
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = protocol.parse_frames_batch(d, o, ln, netif=NetIf.make())
    h, _ = hashcode.flow_hash(out, kind, nat_type, 0)
    n = int(ln.numel())
    rec = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    hf = torch.zeros(n, dtype=torch.int64, device=dev)
    _lib.check("fused", _lib.lib.halo_rx_parse_flow_batch_device(
        d.data_ptr(), o.data_ptr(), ln.data_ptr(), n, 1, NetIf.make(), 0, rec.data_ptr(), None, kind, nat_type,
        hf.data_ptr(), 0, None, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(h.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(hf.cpu().numpy().view(np.uint64), want)
