"""Batch mirror of halo's ``hashcode`` package and the NAT flow-table keys.

``GetHashCodeXXH3`` (hashcode/hashcode.go:15-17, XXH3-64 of hashcode/xxh3.go) hashes one byte
slice per call in the reference; here one call hashes a device-resident batch through
``halo_xxh3_64_batch_device``. ``flow_hash`` builds, from parsed rx records, the 13-byte keys
of ``NatFlowHash`` / ``NatWanFlowHash`` (engine/ipv4_engine.go:442-479) the way
``NatGetFlowByHash`` / ``NatGetFlowByWan`` normalise them (:524-581) and hashes them, plus the
``hashmap.HashMap`` bucket ``hash % buckets`` (hashmap/hashmap.go:64).
"""
from __future__ import annotations

from . import _lib
from ._lib import FLOW_NAT_LAN, FLOW_NAT_WAN, NAT_FULL_CONE, NAT_SYMMETRIC  # noqa: F401

# engine/ipv4_engine.go:423-426
NatTypeSymmetric = NAT_SYMMETRIC
NatTypeFullCone = NAT_FULL_CONE


def _stream(stream):
    import torch

    return (stream if stream is not None else torch.cuda.current_stream()).cuda_stream


def GetHashCodeXXH3(data, offsets, lens, out=None, stream=None):  # noqa: N802 (reference name)
    """XXH3-64 of data[offsets[i] : offsets[i] + lens[i]] for every i (cuda tensors: uint8 data,
    int64 byte offsets, int32 lengths). Returns a cuda int64 tensor (bit pattern of the u64)."""
    import torch

    n = int(lens.numel())
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=data.device)
    rc = _lib.lib.halo_xxh3_64_batch_device(_lib.ptr(data), _lib.ptr(offsets), _lib.ptr(lens), n, _lib.ptr(out),
                                            _stream(stream))
    _lib.check("halo_xxh3_64_batch_device", rc)
    return out


def flow_hash(records, kind: int = FLOW_NAT_LAN, nat_type: int = NatTypeSymmetric, buckets: int = 0,
              stream=None):
    """(hash, bucket) for a cuda uint8 [n, 32] record tensor (parse_frames_batch output), or a
    [n, 16] tensor of compact records (halo_flow_hash_compact_device)."""
    import torch

    width = int(records.shape[1]) if records.dim() == 2 else 32
    assert width in (16, 32), "records: uint8 [n, 32] (full) or [n, 16] (compact)"
    n = int(records.shape[0]) if records.dim() == 2 else int(records.numel()) // 32
    h = torch.empty(n, dtype=torch.int64, device=records.device)
    b = torch.empty(n, dtype=torch.int32, device=records.device) if buckets else None
    fn = "halo_flow_hash_compact_device" if width == 16 else "halo_flow_hash_device"
    rc = getattr(_lib.lib, fn)(_lib.ptr(records), n, kind, nat_type, _lib.ptr(h), buckets, _lib.ptr(b),
                               _stream(stream))
    _lib.check(fn, rc)
    return h, b
