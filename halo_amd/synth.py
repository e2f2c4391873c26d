"""Seeded synthetic receive traffic generated in HBM.

``layout`` (host, C) gives each frame of the global stream its length, protocol and
mutation bit plus packed 4-byte-aligned offsets; ``frames_device`` writes the bytes with the
``halo_synth_frames_device`` kernel. Frame i depends only on (seed, i), so a rank can
generate its shard [first_index, first_index + n) on its own GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import NetIf

SEED = 0x48414C4F  # "HALO"
SIZE_UNIFORM, SIZE_IMIX = 0, 1
PROTO_UDP, PROTO_TCP, PROTO_ICMP, PROTO_MIX = 0, 1, 2, 3


def layout(n: int, *, length: int = 64, size_mode: int = SIZE_UNIFORM, proto_mode: int = PROTO_UDP,
           mutate_shift: int = 0, seed: int = SEED, first_index: int = 0, ragged: bool = True) -> dict:
    lens = np.empty(n, dtype=np.uint16)
    kinds = np.empty(n, dtype=np.uint8)
    offs = np.empty(n, dtype=np.uint32) if ragged else None
    total = ctypes.c_uint64()
    rc = _lib.lib.halo_synth_layout(seed, first_index, n, size_mode, length, proto_mode, mutate_shift,
                                    _lib.ptr(lens), _lib.ptr(offs), _lib.ptr(kinds), ctypes.byref(total))
    _lib.check("halo_synth_layout", rc)
    return {"n": n, "lens": lens, "offsets_dw": offs, "kinds": kinds, "total_bytes": int(total.value),
            "seed": seed, "first_index": first_index}


def frames_device(lay: dict, netif: NetIf, *, device="cuda", stride: int = 0, fill: int | None = None,
                  stream=None) -> dict:
    """Materialise a layout on the GPU. Ragged unless ``stride`` is given.

    Returns dict(bytes, offsets_dw, lens, kinds) of cuda tensors (offsets/lens as int32/int16
    views of the u32/u16 arrays). ``fill`` pre-fills the byte buffer (gap bytes keep it).
    """
    import torch

    n = lay["n"]
    nbytes = stride * n if stride else lay["total_bytes"]
    nbytes = max(16, (nbytes + 15) & ~15)
    buf = (torch.full((nbytes,), fill, dtype=torch.uint8, device=device) if fill is not None
           else torch.empty(nbytes, dtype=torch.uint8, device=device))
    lens = torch.from_numpy(lay["lens"].view(np.int16)).to(device)
    kinds = torch.from_numpy(lay["kinds"]).to(device)
    offs = None
    if not stride:
        offs = torch.from_numpy(lay["offsets_dw"].view(np.int32)).to(device)
    s = (stream or torch.cuda.current_stream()).cuda_stream
    rc = _lib.lib.halo_synth_frames_device(lay["seed"], lay["first_index"], n, _lib.ptr(lens), _lib.ptr(offs),
                                           stride, _lib.ptr(kinds), netif, _lib.ptr(buf), s)
    _lib.check("halo_synth_frames_device", rc)
    return {"bytes": buf, "offsets_dw": offs, "lens": lens, "kinds": kinds, "stride": stride}
