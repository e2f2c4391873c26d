"""ctypes binding of libhalo_rx_cpu.so — halo_rx_parse_batch_cpu (include/halo_rx_cpu.h).

The explicit CPU entry point of SURVEY.md §8b: the receive chain on the calling core, for polls
too small to pay a GPU round trip. It is not a fallback: nothing in
halo_amd's device path imports this module, and libhalo_rx.so never calls the library. Importing
it raises if the library is not built.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import HALO_RX_RECORD_COMPACT, HALO_RX_STATUS_COUNT, LIB_DIR, RECORD16_DTYPE, RESULT_DTYPE, NetIf, check

CPU_LIB_PATH = os.path.join(LIB_DIR, "libhalo_rx_cpu.so")


def _load() -> ctypes.CDLL:
    if not os.path.exists(CPU_LIB_PATH):
        raise ImportError(f"{CPU_LIB_PATH} is missing: build it first (python halo_amd/build.py)")
    L = ctypes.CDLL(CPU_LIB_PATH)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.halo_rx_parse_batch_cpu.restype = ctypes.c_int
    L.halo_rx_parse_batch_cpu.argtypes = [vp, vp, vp, u32, u32, ctypes.POINTER(NetIf), vp, vp]
    L.halo_rx_cpu_version.restype = ctypes.c_char_p
    L.halo_rx_cpu_version.argtypes = []
    return L


lib = _load()


def parse_frames_cpu(data: np.ndarray, offsets: np.ndarray, lens: np.ndarray, *, netif: NetIf,
                     check_sum_enable: bool = True, jumbo: bool = False, l3_start: bool = False,
                     compact: bool = False, out: np.ndarray | None = None,
                     hist: np.ndarray | None = None) -> np.ndarray:
    """Parse + verify n frames in host memory (frame i: lens[i] bytes at data[offsets[i]:]) on the
    calling core; returns the n RESULT_DTYPE records, or RECORD16_DTYPE ones with `compact` (into
    `out` when given). `hist` (u32[14]) is incremented per status."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    n = int(lens.shape[0])
    if offsets.shape[0] != n:
        raise ValueError("offsets and lens differ in length")
    if n and int((offsets + lens).max()) > data.nbytes:
        raise ValueError("a frame reaches past the end of data")
    rec = RECORD16_DTYPE if compact else RESULT_DTYPE
    if out is None:
        out = np.empty(n, dtype=rec)
    if out.dtype != rec or out.shape[0] < n or not out.flags.c_contiguous:
        raise ValueError(f"out must be a contiguous array of n {'RECORD16' if compact else 'RESULT'}_DTYPE records")
    if hist is not None and (hist.dtype != np.uint32 or hist.shape[0] < HALO_RX_STATUS_COUNT
                             or not hist.flags.c_contiguous):
        raise ValueError("hist must be a contiguous u32 array of 14 counters")
    if data.size == 0:  # every frame is empty: any valid address will do (the call needs a non-null one)
        data = np.zeros(4, np.uint8)
    flags = ((1 if check_sum_enable else 0) | (2 if jumbo else 0) | (0x10 if l3_start else 0)
             | (HALO_RX_RECORD_COMPACT if compact else 0))
    p = lambda a: None if a is None or a.size == 0 else a.ctypes.data  # noqa: E731
    check("halo_rx_parse_batch_cpu", lib.halo_rx_parse_batch_cpu(p(data), p(offsets), p(lens), n, flags, netif,
                                                                 p(out), p(hist)))
    return out[:n]
