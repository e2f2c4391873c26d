"""Replay, on the CPU, the host allocations the ring tests registered BEFORE commit 52767bd
(np.zeros heap arrays: RingBuffer memory via _aligned(), RingConsumer's record array) and check
every concurrently live pair of registrations against the registry's rule (no shared page).

Each RingConsumer registered two arrays at once: the ring (128 B header + data area) and its
record array. Prints, per consumer, the page ranges the two registrations pinned and whether
they shared a page, or shared one with the previous consumer's still-unfreed arrays.
Usage: python tools/exp/reg_overlap_replay.py  (no GPU, no library calls)"""
from __future__ import annotations

import mmap

import numpy as np

P = mmap.PAGESIZE
RESULT_ITEMSIZE = 32


def _aligned(nbytes: int, align: int = 64) -> np.ndarray:  # the pre-fix RingBuffer allocation
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def pages(a: np.ndarray):
    lo = a.ctypes.data // P
    hi = (a.ctypes.data + a.nbytes + P - 1) // P
    return lo, hi


def overlap(x, y):
    return x[0] < y[1] and y[0] < x[1]


def main():
    import torch  # noqa: F401  (the test process's allocator state: torch and numpy loaded)

    live = []
    shared = 0
    # the ring sizes of tests/test_gpu_ring.py in file order (golden x9 at 1<<18, stops x12 at 1<<20,
    # laps at 1<<16, unpinned x2 at 1<<18, large at 256 MiB, Wire at 8 MiB)
    sizes = [1 << 18] * 9 + [1 << 20] * 12 + [1 << 16] + [1 << 18] * 2 + [256 << 20, 8 << 20]
    for k, size in enumerate(sizes):
        mem = _aligned(128 + size)
        max_frames = min(size, 256 << 20) // 8
        out = np.zeros(max_frames * RESULT_ITEMSIZE, np.uint8)
        pr, po = pages(mem), pages(out)
        same = overlap(pr, po)
        stale = [j for j, (a, b) in enumerate(live) if overlap(a, pr) or overlap(a, po) or overlap(b, pr)
                 or overlap(b, po)]
        shared += same
        print(f"consumer {k:2d} ring 0x{mem.ctypes.data:x} (+{mem.nbytes}) page off {mem.ctypes.data % P:4d}  "
              f"records 0x{out.ctypes.data:x} (+{out.nbytes}) page off {out.ctypes.data % P:4d}  "
              f"share a page: {same}  with an earlier consumer's pages: {stale}")
        live = [(pr, po)]  # the previous consumer's arrays are freed when the next test rebinds
        del mem, out
    print(f"{shared} of {len(sizes)} consumers registered two ranges that shared a page")


if __name__ == "__main__":
    main()
