"""CPU: the status histogram's trees (rx_parse.hip flush_hist), restated in Python: the two-level tree
(grids above 16384 blocks) and, at the end of the file, the one level of 16-block runs.

Every block adds (1 << 40 | count) to status word k of level-1 slot b % 1024; the add that brings
the slot's arrivals to its block count (g // 1024 + (g % 1024 > s)) moves the slot's total to
level-2 slot s // 32, whose completing add (arrivals = the level-1 slots it covers) moves it to the
caller's counter; each completing thread zeroes its word. The model runs the blocks in random
orders for grids below, at and above 1024 and 32 x 1024 blocks and checks that the caller's counts
are exact, that every slot completes exactly once, and that every word is left zero for the next
launch (the GPU tests check the kernel itself: test_gpu_parity.py
test_histogram_tree_across_grid_sizes_and_launches)."""
from __future__ import annotations

import numpy as np
import pytest

SLOTS, FAN, ONE = 1024, 32, 1 << 40
MASK = ONE - 1


def run_tree(counts: np.ndarray, order: np.ndarray, l1: dict, l2: dict, out: np.ndarray) -> int:
    """counts[b] = block b's count for one status; returns how many level-1 slots completed."""
    g = len(counts)
    used = min(g, SLOTS)
    done = 0
    for b in order:
        s = b % SLOTS
        add = ONE | int(counts[b])
        now = l1.get(s, 0) + add
        l1[s] = now
        if now >> 40 != g // SLOTS + (g % SLOTS > s):
            continue
        done += 1
        l1[s] = 0  # atomicExch(l1, 0)
        first = s & ~(FAN - 1)
        add2 = ONE | (now & MASK)
        t = SLOTS + s // FAN
        now2 = l2.get(t, 0) + add2
        l2[t] = now2
        if now2 >> 40 != min(used - first, FAN):
            continue
        l2[t] = 0
        out[0] += now2 & MASK
    return done


@pytest.mark.parametrize("g", [1, 7, 31, 32, 33, 1023, 1024, 1025, 2047, 4096, 16384, 32 * 1024 + 5, 40000])
def test_tree_counts_exact_and_words_reset(g):
    rng = np.random.default_rng(g)
    l1, l2 = {}, {}
    for launch in range(3):  # launches in a row reuse the words
        counts = rng.integers(0, 64, g)
        out = np.zeros(1, np.int64)
        done = run_tree(counts, rng.permutation(g), l1, l2, out)
        assert out[0] == counts.sum(), (g, launch)
        assert done == min(g, SLOTS)  # every used level-1 slot completed exactly once
        assert all(v == 0 for v in l1.values()) and all(v == 0 for v in l2.values())


RUN = 16  # HALO_HIST_RUNS


def run_runs(counts: np.ndarray, order: np.ndarray, words: dict, out: np.ndarray) -> int:
    """flush_hist for grids up to SLOTS * RUN blocks: block b adds (1 << 40 | count) to word b // RUN;
    the add that brings a run's arrivals to its size (min(RUN, g - RUN * r)) zeroes the word and adds
    the run's total to the caller's counter."""
    g = len(counts)
    done = 0
    for b in order:
        r = b // RUN
        now = words.get(r, 0) + (ONE | int(counts[b]))
        words[r] = now
        if now >> 40 != min(RUN, g - RUN * r):
            continue
        done += 1
        words[r] = 0
        out[0] += now & MASK
    return done


@pytest.mark.parametrize("g", [1, 15, 16, 17, 1023, 8192, 8193, 16383, 16384])
def test_runs_counts_exact_and_words_reset(g):
    rng = np.random.default_rng(g + 7)
    words = {}
    for launch in range(3):
        counts = rng.integers(0, 64, g)
        out = np.zeros(1, np.int64)
        done = run_runs(counts, rng.permutation(g), words, out)
        assert out[0] == counts.sum(), (g, launch)
        assert done == (g + RUN - 1) // RUN  # every run completed exactly once
        assert max(words) < SLOTS and all(v == 0 for v in words.values())
