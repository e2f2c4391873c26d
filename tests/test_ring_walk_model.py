"""CPU: a model of the device record walk's algorithm (ring_rx.hip) — every tile
guesses its entry (the first listed chain that does not stop inside the tile), walks from it, and
one pass links the tiles, walking a tile again from its real entry where the guess was wrong —
checked against the oracle's ReadPacket walk (oracle/halo_ring_oracle.c, itself pinned to the
reference's cgo/ring_buffer.h by tests/test_ring_oracle.py) on spans full of record decoys. The
kernels are checked against the same oracle on the GPU (tests/test_gpu_ring.py); this pins the
induction the link pass relies on, including the wrong-guess and stop cases, where it is cheap to
run many spans."""
from __future__ import annotations

import numpy as np
import pytest

T = 4096  # tile dwords (kTile)
EMPTY, BAD_LEN, PARTIAL, CAPACITY, MAX = 0, 1, 2, 3, 4
TRIES = 4  # kGuessTries


def _tile_tables(w, n_dw, t, half32, cap, lo=0):
    """nxt (position of the next record, or -1 - why) and the listed candidates >= lo."""
    q = np.arange(T, dtype=np.int64)
    a = t * T + q
    ln = np.where(a < n_dw, w[np.minimum(a, n_dw - 1)], 0).astype(np.int64)
    dw = (ln >> 2) + 1 + ((ln & 3) != 0)
    why = np.full(T, -1, np.int64)
    why[(why < 0) & (a >= n_dw)] = EMPTY
    why[(why < 0) & ((ln == 0) | (ln > half32))] = BAD_LEN
    why[(why < 0) & (n_dw - a < dw)] = PARTIAL
    why[(why < 0) & (ln > cap)] = CAPACITY
    nxt = np.where(why < 0, q + dw, -1 - why)
    listed = np.nonzero((why < 0) & (q >= lo))[0]
    return nxt, listed, ln


def _first_break(nxt, listed, i0):
    for i in range(i0, len(listed)):
        if i + 1 >= len(listed) or nxt[listed[i]] != listed[i + 1]:
            return i
    return len(listed) - 1


def _walk(nxt, listed, i0, entry):
    """tile_walk: (records, q) from entry = listed[i0]: the chain of linked candidates, then a
    serial walk past a decoy; nothing when the entry is not listed (it fails the checks)."""
    recs, q = [], entry
    serial = len(listed) > T // 2
    if not serial and i0 < len(listed) and listed[i0] == entry:
        F = _first_break(nxt, listed, i0)
        recs = [int(x) for x in listed[i0:F + 1]]
        q = int(nxt[listed[F]])  # listed positions pass the checks
        serial = q < T and nxt[q] >= 0
    if serial:
        while q < T and nxt[q] >= 0:
            recs.append(q)
            q = int(nxt[q])
    return recs, q


def model_scan(span, used, ring_size, cap, max_frames):
    w = np.frombuffer(span[:used - used % 4].tobytes() + b"\0" * 16, np.uint32).astype(np.int64)
    n_dw = used // 4
    half32 = min(ring_size // 2, 2**32 - 1)
    n_tiles = max(1, (n_dw + T - 1) // T)
    guess = []
    for t in range(n_tiles):  # A: every tile's guess and its walk
        nxt, listed, ln = _tile_tables(w, n_dw, t, half32, cap)
        i0 = 0
        if t > 0:
            k, tries = 0, 0
            while k < len(listed) and tries < TRIES:
                F = _first_break(nxt, listed, k)
                q = int(nxt[listed[F]])
                if not (q < T and nxt[q] < 0):
                    i0 = k
                    break
                k, tries = F + 1, tries + 1
        g = 0 if t == 0 else (int(listed[i0]) if len(listed) else None)
        recs, q = _walk(nxt, listed, i0, g) if g is not None else ([], None)
        guess.append((g, recs, q, nxt, ln))
    # B: link from tile 0 (entry 0); a wrong guess is walked again from the real entry
    offs, lens, e, repaired = [], [], 0, 0
    for t in range(n_tiles):
        g, recs, q, nxt, ln = guess[t]
        if g != e:
            nxt, listed, ln = _tile_tables(w, n_dw, t, half32, cap, lo=e)
            recs, q = _walk(nxt, listed, 0, e)
            repaired += 1
        offs += [t * T + r + 1 for r in recs]
        lens += [int(ln[r]) for r in recs]
        if q < T or t == n_tiles - 1:
            why = int(-1 - nxt[q]) if q < T else EMPTY
            break
        e = q - T
    total = len(offs)
    n = min(total, max_frames)
    stop = MAX if n < total else why
    end = 0
    if n:
        last = offs[n - 1] - 1
        end = 4 * (last + 1 + ((lens[n - 1] + 3) >> 2))
    return (np.array(offs[:n], np.uint32), np.array(lens[:n], np.uint16), stop, end, max(lens[:n], default=0),
            repaired)


def _span(rng, lens, garbage=0.0, pad_decoys=False, corrupt=None):
    lens = np.asarray(lens, np.int64)
    sizes = (4 + lens + 3) & ~3
    starts = np.zeros(len(lens), np.int64)
    starts[1:] = np.cumsum(sizes)[:-1]
    used = int(sizes.sum())
    span = rng.integers(0, 256, used + 16, dtype=np.uint8)
    words = span[:used].view(np.uint32)
    if garbage:
        d = rng.random(words.size) < garbage
        words[d] = rng.integers(1, 1515, int(d.sum()), dtype=np.uint32)
    if pad_decoys:  # the dword before every record: a small "length" (a frame's last bytes + padding)
        words[(starts[1:] // 4) - 1] = rng.integers(1, 400, len(starts) - 1, dtype=np.uint32)
    words[starts // 4] = lens.astype(np.uint32)
    if corrupt is not None:
        words[starts[corrupt[0]] // 4] = corrupt[1]
    return span, used


CASES = [
    ("imix", lambda r: r.choice([64, 570, 1500], 20_000, p=[7 / 12, 4 / 12, 1 / 12]), {}, 1514, 0),
    ("imix_pad_decoys", lambda r: r.choice([64, 570, 1500], 20_000, p=[7 / 12, 4 / 12, 1 / 12]),
     {"pad_decoys": True}, 1514, 0),
    ("decoys_1pct", lambda r: r.integers(1, 1515, 8_000), {"garbage": 0.01}, 1514, 0),
    ("decoys_all", lambda r: r.integers(1, 1515, 4_000), {"garbage": 1.0}, 1514, 0),
    ("bad_len_mid", lambda r: r.integers(1, 1515, 8_000), {"corrupt": (5_000, 0), "pad_decoys": True}, 1514, 0),
    ("capacity_stop", lambda r: list(r.integers(1, 1515, 6_000)) + [1515] + [64] * 500, {"pad_decoys": True}, 1514, 0),
    ("max_frames_cut", lambda r: r.integers(60, 1515, 8_000), {"pad_decoys": True}, 1514, 3_333),
    ("dense", lambda r: r.integers(1, 9, 40_000), {}, 1514, 0),
    ("jumbo", lambda r: r.integers(1, 9015, 3_000), {"pad_decoys": True}, 9014, 0),
]


@pytest.mark.parametrize("name,gen,kw,cap,max_frames", CASES, ids=[c[0] for c in CASES])
def test_guess_and_link_walk_equals_readpacket(oracle_lib, name, gen, kw, cap, max_frames):
    rng = np.random.default_rng(abs(hash(name)) % (2**32))
    span, used = _span(rng, gen(rng), **kw)
    ring_size = 1 << (int(np.ceil(np.log2(max(used, 8)))) + 1)
    for trim in (0, 4, 12):
        u = used - trim
        mf = max_frames or 0xFFFFFFFF
        w_off, w_len, w_stop, w_end, w_ml = oracle_lib.ring_scan(span, u, ring_size, cap, mf)
        off, ln, stop, end, ml, repaired = model_scan(span, u, ring_size, cap, mf)
        assert np.array_equal(off, w_off), (name, trim)
        assert np.array_equal(ln, w_len), (name, trim)
        assert (stop, end, ml) == (w_stop, w_end, w_ml), (name, trim, (stop, end, ml), (w_stop, w_end, w_ml))
        if name == "imix_pad_decoys":
            # a decoy before EVERY record: the guesses skip decoy chains that stop, so few tiles are
            # walked twice (the synthetic IMIX ring of bench.py, where 1.3 % of tiles start with one,
            # needs none: DESIGN.md §14.2)
            tiles = (u // 4 + T - 1) // T
            assert repaired <= max(2, tiles // 10), (repaired, tiles)


@pytest.mark.parametrize("ring_size,cap", [(1 << 12, 1514), (1 << 20, 1514), (1 << 26, 9014), (1 << 14, 16376)])
def test_inner_tile_check_is_readpacket(ring_size, cap):
    """ring_rx.hip tabulate_as<INNER>: in a tile that ends at least one longest record (lim =
    min(size / 2, capacity), (lim + 7) / 4 dwords) before the span does, a position passes
    ReadPacket's four checks exactly when 1 <= len <= lim, and its record is (len + 7) >> 2 dwords
    — the shortcut the guess kernel takes instead of record_dwords."""
    rng = np.random.default_rng(ring_size ^ cap)
    half32 = min(ring_size // 2, 2**32 - 1)
    lim = min(half32, cap)
    lim_dw = (lim + 7) // 4
    n_dw = 50 * T
    for t in (0, 3, 47):
        if t * T + T + lim_dw > n_dw:
            continue
        a = t * T + rng.integers(0, T, 20000)
        ln = np.concatenate([rng.integers(0, 2 * lim + 8, 19000), rng.integers(0, 2**32, 1000, dtype=np.uint64)])
        ln = ln.astype(np.int64)
        dw = (ln >> 2) + 1 + ((ln & 3) != 0)
        full = (a < n_dw) & (ln != 0) & (ln <= half32) & (n_dw - a >= dw) & (ln <= cap)
        short = ((ln - 1) & 0xFFFFFFFF) < lim
        assert np.array_equal(full, short)
        assert np.array_equal(dw[full], (ln[full] + 7) >> 2)
