"""CPU: the schedule of flow_hash.hip's run kernel (xxh3_run_kernel), restated in Python and checked
against the independent XXH3 restatement (oracle/ref_xxh3_py.py, pinned to the published sanity
vectors). The kernel reorders hashLong (hashcode/xxh3.go:132-209) into batches of B stripes with
the last stripe as one more term of the final block, scrambles when a batch closes a full block, and
splits hashMedium / hashLarge (:94-129) into per-lane term pairs; a window's strings are split into
16 contiguous runs balanced by iteration count. This model follows those rules step by step (the
GPU tests check the kernel itself bit-exactly)."""
from __future__ import annotations

import numpy as np

from oracle.ref_xxh3_py import M64, P32, P64, SECRET, _aval, _mulfold, _r64, xxh3_64


def _term(lo, hi, s0, s1):
    return _mulfold(lo ^ s0, hi ^ s1)


B = 8  # HALO_XXH3_RUN_B


def run_cost(n: int) -> int:
    return ((n - 1) // 64 + B) // B if n > 240 else 1


def model_long(d: bytes) -> int:
    n = len(d)
    T, nb = (n - 1) // 64, (n - 1) // 1024
    acc = [P32[2], P64[0], P64[1], P64[2], P64[3], P32[1], P64[4], P32[0]]
    st = 0
    iters = 0
    while True:
        iters += 1
        for u in range(B):
            x = st + u
            if x > T:
                continue
            off, soff = (64 * x, 8 * (x & 15)) if x < T else (n - 64, 121)
            for j in range(8):
                v = _r64(d, off + 8 * j)
                k = v ^ _r64(SECRET, soff + 8 * j)
                acc[j ^ 1] = (acc[j ^ 1] + v) & M64
                acc[j] = (acc[j] + (k & 0xFFFFFFFF) * (k >> 32)) & M64
        st += B
        if st % 16 == 0 and st // 16 <= nb:
            for j in range(8):
                a = acc[j] ^ (acc[j] >> 47)
                a ^= _r64(SECRET, 128 + 8 * j)
                acc[j] = (a * P32[0]) & M64
        if st > T:
            break
    assert iters == run_cost(n)
    r = (n * P64[0]) & M64
    for i in range(4):
        r = (r + _mulfold(acc[2 * i] ^ _r64(SECRET, 11 + 16 * i), acc[2 * i + 1] ^ _r64(SECRET, 19 + 16 * i))) & M64
    return _aval(r)


def model_mid(d: bytes) -> int:
    """17..240 B on 4 lanes: lane j's loads u = 0..3 and the terms it adds, summed over the quad."""
    n = len(d)
    sec = lambda o: _r64(SECRET, o)  # noqa: E731
    if n <= 128:
        lv = 4 if n > 96 else 3 if n > 64 else 2 if n > 32 else 1
        t = 0
        for j in range(4):
            if j < lv:
                a, b = 16 * j, n - 16 - 16 * j
                t += _term(_r64(d, a), _r64(d, a + 8), sec(32 * j), sec(32 * j + 8))
                t += _term(_r64(d, b), _r64(d, b + 8), sec(32 * j + 16), sec(32 * j + 24))
        return _aval(((n * P64[0]) + t) & M64)
    nmid = ((n & ~15) - 128) // 16
    t01 = t23 = 0
    for j in range(4):
        for u in range(2):
            t = 2 * j + u
            t01 += _term(_r64(d, 16 * t), _r64(d, 16 * t + 8), sec(16 * t), sec(16 * t + 8))
            if t < nmid:
                o = 128 + 16 * t
                t23 += _term(_r64(d, o), _r64(d, o + 8), sec(3 + 16 * t), sec(11 + 16 * t))
            elif t == nmid:
                t23 += _term(_r64(d, n - 16), _r64(d, n - 8), sec(119), sec(127))
    acc = _aval(((n * P64[0]) + t01) & M64)
    return _aval((acc + t23) & M64)


def runs(lens, groups: int = 16):
    """The kernel's split of a window into contiguous runs: group g takes the strings whose cost
    starts in [ceil(g * total / 16), ceil((g + 1) * total / 16))."""
    w = np.array([run_cost(int(x)) for x in lens], np.int64)
    pref = np.concatenate([[0], np.cumsum(w)[:-1]])
    total = int(w.sum())
    starts = [int(np.searchsorted(pref, -(-g * total // groups))) for g in range(groups)] + [len(lens)]
    return [(starts[g], starts[g + 1]) for g in range(groups)], w


def test_long_and_mid_schedules_equal_xxh3():
    rng = np.random.default_rng(0x5852)
    sizes = [17, 31, 32, 33, 64, 65, 96, 97, 128, 129, 143, 144, 239, 240, 241, 255, 256, 257, 1023, 1024,
             1025, 1087, 1088, 1089, 2048, 2049, 3000, 4096, 4097, 9000]
    sizes += [int(x) for x in rng.integers(17, 3000, 120)]
    for n in sizes:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        want = xxh3_64(d)
        got = model_long(d) if n > 240 else model_mid(d)
        assert got == want, n


def test_runs_cover_the_window_once_and_balance():
    rng = np.random.default_rng(0x52554E)
    for cnt in (1, 2, 15, 16, 17, 64, 200, 256):
        lens = rng.integers(0, 1401, cnt)
        rs, w = runs(lens)
        covered = [i for a, b in rs for i in range(a, b)]
        assert covered == list(range(cnt))  # contiguous, in order, each string once
        if cnt >= 64:
            loads = [int(w[a:b].sum()) for a, b in rs]
            assert max(loads) <= int(w.sum()) / 16 + int(w.max())  # within one string of the mean
