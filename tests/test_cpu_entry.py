"""CPU: halo_rx_parse_batch_cpu (include/halo_rx_cpu.h, libhalo_rx_cpu.so) — SURVEY.md §8b's CPU
entry point, product code independent of the oracle — against the committed golden fixtures
(Ethernet frames and LoChan packets, flags 0-3), against the C oracle on the structured fuzz
corpus and on synthetic IMIX / jumbo batches at unaligned offsets, its argument checks, its read
contract (no byte outside a frame, none of a frame failing the length check) and its separation
from libhalo_rx.so (not a fallback: the GPU library neither exports nor links it)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

import numpy as np
import pytest

from tests.helpers import assert_records_equal, expected_records, golden_arrays, lo_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "halo_rx_cpu.h")
L3 = 0x10


@pytest.fixture(scope="module")
def cpu():
    from halo_amd import cpu

    return cpu


def _byte_offsets(offs_dw):
    return offs_dw.astype(np.uint64) * 4


def test_exports_and_separation(cpu):
    from halo_amd import _lib

    declared = sorted(set(re.findall(r"HALO_API\s+[\w\s\*]+?\b(halo_\w+)\s*\(", open(HEADER).read())))
    assert declared == ["halo_rx_cpu_version", "halo_rx_parse_batch_cpu"]
    nm = lambda p: {ln.split()[-1] for ln in subprocess.run(  # noqa: E731
        ["nm", "-D", "--defined-only", p], capture_output=True, text=True, check=True).stdout.splitlines() if " T " in ln}
    assert set(declared) <= nm(cpu.CPU_LIB_PATH)
    assert not set(declared) & nm(_lib.LIB_PATH)  # the GPU library has no CPU entry point
    needed = subprocess.run(["readelf", "-d", cpu.CPU_LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "amdhip" not in needed and "halo_rx.so" not in needed
    assert b"no HIP" in cpu.lib.halo_rx_cpu_version()


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_golden_frames(cpu, golden, flags):
    from halo_amd._lib import RESULT_DTYPE, NetIf

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    hist = np.zeros(14, np.uint32)
    got = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                               jumbo=bool(flags & 2), hist=hist)
    want = expected_records(meta, flags, RESULT_DTYPE)
    assert_records_equal(got, want, names, f"cpu entry flags={flags}")
    assert np.array_equal(hist, np.bincount(want["status"], minlength=14))


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_golden_lochan_packets(cpu, flags):
    from halo_amd._lib import RESULT_DTYPE, NetIf

    meta, blob = lo_golden(ROOT)
    data, offs, lens, names = golden_arrays(meta, blob, key="packets")
    got = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                               jumbo=bool(flags & 2), l3_start=True)
    assert_records_equal(got, expected_records(meta, flags, RESULT_DTYPE, key="packets"), names,
                         f"cpu entry L3 flags={flags}")


def _unaligned(data, offs_dw, lens, seed):
    """The same frames repacked at offsets of every residue mod 8 (the CPU entry takes any alignment)."""
    rng = np.random.default_rng(seed)
    lead = rng.integers(0, 8, len(lens))
    sizes = lens.astype(np.int64) + lead
    start = np.zeros(len(lens), np.int64)
    start[1:] = np.cumsum(sizes)[:-1]
    out = np.zeros(int(sizes.sum()) + 8, np.uint8)
    src = offs_dw.astype(np.int64) * 4
    for i in range(len(lens)):
        b = start[i] + lead[i]
        out[b:b + lens[i]] = data[src[i]:src[i] + lens[i]]
    return out, (start + lead).astype(np.uint64)


@pytest.fixture(scope="module")
def fuzz(oracle_lib):
    ni = oracle_lib.NetIf.make()
    return oracle_lib.fuzz_batch(0xF022, 60_000, ni)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_fuzz_corpus_matches_oracle(cpu, oracle_lib, fuzz, flags):
    from halo_amd._lib import NetIf

    data, offs, lens = fuzz
    want, whist = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), flags, offsets_dw=offs, threads=4)
    hist = np.zeros(14, np.uint32)
    got = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                               jumbo=bool(flags & 2), hist=hist)
    assert_records_equal(got, want, None, f"fuzz flags={flags}")
    assert np.array_equal(hist, whist)
    udata, uoffs = _unaligned(data, offs, lens, flags)
    got2 = cpu.parse_frames_cpu(udata, uoffs, lens, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                                jumbo=bool(flags & 2))
    assert_records_equal(got2, want, None, f"fuzz unaligned flags={flags}")


@pytest.mark.parametrize("flags", [0, 1, 3])
def test_fuzz_corpus_compact_records(cpu, oracle_lib, fuzz, flags):
    """HALO_RX_RECORD_COMPACT: each 16-byte record is the packing (compact_of) of the full record,
    for Ethernet frames and LoChan packets; the histogram is unchanged."""
    from halo_amd._lib import NetIf, compact_of
    from tests.helpers import strip_ethernet

    for l3, (data, offs, lens) in ((False, fuzz), (True, strip_ethernet(*fuzz))):
        kw = dict(netif=NetIf.make(), check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2), l3_start=l3)
        full = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, **kw)
        h16 = np.zeros(14, np.uint32)
        c16 = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, compact=True, hist=h16, **kw)
        assert c16.tobytes() == compact_of(full).tobytes(), (l3, flags)
        assert np.array_equal(h16, np.bincount(full["status"], minlength=14))


@pytest.mark.parametrize("flags", [1, 3])
def test_fuzz_corpus_as_lochan_packets_matches_oracle(cpu, oracle_lib, fuzz, flags):
    from halo_amd._lib import NetIf
    from tests.helpers import strip_ethernet

    data, offs, lens = strip_ethernet(*fuzz)
    want, _ = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(), flags | L3, offsets_dw=offs, threads=4)
    got = cpu.parse_frames_cpu(data, _byte_offsets(offs), lens, netif=NetIf.make(), check_sum_enable=bool(flags & 1),
                               jumbo=bool(flags & 2), l3_start=True)
    assert_records_equal(got, want, None, f"fuzz L3 flags={flags}")


@pytest.mark.parametrize("size_mode,length,jumbo", [(1, 64, False), (0, 1514, False), (0, 9014, True)])
def test_synthetic_batches_match_oracle(cpu, oracle_lib, size_mode, length, jumbo):
    """IMIX / 1514 B / 9014 B TCP-UDP-ICMP batches with one frame in 16 mutated, at unaligned offsets."""
    from halo_amd import synth
    from halo_amd._lib import NetIf

    n = 6000 if length < 9000 else 800
    lay = synth.layout(n, length=length, size_mode=size_mode, proto_mode=3, mutate_shift=4, first_index=4321)
    on = oracle_lib.NetIf.make()
    data = oracle_lib.synth_batch(synth.SEED, 4321, lay["lens"], lay["kinds"], on, offsets_dw=lay["offsets_dw"])
    fl = 1 | (2 if jumbo else 0)
    want, _ = oracle_lib.rx_batch(data, lay["lens"], on, fl, offsets_dw=lay["offsets_dw"])
    assert np.count_nonzero(want["status"]) > n // 40 and np.count_nonzero(want["status"] == 0) > n // 2
    udata, uoffs = _unaligned(data, lay["offsets_dw"], lay["lens"], length)
    got = cpu.parse_frames_cpu(udata, uoffs, lay["lens"], netif=NetIf.make(), jumbo=jumbo)
    assert_records_equal(got, want, None, f"synthetic {length} B")


def test_empty_frames_and_empty_buffer(cpu):
    """A batch whose frames are all empty (no data bytes at all) parses: ETH_LEN, or IP_LEN as LoChan
    packets, and no byte is read."""
    from halo_amd._lib import NetIf

    for l3, want in ((False, 1), (True, 3)):
        got = cpu.parse_frames_cpu(np.zeros(0, np.uint8), np.zeros(3, np.uint64), np.zeros(3, np.uint16),
                                   netif=NetIf.make(), l3_start=l3)
        assert list(got["status"]) == [want] * 3


def test_argument_checks(cpu):
    from halo_amd import _lib

    L, ni = cpu.lib, _lib.NetIf.make()
    buf = np.zeros(64, np.uint8)
    offs = np.zeros(1, np.uint64)
    lens = np.full(1, 64, np.uint16)
    out = np.zeros(1, _lib.RESULT_DTYPE)
    a = (buf.ctypes.data, offs.ctypes.data, lens.ctypes.data)
    assert L.halo_rx_parse_batch_cpu(None, None, None, 0, 1, ni, None, None) == _lib.HALO_OK
    assert L.halo_rx_parse_batch_cpu(*a, 1, 1, None, out.ctypes.data, None) == _lib.HALO_E_INVAL
    assert L.halo_rx_parse_batch_cpu(None, offs.ctypes.data, lens.ctypes.data, 1, 1, ni, out.ctypes.data,
                                     None) == _lib.HALO_E_INVAL
    assert L.halo_rx_parse_batch_cpu(*a, 1, 1, ni, None, None) == _lib.HALO_E_INVAL
    assert L.halo_rx_parse_batch_cpu(*a, 1, 1 | 0x20, ni, out.ctypes.data, None) == _lib.HALO_E_INVAL
    # kernel-choice bits are accepted and change nothing
    assert L.halo_rx_parse_batch_cpu(*a, 1, 1 | _lib.HALO_RX_UNIFORM_LEN | _lib.variant_flags(16), ni,
                                     out.ctypes.data, None) == _lib.HALO_OK
    assert out["status"][0] == 2  # all-zero frame: EtherType 0 is not whitelisted


_READ_CONTRACT = r"""
import ctypes, mmap, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from halo_amd import cpu
from halo_amd._lib import NetIf, RESULT_DTYPE
from oracle import oracle as O
P = mmap.PAGESIZE
libc = ctypes.CDLL(None)
libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
mm = mmap.mmap(-1, 3 * P)
base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
arr = np.frombuffer(mm, dtype=np.uint8)
ni = NetIf.make()
# a valid 61 B UDP frame (odd length: the checksum tail) ending exactly where page 1 ends
f = O.synth_frame(7, 7, 61, 1, O.NetIf.make())
end = 2 * P
arr[end - 61:end] = np.frombuffer(f, np.uint8)
assert libc.mprotect(base + 2 * P, P, 0) == 0   # page 2: no access
assert libc.mprotect(base, P, 0) == 0           # page 0: no access
offs = np.array([end - 61, 2 * P + 16, P - 30, end - 61], np.uint64)
lens = np.array([61, 30, 20, 0], np.uint16)    # frames 1-2: below 42 B, inside no-access pages
out = np.zeros(4, RESULT_DTYPE)
hist = np.zeros(14, np.uint32)
rc = cpu.lib.halo_rx_parse_batch_cpu(base, offs.ctypes.data, lens.ctypes.data, 4, 1, ni, out.ctypes.data,
                                     hist.ctypes.data)
assert rc == 0, rc
want = O.rx_frame(f, O.NetIf.make(), 1)
assert out[0].tobytes() == want.tobytes(), (out[0], want)
assert list(out["status"]) == [want["status"], 1, 1, 1], out["status"]
assert want["status"] == 0 and want["payload_len"] > 0
# the same packet's IPv4 part as a LoChan packet ending at the page end; a 10 B packet in page 2
pk = f[14:]
arr[end - len(pk):end] = np.frombuffer(pk, np.uint8)
offs = np.array([end - len(pk), 2 * P + 8], np.uint64)
lens = np.array([len(pk), 10], np.uint16)
rc = cpu.lib.halo_rx_parse_batch_cpu(base, offs.ctypes.data, lens.ctypes.data, 2, 1 | 0x10, ni, out.ctypes.data, None)
assert rc == 0 and out["status"][1] == 3, (rc, out["status"][:2])
print("ok")
"""


def test_read_contract_guard_pages(cpu, oracle_lib):
    """Frames ending at a page followed by a no-access page parse without touching it, and frames
    failing ParseEthFrm's (ParseIpv4Pkt's, for LoChan packets) length check are never read — they may
    point into a no-access page. In a child process: a violation is a segmentation fault there."""
    r = subprocess.run([sys.executable, "-c", _READ_CONTRACT, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
