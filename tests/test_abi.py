"""CPU: the C-ABI library loads, exports every symbol include/halo_rx.h declares, agrees
with the header on struct layout, refuses bad arguments, and has no CPU compute fallback.
Also the pure-host pieces of the ABI: halo_rx_dispatch and halo_synth_layout."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "halo_rx.h")


def _declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"HALO_API\s+[\w\s\*]+?\b(halo_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from halo_amd import _lib

    syms = _declared_symbols()
    assert len(syms) >= 12
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:
        assert hasattr(_lib.lib, s)


def test_result_struct_layout_matches_header(tmp_path):
    from halo_amd._lib import RESULT_DTYPE, NetIf

    src = tmp_path / "layout.c"
    fields = list(RESULT_DTYPE.names)
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "halo_rx.h"\nint main(void){\n'
        + "".join(f'printf("%zu\\n", offsetof(halo_rx_result_t, {f}));\n' for f in fields)
        + 'printf("%zu\\n%zu\\n%zu\\n", sizeof(halo_rx_result_t), sizeof(halo_rx_netif_t), '
          'offsetof(halo_rx_netif_t, ip));\nreturn 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[:len(fields)] == [RESULT_DTYPE.fields[f][1] for f in fields]
    assert vals[len(fields)] == RESULT_DTYPE.itemsize == 32
    assert vals[len(fields) + 1] == ctypes.sizeof(NetIf)
    assert vals[len(fields) + 2] == NetIf.ip.offset


def test_status_and_error_names():
    from halo_amd import _lib

    for code, name in enumerate(_lib.STATUS_NAMES):
        assert _lib.lib.halo_rx_status_name(code).decode() == name
    assert _lib.lib.halo_rx_status_name(99).decode() == "UNKNOWN"
    assert _lib.strerror(_lib.HALO_E_ARCH) == "device is not gfx950"
    assert b"gfx950" in _lib.lib.halo_rx_version()


def test_argument_validation_without_gpu():
    from halo_amd import _lib

    L, n = _lib.lib, _lib.NetIf.make()
    buf = np.zeros(64, np.uint8)
    out = np.zeros(64, np.uint8)
    # empty batch is a no-op success; a null netif / output is always INVAL
    assert L.halo_rx_parse_batch_device(None, None, None, 0, 1, n, 0, out.ctypes.data, None, None) == 0
    assert L.halo_rx_parse_batch_device(None, None, None, 0, 1, None, 0, out.ctypes.data, None, None) == -1
    assert L.halo_rx_parse_batch_device(None, None, None, 1, 1, n, 0, out.ctypes.data, None, None) == -1
    assert L.halo_rx_parse_batch_device(buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 1, 0x20, n, 0,
                                        out.ctypes.data, None, None) == -1  # unknown flag bit
    assert L.halo_rx_parse_batch_device(buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 1, 1, n, 0,
                                        out.ctypes.data + 4, None, None) == -1  # misaligned output
    assert L.halo_rx_parse_strided_device(buf.ctypes.data, 6, None, 60, 2, 1, n, out.ctypes.data, None,
                                          None) == -1  # stride not a multiple of 4
    for v in (7,):  # HALO_RX_VARIANT_* codes end at STREAM = 6
        assert L.halo_rx_parse_batch_device(buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 1,
                                            1 | (v << _lib.HALO_RX_VARIANT_SHIFT), n, 0, out.ctypes.data, None,
                                            None) == -1
    assert not hasattr(_lib.lib, "halo_rx_tune_variant")  # no process-wide override: per call only
    assert L.halo_rx_parse_strided_device(buf.ctypes.data, 60, None, 64, 2, 1, n, out.ctypes.data, None,
                                          None) == -1  # overlapping uniform frames


def test_no_cpu_fallback_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from halo_amd import _lib

    L, n = _lib.lib, _lib.NetIf.make()
    buf = np.zeros(128, np.uint8)
    out = np.zeros(64, np.uint8)
    offs = np.zeros(1, np.uint32)
    lens = np.full(1, 64, np.uint16)
    assert L.halo_rx_init(0) == _lib.HALO_E_NODEV
    rc = L.halo_rx_parse_batch_device(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1, 1, n, 0,
                                      out.ctypes.data, None, None)
    assert rc == _lib.HALO_E_NODEV


def test_dispatch_matches_oracle_engine(golden, oracle_lib):
    """halo_rx_dispatch (records -> engine action) == the oracle's independent re-derivation."""
    from halo_amd import engine
    from halo_amd._lib import NetIf
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, names = golden_arrays(meta, blob)
    for nat in (False, True):
        on = oracle_lib.NetIf.make(nat_enable=nat)
        hn = NetIf.make(nat_enable=nat)
        for fl in (0, 1, 2, 3):
            recs, _ = oracle_lib.rx_batch(data, lens, on, fl, offsets_dw=offs)
            got = engine.dispatch(recs, hn)
            want = oracle_lib.engine_batch(data, lens, on, fl, offsets_dw=offs)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, [(names[i], got[i], want[i]) for i in bad[:5]]


@pytest.mark.parametrize("size_mode,proto_mode", [(0, 0), (0, 1), (0, 2), (1, 3)])
def test_synth_layout_matches_oracle_twin(oracle_lib, size_mode, proto_mode):
    from halo_amd import synth

    lay = synth.layout(3000, length=128, size_mode=size_mode, proto_mode=proto_mode, mutate_shift=4,
                       first_index=777)
    offs = lay["offsets_dw"].astype(np.int64) * 4
    assert offs[0] == 0 and np.all(np.diff(offs) == ((lay["lens"][:-1].astype(np.int64) + 3) & ~3))
    assert lay["total_bytes"] == offs[-1] + ((int(lay["lens"][-1]) + 3) & ~3)
    for k in range(0, 3000, 37):
        L, kind = oracle_lib.synth_kind(synth.SEED, 777 + k, size_mode, 128, proto_mode, 4)
        assert (L, kind) == (int(lay["lens"][k]), int(lay["kinds"][k]))
    if size_mode == 1:
        big = synth.layout(120000, size_mode=1, proto_mode=3)
        frac = np.bincount(np.searchsorted([64, 570, 1500], big["lens"]), minlength=3) / 120000
        assert np.allclose(frac, [7 / 12, 4 / 12, 1 / 12], atol=0.01)
        pf = np.bincount(big["kinds"] & 3, minlength=3) / 120000
        assert np.allclose(pf, [0.5, 0.4, 0.1], atol=0.01)


def test_synth_twin_frames_verify(oracle_lib):
    """Frames of the generator spec (host twin) verify clean, and every mutated frame fails."""
    from halo_amd import synth

    n = oracle_lib.NetIf.make()
    lay = synth.layout(600, size_mode=1, proto_mode=3, mutate_shift=2)
    data = oracle_lib.synth_batch(synth.SEED, 0, lay["lens"], lay["kinds"], n, offsets_dw=lay["offsets_dw"])
    recs, _ = oracle_lib.rx_batch(data, lay["lens"], n, 1, offsets_dw=lay["offsets_dw"])
    mutated = (lay["kinds"] & 0x80) != 0
    assert mutated.sum() > 50
    assert np.all(recs["status"][~mutated] == 0)
    assert np.all(recs["status"][mutated] != 0)


def test_dispatch_compact_matches_full(golden, oracle_lib):
    """halo_rx_dispatch_compact on the compact form of each record == halo_rx_dispatch."""
    from halo_amd import _lib
    from halo_amd._lib import NetIf, compact_of
    from tests.helpers import golden_arrays

    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    for nat in (False, True):
        hn = NetIf.make(nat_enable=nat)
        for fl in (0, 1, 2, 3):
            recs, _ = oracle_lib.rx_batch(data, lens, oracle_lib.NetIf.make(nat_enable=nat), fl, offsets_dw=offs)
            full = np.empty(len(recs), np.uint8)
            comp = np.empty(len(recs), np.uint8)
            c16 = compact_of(recs)
            assert _lib.lib.halo_rx_dispatch(recs.ctypes.data, len(recs), hn, full.ctypes.data, None) == 0
            assert _lib.lib.halo_rx_dispatch_compact(c16.ctypes.data, len(recs), hn, comp.ctypes.data, None) == 0
            assert np.array_equal(full, comp)


def test_tx_op_struct_layout_and_validation(tmp_path):
    """halo_tx_op_t matches TX_OP_DTYPE; halo_tx_fixup_batch_device validates before touching
    a device and has no CPU fallback."""
    import torch

    from halo_amd import _lib
    from halo_amd._lib import TX_OP_DTYPE

    src = tmp_path / "txl.c"
    fields = [f for f in TX_OP_DTYPE.names]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "halo_rx.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(halo_tx_op_t, {f}));\n' for f in fields)
                   + 'printf("%zu\\n", sizeof(halo_tx_op_t));\nreturn 0;}\n')
    exe = tmp_path / "txl"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals == [TX_OP_DTYPE.fields[f][1] for f in fields] + [16]
    L = _lib.lib
    buf = np.zeros(128, np.uint8)
    ops = np.zeros(1, TX_OP_DTYPE)
    offs = np.zeros(1, np.uint32)
    lens = np.full(1, 64, np.uint16)
    assert L.halo_tx_fixup_batch_device(None, None, None, 0, None, 1, 0, None, None) == 0
    assert L.halo_tx_fixup_batch_device(buf.ctypes.data, None, None, 1, ops.ctypes.data, 1, 0, None, None) == -1
    assert L.halo_tx_fixup_batch_device(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1, ops.ctypes.data,
                                        0x4, 0, None, None) == -1  # only CSUM_ENABLE is defined here
    if not torch.cuda.is_available():
        rc = L.halo_tx_fixup_batch_device(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1,
                                          ops.ctypes.data, 1, 0, None, None)
        assert rc == _lib.HALO_E_NODEV


def test_host_registration_rules_before_any_hip_call():
    """halo_rx_host_register / ring attach with HALO_RING_REGISTER refuse, before any HIP call, a
    base that is not page-aligned, a size that is not whole pages, and unregistering anything that
    is not the base of a live registration (registrations pin whole pages)."""
    import mmap

    import torch

    from halo_amd import _lib

    L, P = _lib.lib, mmap.PAGESIZE
    a = _lib.host_array(4 * P)
    base = a.ctypes.data
    assert base % P == 0
    assert L.halo_rx_host_register(None, P) == _lib.HALO_E_INVAL
    assert L.halo_rx_host_register(base, 0) == _lib.HALO_E_INVAL
    assert L.halo_rx_host_register(base + 64, P) == _lib.HALO_E_INVAL      # base inside a page
    assert L.halo_rx_host_register(base, P + 100) == _lib.HALO_E_INVAL     # a partial last page
    assert L.halo_rx_host_unregister(None) == _lib.HALO_E_INVAL
    assert L.halo_rx_host_unregister(base) == _lib.HALO_E_INVAL           # never registered
    assert _lib.registered_count() == 0 and _lib.registrations() == []
    # a ring that does not start on a page boundary cannot be attached with RING_REGISTER
    mem = a[64:64 + 128 + 4096]
    assert L.halo_ring_create(mem.ctypes.data, mem.nbytes) == 0
    h = ctypes.c_void_p()
    rc = L.halo_rx_ring_attach(0, mem.ctypes.data, 0, 1514, 0, 0, _lib.RING_REGISTER, ctypes.byref(h))
    assert rc == _lib.HALO_E_INVAL and not h.value
    if not torch.cuda.is_available():
        assert L.halo_rx_host_register(base, 2 * P) == _lib.HALO_E_NODEV   # valid range, no device
        assert _lib.registered_count() == 0


def test_tx_build_desc_layout_and_validation(tmp_path):
    """halo_tx_build_desc_t matches BUILD_DESC_DTYPE (and the oracle's copy); the build entry
    point validates before touching a device and has no CPU fallback."""
    import torch

    from halo_amd import _lib
    from halo_amd._lib import BUILD_DESC_DTYPE
    from oracle import oracle as O

    assert O.BUILD_DESC_DTYPE == BUILD_DESC_DTYPE
    fields = [f for f in BUILD_DESC_DTYPE.names if f != "dst_mac"] + ["dst_mac"]
    src = tmp_path / "bdl.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "halo_rx.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(halo_tx_build_desc_t, {f}));\n' for f in fields)
                   + 'printf("%zu\\n", sizeof(halo_tx_build_desc_t));\nreturn 0;}\n')
    exe = tmp_path / "bdl"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals == [BUILD_DESC_DTYPE.fields[f][1] for f in fields] + [40]
    L, n = _lib.lib, _lib.NetIf.make()
    d = np.zeros(4, BUILD_DESC_DTYPE)
    buf = np.zeros(4096, np.uint8)
    ws = np.zeros(64, np.uint64)
    ip = np.zeros(4, np.uint16)
    lens = np.zeros(4, np.uint16)
    wsb = int(L.halo_tx_build_workspace(4))
    assert wsb == 8 and int(L.halo_tx_build_workspace(513)) == 40  # u32: rejections, then one per 64-descriptor tile
    args = lambda stride=64, flags=1, wsbytes=wsb: (d.ctypes.data, 4, buf.ctypes.data, flags, n, 0, buf.ctypes.data,  # noqa: E731
                                                  stride, lens.ctypes.data, None, ip.ctypes.data, ws.ctypes.data,
                                                  wsbytes, None)
    assert L.halo_tx_build_batch_device(None, 0, None, 1, n, 0, None, 64, None, None, None, None, 0, None) == 0
    assert L.halo_tx_build_batch_device(*args(stride=62)) == -1  # not a multiple of 4
    assert L.halo_tx_build_batch_device(*args(stride=56)) == -1  # below the 60 B minimum frame
    assert L.halo_tx_build_batch_device(*args(flags=2)) == -1    # only CSUM_ENABLE applies
    assert L.halo_tx_build_batch_device(*args(wsbytes=4)) == -1  # workspace too small
    if not torch.cuda.is_available():
        assert L.halo_tx_build_batch_device(*args()) == _lib.HALO_E_NODEV


def test_round4_structs_and_validation(tmp_path):
    """halo_rx_host_stats_t / halo_rx_batch_desc_t agree with the Python mirrors; the round-4 entry
    points refuse bad arguments before touching a device."""
    import ctypes

    from halo_amd import _lib

    src = tmp_path / "l4.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "halo_rx.h"\nint main(void){\n'
        + "".join(f'printf("%zu\\n", offsetof(halo_rx_host_stats_t, {f}));\n' for f in _lib.HOST_STATS_DTYPE.names)
        + 'printf("%zu\\n%zu\\n%zu\\n%zu\\n", sizeof(halo_rx_host_stats_t), sizeof(halo_rx_batch_desc_t), '
          'offsetof(halo_rx_batch_desc_t, d_out), offsetof(halo_rx_batch_desc_t, n));\nreturn 0;}\n')
    exe = tmp_path / "l4"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    names = _lib.HOST_STATS_DTYPE.names
    assert vals[:len(names)] == [_lib.HOST_STATS_DTYPE.fields[f][1] for f in names]
    assert vals[len(names)] == _lib.HOST_STATS_DTYPE.itemsize
    assert vals[len(names) + 1:] == [ctypes.sizeof(_lib.BatchDesc), _lib.BatchDesc.d_out.offset, _lib.BatchDesc.n.offset]
    L, n = _lib.lib, _lib.NetIf.make()
    assert L.halo_rx_host_ctx_set_resident(None, 64, 0) == _lib.HALO_E_INVAL
    assert L.halo_rx_host_ctx_set_service_timeout(None, 1) == _lib.HALO_E_INVAL
    assert L.halo_rx_host_ctx_get_stats(None, None) == _lib.HALO_E_INVAL
    assert L.halo_rx_ring_set_service_timeout(None, 1) == _lib.HALO_E_INVAL
    descs = (_lib.BatchDesc * 33)()
    assert L.halo_rx_parse_batches_device(None, 1, 1, n, 64, None, None) == _lib.HALO_E_INVAL
    assert L.halo_rx_parse_batches_device(ctypes.cast(descs, ctypes.c_void_p), 0, 1, n, 64, None, None) == _lib.HALO_E_INVAL
    assert L.halo_rx_parse_batches_device(ctypes.cast(descs, ctypes.c_void_p), 33, 1, n, 64, None, None) == _lib.HALO_E_INVAL
    # all batches empty: nothing to do
    assert L.halo_rx_parse_batches_device(ctypes.cast(descs, ctypes.c_void_p), 32, 1, n, 64, None, None) == 0
    buf = np.zeros(64, np.uint8)
    descs[0] = _lib.BatchDesc(buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data + 4, 1, 0)
    assert L.halo_rx_parse_batches_device(ctypes.cast(descs, ctypes.c_void_p), 1, 1, n, 64, None,
                                          None) == _lib.HALO_E_INVAL  # misaligned records
    assert L.halo_flow_hash_compact_device(None, 0, 2, 0, None, 0, None, None) == _lib.HALO_E_INVAL
