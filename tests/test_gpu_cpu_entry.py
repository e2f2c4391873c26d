"""GPU: the CPU entry point (halo_rx_parse_batch_cpu, libhalo_rx_cpu.so) and the device entry point
(halo_rx_parse_batch_device, libhalo_rx.so) give the same records, byte for byte, on the same
frames: the structured fuzz corpus under every flags word (Ethernet frames and, stripped, LoChan
packets) and the bench's config-2 / IMIX / jumbo batches generated on the device. A caller that
routes small polls to the CPU and large ones to the GPU sees one record
format and one set of verdicts."""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import assert_records_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _gpu(dev, data, offs_dw, lens, flags, compact=False):
    import torch

    from halo_amd import _lib
    from halo_amd._lib import RESULT_DTYPE, NetIf

    n = len(lens)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs_dw.view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = torch.full((n, 16 if compact else 32), 0xEE, dtype=torch.uint8, device=dev)
    _lib.check("halo_rx_parse_batch_device", _lib.lib.halo_rx_parse_batch_device(
        d.data_ptr(), o.data_ptr(), ln.data_ptr(), n, flags | (_lib.HALO_RX_RECORD_COMPACT if compact else 0),
        NetIf.make(), 0, out.data_ptr(), None, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(_lib.RECORD16_DTYPE if compact else RESULT_DTYPE).reshape(n)


def _cpu(data, offs_dw, lens, flags, compact=False):
    from halo_amd import cpu
    from halo_amd._lib import NetIf

    return cpu.parse_frames_cpu(data, offs_dw.astype(np.uint64) * 4, lens, netif=NetIf.make(),
                                check_sum_enable=bool(flags & 1), jumbo=bool(flags & 2), l3_start=bool(flags & 0x10),
                                compact=compact)


@pytest.fixture(scope="module")
def fuzz(oracle_lib):
    return oracle_lib.fuzz_batch(0xC0E, 1 << 17, oracle_lib.NetIf.make())


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_fuzz_cpu_entry_equals_gpu(dev, fuzz, flags):
    data, offs, lens = fuzz
    assert_records_equal(_cpu(data, offs, lens, flags), _gpu(dev, data, offs, lens, flags), None,
                         f"fuzz flags={flags}")


@pytest.mark.parametrize("flags", [0, 1, 3])
def test_fuzz_compact_cpu_entry_equals_gpu(dev, fuzz, flags):
    """HALO_RX_RECORD_COMPACT on both sides: the 16-byte records match byte for byte."""
    data, offs, lens = fuzz
    got, want = _cpu(data, offs, lens, flags, compact=True), _gpu(dev, data, offs, lens, flags, compact=True)
    assert got.tobytes() == want.tobytes(), np.nonzero(got != want)[0][:8]


@pytest.mark.parametrize("flags", [1, 3])
def test_fuzz_lochan_cpu_entry_equals_gpu(dev, fuzz, flags):
    from tests.helpers import strip_ethernet

    data, offs, lens = strip_ethernet(*fuzz)
    assert_records_equal(_cpu(data, offs, lens, flags | 0x10), _gpu(dev, data, offs, lens, flags | 0x10), None,
                         f"fuzz L3 flags={flags}")


@pytest.mark.parametrize("n,length,size_mode,jumbo", [(1 << 20, 64, 0, False), (1 << 17, 64, 1, False),
                                                     (4096, 9014, 0, True)])
def test_bench_batches_cpu_entry_equals_gpu(dev, n, length, size_mode, jumbo):
    from halo_amd import synth
    from halo_amd._lib import NetIf

    lay = synth.layout(n, length=length, size_mode=size_mode, proto_mode=3 if size_mode else 0, mutate_shift=5)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    data = fr["bytes"].cpu().numpy()
    flags = 1 | (2 if jumbo else 0)
    got = _cpu(data, lay["offsets_dw"], lay["lens"], flags)
    want = _gpu(dev, data, lay["offsets_dw"], lay["lens"], flags)
    assert np.count_nonzero(want["status"]) > 0
    assert_records_equal(got, want, None, f"{n} x {length} B")
