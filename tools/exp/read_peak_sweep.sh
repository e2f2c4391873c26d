for b in 1024 2048 4096 8192; do HALO_READ_PEAK_BLOCKS=$b timeout -k 5 120 python -c "
import torch, bench, os
from halo_amd import _lib
_lib.check('i', _lib.lib.halo_rx_init(0))
d = bench.Dist()
print(os.environ['HALO_READ_PEAK_BLOCKS'], [bench.measure_read_peak(torch.device('cuda', 0), d, gib=g) for g in (2, 8)])
" 2>&1 | tail -1 || exit 1; done
