"""halo_amd — MI355X-native receive parse-and-checksum engine for halo's rx path.

The hot path (protocol.Parse* + GetCheckSum driven by engine.RxEthernet/RxIpv4) runs as
hand-written HIP kernels for gfx950 behind the C ABI in include/halo_rx.h; this package is
the thin Python host side over that ABI (ctypes). See DESIGN.md.
"""
from . import _lib  # noqa: F401  (raises if libhalo_rx.so is not built: no CPU fallback)
from ._lib import ACTION, ACTION_NAMES, RESULT_DTYPE, STATUS, STATUS_NAMES, NetIf, HaloError  # noqa: F401

__all__ = ["ACTION", "ACTION_NAMES", "RESULT_DTYPE", "STATUS", "STATUS_NAMES", "NetIf", "HaloError"]
