"""ctypes binding of libhalo_rx.so — the C ABI declared in include/halo_rx.h.

The shared library is built in-tree (``__graft_entry__.build()`` or
``python -m halo_amd.build``) and loaded from ``halo_amd/lib/``. There is no CPU
fallback: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# HALO_RX_LIB overrides the library path (A/B experiments with alternative builds only)
LIB_PATH = os.environ.get("HALO_RX_LIB") or os.path.join(LIB_DIR, "libhalo_rx.so")

# ---- constants mirrored from include/halo_rx.h ---------------------------------------
HALO_OK = 0
HALO_E_INVAL = -1
HALO_E_NODEV = -2
HALO_E_ARCH = -3
HALO_E_HIP = -4
HALO_E_NOMEM = -5
HALO_E_RANGE = -6

HALO_RX_CSUM_ENABLE = 0x1
HALO_RX_JUMBO_EXT = 0x2
HALO_RX_RECORD_COMPACT = 0x4
HALO_RX_UNIFORM_LEN = 0x8
HALO_RX_L3_START = 0x10  # LoChan packets: every buffer starts at its IPv4 header
HALO_RX_VARIANT_SHIFT = 8
# lanes per frame -> HALO_RX_VARIANT_* (0 = automatic, -1 = the size-class mix kernel,
# -2 = the byte-stream kernel)
_VARIANT_CODE = {0: 0, 1: 1, 4: 2, 8: 3, 16: 4, -1: 5, -2: 6}


def variant_flags(lanes_per_frame: int) -> int:
    """The flags bits that force a kernel variant for one call (HALO_RX_VARIANT_*)."""
    return _VARIANT_CODE[lanes_per_frame] << HALO_RX_VARIANT_SHIFT

STATUS_NAMES = (
    "OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
    "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM",
)
STATUS = {name: code for code, name in enumerate(STATUS_NAMES)}
HALO_RX_STATUS_COUNT = len(STATUS_NAMES)

F_MAC_MATCH = 0x01
F_IP_BCAST = 0x02
F_DST_IS_OWN = 0x04

ACTION_NAMES = (
    "DROP_ETH", "IGNORE_MAC", "ARP", "IGNORE_TYPE", "DROP_IP", "BCAST_UDP", "DROP_BCAST_UDP",
    "IGNORE_BCAST", "FORWARD", "LOCAL_ICMP", "LOCAL_UDP", "LOCAL_TCP", "DROP_L4", "LO_NOT_OWN",
)
ACTION = {name: code for code, name in enumerate(ACTION_NAMES)}
HALO_RX_ACT_COUNT = len(ACTION_NAMES)

# halo_rx_result_t (32 bytes, little-endian)
RESULT_DTYPE = np.dtype([
    ("status", "u1"), ("flags", "u1"), ("ethertype", "<u2"),
    ("ip_proto", "u1"), ("l4_aux", "u1"), ("ip_total_len", "<u2"),
    ("src_ip", "<u4"), ("dst_ip", "<u4"),
    ("sport", "<u2"), ("dport", "<u2"),
    ("payload_off", "<u2"), ("payload_len", "<u2"),
    ("l4_seq", "<u4"), ("l4_ack", "<u4"),
])
assert RESULT_DTYPE.itemsize == 32

# halo_rx_record16_t (16 bytes): flags bits 4-5 hold the EtherType class
RECORD16_DTYPE = np.dtype([
    ("status", "u1"), ("flags", "u1"), ("ip_proto", "u1"), ("l4_aux", "u1"),
    ("src_ip", "<u4"), ("dst_ip", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
])
assert RECORD16_DTYPE.itemsize == 16
ET_CLASS = {0x0800: 0x00, 0x0806: 0x10, 0x86DD: 0x20, 0x05DC: 0x30}


def compact_of(full: np.ndarray) -> np.ndarray:
    """The halo_rx_record16_t a full record maps to (host-side reference of the packing)."""
    out = np.zeros(full.shape[0], dtype=RECORD16_DTYPE)
    for f in ("status", "ip_proto", "l4_aux", "src_ip", "dst_ip", "sport", "dport"):
        out[f] = full[f]
    cls = np.zeros(full.shape[0], dtype=np.uint8)
    for et, c in ET_CLASS.items():
        cls[full["ethertype"] == et] = c
    out["flags"] = full["flags"] | cls
    return out

# halo_tx_op_t (16 bytes): per-frame steps of halo_tx_fixup_batch_device
TX_OP_DTYPE = np.dtype([("steps", "u1"), ("pad", "u1"), ("dst_port", "<u2"), ("dst_ip", "<u4"),
                        ("src_port", "<u2"), ("pad2", "<u2"), ("src_ip", "<u4")])
assert TX_OP_DTYPE.itemsize == 16
TX_NAT_DST, TX_TTL, TX_NAT_SRC, TX_RECALC, TX_DPDK_FILL = 0x01, 0x02, 0x04, 0x08, 0x10
TX_R_TTL_ALIVE, TX_R_SKIPPED, TX_R_OVERRUN = 0x01, 0x02, 0x04
# halo_tx_build_desc_t (40 bytes): one locally originated packet for halo_tx_build_batch_device
BUILD_DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("payload_len", "<u2"), ("proto", "u1"), ("aux", "u1"),
                             ("src_port", "<u2"), ("dst_port", "<u2"), ("src_ip", "<u4"), ("dst_ip", "<u4"),
                             ("seq", "<u4"), ("ack", "<u4"), ("dst_mac", "u1", (6,)), ("mode", "u1"),
                             ("pad", "u1")])
assert BUILD_DESC_DTYPE.itemsize == 40
TX_BUILD_ETH, TX_BUILD_LOOPBACK = 0, 1   # HALO_TX_BUILD_*
DEEP_NAT_DTYPE = np.dtype([("lan_ip", "<u4"), ("lan_port", "<u2"), ("found", "u1"), ("pad", "u1")])  # halo_tx_deep_nat_t
TX_B_OK, TX_B_PAYLOAD_LEN, TX_B_PROTO, TX_B_SLOT = 0, 1, 2, 3
FLOW_NAT_LAN, FLOW_NAT_WAN = 0, 1        # HALO_FLOW_*
NAT_SYMMETRIC, NAT_FULL_CONE = 0, 1      # HALO_NAT_* (engine.NatTypeSymmetric / NatTypeFullCone)
ROUTE_DTYPE = np.dtype([("dst_ip", "<u4"), ("network_mask", "<u4"), ("next_hop", "<u4"), ("netif", "<u4")])
ROUTE_NONE, ROUTE_PANIC = 0xFFFFFFFF, 0xFFFFFFFE  # HALO_ROUTE_*
# halo_rx_ring_scan_t (24 bytes) and HALO_RING_STOP_* / HALO_RING_REGISTER
RING_SCAN_DTYPE = np.dtype([("n_frames", "<u4"), ("stop", "<u4"), ("end_bytes", "<u8"), ("max_len", "<u4"),
                            ("pad", "<u4")])
assert RING_SCAN_DTYPE.itemsize == 24
# halo_rx_ring_stats_t (8 x u64)
RING_STATS_DTYPE = np.dtype([(k, "<u8") for k in ("polls", "frames", "small_polls", "service_requests",
                                                  "service_launches", "walk_ns", "wait_ns", "service_gpu_ns")])
# halo_rx_host_stats_t (8 x u64)
HOST_STATS_DTYPE = np.dtype([(k, "<u8") for k in ("calls", "frames", "resident_calls", "resident_parked",
                                                  "service_launches", "pack_ns", "wait_ns", "service_gpu_ns")])
RING_STOP_NAMES = ("EMPTY", "BAD_LEN", "PARTIAL", "CAPACITY", "MAX", "BAD_CURSOR")
RING_STOP = {name: code for code, name in enumerate(RING_STOP_NAMES)}
RING_REGISTER = 0x1
RING_PERSISTENT = 0x2  # HALO_RING_PERSISTENT: small polls served by a resident consumer kernel

def host_array(shape, dtype=np.uint8) -> np.ndarray:
    """A zeroed host array on pages of its own: an anonymous mmap, page-aligned, its size rounded
    up to whole pages, unmapped when the array is freed. For every buffer handed to
    ``halo_rx_host_register`` or attached with ``RING_REGISTER``: hipHostRegister pins whole pages,
    so a heap array (np.zeros) can share its first or last page with an unrelated allocation that
    outlives the registration, and a later transfer that pins that neighbour in place then meets a
    stale mapping. Pages that only this array uses go back to the OS with it."""
    import mmap

    dt = np.dtype(dtype)
    shape = (shape,) if isinstance(shape, (int, np.integer)) else tuple(shape)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    size = max(mmap.PAGESIZE, -(-nbytes // mmap.PAGESIZE) * mmap.PAGESIZE)
    buf = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    return np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dt).reshape(shape)

def host_pages(nbytes: int) -> int:
    """The whole-page size host_array maps for `nbytes` (what a registration of it covers)."""
    import mmap

    return max(mmap.PAGESIZE, -(-int(nbytes) // mmap.PAGESIZE) * mmap.PAGESIZE)


_leaked: list = []  # host arrays whose registration could not be removed: never freed


class registered:
    """``with registered(arr):`` — halo_rx_host_register over the whole pages of a host_array for
    the block, unregistered on exit even when the block raises. If the unregistration fails the
    array is kept alive for the rest of the process (its pages may still be mapped for the
    device) and HaloError is raised."""

    def __init__(self, arr: np.ndarray):
        self.arr = arr

    def __enter__(self):
        check("halo_rx_host_register", lib.halo_rx_host_register(self.arr.ctypes.data, host_pages(self.arr.nbytes)))
        return self.arr

    def __exit__(self, *exc):
        rc = lib.halo_rx_host_unregister(self.arr.ctypes.data)
        if rc != HALO_OK:
            _leaked.append(self.arr)
            if exc[0] is None:
                check("halo_rx_host_unregister", rc)
        return False


def registered_count() -> int:
    """Live host registrations made through the library (halo_rx_host_registered_count)."""
    return int(lib.halo_rx_host_registered_count())


def registrations() -> list:
    """(base, bytes) of every live registration, in address order."""
    n = int(lib.halo_rx_host_registrations(None, None, 0))
    bases = (ctypes.c_void_p * max(n, 1))()
    sizes = (ctypes.c_uint64 * max(n, 1))()
    n = int(lib.halo_rx_host_registrations(bases, sizes, n))
    return [(int(bases[i] or 0), int(sizes[i])) for i in range(n)]


RING_HEADER = 128  # sizeof(RingBuffer), mem/ring_buffer.go:18-26


class NetIf(ctypes.Structure):
    """halo_rx_netif_t — engine.NetIfConfig's MacAddr / IpAddr / NatEnable."""

    _fields_ = [
        ("mac", ctypes.c_uint8 * 6),
        ("pad", ctypes.c_uint8 * 2),
        ("ip", ctypes.c_uint32),
        ("nat_enable", ctypes.c_uint32),
    ]

    @classmethod
    def make(cls, mac: str = "AA:AA:AA:AA:AA:AA", ip: str = "192.168.100.100", nat_enable: bool = False):
        """Parse addresses like protocol.ParseMacAddr / ParseIpAddr (protocol/utils.go:57-82)."""
        n = cls()
        for i, part in enumerate(mac.split(":")[:6]):
            n.mac[i] = int(part, 16)
        a = [int(x) for x in ip.split(".")[:4]]
        n.ip = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]  # IpAddrToU (utils.go:34-44)
        n.nat_enable = 1 if nat_enable else 0
        return n


class BatchDesc(ctypes.Structure):
    """halo_rx_batch_desc_t — one batch of halo_rx_parse_batches_device."""

    _fields_ = [("d_bytes", ctypes.c_void_p), ("d_offsets_dw", ctypes.c_void_p), ("d_lens", ctypes.c_void_p),
                ("d_out", ctypes.c_void_p), ("n", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


assert ctypes.sizeof(BatchDesc) == 40

_u8p = ctypes.c_void_p
_PROTOS = {
    "halo_rx_version": (ctypes.c_char_p, []),
    "halo_rx_init": (ctypes.c_int, [ctypes.c_int]),
    "halo_rx_debug_hist_keys": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_uint32]),
    "halo_rx_device_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "halo_rx_release": (ctypes.c_int, [ctypes.c_int]),
    "halo_rx_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "halo_rx_status_name": (ctypes.c_char_p, [ctypes.c_int]),
    "halo_rx_parse_batch_device": (ctypes.c_int, [
        _u8p, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf), ctypes.c_uint32,
        _u8p, _u8p, ctypes.c_void_p]),
    "halo_rx_parse_strided_device": (ctypes.c_int, [
        _u8p, ctypes.c_uint64, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.POINTER(NetIf), _u8p, _u8p, ctypes.c_void_p]),
    "halo_rx_parse_batches_device": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf), ctypes.c_uint32, _u8p,
        ctypes.c_void_p]),
    "halo_rx_host_ctx_create": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "halo_rx_host_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "halo_rx_host_ctx_set_zero_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "halo_rx_host_ctx_set_resident": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    "halo_rx_host_ctx_set_service_timeout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "halo_rx_host_ctx_get_stats": (ctypes.c_int, [ctypes.c_void_p, _u8p]),
    "halo_rx_parse_batch_host": (ctypes.c_int, [
        ctypes.c_void_p, _u8p, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf),
        _u8p, _u8p]),
    "halo_rx_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "halo_rx_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
    "halo_rx_host_registered_count": (ctypes.c_uint32, []),
    "halo_rx_host_registrations": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "halo_rx_dispatch": (ctypes.c_int, [_u8p, ctypes.c_uint32, ctypes.POINTER(NetIf), _u8p, _u8p]),
    "halo_rx_dispatch_compact": (ctypes.c_int, [_u8p, ctypes.c_uint32, ctypes.POINTER(NetIf), _u8p, _u8p]),
    "halo_rx_dispatch_loopback": (ctypes.c_int, [_u8p, ctypes.c_uint32, ctypes.POINTER(NetIf), _u8p, _u8p]),
    "halo_tx_icmp_deep_nat_batch_device": (ctypes.c_int, [
        _u8p, _u8p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p, _u8p, ctypes.c_void_p]),
    "halo_tx_fixup_batch_device": (ctypes.c_int, [
        _u8p, _u8p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_tx_build_workspace": (ctypes.c_uint64, [ctypes.c_uint32]),
    "halo_tx_build_batch_device": (ctypes.c_int, [
        _u8p, ctypes.c_uint32, _u8p, ctypes.c_uint32, ctypes.POINTER(NetIf), ctypes.c_uint32, _u8p, ctypes.c_uint32,
        _u8p, _u8p, _u8p, _u8p, ctypes.c_uint64, ctypes.c_void_p]),
    "halo_xxh3_64_batch_device": (ctypes.c_int, [_u8p, _u8p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_rx_parse_flow_batch_device": (ctypes.c_int, [
        _u8p, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf), ctypes.c_uint32, _u8p, _u8p,
        ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_rx_parse_route_batch_device": (ctypes.c_int, [
        _u8p, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf), ctypes.c_uint32, _u8p, _u8p,
        ctypes.c_void_p, _u8p, ctypes.c_void_p]),
    "halo_flow_hash_device": (ctypes.c_int, [
        _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_flow_hash_compact_device": (ctypes.c_int, [
        _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_route_table_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "halo_route_table_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "halo_route_update": (ctypes.c_int, [ctypes.c_void_p, _u8p, _u8p, ctypes.POINTER(ctypes.c_uint32)]),
    "halo_route_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, _u8p]),
    "halo_route_sync_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "halo_route_lookup_device": (ctypes.c_int, [ctypes.c_void_p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_route_lookup_records_device": (ctypes.c_int, [
        ctypes.c_void_p, _u8p, ctypes.c_uint32, _u8p, ctypes.c_void_p]),
    "halo_rx_shard_multi": (ctypes.c_int, [
        _u8p, ctypes.c_uint32, _u8p, _u8p, _u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(NetIf), _u8p,
        _u8p, _u8p]),
    "halo_rx_ring_attach": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "halo_rx_ring_detach": (ctypes.c_int, [ctypes.c_void_p]),
    "halo_rx_ring_poll": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(NetIf), _u8p, _u8p, _u8p, _u8p]),
    "halo_rx_ring_commit": (ctypes.c_int, [ctypes.c_void_p]),
    "halo_rx_ring_get_stats": (ctypes.c_int, [ctypes.c_void_p, _u8p]),
    "halo_rx_ring_set_small_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "halo_rx_ring_set_service_timeout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "halo_rx_ring_scan_workspace": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32]),
    "halo_rx_ring_scan_device": (ctypes.c_int, [
        _u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p, _u8p, _u8p,
        ctypes.c_uint64, ctypes.c_void_p]),
    "halo_ring_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "halo_ring_write_batch": (ctypes.c_int, [
        ctypes.c_void_p, _u8p, _u8p, _u8p, ctypes.c_uint32, _u8p, ctypes.POINTER(ctypes.c_uint32)]),
    "halo_synth_layout": (ctypes.c_int, [
        ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p, _u8p, ctypes.POINTER(ctypes.c_uint64)]),
    "halo_synth_frames_device": (ctypes.c_int, [
        ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _u8p, _u8p, ctypes.c_uint64, _u8p,
        ctypes.POINTER(NetIf), _u8p, ctypes.c_void_p]),
}


class HaloError(RuntimeError):
    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed: {code} ({strerror(code)})")
        self.code = code


def _same_hip_runtime_as_torch() -> None:
    """One HIP runtime per process. libhalo_rx.so needs libamdhip64.so.7; PyTorch-ROCm ships its own
    copy (same soname) and links it by the name libamdhip64.so. Whichever loads first decides: if
    torch comes first, our library binds to torch's copy; if we came first with /opt/rocm's, torch
    would later load its copy as a SECOND runtime, and the two fight over the device (every call
    here then fails with HALO_E_NODEV). So when torch is installed, load its runtime first (without
    importing torch). Processes without torch (a cgo host) use the system runtime."""
    import importlib.util

    if "torch" in __import__("sys").modules:
        return
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    rt = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
    _same_hip_runtime_as_torch()
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def strerror(code: int) -> str:
    return lib.halo_rx_strerror(code).decode()


def check(fn: str, code: int) -> None:
    if code != HALO_OK:
        raise HaloError(fn, code)


def device_synchronize(device: int = 0) -> None:
    """hipDeviceSynchronize for `device` after parking this library's resident consumers there
    (halo_rx_device_synchronize): use it instead of torch.cuda.synchronize() while a persistent ring
    or a resident host context is live, which a plain device sync would wait on."""
    check("halo_rx_device_synchronize", lib.halo_rx_device_synchronize(device))


def ptr(x) -> int | None:
    """Device/host address of a torch tensor or numpy array (None for None)."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data
