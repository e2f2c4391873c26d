"""Batch mirror of halo's ``engine.RouteTable``.

``RouteTable.AddRoute / DeleteRoute / UpdateRoute`` (engine/ipv4_engine.go:293-348) edit the
host-side trie through the C ABI (``halo_route_update``); ``sync()`` compiles it into the
device's DIR-24-8 table; ``FindRoute`` looks up a whole device-resident batch of addresses (or the
``dst_ip`` of parsed rx records) on the GPU and returns route ids, ``ROUTE_NONE`` where the
reference returns nil and ``ROUTE_PANIC`` where its ECMP pick divides by an emptied list.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import ROUTE_DTYPE, ROUTE_NONE, ROUTE_PANIC  # noqa: F401


def ip_u(s: str) -> int:
    """protocol.ParseIpAddr + IpAddrToU (protocol/utils.go:34-44, :71-82)."""
    a = [int(x) for x in s.split(".")]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


class RouteTable:
    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _lib.check("halo_route_table_create", _lib.lib.halo_route_table_create(ctypes.byref(h)))
        self._t = h
        self.device = device

    def close(self):
        if self._t:
            _lib.lib.halo_route_table_destroy(self._t)
            self._t = None

    def __del__(self):
        self.close()

    @staticmethod
    def entry(dst_ip: int, network_mask: int, next_hop: int = 0, netif: int = 0) -> np.ndarray:
        return np.array([(dst_ip, network_mask, next_hop, netif)], ROUTE_DTYPE)

    def UpdateRoute(self, old: np.ndarray, new: np.ndarray | None) -> int | None:  # noqa: N802
        rid = ctypes.c_uint32(ROUTE_NONE)
        _lib.check("halo_route_update", _lib.lib.halo_route_update(
            self._t, _lib.ptr(old), None if new is None else _lib.ptr(new), ctypes.byref(rid)))
        return None if new is None else int(rid.value)

    def AddRoute(self, route: np.ndarray) -> int:  # noqa: N802
        return self.UpdateRoute(route, route)

    def DeleteRoute(self, route: np.ndarray) -> None:  # noqa: N802
        self.UpdateRoute(route, None)

    def get(self, route_id: int) -> np.ndarray:
        out = np.zeros(1, ROUTE_DTYPE)
        _lib.check("halo_route_get", _lib.lib.halo_route_get(self._t, route_id, _lib.ptr(out)))
        return out

    def sync(self):
        _lib.check("halo_route_sync_device", _lib.lib.halo_route_sync_device(self._t, self.device))

    def FindRoute(self, ips, out=None, stream=None):  # noqa: N802
        """Route ids for a cuda uint32 (int32-viewed) address tensor (16-byte aligned)."""
        import torch

        n = int(ips.numel())
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=ips.device)
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        _lib.check("halo_route_lookup_device",
                   _lib.lib.halo_route_lookup_device(self._t, _lib.ptr(ips), n, _lib.ptr(out), s))
        return out

    def FindRouteRecords(self, records, out=None, stream=None):  # noqa: N802
        """FindRoute(ipv4DstAddr) for parsed records (cuda uint8 [n, 32])."""
        import torch

        n = int(records.shape[0])
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=records.device)
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        _lib.check("halo_route_lookup_records_device",
                   _lib.lib.halo_route_lookup_records_device(self._t, _lib.ptr(records), n, _lib.ptr(out), s))
        return out
