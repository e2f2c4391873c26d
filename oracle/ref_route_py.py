"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of engine.RouteTable (§8f row f4).

Independent of oracle/halo_route_oracle.c; written from engine/ipv4_engine.go:270-383 with Go's
byte-slice addresses (``DstIpAddr[i/8] >> (7 - i%8)``), the maskSize loop as written (a Go
uint32 shifted by 32 is 0), and Go's hash/fnv FNV-1a 32 (engine/engine.go:159). Used to generate
tests/golden/route.json and to cross-check the C restatement.
"""
from __future__ import annotations

NONE, PANIC = 0xFFFFFFFF, 0xFFFFFFFE


class _Node:
    __slots__ = ("route_list", "left", "right")

    def __init__(self):
        self.route_list = None  # nil
        self.left = None
        self.right = None


def _b4(u: int) -> bytes:
    return int(u).to_bytes(4, "big")


def fnv32a(data: bytes) -> int:
    h = 0x811C9DC5
    for b in data:
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


class RouteTable:
    def __init__(self):
        self.root = _Node()
        self.routes = []  # id -> (dst, mask, next_hop, netif) as IpAddrToU values / netif id

    def update(self, old, new=None):
        dst, mask = _b4(old[0]), int(old[1])
        node, mask_size = self.root, 0
        if mask != 0:
            for i in range(1, 33):
                mask_size += 1
                if (mask << i) & 0xFFFFFFFF == 0:
                    break
        for i in range(mask_size):
            bit = (dst[i // 8] >> (7 - i % 8)) & 1
            if bit == 0:
                if node.left is None:
                    node.left = _Node()
                node = node.left
            else:
                if node.right is None:
                    node.right = _Node()
                node = node.right
        new_list = []
        for rid in node.route_list or []:
            if tuple(self.routes[rid]) == tuple(int(x) for x in old):
                continue
            new_list.append(rid)
        rid = None
        if new is not None:
            rid = len(self.routes)
            self.routes.append(tuple(int(x) for x in new))
            new_list.append(rid)
        node.route_list = new_list
        return rid

    def add(self, r):
        return self.update(r, r)

    def delete(self, r):
        self.update(r, None)

    def find(self, ip: int) -> int:
        b = _b4(ip)
        node, last = self.root, None
        for i in range(32):
            if node.route_list is not None:
                last = node.route_list
            bit = (b[i // 8] >> (7 - i % 8)) & 1
            nxt = node.left if bit == 0 else node.right
            if nxt is None:
                break
            node = nxt
        if node.route_list is not None:
            last = node.route_list
        if last is None:
            return NONE
        if len(last) == 0:
            return PANIC  # Go: integer divide by zero
        return last[fnv32a(b) % len(last)]
