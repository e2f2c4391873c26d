"""GPU parity for §8f row f4: the DIR-24-8 lookup compiled from the host trie
(halo_route_sync_device + halo_route_lookup_*_device) against the committed fixtures and the C
oracle, bit-exact route ids (incl. HALO_ROUTE_NONE / HALO_ROUTE_PANIC)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a device"
    from halo_amd import _lib

    _lib.check("halo_rx_init", _lib.lib.halo_rx_init(0))
    return torch.device("cuda:0")


def _replay_both(ops, oracle_lib):
    from halo_amd.route import RouteTable

    g, o = RouteTable(0), oracle_lib.RouteTable()
    for op in ops:
        if op[0] == "add":
            assert g.AddRoute(RouteTable.entry(*op[1])) == o.add(op[1])
        elif op[0] == "del":
            g.DeleteRoute(RouteTable.entry(*op[1]))
            o.delete(op[1])
        else:
            assert g.UpdateRoute(RouteTable.entry(*op[1]), RouteTable.entry(*op[2])) == o.update(op[1], op[2])
    return g, o


def _lookup(dev, g, ips):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(ips, np.uint32).view(np.int32)).to(dev)
    out = g.FindRoute(t)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_route_fixture_scenarios(dev, oracle_lib):
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "route.json")))
    for s in meta["scenarios"]:
        g, _ = _replay_both(s["ops"], oracle_lib)
        g.sync()
        got = _lookup(dev, g, np.array(s["lookups"], np.uint32))
        assert got.tolist() == s["expect"], s["name"]


def test_route_large_table_and_resync(dev, oracle_lib):
    """200k prefixes (BGP-like length mix, ECMP groups, /25-/32 under /24 blocks), 2M lookups;
    then delete / update a slice and re-sync: the device table follows the trie."""
    rng = np.random.default_rng(7)
    n = 200_000
    plen = rng.choice([8, 12, 16, 19, 20, 21, 22, 23, 24, 24, 24, 24, 25, 26, 28, 30, 32], n)
    mask = np.where(plen > 0, (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF, 0).astype(np.uint32)
    dst = (rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) & mask)
    ops = [("add", [0, 0, 1, 0])]
    for k in range(n):
        ops.append(("add", [int(dst[k]), int(mask[k]), int(k + 10), int(k % 4)]))
        if k % 9 == 0:
            ops.append(("add", [int(dst[k]), int(mask[k]), int(k + 11), int(k % 4)]))
    g, o = _replay_both(ops, oracle_lib)
    g.sync()
    ips = np.concatenate([rng.integers(0, 1 << 32, 1 << 20, dtype=np.uint64).astype(np.uint32),
                          (dst[rng.integers(0, n, 1 << 20)] | rng.integers(0, 256, 1 << 20).astype(np.uint32))])
    assert np.array_equal(_lookup(dev, g, ips), o.find_batch(ips))
    for k in range(0, n, 50):
        r = [int(dst[k]), int(mask[k]), int(k + 10), int(k % 4)]
        if k % 100 == 0:
            g.DeleteRoute(g.entry(*r))
            o.delete(r)
        else:
            new = [int(dst[k]), int(mask[k]), 7, 3]
            assert g.UpdateRoute(g.entry(*r), g.entry(*new)) == o.update(r, new)
    g.sync()
    assert np.array_equal(_lookup(dev, g, ips), o.find_batch(ips))


def test_route_lookup_from_records(dev, oracle_lib):
    """FindRoute(ipv4DstAddr) straight from parsed rx records (IMIX batch)."""
    import torch

    from halo_amd import protocol, synth
    from halo_amd._lib import NetIf

    ops = [("add", [0, 0, 1, 0]), ("add", [0xC0A86400, 0xFFFFFF00, 0, 1]), ("add", [0xC0A86464, 0xFFFFFFFF, 0, 2]),
           ("add", [0x0A000000, 0xFF000000, 5, 3]), ("add", [0x0A000000, 0xFF000000, 6, 3])]
    g, o = _replay_both(ops, oracle_lib)
    g.sync()
    lay = synth.layout(100_000, size_mode=1, proto_mode=3, first_index=99)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    out = protocol.parse_frames_batch(fr["bytes"], fr["offsets_dw"], fr["lens"], netif=NetIf.make(),
                                      max_len_hint=1500)
    rid = g.FindRouteRecords(out)
    torch.cuda.synchronize()
    recs = protocol.records(out)
    assert np.array_equal(rid.cpu().numpy().view(np.uint32), o.find_batch(recs["dst_ip"]))


@pytest.mark.parametrize("variant", [0, 1, 4, 8, 16, -1, -2])
def test_fused_parse_route(dev, oracle_lib, golden, variant):
    """halo_rx_parse_route_batch_device: records identical to the plain parse (full and compact)
    and route ids identical to the oracle's FindRoute of each record's dst — golden frames and
    IMIX, a table with a /32 to the NetIf, a /24, an ECMP group, an emptied list and a default."""
    import torch

    from halo_amd import _lib, protocol, synth
    from halo_amd._lib import NetIf
    from tests.helpers import golden_arrays

    ops = [("add", [0, 0, 1, 0]), ("add", [0xC0A86400, 0xFFFFFF00, 0, 1]), ("add", [0xC0A86464, 0xFFFFFFFF, 0, 2]),
           ("add", [0x0A000000, 0xFF000000, 5, 3]), ("add", [0x0A000000, 0xFF000000, 6, 3]),
           ("add", [0x0A800000, 0xFF800000, 9, 1]), ("del", [0x0A800000, 0xFF800000, 9, 1])]
    g, o = _replay_both(ops, oracle_lib)
    g.sync()
    meta, blob = golden
    data, offs, lens, _ = golden_arrays(meta, blob)
    lay = synth.layout(60_000, size_mode=1, proto_mode=3, mutate_shift=4, first_index=777)
    fr = synth.frames_device(lay, NetIf.make(), device=dev)
    batches = [(torch.from_numpy(data).to(dev), torch.from_numpy(offs.view(np.int32)).to(dev),
                torch.from_numpy(lens.view(np.int16)).to(dev), 0), (fr["bytes"], fr["offsets_dw"], fr["lens"], 1500)]
    stream = torch.cuda.current_stream().cuda_stream
    vf = _lib.variant_flags(variant)
    for d, o_, ln, hint in batches:
        n = int(ln.numel())
        full = protocol.parse_frames_batch(d, o_, ln, netif=NetIf.make(), max_len_hint=hint)
        want_ids = o.find_batch(protocol.records(full)["dst_ip"])
        for compact in (False, True):
            flags = 1 | vf | (_lib.HALO_RX_RECORD_COMPACT if compact else 0)
            width = 16 if compact else 32
            ref = torch.empty((n, width), dtype=torch.uint8, device=dev)
            _lib.check("parse", _lib.lib.halo_rx_parse_batch_device(
                d.data_ptr(), o_.data_ptr(), ln.data_ptr(), n, flags, NetIf.make(), hint, ref.data_ptr(), None,
                stream))
            got = torch.full((n, width), 0xEE, dtype=torch.uint8, device=dev)
            rid = torch.zeros(n, dtype=torch.int32, device=dev)
            _lib.check("fused", _lib.lib.halo_rx_parse_route_batch_device(
                d.data_ptr(), o_.data_ptr(), ln.data_ptr(), n, flags, NetIf.make(), hint, got.data_ptr(), None,
                g._t, rid.data_ptr(), stream))
            torch.cuda.synchronize()
            assert torch.equal(got, ref), (variant, compact)
            assert np.array_equal(rid.cpu().numpy().view(np.uint32), want_ids), (variant, compact)
    assert _lib.lib.halo_rx_parse_route_batch_device(None, None, None, 0, 1, NetIf.make(), 0, None, None, None,
                                                     None, None) == _lib.HALO_E_INVAL  # no table


def test_route_validation(dev):
    import ctypes

    import torch

    from halo_amd import _lib
    from halo_amd.route import RouteTable

    g = RouteTable(0)
    ips = torch.zeros(8, dtype=torch.int32, device=dev)
    rc = _lib.lib.halo_route_lookup_device(g._t, ips.data_ptr(), 8, ips.data_ptr(), None)
    assert rc == _lib.HALO_E_INVAL  # not synced yet
    assert _lib.lib.halo_route_get(g._t, 5, ctypes.c_void_p(ips.data_ptr())) == _lib.HALO_E_RANGE


def test_concurrent_sync_and_lookups(dev):
    """Syncs on one thread, lookups on another stream and thread (a sync could rewrite
    the generation a lookup had taken its view of but not yet launched on). Every launch must see
    exactly one published table: all of its 64k addresses (inside 10.1.0.0/16) get the same id, the
    /8's or the /16 route current at some sync."""
    import threading

    import torch

    from halo_amd.route import RouteTable, ip_u

    t = RouteTable(dev.index or 0)
    base_id = t.AddRoute(t.entry(ip_u("10.0.0.0"), ip_u("255.0.0.0"), ip_u("192.168.1.1"), 1))
    t.sync()
    valid = {base_id}
    lock = threading.Lock()
    stop = threading.Event()
    errors = []
    n = 1 << 16
    ips = torch.from_numpy((np.uint32(ip_u("10.1.0.0")) + np.arange(n, dtype=np.uint32)).view(np.int32)).to(dev)

    def syncer():
        try:
            route = t.entry(ip_u("10.1.0.0"), ip_u("255.255.0.0"), ip_u("192.168.1.2"), 2)
            for k in range(60):
                if k % 2 == 0:
                    rid = t.AddRoute(route)
                    with lock:
                        valid.add(rid)
                else:
                    t.DeleteRoute(route)  # leaves an emptied list: lookups there panic (ROUTE_PANIC)
                t.sync()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
        finally:
            stop.set()

    def looker():
        s = torch.cuda.Stream(device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        launches = 0
        try:
            while not stop.is_set() or launches < 5:
                with torch.cuda.stream(s):
                    t.FindRoute(ips, out=out, stream=s)
                s.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                launches += 1
                u = np.unique(got)
                with lock:
                    ok = len(u) == 1 and (int(u[0]) in valid or int(u[0]) == 0xFFFFFFFE)
                if not ok:
                    errors.append(f"launch {launches}: ids {u[:8]}")
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=syncer), threading.Thread(target=looker)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    t.close()
    assert not errors, errors[:3]
