"""CPU: the route-lookup restatements (§8f row f4) — the C oracle against the committed
fixtures made by the independent Python restatement (including the reference's example route
lists), and the two against each other on fuzzed update sequences."""
from __future__ import annotations

import json
import os
import random

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _replay(table, ops):
    for op in ops:
        if op[0] == "add":
            table.add(op[1])
        elif op[0] == "del":
            table.delete(op[1])
        else:
            table.update(op[1], op[2])


def test_c_oracle_matches_route_fixtures(oracle_lib):
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "route.json")))
    for s in meta["scenarios"]:
        t = oracle_lib.RouteTable()
        _replay(t, s["ops"])
        got = t.find_batch(np.array(s["lookups"], np.uint32))
        assert got.tolist() == s["expect"], s["name"]


def test_c_and_python_route_tables_agree_fuzz(oracle_lib):
    from oracle import ref_route_py as RR

    rnd = random.Random(77)
    for trial in range(20):
        c, py = oracle_lib.RouteTable(), RR.RouteTable()
        live = []
        for _ in range(rnd.randrange(1, 120)):
            plen = rnd.randrange(33)
            mask = ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF) if plen else 0
            r = [rnd.getrandbits(32) & (mask if rnd.random() < 0.8 else 0xFFFFFFFF), mask, rnd.getrandbits(8),
                 rnd.randrange(3)]
            k = rnd.random()
            if k < 0.7 or not live:
                assert c.add(r) == py.add(r)
                live.append(r)
            elif k < 0.85:
                v = live.pop(rnd.randrange(len(live)))
                c.delete(v)
                py.delete(v)
            else:
                v = live.pop(rnd.randrange(len(live)))
                assert c.update(v, r) == py.update(v, r)
                live.append(r)
        ips = [rnd.getrandbits(32) for _ in range(300)] + [(r[0] | rnd.getrandbits(4)) for r in live]
        assert c.find_batch(np.array(ips, np.uint32)).tolist() == [py.find(ip) for ip in ips], trial


def test_route_semantics_spot_checks(oracle_lib):
    """Longest prefix wins; ECMP members are picked by fnv32a(ip) % n in insertion order; deleting
    every member of a prefix leaves an empty (non-nil) list that still ends the lookup."""
    from oracle import ref_route_py as RR

    t = oracle_lib.RouteTable()
    d = t.add((0, 0, 1, 0))
    a = t.add((0x0A000000, 0xFF000000, 2, 0))
    b = t.add((0x0A000000, 0xFF000000, 3, 0))
    c = t.add((0x0A010000, 0xFFFF0000, 4, 0))
    assert t.find(0x0B000001) == d
    assert t.find(0x0A010203) == c
    ip = 0x0A020304
    assert t.find(ip) == [a, b][RR.fnv32a(ip.to_bytes(4, "big")) % 2]
    t.delete((0x0A010000, 0xFFFF0000, 4, 0))
    assert t.find(0x0A010203) == RR.PANIC
    assert t.find(0x0A020304) in (a, b)
