"""Generate the committed route-lookup fixtures (§8f row f4): tests/golden/route.json.

Expected route ids come from oracle/ref_route_py.py (pure-Python restatement of
engine.RouteTable). Scenarios: the reference's own example route lists (example/example.go:146-
152, :368-374 plus the direct routes engine/engine.go:259-273 installs), then a seeded mix of
prefixes /0../32 with ECMP groups, deletions that empty a list (the reference's divide-by-zero),
UpdateRoute with a different new prefix (stored at the old prefix's node), non-contiguous masks
and destinations with bits past the mask. Each scenario lists its operations and lookups.

    python tests/gen_golden_route.py
"""
from __future__ import annotations

import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_route_py as RR  # noqa: E402


def u(s):
    a = [int(x) for x in s.split(".")]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


def run(ops, lookups):
    t = RR.RouteTable()
    for op in ops:
        if op[0] == "add":
            t.add(op[1])
        elif op[0] == "del":
            t.delete(op[1])
        else:
            t.update(op[1], op[2])
    return [t.find(ip) for ip in lookups]


def example_scenario():
    # example/example.go:146-152 (EthernetRouter): one static /32 via wan0, then the direct
    # routes of the interfaces (engine/engine.go:259-273; NextHop nil -> 0)
    ops = [("add", [u("114.114.114.114"), u("255.255.255.255"), u("192.168.100.1"), 1]),
           ("add", [u("192.168.100.0"), u("255.255.255.0"), 0, 1]),
           ("add", [u("192.168.111.0"), u("255.255.255.0"), 0, 2]),
           # DHCP default route (engine/dhcp_engine.go:402-407)
           ("add", [0, 0, u("192.168.100.1"), 1])]
    lookups = [u("114.114.114.114"), u("114.114.114.115"), u("192.168.100.7"), u("192.168.111.255"),
               u("8.8.8.8"), u("192.168.101.1"), 0, 0xFFFFFFFF]
    return {"name": "example_router", "ops": ops, "lookups": lookups}


def random_scenario(seed, n_routes, n_lookups, churn, default=True):
    rnd = random.Random(seed)
    ops, live = [], []
    for k in range(n_routes):
        plen = rnd.choice([0 if default else 8, 1 if default else 9, 7, 8, 9, 12, 15, 16, 17, 20, 23, 24, 24, 24, 25, 26, 28, 30, 31, 32])
        mask = ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF) if plen else 0
        if rnd.random() < 0.05 and mask:
            mask ^= 1 << rnd.randrange(32 - plen + 1, 32) if plen > 1 else 0  # non-contiguous
        dst = rnd.getrandbits(32)
        if rnd.random() < 0.7:
            dst &= mask  # canonical most of the time
        r = [dst, mask, rnd.getrandbits(32) if rnd.random() < 0.8 else 0, rnd.randrange(4)]
        ops.append(("add", r))
        live.append(r)
        if rnd.random() < 0.2:  # ECMP sibling: same prefix, another next hop
            r2 = [dst, mask, rnd.getrandbits(32), rnd.randrange(4)]
            ops.append(("add", r2))
            live.append(r2)
        if churn and rnd.random() < churn and live:
            victim = live.pop(rnd.randrange(len(live)))
            if rnd.random() < 0.5:
                ops.append(("del", victim))
            else:
                plen2 = rnd.randrange(33)
                m2 = ((0xFFFFFFFF << (32 - plen2)) & 0xFFFFFFFF) if plen2 else 0
                new = [rnd.getrandbits(32) & m2, m2, rnd.getrandbits(32), rnd.randrange(4)]
                ops.append(("upd", victim, new))
                live.append(new)
        if rnd.random() < 0.03:  # delete something that was never added (creates an empty list)
            ops.append(("del", [rnd.getrandbits(32), 0xFFFFFF00, 1, 0]))
    lookups = []
    for _ in range(n_lookups):
        if live and rnd.random() < 0.6:
            r = rnd.choice(live)
            ip = (r[0] & r[1]) | (rnd.getrandbits(32) & ~r[1] & 0xFFFFFFFF)
        else:
            ip = rnd.getrandbits(32)
        lookups.append(ip)
    return {"name": f"random_{seed}", "ops": ops, "lookups": lookups}


def main():
    scen = [example_scenario(), random_scenario(1, 40, 400, 0.0), random_scenario(2, 300, 2000, 0.1),
            random_scenario(3, 2000, 4000, 0.2), random_scenario(4, 500, 3000, 0.15, default=False)]
    for s in scen:
        s["expect"] = run(s["ops"], s["lookups"])
    with open(os.path.join(ROOT, "tests", "golden", "route.json"), "w") as fh:
        json.dump({"scenarios": scen}, fh, separators=(",", ":"))
    print({s["name"]: (len(s["ops"]), len(s["lookups"]), sum(e == RR.PANIC for e in s["expect"]),
                       sum(e == RR.NONE for e in s["expect"])) for s in scen})


if __name__ == "__main__":
    main()
