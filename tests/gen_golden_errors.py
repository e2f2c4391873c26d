"""Generate tests/golden/error_text.json: the error strings the reference's receive parsers return,
read as data from the Go source (the `errors.New("...")` literal at each check's file:line). Runs
in the build container only (needs /root/reference); the JSON is committed.

    python tests/gen_golden_errors.py
"""
from __future__ import annotations

import json
import os
import re

REF = "/root/reference/protocol"
# (status, ip protocol or None, file, line): the check of SURVEY.md §8a each status stands for
SITES = [
    ("ETH_LEN", None, "ethernet.go", 32), ("ETH_TYPE", None, "ethernet.go", 49),
    ("IP_LEN", None, "ipv4.go", 50), ("IP_VER", None, "ipv4.go", 53), ("IP_FRAG", None, "ipv4.go", 60),
    ("IP_PROTO", None, "ipv4.go", 71), ("IP_HDR_CKSUM", None, "ipv4.go", 76),
    ("L4_LEN", 17, "udp.go", 23), ("L4_LEN", 6, "tcp.go", 38), ("L4_LEN", 1, "icmp.go", 35),
    ("ICMP_TYPE", 1, "icmp.go", 46), ("ICMP_CODE", 1, "icmp.go", 50),
    ("L4_CKSUM", 17, "udp.go", 43), ("L4_CKSUM", 6, "tcp.go", 64), ("L4_CKSUM", 1, "icmp.go", 54),
]


def main():
    out = []
    for status, proto, fn, line in SITES:
        src = open(os.path.join(REF, fn), encoding="utf-8").read().splitlines()[line - 1]
        m = re.search(r'errors\.New\("([^"]*)"\)', src)
        assert m, (fn, line, src)
        out.append({"status": status, "ip_proto": proto, "site": f"protocol/{fn}:{line}", "text": m.group(1)})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "error_text.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {len(out)} error strings to {path}")


if __name__ == "__main__":
    main()
