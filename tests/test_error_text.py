"""CPU: every status a record can carry maps to the exact error string the reference function that
failed returns (tests/golden/error_text.json, read from the Go source by tests/gen_golden_errors.py),
per protocol where the reference has one string per protocol (the L4 length checks)."""
from __future__ import annotations

import json
import os

from halo_amd import protocol
from halo_amd._lib import STATUS, STATUS_NAMES

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "error_text.json")


def test_error_text_matches_reference_strings():
    sites = json.load(open(GOLDEN))
    assert len(sites) == 15
    for e in sites:
        protos = [e["ip_proto"]] if e["ip_proto"] is not None else [protocol.IPH_PROTO_UDP, protocol.IPH_PROTO_TCP,
                                                                     protocol.IPH_PROTO_ICMP]
        for p in protos:
            assert protocol.error_text(STATUS[e["status"]], p) == e["text"], (e["site"], p)
    # every status is covered: OK and the build-defined totalLen statuses have no reference string
    covered = {e["status"] for e in sites}
    for code, name in enumerate(STATUS_NAMES):
        if name in ("OK", "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN"):
            assert protocol.error_text(code) is None
        else:
            assert name in covered, name
    # the three L4 length strings differ: the protocol decides
    texts = {protocol.error_text(STATUS["L4_LEN"], p) for p in (1, 6, 17)}
    assert len(texts) == 3
