"""Shared helpers for the parity tests."""
from __future__ import annotations

import numpy as np

FIELDS = ["status", "flags", "ethertype", "ip_proto", "l4_aux", "ip_total_len", "src_ip", "dst_ip", "sport",
          "dport", "payload_off", "payload_len", "l4_seq", "l4_ack"]
STATUS_NAMES = ["OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
                "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM"]


def golden_arrays(meta, blob):
    """(data, offsets_dw, lens, names) for the golden frames (4-byte aligned, ragged)."""
    fr = meta["frames"]
    offs = np.array([e["offset"] for e in fr], dtype=np.uint64)
    assert np.all(offs % 4 == 0)
    lens = np.array([e["len"] for e in fr], dtype=np.uint16)
    return blob, (offs // 4).astype(np.uint32), lens, [e["name"] for e in fr]


def expected_records(meta, flags: int, dtype) -> np.ndarray:
    fr = meta["frames"]
    out = np.zeros(len(fr), dtype=dtype)
    for i, e in enumerate(fr):
        r = e["expect"][str(flags)]
        for f in FIELDS:
            out[i][f] = r[f]
    return out


def assert_records_equal(got: np.ndarray, want: np.ndarray, names=None, what=""):
    """Bit-exact comparison of two halo_rx_result_t arrays with a readable diff."""
    assert got.shape == want.shape, (got.shape, want.shape)
    gb = np.ascontiguousarray(got).view(np.uint8).reshape(-1, 32)
    wb = np.ascontiguousarray(want).view(np.uint8).reshape(-1, 32)
    bad = np.nonzero(np.any(gb != wb, axis=1))[0]
    if bad.size:
        lines = [f"{what}: {bad.size} of {got.shape[0]} records differ"]
        for i in bad[:8]:
            nm = names[i] if names is not None else str(i)
            diffs = [f"{f}: got {got[i][f]} want {want[i][f]}" for f in FIELDS if got[i][f] != want[i][f]]
            lines.append(f"  [{i}] {nm}: " + "; ".join(diffs))
        raise AssertionError("\n".join(lines))
