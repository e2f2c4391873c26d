"""Shared helpers for the parity tests."""
from __future__ import annotations

import numpy as np

FIELDS = ["status", "flags", "ethertype", "ip_proto", "l4_aux", "ip_total_len", "src_ip", "dst_ip", "sport",
          "dport", "payload_off", "payload_len", "l4_seq", "l4_ack"]
STATUS_NAMES = ["OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
                "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM"]


def golden_arrays(meta, blob, key="frames"):
    """(data, offsets_dw, lens, names) for the golden frames (4-byte aligned, ragged); key
    "packets" for the LoChan fixtures (lo_golden)."""
    fr = meta[key]
    offs = np.array([e["offset"] for e in fr], dtype=np.uint64)
    assert np.all(offs % 4 == 0)
    lens = np.array([e["len"] for e in fr], dtype=np.uint16)
    return blob, (offs // 4).astype(np.uint32), lens, [e["name"] for e in fr]


def expected_records(meta, flags: int, dtype, key="frames") -> np.ndarray:
    fr = meta[key]
    out = np.zeros(len(fr), dtype=dtype)
    for i, e in enumerate(fr):
        r = e["expect"][str(flags)]
        for f in FIELDS:
            out[i][f] = r[f]
    return out


def lo_golden(root):
    """The LoChan packet fixtures (tests/gen_golden_lo.py): (meta, blob); entries under "packets"."""
    import json
    import os

    g = os.path.join(root, "tests", "golden")
    with open(os.path.join(g, "lo_packets.json")) as fh:
        meta = json.load(fh)
    return meta, np.fromfile(os.path.join(g, "lo_packets.bin"), dtype=np.uint8)


def strip_ethernet(data: np.ndarray, offsets_dw: np.ndarray, lens: np.ndarray):
    """Frames -> their Ethernet payloads (what Ipv4RouteForward puts in LoChan,
    engine/ipv4_engine.go:195-200), repacked at 4-byte-aligned starts: (data, offsets_dw, lens).
    Frames shorter than 14 bytes become empty packets."""
    plens = np.maximum(lens.astype(np.int64) - 14, 0)
    sizes = (plens + 3) & ~3
    offs = np.zeros(len(lens), dtype=np.int64)
    if len(lens):
        offs[1:] = np.cumsum(sizes)[:-1]
    out = np.zeros(int(sizes.sum()) + 16, dtype=np.uint8)
    for i in range(len(lens)):
        src = int(offsets_dw[i]) * 4 + 14
        out[offs[i]:offs[i] + plens[i]] = data[src:src + plens[i]]
    return out, (offs // 4).astype(np.uint32), plens.astype(np.uint16)


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


def tx_golden(root):
    """The §8f f2 fixtures: (meta, frames blob, expected header bytes [entries, 2, 52])."""
    import json
    import os

    g = os.path.join(root, "tests", "golden")
    with open(os.path.join(g, "tx.json")) as fh:
        meta = json.load(fh)
    blob = np.fromfile(os.path.join(g, "tx_frames.bin"), dtype=np.uint8)
    exp = np.fromfile(os.path.join(g, "tx_expect.bin"), dtype=np.uint8).reshape(len(meta["entries"]), 2,
                                                                                 meta["hdr_bytes"])
    return meta, blob, exp


def tx_batch_arrays(meta, blob, op_dtype, entries=None):
    """Lay the fixture entries out as one ragged batch: (data, offsets_dw, lens, ops, originals)."""
    ents = meta["entries"] if entries is None else [meta["entries"][k] for k in entries]
    frs = meta["frames"]
    lens = np.array([frs[e["frame"]]["len"] for e in ents], dtype=np.uint16)
    sizes = (lens.astype(np.int64) + 3) & ~3
    offs = np.zeros(len(ents), dtype=np.int64)
    if len(ents):
        offs[1:] = np.cumsum(sizes)[:-1]
    data = np.zeros(max(16, int(sizes.sum()) + 16), dtype=np.uint8)
    originals = []
    for k, e in enumerate(ents):
        f = frs[e["frame"]]
        src = blob[f["offset"]:f["offset"] + f["len"]]
        data[offs[k]:offs[k] + f["len"]] = src
        originals.append(src)
    ops = np.zeros(len(ents), dtype=op_dtype)
    for k, e in enumerate(ents):
        ops[k]["steps"], ops[k]["dst_ip"], ops[k]["dst_port"], ops[k]["src_ip"], ops[k]["src_port"] = e["op"]
    return data, (offs // 4).astype(np.uint32), lens, ops, originals


def assert_tx_equal(data, offsets_dw, lens, results, meta, exp, flag, entries=None, what=""):
    """Rewritten frames == fixture (header bytes) and untouched past byte 51; result bytes equal."""
    ents = meta["entries"] if entries is None else [meta["entries"][k] for k in entries]
    idx = range(len(meta["entries"])) if entries is None else entries
    hb = meta["hdr_bytes"]
    bad = []
    for k, (ek, e) in enumerate(zip(idx, ents)):
        L = int(lens[k])
        o = int(offsets_dw[k]) * 4
        got = data[o:o + min(L, hb)]
        want = exp[ek, flag, :min(L, hb)]
        if not np.array_equal(got, want) or int(results[k]) != e["result"][str(flag)]:
            bad.append((k, meta["frames"][e["frame"]]["name"], e["op"][0], got.tobytes().hex(),
                        want.tobytes().hex(), int(results[k]), e["result"][str(flag)]))
    assert not bad, f"{what}: {len(bad)} of {len(ents)} entries differ; first: {bad[:3]}"


def build_golden(root):
    """The §8f f2 Build* fixtures: (descriptor array, payload bytes, meta, expected frames blob)."""
    import json
    import os

    from oracle.oracle import BUILD_DESC_DTYPE

    g = os.path.join(root, "tests", "golden")
    with open(os.path.join(g, "tx_build.json")) as fh:
        meta = json.load(fh)
    desc = np.zeros(len(meta["descs"]), dtype=BUILD_DESC_DTYPE)
    for i, d in enumerate(meta["descs"]):
        for k, v in d.items():
            desc[i][k] = v
    payload = np.fromfile(os.path.join(g, "tx_build_payload.bin"), dtype=np.uint8)
    expect = np.fromfile(os.path.join(g, "tx_build_expect.bin"), dtype=np.uint8)
    return desc, payload, meta, expect


def assert_build_equal(frames, lens, res, ip_end, run, expect, what="", names=None):
    """Built frames / lengths / results / final iphId == one fixture run (frames compared up to
    each expected length)."""
    want_lens = np.array(run["lens"], dtype=np.uint16)
    want_res = np.array(run["results"], dtype=np.uint8)
    bad_res = np.nonzero(np.asarray(res) != want_res)[0]
    assert bad_res.size == 0, f"{what}: results differ at {bad_res[:8]} got {np.asarray(res)[bad_res[:8]]}"
    bad_len = np.nonzero(np.asarray(lens) != want_lens)[0]
    assert bad_len.size == 0, f"{what}: lengths differ at {bad_len[:8]}"
    for i, (o, ln) in enumerate(zip(run["expect_offsets"], run["lens"])):
        got = bytes(frames[i][:ln])
        want = bytes(expect[o:o + ln])
        if got != want:
            k = next(j for j in range(ln) if got[j] != want[j])
            raise AssertionError(f"{what}: frame {i} differs first at byte {k}: got {got[k:k+8].hex()} "
                                 f"want {want[k:k+8].hex()}")
    assert ip_end == run["ip_id_end"], (what, ip_end, run["ip_id_end"])
