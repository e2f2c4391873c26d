#!/usr/bin/env python3
"""Summarise a tools/gpu_session.sh profiling session (kt, kfetch, kwrite, ksq steps) into
per-workload numbers and write profiles/pmc_summary.json (read by bench.py for `traffic`).

    python tools/pmc_summary.py gpurun_out/<tag> [--out profiles/pmc_summary.json] [--only W1,W2]

(--only: the session ran tools/prof_kernels.py with that workload filter, PK_ARGS.)

rx_* / tx_fixup_* dispatches are attributed to tools/prof_kernels.py's WORKLOADS in launch order.
HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from separate
--pmc passes; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read,
so read bytes = 2 x FETCH_SIZE x 1024 (the calibration column checks that against the bytes
each launch must read: frames + metadata).
"""
from __future__ import annotations

import csv
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as fh:
        return list(csv.DictReader(fh))


def alg_bytes():
    """(read bytes, written bytes) per launch for each profiled workload."""
    from halo_amd import synth
    from tools.prof_kernels import WORKLOADS

    out = {}
    for name, kw, n, _rot, _launches, slen, _flags, _hint in WORKLOADS:  # noqa: B007
        kw = dict(kw)
        kw.pop("strided", None)
        lay = synth.layout(n, **kw, ragged=not slen)
        frames = int(lay["lens"].astype("int64").sum())
        meta = 0 if slen else 6 * n
        if name.startswith("flow_hash"):  # record bytes 0..19 (compact: the 16 B record) in; hash + bucket out
            out[name] = ((16 if name.endswith("_compact") else 20) * n, 12 * n)
            continue
        if name == "config2_batch_stream":  # `rot` batches per launch
            out[name] = (_rot * (frames + meta), _rot * 32 * n)
            continue
        if name.startswith("lo_drain"):  # 50 B packets + offset/len in, 32 B record out
            out[name] = (56 * n, 32 * n)
            continue
        if name.startswith("tx_build"):  # descriptor + payload in; frame + length + result out
            plen = _hint
            flen = max(60, 42 + plen)
            out[name] = ((40 + plen) * n, (flen + 3) * n)
            continue
        if name.startswith("ring_scan"):  # the ring span (u32 length + frame, dword aligned) in; 6 B per record out
            lens = lay["lens"].astype("int64")
            out[name] = (int((4 + ((lens + 3) & ~3)).sum()), 6 * n)
            continue
        if name.startswith("tx_"):  # + 16 B op in; 1 B result + 20 B of rewritten header out
            import bench

            out[name] = (frames + meta + 16 * n, (1 + bench.TX_WRITE_BYTES) * n)
        else:
            out[name] = (frames + meta, 32 * n)
    return out


def main():
    if len(sys.argv) < 2 or not os.path.isdir(sys.argv[1]):
        sys.exit(__doc__)
    sess = sys.argv[1]
    out_path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(
        ROOT, "profiles", "pmc_summary.json")
    from tools.prof_kernels import WORKLOADS

    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    order = []
    for name, _kw, _n, _rot, launches, *_ in WORKLOADS:
        if (only is None or name in only) and not name.startswith(("ring_", "probe_")):  # the ring walk: below; probes: not ours
            order += [name] * launches

    def family(w):
        if w.startswith("flow_hash"):
            return "flow_hash_kernel"
        if w.startswith("tx_build"):
            return "tx_build_"
        return "tx_fixup" if w.startswith("tx_") else "rx_"

    def attribute(rows, key="Dispatch_Id"):
        """dispatch id -> workload: each kernel family's dispatches in launch order."""
        amap = {}
        for fam in ("rx_", "tx_fixup", "flow_hash_kernel", "tx_build_"):
            disp = sorted({int(r[key]) for r in rows if fam in r["Kernel_Name"]})
            ws = [w for w in order if family(w) == fam]
            # (the flow-hash workload's one preparatory parse comes after every rx workload's
            # launches, WORKLOADS order, so it falls outside ws and is not attributed)
            amap.update({d: ws[k] for k, d in enumerate(disp) if k < len(ws)})
        return amap

    res = defaultdict(lambda: defaultdict(list))
    kt = _rows(os.path.join(sess, "kt", "run_kernel_trace.csv"))
    amap = attribute(kt)
    for r in kt:
        d = int(r["Dispatch_Id"])
        if d in amap:
            w = amap[d]
            res[w]["duration_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            res[w]["kernel"] = [r["Kernel_Name"]]
            res[w]["vgpr"] = [int(r["VGPR_Count"])]
            res[w]["sgpr"] = [int(r["SGPR_Count"])]
    for step in ("kfetch", "kwrite", "ksq", "krd", "kwrq"):
        rows = _rows(os.path.join(sess, step, "run_counter_collection.csv"))
        amap = attribute(rows)
        per = defaultdict(dict)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in amap:
                per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for d, cs in per.items():
            for c, v in cs.items():
                res[amap[d]][c].append(v)
    # the ring walk: three kernels per walk (guess, link, copy) — a workload's counters are summed
    # over its walks' dispatches and divided by the walks; durations are kept per kernel
    ring_order = []
    for name, _kw, _n, _rot, launches, *_ in WORKLOADS:
        if (only is None or name in only) and name.startswith("ring_"):
            ring_order += [name] * launches

    def ring_attr(rows):
        disp = sorted({int(r["Dispatch_Id"]) for r in rows if "ring_" in r["Kernel_Name"]})
        return {d: ring_order[k // 3] for k, d in enumerate(disp) if k // 3 < len(ring_order)}

    ring = defaultdict(lambda: defaultdict(float))
    ring_kernels = defaultdict(lambda: defaultdict(list))
    amap = ring_attr(kt)
    for r in kt:
        d = int(r["Dispatch_Id"])
        if d in amap:
            short = re.search(r"ring_\w+?_kernel", r["Kernel_Name"]).group(0)
            ring_kernels[amap[d]][short].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for step in ("kfetch", "kwrite", "ksq", "krd", "kwrq"):
        rows = _rows(os.path.join(sess, step, "run_counter_collection.csv"))
        amap = ring_attr(rows)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in amap:
                ring[amap[d]][r["Counter_Name"]] += float(r["Counter_Value"])
    for w in set(ring) | set(ring_kernels):
        walks = ring_order.count(w)
        for c, v in ring[w].items():
            res[w][c].append(v / walks)
        per = {k: round(sum(v) / len(v) / 1e3, 3) for k, v in ring_kernels[w].items()}
        if per:
            res[w]["duration_ns"].append(1e3 * sum(per.values()))
            res[w]["kernel"] = [" + ".join(per)]
            res[w]["kernels_us"] = [per]
    algs = alg_bytes()
    summary = {}
    for w, m in res.items():
        avg = {k: (sum(v) / len(v) if v and not isinstance(v[0], (str, dict)) else v[0]) for k, v in m.items()}
        rd_alg, wr_alg = algs[w]
        s = {"kernel": avg.get("kernel"), "vgpr": avg.get("vgpr"), "sgpr": avg.get("sgpr"),
             **({"kernels_us": m["kernels_us"][0]} if "kernels_us" in m else {}),
             "launches": len(m.get("duration_ns", [])),
             "avg_duration_us": round(avg["duration_ns"] / 1e3, 3) if "duration_ns" in avg else None,
             "alg_read_bytes": rd_alg, "alg_write_bytes": wr_alg}
        if "duration_ns" in avg:
            s["alg_GBps"] = round((rd_alg + wr_alg) / avg["duration_ns"], 1)
        if "FETCH_SIZE" in avg:
            raw = avg["FETCH_SIZE"] * 1024
            s["fetch_bytes_raw"] = int(raw)
            s["fetch_bytes_corrected_x2"] = int(2 * raw)
            s["fetch_over_alg_read_raw"] = round(raw / rd_alg, 3)
        if "WRITE_SIZE" in avg:
            s["write_bytes"] = int(avg["WRITE_SIZE"] * 1024)
            s["write_over_alg"] = round(avg["WRITE_SIZE"] * 1024 / wr_alg, 3)
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            s["hbm_bytes_per_launch"] = int(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024)
        # exact request bytes from the L2's memory-side request counters by size (krd / kwrq passes):
        # no calibration factor needed (FETCH_SIZE tallies a 128-byte request as 64 bytes on gfx950)
        r32, r64, r128 = (avg.get(f"TCC_EA0_RDREQ_{b}B_sum") for b in (32, 64, 128))
        if r32 is not None and r64 is not None and r128 is not None:
            s["read_bytes_by_request_size"] = int(32 * r32 + 64 * r64 + 128 * r128)
            s["read_over_alg"] = round(s["read_bytes_by_request_size"] / rd_alg, 4)
            if avg.get("TCC_EA0_RDREQ_sum"):
                s["rdreq_sizes_cover_all"] = round((r32 + r64 + r128) / avg["TCC_EA0_RDREQ_sum"], 4)
        w_all, w64 = avg.get("TCC_EA0_WRREQ_sum"), avg.get("TCC_EA0_WRREQ_64B_sum")
        if w_all is not None and w64 is not None:
            s["write_bytes_by_request_size"] = int(64 * w64 + 32 * (w_all - w64))
            s["write_requests_64B"] = int(w64)
        if "read_bytes_by_request_size" in s:
            wb = s.get("write_bytes_by_request_size", s.get("write_bytes"))
            if wb is not None:
                s["hbm_bytes_per_launch"] = s["read_bytes_by_request_size"] + wb
                s["hbm_bytes_method"] = "TCC_EA0_RDREQ_{32,64,128}B + TCC_EA0_WRREQ(_64B) request sizes"
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                  "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"):
            if c in avg:
                s[c] = avg[c]
        if "SQ_WAVES" in avg and avg["SQ_WAVES"]:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS"):
                if c in avg:
                    s[c + "_per_wave"] = round(avg[c] / avg["SQ_WAVES"], 1)
        if "SQ_WAIT_ANY" in avg and avg.get("SQ_WAVE_CYCLES"):
            s["wait_frac"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 3)
        # (GRBM_GUI_ACTIVE / duration is not a clock: the counter's window is wider than the kernel,
        # so round 3's "eff_clock_GHz" read 3-4 GHz on a 2.4 GHz part; it is not reported)
        summary[w] = s
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    merged = {}
    if "--merge" in sys.argv and os.path.exists(out_path):  # keep other workloads' entries
        merged = json.load(open(out_path))
    merged.update(summary)
    merged.setdefault("sessions", {})
    for w in summary:
        merged["sessions"][w] = os.path.basename(sess.rstrip("/"))
    merged.pop("session", None)
    with open(out_path, "w") as fh:
        json.dump(merged, fh, indent=1)
    for w, s in summary.items():
        print(w, json.dumps(s))


if __name__ == "__main__":
    main()
