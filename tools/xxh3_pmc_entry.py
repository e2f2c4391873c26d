"""Refresh the `xxh3_kcp_1M` entry of profiles/pmc_summary.json from one GPU session's ktxx / rdxx /
wrxx / sqxx passes over tools/exp/bench_xxh3.py (tools/gpu_session.sh): xxh3_run_kernel's average
duration, request-size read/write bytes and SQ counters, per launch.
usage: python tools/xxh3_pmc_entry.py gpurun_out/<session>"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "xxh3_run_kernel"
ALG_BYTES = 767981337  # bench.py xxh3_secondary: string bytes + 8 B metadata + 8 B hash per string


def per_dispatch(path):
    d = defaultdict(dict)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if KERNEL in r["Kernel_Name"]:
                d[int(r["Dispatch_Id"])][r["Counter_Name"]] = d[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
    return d


def avg(d, c):
    v = [x[c] for x in d.values() if c in x]
    return sum(v) / len(v) if v else None


def main():
    sess = sys.argv[1].rstrip("/")
    with open(os.path.join(sess, "ktxx", "run_kernel_trace.csv")) as fh:
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(fh) if KERNEL in r["Kernel_Name"]]
    rd = per_dispatch(os.path.join(sess, "rdxx", "run_counter_collection.csv"))
    wr = per_dispatch(os.path.join(sess, "wrxx", "run_counter_collection.csv"))
    sq = per_dispatch(os.path.join(sess, "sqxx", "run_counter_collection.csv"))
    rbytes = int(32 * avg(rd, "TCC_EA0_RDREQ_32B_sum") + 64 * avg(rd, "TCC_EA0_RDREQ_64B_sum") +
                 128 * avg(rd, "TCC_EA0_RDREQ_128B_sum"))
    w_all, w64 = avg(wr, "TCC_EA0_WRREQ_sum"), avg(wr, "TCC_EA0_WRREQ_64B_sum")
    wbytes = int(64 * w64 + 32 * (w_all - w64))
    waves = avg(sq, "SQ_WAVES")
    entry = {
        "kernels": [KERNEL],
        "workload": "tools/exp/bench_xxh3.py: 1M strings of 24..1400 B packed one byte apart (bench.py xxh3_secondary)",
        "launches": len(dur),
        "avg_duration_us": {KERNEL: round(sum(dur) / len(dur) / 1e3, 3)},
        "read_bytes_by_request_size": rbytes,
        "write_bytes_by_request_size": wbytes,
        "hbm_bytes_per_launch": rbytes + wbytes,
        "alg_bytes_per_launch": ALG_BYTES,
        "hbm_over_alg": round((rbytes + wbytes) / ALG_BYTES, 4),
        "hbm_bytes_method": "TCC_EA0_RDREQ_{32,64,128}B + TCC_EA0_WRREQ(_64B) request sizes, averaged over the launches",
        "SQ_WAVES": waves,
        "SQ_INSTS_VALU_per_wave": round(avg(sq, "SQ_INSTS_VALU") / waves, 1),
        "SQ_INSTS_VMEM_RD_per_wave": round(avg(sq, "SQ_INSTS_VMEM_RD") / waves, 1),
        "SQ_INSTS_LDS_per_wave": round(avg(sq, "SQ_INSTS_LDS") / waves, 1),
        "wait_frac": round(avg(sq, "SQ_WAIT_ANY") / avg(sq, "SQ_WAVE_CYCLES"), 3),
    }
    out = os.path.join(ROOT, "profiles", "pmc_summary.json")
    summary = json.load(open(out))
    summary["xxh3_kcp_1M"] = entry
    summary.setdefault("sessions", {})["xxh3_kcp_1M"] = os.path.basename(sess)
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(entry))


if __name__ == "__main__":
    main()
