"""Per-kernel SQ / TCC counter summary of one or more rocprofv3 --pmc passes (tools only):
    python tools/exp/sq_per_kernel.py <dir with run_counter_collection.csv> [...] [--kt <kt dir>]
Sums each counter over a kernel's dispatches, and prints per-dispatch and per-wave figures
(VALU / VMEM / LDS instructions per wave, wave cycles, waits), the average resident waves per
SIMD (SQ_WAVE_CYCLES x 4 quad-cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)... see the
note printed) and, with --kt, the average kernel duration from the kernel trace."""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("halo::", "")
    return re.sub(r"\(.*", "", name).replace("void ", "")


def main():
    args = sys.argv[1:]
    kt = None
    if "--kt" in args:
        i = args.index("--kt")
        kt = args[i + 1]
        del args[i:i + 2]
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    vgpr = {}
    for d in args:
        for row in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            k = short(row["Kernel_Name"]) + f" grid={row['Grid_Size']}"
            per[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add((d, row["Dispatch_Id"]))
            vgpr[k] = (row["VGPR_Count"], row["Accum_VGPR_Count"], row["SGPR_Count"], row["LDS_Block_Size"],
                       row["Workgroup_Size"])
    dur = defaultdict(list)
    if kt:
        for row in csv.DictReader(open(os.path.join(kt, "run_kernel_trace.csv"))):
            dur[short(row["Kernel_Name"]) + f" grid={row['Grid_Size_X']}"].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    for k, c in per.items():
        if "probe" in k and "stream_rw" not in k:
            continue
        ndisp = max(1, len(disp[k]) // max(1, len(args)))
        w = c.get("SQ_WAVES", 0) or 1
        line = [f"{k}  dispatches/pass={ndisp} vgpr/agpr/sgpr/lds/wg={vgpr[k]}"]
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                     "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                     "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
            if name in c:
                line.append(f"{name}/wave={c[name] / w:.1f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
            line.append(f"wait_any_frac={c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_INST_ANY" in c:
            line.append(f"wait_inst_frac={c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAVE_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # waves resident per SIMD on average while the GPU was busy: wave quad-cycles x 4 over
            # (GUI_ACTIVE summed over 8 XCDs / 8) x 1024 SIMDs
            line.append(f"waves_per_simd={c['SQ_WAVE_CYCLES'] * 4 / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
        if "SQ_WAVES" in c:
            line.append(f"waves/dispatch={c['SQ_WAVES'] / ndisp:.0f}")
        if dur.get(k):
            line.append(f"avg_us={sum(dur[k]) / len(dur[k]):.2f} (n={len(dur[k])})")
        print("\n  ".join(line))


if __name__ == "__main__":
    main()
