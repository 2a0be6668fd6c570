#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel: counters
averaged over dispatches, plus per-wave instruction counts and the
issue / wait split of wave cycles (SQ_* cycle counters are quad-cycles).
With the LDS / occupancy pass (SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE,
GRBM_GUI_ACTIVE): the bank-conflict share of LDS cycles (conflict cycles /
all LDS-array cycles, MI355X_MICROARCH.md "LDS") and the mean resident waves
per SIMD = 4 SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs) / 1024 SIMDs."""
import csv
import sys
from collections import defaultdict


def main(path, out=None):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
        dur[k][row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    lds_pass = any("SQ_LDS_IDX_ACTIVE" in acc[k] for k in acc)
    fetch_pass = any("FETCH_SIZE" in acc[k] for k in acc)
    if fetch_pass:  # FETCH_SIZE is in KB (MI355X_MICROARCH.md, rocprofv3 section)
        # gfx950: FETCH_SIZE = TCC_EA0_RDREQ x 64 B while the requests are 128 B, so a 16-B-per-lane read (every
        # bulk load of these kernels: registry records, line records) reports half its bytes -- doubled here
        lines = [f"# rocprofv3 --pmc FETCH_SIZE summary of {path} (per dispatch averages; 'corrected' = x2, the "
                 "gfx950 correction for 16-B/lane reads, MI355X_MICROARCH.md HBM section)",
                 "| kernel | disp | ms | FETCH_SIZE KB/dispatch (raw) | MB/dispatch (raw) | MB/dispatch (corrected) | "
                 "GB/s (corrected) |",
                 "|---|---|---|---|---|---|---|"]
        for k in sorted(acc, key=lambda k: -sum(dur[k].values())):
            n = len(disp[k])
            kb = acc[k].get("FETCH_SIZE", 0) / n
            ms = sum(dur[k].values()) / n
            lines.append(f"| {k} | {n} | {ms:.3f} | {kb:.0f} | {kb * 1024 / 1e6:.2f} | {2 * kb * 1024 / 1e6:.2f} | "
                         f"{2 * kb * 1024 / (ms * 1e-3) / 1e9 if ms else 0:.1f} |")
        text = "\n".join(lines) + "\n"
        if out:
            open(out, "w").write(text)
        print(text)
        return
    if lds_pass:
        lines = [f"# rocprofv3 --pmc LDS / occupancy summary of {path} (per dispatch averages)",
                 "| kernel | disp | ms | waves | LDS instr/wave | LDS-array cycles | bank-conflict cycles | "
                 "conflict % of LDS cycles | mean waves/SIMD |",
                 "|---|---|---|---|---|---|---|---|---|"]
    else:
        lines = [f"# rocprofv3 --pmc summary of {path} (per dispatch averages)",
                 "| kernel | disp | ms | waves | VALU/wave | SALU/wave | LDS/wave | active% | wait% | issue-stall% |",
                 "|---|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(acc, key=lambda k: -sum(dur[k].values())):
        c = acc[k]
        n = len(disp[k])
        w = c.get("SQ_WAVES", 0) or 1
        cyc = c.get("SQ_WAVE_CYCLES", 0) or 1
        if lds_pass:
            idx = c.get("SQ_LDS_IDX_ACTIVE", 0)
            bc = c.get("SQ_LDS_BANK_CONFLICT", 0)
            gui = c.get("GRBM_GUI_ACTIVE", 0)
            occ = 4 * cyc / (gui / 8) / 1024 if gui else float("nan")
            lines.append(f"| {k} | {n} | {sum(dur[k].values()) / n:.3f} | {w / n:.0f} | "
                         f"{c.get('SQ_INSTS_LDS', 0) / w:.0f} | {idx / n:.3g} | {bc / n:.3g} | "
                         f"{100 * bc / idx if idx else 0:.1f} | {occ:.2f} |")
            continue
        lines.append(
            f"| {k} | {n} | {sum(dur[k].values()) / n:.3f} | {w / n:.0f} | {c.get('SQ_INSTS_VALU', 0) / w:.0f} | "
            f"{c.get('SQ_INSTS_SALU', 0) / w:.0f} | {c.get('SQ_INSTS_LDS', 0) / w:.0f} | "
            f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.1f} | {100 * c.get('SQ_WAIT_ANY', 0) / cyc:.1f} | "
            f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / cyc:.1f} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
