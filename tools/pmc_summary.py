#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel: counters
averaged over dispatches, plus per-wave instruction counts and the
issue / wait split of wave cycles (SQ_* cycle counters are quad-cycles)."""
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
    lines = [f"# rocprofv3 --pmc summary of {path} (per dispatch averages)",
             "| kernel | disp | ms | waves | VALU/wave | SALU/wave | LDS/wave | active% | wait% | issue-stall% |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(acc, key=lambda k: -sum(dur[k].values())):
        c = acc[k]
        n = len(disp[k])
        w = c.get("SQ_WAVES", 0) or 1
        cyc = c.get("SQ_WAVE_CYCLES", 0) or 1
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
