#!/usr/bin/env python3
"""Per-kernel wave residency from a rocprofv3 --pmc counter_collection.csv that holds SQ_WAVES and SQ_WAVE_CYCLES
(quad-cycles, 2.4 GHz): mean ms a wave of the kernel stays resident, and the sampled SIMD-ms per dispatch.  In a
pipeline of one-wave-per-SIMD kernels the chip is slot-bound, and residency x waves is what a kernel costs it."""
import collections
import csv
import sys


def main(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("bls::", "")
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    print("| kernel | dispatches | sampled waves/dispatch | ms resident per wave | sampled SIMD-ms/dispatch | VALU/wave |")
    print("|---|---|---|---|---|---|")
    for k in sorted(acc, key=lambda k: -acc[k]["SQ_WAVE_CYCLES"]):
        n = len(disp[k])
        w = acc[k]["SQ_WAVES"] / n
        wc = acc[k]["SQ_WAVE_CYCLES"] / n * 4 / 2.4e6
        if wc < 0.5:
            continue
        print(f"| {k} | {n} | {w:.0f} | {wc / max(w, 1):.3f} | {wc:.1f} | {acc[k]['SQ_INSTS_VALU'] / n / max(w, 1):.0f} |")


if __name__ == "__main__":
    main(sys.argv[1])
