#!/usr/bin/env python3
"""Write tools/pmc_traffic.json from a rocprofv3 --pmc FETCH_SIZE pass (build-time tool).

bytes_per_dispatch[k] = FETCH_SIZE (KB) x 1024 x 2 averaged over the dispatches of the kernel bench.py's
profile entry k names: the x2 is the gfx950 correction for 16-B-per-lane reads (MI355X_MICROARCH.md, HBM
section: FETCH_SIZE tallies the 128-B requests at 64 B), which tools/microbench/fetchcal.hip measured to hold for
4-B-per-lane coalesced reads too (profiles/r05r_fetchcal.txt: a 1 GiB read reports exactly 1/2).  The file records the libblsmi355x.so hash of the
profiled build; bench.py reports `traffic` only when it matches the library it runs.
Usage: python3 tools/pmc_traffic.py <fetch counter_collection.csv> <source label> <lib sha256_16>"""
import csv
import json
import os
import sys
from collections import defaultdict

SYMBOLS = {"miller": "k_miller_acc4q<4>", "miller_lines": "k_miller_lines2", "fav_gather": "k_fav_gather_q<16>"}


def main(path, label, sha):
    kb, disp = defaultdict(float), defaultdict(set)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != "FETCH_SIZE":
            continue
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("bls::", "")
        kb[k] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    out = {"source": f"{label} (rocprofv3 --pmc FETCH_SIZE in KB x 1024 x 2: the gfx950 read correction, which holds "
                     "for these kernels' 4-B/lane loads too: profiles/r05r_fetchcal.txt)",
           "lib_sha256_16": sha,
           "bytes_per_dispatch": {e: round(kb[s] * 1024 * 2 / len(disp[s])) for e, s in SYMBOLS.items() if disp[s]}}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_traffic.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:4])
