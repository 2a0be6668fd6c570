#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd SQLite) into a
per-kernel table (calls, total/avg/min/max duration, VGPRs, scratch), and
optionally a JSON of per-kernel average durations (bench.py reads the
committed copy, profiles/rocprof_kernel_avg.json, to set its live hipEvent
roofline figure beside the rocprof one)."""
import json
import sqlite3
import sys


def _lib_sha():
    """sha256 (16 hex) of the in-tree libblsmi355x.so that was profiled: bench.py reports the rocprof figures
    only for the same build"""
    import hashlib
    import os
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "eth-consensus-specs_amd",
                       "libblsmi355x.so")
    try:
        return hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def main(db, out=None, out_json=None, source=None):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(scratch_size), max(grid_x), max(workgroup_x) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats summary of {db}",
             "| kernel | calls | total ms | avg ms | min ms | max ms | % | VGPR | AGPR | scratch B/lane | grid | wg |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for name, n, tot, avg, mn, mx, vg, ag, scr, gx, wg in rows:
        short = name.split("(")[0].replace("void ", "")
        lines.append(f"| {short} | {n} | {tot/1e6:.3f} | {avg/1e6:.4f} | {mn/1e6:.4f} | {mx/1e6:.4f} | "
                     f"{100*tot/total:.1f} | {vg} | {ag} | {scr} | {gx} | {wg} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    if out_json:
        sym = lambda n: n.split("(")[0].replace("void ", "").replace("bls::", "")  # noqa: E731
        avg = {sym(r[0]): round(r[3] / 1e6, 4) for r in rows}
        # per (kernel, grid): one kernel launched at several sizes (e.g. k_miller_acc4q<2> for C2's 10,000 pairs
        # and C4's 125,000) has one average per launch size; bench.py reads the entry of its own launch
        by_grid: dict = {}
        for name, grid, n, a in c.execute("select name, grid_x, count(*), avg(duration) from kernels "
                                          "group by name, grid_x"):
            by_grid.setdefault(sym(name), {})[str(grid)] = {"calls": n, "avg_ms": round(a / 1e6, 4)}
        with open(out_json, "w") as fh:
            json.dump({"source": source or out or db, "avg_ms": avg, "avg_ms_by_grid": by_grid,
                       "lib_sha256_16": _lib_sha()}, fh, indent=1, sort_keys=True)
    print(text)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1] if len(a) > 1 else None, a[2] if len(a) > 2 else None, a[3] if len(a) > 3 else None)
