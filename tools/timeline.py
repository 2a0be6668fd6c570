#!/usr/bin/env python3
"""Concurrency view of a rocprofv3 --kernel-trace database over the bench's timed region.

The window runs from the start of the (skip+1)-th to the end of the (skip+steps)-th dispatch of the
anchor kernel (one per FAV batch).  Reports the fraction of the window with >= 1 kernel running, the
time-averaged number of concurrent kernels, and per kernel its summed duration and wave-milliseconds
(waves x duration: what the launch asks of the chip while it runs).
Usage: timeline.py DB [anchor-substring] [skip] [steps]"""
import sqlite3
import sys


def main(db, anchor="k_miller_acc4", skip=2, steps=40):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    anc = [r for r in rows if anchor in r[0]]
    if len(anc) < skip + steps:
        raise SystemExit(f"{len(anc)} anchor dispatches, need {skip + steps}")
    t0, t1 = anc[skip][1], anc[skip + steps - 1][2]
    win = [(n, max(s, t0), min(e, t1), gx, wg) for n, s, e, gx, wg in rows if e > t0 and s < t1]
    ev = sorted([(s, 1) for _, s, _, _, _ in win] + [(e, -1) for _, _, e, _, _ in win])
    busy = area = 0
    cur, last = 0, t0
    for t, d in ev:
        if cur > 0:
            busy += t - last
        area += cur * (t - last)
        cur += d
        last = t
    span = t1 - t0
    per = {}
    for n, s, e, gx, wg in win:
        k = n.split("(")[0].replace("void ", "").replace("bls::", "")
        p = per.setdefault(k, [0, 0.0, 0])
        p[0] += e - s
        p[1] += (gx / 64) * (e - s) / 1e6
        p[2] += 1
    print(f"window {span/1e6:.2f} ms over {steps} batches ({span/1e6/steps:.3f} ms/batch); busy {100*busy/span:.1f} %; "
          f"mean concurrent kernels {area/span:.2f}")
    print("| kernel | calls | ms/batch | wave-ms/batch | share of wave-ms |")
    print("|---|---|---|---|---|")
    tot = sum(p[1] for p in per.values())
    for k, (d, w, n) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"| {k} | {n} | {d/1e6/steps:.3f} | {w/steps:.0f} | {100*w/tot:.1f} % |")
    print(f"total wave-ms/batch {tot/steps:.0f}; chip = 1024 SIMDs x {span/1e6/steps:.3f} ms = "
          f"{1024*span/1e6/steps:.0f} SIMD-ms/batch")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1] if len(a) > 1 else "k_miller_acc4", int(a[2]) if len(a) > 2 else 2,
         int(a[3]) if len(a) > 3 else 40)
