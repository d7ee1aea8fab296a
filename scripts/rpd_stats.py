#!/usr/bin/env python3
"""Per-kernel summary (count, mean/median us, total ms, scratch) of a
rocprofv3 --kernel-trace database (rocpd sqlite: <dir>/*_results.db).
usage: python scripts/rpd_stats.py gpurun_out/pr_main [--skip 0]"""
import glob
import sqlite3
import statistics
import sys


def stats(d):
    db = sorted(glob.glob(f"{d}/**/*results.db", recursive=True))[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, scratch_size, vgpr_count from kernels order by start").fetchall()
    agg = {}
    for name, dur, gx, gy, scr, vg in rows:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        a = agg.setdefault(short, {"n": 0, "d": [], "scratch": scr, "vgpr": vg, "grid": (gx, gy)})
        a["n"] += 1
        a["d"].append(dur / 1e3)
    return agg


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print("==", d)
        agg = stats(d)
        for k, a in sorted(agg.items(), key=lambda kv: -sum(kv[1]["d"])):
            print(f"{sum(a['d'])/1e3:9.3f} ms  n={a['n']:4d}  mean={statistics.mean(a['d']):9.2f} us  "
                  f"med={statistics.median(a['d']):9.2f}  scr={a['scratch']} vgpr={a['vgpr']} grid={a['grid']}  {k[:110]}")
