#!/usr/bin/env python3
"""Per-launch timeline of one sort from a rocprofv3 kernel trace: every
kernel of the last sort (from its thrs_zero_ranges on), its duration and the
idle gap before it.  usage: python scripts/gaps.py <dir with *kernel_trace.csv> [--sort -1]"""
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    which = int(sys.argv[sys.argv.index("--sort") + 1]) if "--sort" in sys.argv else -1
    path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "thrs_zero_ranges" in r["Kernel_Name"]]
    i0 = starts[which]
    i1 = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
    seq = [r for r in rows[i0:i1] if "thrs_" in r["Kernel_Name"]]
    t0 = int(seq[0]["Start_Timestamp"])
    prev = t0
    out = []
    for r in seq:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        out.append({"kernel": r["Kernel_Name"].split("(")[0][:60], "start_us": round((s - t0) / 1e3, 2),
                    "dur_us": round((e - s) / 1e3, 2), "gap_us": round((s - prev) / 1e3, 2)})
        prev = e
    for o in out:
        print(json.dumps(o))
    tot = (prev - t0) / 1e3
    busy = sum(o["dur_us"] for o in out)
    print(json.dumps({"launches": len(out), "span_us": round(tot, 1), "busy_us": round(busy, 1),
                      "gaps_us": round(tot - busy, 1),
                      "small_us": round(sum(o["dur_us"] for o in out if o["dur_us"] < 50), 1)}))


if __name__ == "__main__":
    main()
