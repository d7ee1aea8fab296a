#!/usr/bin/env python3
"""rocprof-vs-event gap: for a scripts/profile.sh directory, the per-launch
times bench.py measured with HIP events (its bench line, run under rocprofv3)
against the kernel durations rocprofv3 recorded for the same command
(bench/run_kernel_trace.csv; launches under 20 us -- gated no-ops -- left out).
usage: python scripts/event_gap.py gpurun_out/prof_r05_c2 [...]"""
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    n = name.replace("thrs_dev::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main():
    for d in sys.argv[1:]:
        b = json.load(open(os.path.join(d, "bench.json")))
        tr = glob.glob(os.path.join(d, "bench", "*kernel_trace.csv"))[0]
        durs = {}
        for r in csv.DictReader(open(tr)):
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if us >= 20 and "thrs_" in r["Kernel_Name"]:
                durs.setdefault(short(r["Kernel_Name"]), []).append(us)
        kinds = b["roofline"]["kinds"]
        ev = {"pass": kinds["pass"].get("by_launch_ms") or [kinds["pass"]["avg_launch_ms"]],
              "local": [kinds["local"]["avg_launch_ms"]]}
        prof = {k: round(statistics.mean(v) / 1e3, 4) for k, v in durs.items()}
        print(json.dumps({"dir": d, "ms_per_step_under_rocprof": b["ms_per_step"], "events_ms": ev,
                          "rocprof_ms": prof}))


if __name__ == "__main__":
    main()
