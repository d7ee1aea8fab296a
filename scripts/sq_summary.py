#!/usr/bin/env python3
"""Per-kernel averages of the SQ counters collected by scripts/sqprof.sh
(kernels keyed by their demangled name, template arguments included)."""
import glob
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(__file__))
from prof_summary import col, read_csv  # noqa: E402

d = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in read_csv(p):
        name = col(r, "Kernel_Name", "Kernel-Name", "KernelName").replace("thrs_dev::", "").replace(
            "(anonymous namespace)::", "").split("(")[0]
        disp = col(r, "Dispatch_Id", "Dispatch-Id", "DispatchId", "Correlation_Id")
        per[(name, p, disp)][col(r, "Counter_Name", "Counter-Name", "CounterName")] += float(
            col(r, "Counter_Value", "Counter-Value", "CounterValue"))
agg = defaultdict(lambda: defaultdict(list))
for (name, _, _), cs in per.items():
    for c, v in cs.items():
        agg[name][c].append(v)
for name, cs in sorted(agg.items()):
    if "thrs" not in name:
        continue
    vals = {c: statistics.median(v) for c, v in cs.items()}
    if vals.get("SQ_WAVES", 1e9) < 1000 and "plan" not in name:
        continue
    print(name[:90])
    print("   " + "  ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(vals.items())))
