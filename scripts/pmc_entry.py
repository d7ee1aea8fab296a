#!/usr/bin/env python3
"""Add / refresh a profiles/pmc_traffic.json entry from a scripts/profile.sh
summary (scripts/prof_summary.py output): the pass kernel's, the local sort's
and the bucket histogram's HBM bytes per launch (gated no-op launches are
already excluded by prof_summary).
usage: python scripts/pmc_entry.py <workload> <profiles/rNN_x/summary.json> "<kernel version text>"
"""
import json
import sys

wl, src, version = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.load(open(src))
k = d["kernels"]
passes = [v for n, v in k.items() if n.startswith("thrs_pass_seg") or n.startswith("thrs_pass_xb") or n == "thrs_pass"]
if not passes:
    raise SystemExit("no pass kernel in " + src)
p = max(passes, key=lambda v: v["calls"] * v["avg_ns"])
local = {n: v for n, v in k.items() if n.startswith("thrs_local")}
ln, lv = max(local.items(), key=lambda kv: kv[1]["calls"] * kv[1]["avg_ns"]) if local else (None, None)
entry = {"source": src, "kernel_version": version,
         "thrs_pass_bytes_per_launch": p["hbm_bytes"], "thrs_pass_fetch_bytes": p["fetch_bytes"],
         "thrs_pass_write_bytes": p["write_bytes"], "thrs_pass_avg_ns": p["avg_ns"]}
if ln:
    entry.update({"local_kernel": ln, "local_bytes_per_launch": lv["hbm_bytes"], "local_avg_ns": lv["avg_ns"]})
if "thrs_hist_joint" in k:
    entry["thrs_hist_joint_bytes_per_launch"] = k["thrs_hist_joint"]["hbm_bytes"]
entry["calibration"] = d.get("calibration")
entry["method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (scripts/profile.sh); FETCH_SIZE x2 per "
                   "the gfx950 calibration copies, WRITE_SIZE x1; gated (fallback-only) launches excluded; the pass "
                   "figure averages the two top-digit launches")
path = "profiles/pmc_traffic.json"
t = json.load(open(path))
t[wl] = entry
json.dump(t, open(path, "w"), indent=1)
print(wl, json.dumps(entry)[:300])
