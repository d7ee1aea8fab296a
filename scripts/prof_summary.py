#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into JSON.

* kernel durations: from the --kernel-trace/--stats pass (average ns per
  dispatch, by kernel family).
* HBM bytes: FETCH_SIZE / WRITE_SIZE (KiB units) from their own --pmc passes,
  CALIBRATED against the known-byte copies profile_run.py performs first
  (1 GiB read + 1 GiB written per dispatch at 16 B/lane and at 4 B/lane):
  the MI355X guide notes FETCH_SIZE reads exactly half of a 16-B streaming read
  on gfx950 and other widths are uncalibrated, so each kernel's raw counter is
  scaled by the factor of the copy with its dominant access width.
usage: python scripts/prof_summary.py <dir>  (prints JSON)
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

FAMILIES = ["thrs_pass_seg", "thrs_pass_xb", "thrs_pass", "thrs_hist_joint", "thrs_hist", "thrs_scan", "thrs_plan",
            "thrs_local_count16", "thrs_local16", "thrs_local64", "thrs_local_pairs", "thrs_local", "thrs_copy_gated", "thrs_digit_hist",
            "thrs_err_publish", "k_fill_dist",
            "k_copy_u128", "k_copy_u32", "k_fill", "k_iota", "k_sorted", "k_fingerprint", "thrs_probe"]
# dominant global access width per family, for counter calibration
WIDTH16 = {"thrs_hist": True, "thrs_hist_joint": True, "k_copy_u128": True}
# launches of the 3-HBM-pass path that exit at once unless the fallback flag
# is set (the low-digit passes and their histogram): reported apart
GATED = ("thrs_pass", "thrs_hist", "thrs_pass_seg", "thrs_hist_joint")  # pass_seg: the fallback-only (mode 1) launch; hist_joint: the squeeze's second histogram
GATED_NS = 100_000           # shorter than this = a gated launch that exited
GATED_KIB = 1024             # FETCH_SIZE / WRITE_SIZE below 1 MiB = the same
GIB = 1 << 30


def family(name: str) -> str:
    for f in FAMILIES:
        if f in name:
            return f
    return name[:60]


def find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(f"none of {names} in {list(row)[:12]}")


def durations(d):
    out = defaultdict(list)
    for p in find(d, "*kernel_trace.csv"):
        for r in read_csv(p):
            name = col(r, "Kernel_Name", "Kernel-Name", "KernelName")
            t0 = int(col(r, "Start_Timestamp", "Start-Timestamp", "BeginNs"))
            t1 = int(col(r, "End_Timestamp", "End-Timestamp", "EndNs"))
            fam = family(name)
            if fam in GATED and t1 - t0 < GATED_NS:
                fam += "_gated"
            out[fam].append(t1 - t0)
    return out


def counters(d):
    """family -> counter -> list of per-dispatch values (summed over dimensions)."""
    per = defaultdict(lambda: defaultdict(float))   # (family, dispatch, counter) -> value
    for p in find(d, "*counter_collection.csv"):
        for r in read_csv(p):
            name = col(r, "Kernel_Name", "Kernel-Name", "KernelName")
            disp = col(r, "Dispatch_Id", "Dispatch-Id", "DispatchId", "Correlation_Id")
            cname = col(r, "Counter_Name", "Counter-Name", "CounterName")
            val = float(col(r, "Counter_Value", "Counter-Value", "CounterValue"))
            per[(family(name), disp)][cname] += val
    out = defaultdict(lambda: defaultdict(list))
    for (fam, _), cs in per.items():
        if fam in GATED and all(v < (GATED_KIB if c in ("FETCH_SIZE", "WRITE_SIZE") else 1e5) for c, v in cs.items()):
            fam += "_gated"
        for c, v in cs.items():
            out[fam][c].append(v)
    return out


def main(d):
    res = {"dir": d, "kernels": {}, "calibration": {}}
    dur = durations(os.path.join(d, "trace"))
    for fam, xs in dur.items():
        res["kernels"].setdefault(fam, {})
        res["kernels"][fam].update({"calls": len(xs), "avg_ns": round(statistics.mean(xs)),
                                    "min_ns": min(xs), "max_ns": max(xs)})
    raw = {}
    for sub in sorted(glob.glob(os.path.join(d, "pmc_*"))):
        if not os.path.isdir(sub):
            continue
        for fam, cs in counters(sub).items():
            for c, vals in cs.items():
                raw.setdefault(fam, {})[c] = statistics.mean(vals)
    # calibration: copies move exactly 1 GiB in and 1 GiB out per dispatch
    cal = {}
    for fam in ("k_copy_u128", "k_copy_u32"):
        c = raw.get(fam, {})
        if c.get("FETCH_SIZE"):
            cal[fam + ".fetch"] = GIB / (c["FETCH_SIZE"] * 1024.0)
        if c.get("WRITE_SIZE"):
            cal[fam + ".write"] = GIB / (c["WRITE_SIZE"] * 1024.0)
    res["calibration"] = {k: round(v, 4) for k, v in cal.items()}
    for fam, c in raw.items():
        k = res["kernels"].setdefault(fam, {})
        k["raw"] = {n: round(v, 1) for n, v in c.items()}
        ref = "k_copy_u128" if WIDTH16.get(fam) else "k_copy_u32"
        fb = c.get("FETCH_SIZE")
        wb = c.get("WRITE_SIZE")
        if fb is not None:
            k["fetch_bytes"] = round(fb * 1024.0 * cal.get(ref + ".fetch", 1.0))
        if wb is not None:
            k["write_bytes"] = round(wb * 1024.0 * cal.get(ref + ".write", 1.0))
        if fb is not None and wb is not None:
            k["hbm_bytes"] = k["fetch_bytes"] + k["write_bytes"]
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            k["l2_hit_rate"] = round(h / (h + m), 4)
        if "avg_ns" in k and "hbm_bytes" in k:
            k["hbm_GBps"] = round(k["hbm_bytes"] / k["avg_ns"], 1)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
