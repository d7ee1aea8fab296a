#!/usr/bin/env python3
"""Per-tile phase timeline of the bucket path's two segmented top-digit passes
(thrs_pass_seg) from a -DTHRS_STAMPS build (exp/variants/libthrs_stamps.so).

Pass 0 = pass A (second digit, position segments, split codec), pass 1 = pass
B (top digit, second-digit segments, planes codec).  Stamps (s_memrealtime,
100 MHz) per tile id (segment chain + ticket):
  0 claim, 1 keys issued, 2 counted (+barrier), 3 scanned, 4 ranked + staged,
  5 look-back done (+barrier), 6 write-out drained; 7 = xcc | seg << 4 |
  max rounds << 8 | max depth << 24 | max stalls << 40; 8..11 walk end per
  walker wave; 12..15 barrier arrival per walker wave; 16 walk start, 17 first
  window consumed (digit 0's thread).
usage: python scripts/seg_stamps.py [--n N] [--opt planes=off] [--out gpurun_out/seg_stamps.json]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402
from sweep import load  # noqa: E402

NAMES = ["claim+issue", "load+count", "scan", "rank+stage", "lookback", "writeout"]
SEG_PAD = 8 * 17  # kSegTilePad


def q(x):
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return None
    return {"med": round(float(np.median(x)), 2), "p10": round(float(np.percentile(x, 10)), 2),
            "p90": round(float(np.percentile(x, 90)), 2), "mean": round(float(x.mean()), 2)}


def analyse(a, tile):
    used = a[:, 0] > 0
    ids = np.nonzero(used)[0]
    a = a[used].astype(np.int64)
    t0 = a[:, 0].min()
    us = lambda x: x * 0.01  # noqa: E731
    rep = {"tiles": int(len(ids)), "span_us": round(float(us(a[:, 6].max() - t0)), 1)}
    rep["phases_us"] = {NAMES[i]: q(us(a[:, i + 1] - a[:, i])) for i in range(6)}
    rep["life_us"] = q(us(a[:, 6] - a[:, 0]))
    seg = (a[:, 7] >> 4) & 0xF
    xcc = a[:, 7] & 0xF
    rounds = (a[:, 7] >> 8) & 0xFFFF
    depth = (a[:, 7] >> 24) & 0xFFFF
    stalls = (a[:, 7] >> 40) & 0xFFFFFF
    rep["stolen_frac"] = round(float((seg != xcc).mean()), 4)
    m = (a[:, 16] > 0) & (a[:, 17] > 0)
    rep["walk_us"] = {"rank_end_to_walk_start": q(us(a[m, 16] - a[m, 4])),
                      "first_round": q(us(a[m, 17] - a[m, 16])),
                      "rest": q(us(a[m, 5] - a[m, 17]))}
    # per segment: how tiles progress, walk length, depth, stalls
    per = []
    for s in range(8):
        k = seg == s
        if not k.any():
            per.append(None)
            continue
        b = a[k]
        order = np.argsort(b[:, 0])
        per.append({"tiles": int(k.sum()), "stolen": int((xcc[k] != s).sum()),
                    "first_claim_us": round(float(us(b[:, 0].min() - t0)), 1),
                    "last_done_us": round(float(us(b[:, 6].max() - t0)), 1),
                    "lookback_us": q(us(b[:, 5] - b[:, 4])), "life_us": q(us(b[:, 6] - b[:, 0])),
                    "rounds": q(rounds[k]), "depth": q(depth[k]), "stalls": q(stalls[k]),
                    # claim-to-claim interval within the segment (dispatch rate)
                    "claim_gap_us": q(us(np.diff(b[order, 0])))})
    rep["per_segment"] = per
    rep["rounds"], rep["depth"], rep["stalls"] = q(rounds), q(depth), q(stalls)
    # tiles in flight and CU concurrency over time
    ts = np.linspace(t0, a[:, 6].max(), 50)[5:45:5]
    rep["inflight"] = [int(((a[:, 0] <= t) & (a[:, 6] > t)).sum()) for t in ts]
    # tiles whose walk waited for a predecessor that had not published yet:
    # time from own rank end to predecessor-in-chain (id-1) aggregate (stamp 2)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--opt", default="")
    ap.add_argument("--lib", default=os.path.join(ROOT, "exp", "variants", "libthrs_stamps.so"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "seg_stamps.json"))
    a = ap.parse_args()
    n = a.n
    L = load(a.lib)
    L.thrs_debug_set_stamps.argtypes = [ctypes.c_void_p]
    L.thrs_debug_tile_keys.argtypes = [ctypes.c_int, ctypes.c_int]
    L.thrs_debug_tile_keys.restype = ctypes.c_uint64
    L.thrs_sort_keys_ex.argtypes = [ctypes.POINTER(T._CConfig), ctypes.POINTER(T._COptions), ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    o = T.Options()
    for kv in filter(None, a.opt.split(",")):
        k, v = kv.split("=")
        setattr(o, k, v)
    cfg = T._CConfig(1, 0, 0, 0)
    d = T._CTempDef()
    L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
    tmp = torch.empty(d.pSumBuffer + d.keyOutBuffer, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    tile = int(L.thrs_debug_tile_keys(0, 0))
    rows = (n + tile - 1) // tile + SEG_PAD
    stamps = torch.zeros(2 * rows * 24, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    reps = []
    for it in range(3):
        TU.fill_keys(0, keys, n, start=it * n)
        stamps.zero_()
        L.thrs_debug_set_stamps(stamps.data_ptr() if it >= 1 else None)
        torch.cuda.synchronize()
        rc = L.thrs_sort_keys_ex(ctypes.byref(cfg), ctypes.byref(o._c()), keys.data_ptr(), n, tmp.data_ptr(), 0, 32,
                                 s.cuda_stream)
        torch.cuda.synchronize()
        assert rc == 0, rc
        if it >= 1:
            st = stamps.cpu().numpy().reshape(2, rows, 24)
            rep = {"n": n, "tile": tile, "opt": a.opt, "iter": it, "passes": [analyse(st[p], tile) for p in range(2)]}
            reps.append(rep)
            for p in range(2):
                r = rep["passes"][p]
                print(json.dumps({"iter": it, "pass": "AB"[p], "span_us": r["span_us"], "life": r["life_us"],
                                  "phases": {k: v["med"] for k, v in r["phases_us"].items()},
                                  "walk": r["walk_us"], "depth": r["depth"], "stalls": r["stalls"],
                                  "stolen": r["stolen_frac"], "inflight": r["inflight"]}), flush=True)
    L.thrs_debug_set_stamps(None)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(reps, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
