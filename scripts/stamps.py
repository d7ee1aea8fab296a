#!/usr/bin/env python3
"""Per-tile phase timeline of the pass kernel from a -DTHRS_STAMPS build
(build/variants/libthrs_stamps.so).  Stamps are s_memrealtime (100 MHz):
  0 entry, 1 tile id known, 2 keys loaded, 3 ranked (+barrier),
  4 scan+LDS scatter done (thread 0), 5 look-back done (+barrier),
  6 write-out drained (thread 0); slot 7 = XCC id.
usage: python scripts/stamps.py [--workload c2] [--n N]
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
from sweep import WL, load  # noqa: E402

NAMES = ["tileid", "load+hist", "agg+scan", "rank", "lookback", "writeout"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "variants", "libthrs_stamps.so"))
    a = ap.parse_args()
    kt, vb, n = WL[a.workload]
    n = a.n or n
    kb = 4 if kt in (0, 2) else 8
    L = load(a.lib)
    L.thrs_debug_set_stamps.argtypes = [ctypes.c_void_p]
    cfg = T._CConfig(1, kt, {0: 0, 4: 0, 8: 1, 16: 2}[vb], 0)
    d = T._CTempDef()
    L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
    tmp = torch.empty(d.pSumBuffer + d.keyOutBuffer + d.valueOutBuffer, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
    vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
    L.thrs_debug_tile_keys.argtypes = [ctypes.c_int, ctypes.c_int]
    L.thrs_debug_tile_keys.restype = ctypes.c_uint64
    tile = int(L.thrs_debug_tile_keys(kt, vb))
    ntiles = (n + tile - 1) // tile
    passes = kb
    stamps = torch.zeros(passes * ntiles * 24, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    for it in range(2):
        TU.fill_keys(kt, keys, n, start=it * n)
        if vb:
            TU.iota(vb, vals, n)
        L.thrs_debug_set_stamps(stamps.data_ptr() if it == 1 else None)
        torch.cuda.synchronize()
        if vb:
            rc = L.thrs_sort_pairs(ctypes.byref(cfg), keys.data_ptr(), vals.data_ptr(), n, tmp.data_ptr(), 0, kb * 8,
                                   s.cuda_stream)
        else:
            rc = L.thrs_sort_keys(ctypes.byref(cfg), keys.data_ptr(), n, tmp.data_ptr(), 0, kb * 8, s.cuda_stream)
        torch.cuda.synchronize()
        assert rc == 0
    L.thrs_debug_set_stamps(None)
    st = stamps.cpu().numpy().reshape(passes, ntiles, 24)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "stamps_pass0.npy"), st[0])
    report = {"n": n, "tile": tile, "ntiles": ntiles, "passes": []}
    for p in range(passes):
        a_ = st[p].astype(np.int64)
        t0 = a_[:, 0].min()
        dur = {}
        for i in range(6):
            x = (a_[:, i + 1] - a_[:, i]) * 10.0 / 1000.0   # 100 MHz ticks -> us
            dur[NAMES[i]] = {"med_us": round(float(np.median(x)), 3), "p90_us": round(float(np.percentile(x, 90)), 3),
                             "mean_us": round(float(x.mean()), 3)}
        life = (a_[:, 6] - a_[:, 0]) * 0.01
        span = (a_[:, 6].max() - t0) * 0.01
        # tiles in flight over time (sampled)
        ts = np.linspace(t0, a_[:, 6].max(), 200)
        inflight = [int(((a_[:, 0] <= t) & (a_[:, 6] > t)).sum()) for t in ts[20:180:20]]
        # dispatch order vs tile id
        order_lag = (a_[:, 1] - a_[:, 0]) * 0.01
        xcc = a_[:, 7] & 0xFF
        rounds = (a_[:, 7] >> 8) & 0xFFFF
        depth = (a_[:, 7] >> 24) & 0xFFFF
        stalls = (a_[:, 7] >> 40) & 0xFFFFFF
        # look-back dynamics: lag = tile id -> own prefix published; age of the
        # predecessor prefix that ended the walk, at the moment the walk ended
        lag = (a_[:, 5] - a_[:, 1]) * 0.01
        ids = np.arange(ntiles)
        pred = ids - 1 - depth
        ok = (pred >= 0) & (ids > 0)
        age = (a_[ids[ok], 5] - a_[pred[ok], 5]) * 0.01
        if age.size == 0:
            age = np.zeros(1)
        walk_start = (a_[:, 4] - a_[:, 0]) * 0.01
        frontier = {"lag_med_us": round(float(np.median(lag)), 2), "lag_p90_us": round(float(np.percentile(lag, 90)), 2),
                    "found_prefix_age_med_us": round(float(np.median(age)), 2),
                    "found_prefix_age_p10_us": round(float(np.percentile(age, 10)), 2),
                    "walk_start_after_entry_med_us": round(float(np.median(walk_start)), 2),
                    "tiles_per_us": round(ntiles / float(span), 2)}
        walk = {}

        def q(x):
            return {"med_us": round(float(np.median(x)), 3), "p90_us": round(float(np.percentile(x, 90)), 3)}
        m = (a_[:, 16] > 0) & (a_[:, 17] > 0) & (a_[:, 18] > 0)
        if m.any():
            walk = {"rank_end_to_walk_issue": q((a_[m, 16] - a_[m, 4]) * 0.01),
                    "first_window_roundtrip": q((a_[m, 17] - a_[m, 16]) * 0.01),
                    "rest_of_walk": q((a_[m, 18] - a_[m, 17]) * 0.01),
                    "walk_end_to_barrier": q((a_[m, 5] - a_[m, 18]) * 0.01)}
        we, ba = a_[:, 8:12], a_[:, 12:16]
        m = (we > 0).all(axis=1) & (ba > 0).all(axis=1)
        if m.any():
            walk["walk_end_per_wave_med_after_rank"] = [round(float(np.median((we[m, i] - a_[m, 4]) * 0.01)), 2)
                                                        for i in range(4)]
            walk["barrier_arrival_per_wave_med_after_rank"] = [
                round(float(np.median((ba[m, i] - a_[m, 4]) * 0.01)), 2) for i in range(4)]
            walk["barrier_release_after_rank"] = q((a_[m, 5] - a_[m, 4]) * 0.01)
        report["passes"].append({"pass": p, "kernel_span_us": round(float(span), 1), "frontier": frontier, "walk": walk,
                                 "tile_life_med_us": round(float(np.median(life)), 2),
                                 "tile_life_p90_us": round(float(np.percentile(life, 90)), 2),
                                 "phases": dur, "inflight_samples": inflight,
                                 "max_rounds_med": float(np.median(rounds)), "max_rounds_p90": float(np.percentile(rounds, 90)),
                                 "max_depth_med": float(np.median(depth)), "max_depth_p90": float(np.percentile(depth, 90)),
                                 "max_stalls_med": float(np.median(stalls)), "max_stalls_p90": float(np.percentile(stalls, 90)),
                                 "xcc_hist": np.bincount(xcc.astype(np.int64), minlength=8).tolist(),
                                 "start_spread_first_1024_us": round(float((a_[:1024, 0].max() - a_[:1024, 0].min()) * 0.01), 2)})
        print(json.dumps(report["passes"][-1]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(report, open(os.path.join(ROOT, "gpurun_out", "stamps.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
