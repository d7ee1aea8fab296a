#!/usr/bin/env python3
"""Diagnostic: test_hybrid_paths_vs_oracle's loop for one configuration,
printing every case (dist, n, window) and whether it failed.
usage: python scripts/diag_hybrid.py [--lib path] [--seg none|auto|top_only] [--geom big]"""
import argparse
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--seg", default="none")
ap.add_argument("--geom", default="big")
ap.add_argument("--desc", type=int, default=0)
a = ap.parse_args()
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
if a.lib:
    T.LIB_PATH = os.path.abspath(a.lib)
from oracle import oracle as O  # noqa: E402
from test_gpu_parity import gpu_sort, make_sorter  # noqa: E402

rs = make_sorter(O.U32, 0, bool(a.desc), path="bucket", segmented=a.seg, localGeometry=a.geom)
dists = {
    "uniform": lambda k: k,
    "low20": lambda k: k & np.array(0xFFFFF, k.dtype),
    "top_skew": lambda k: k | np.array(0x7F000000, k.dtype),
    "ties": lambda k: k & np.array(0xFF00FF00, k.dtype),
    "const": lambda k: np.full_like(k, k[0]),
}
j = 0
bad = 0
for name, f in dists.items():
    for n in [1, 100, 18432, 18433, 70001, 300007, 1 << 20]:
        for (s, e) in [(0, 32), (8, 32), (0, 24), (4, 28)]:
            j += 1
            if j % 2 and n >= 300007 and (s, e) != (0, 32):
                continue
            keys = f(O.randomize_np(O.U32, O.splitmix64_stream(7777 * j, n)))
            try:
                k, _ = gpu_sort(torch, rs, {"keys": keys, "values": None}, O.U32, 0, s, e)
                ek, _ = O.lsd_sort(O.U32, keys, None, s, e, bool(a.desc))
                ok = np.array_equal(k, ek)
                msg = "ok" if ok else "MISMATCH"
            except Exception as ex:  # noqa: BLE001
                ok, msg = False, f"ERROR {ex}"
            if not ok:
                bad += 1
                print(name, n, (s, e), msg, flush=True)
print("bad cases:", bad)
