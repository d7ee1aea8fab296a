#!/usr/bin/env python3
"""Workload run under rocprofv3 (one process): calibration copies with known
byte counts (1 GiB at 16 B/lane and at 4 B/lane), then K sorts of the bench
workload (fresh inputs).  The profiler attributes per-kernel time and counters;
scripts/prof_summary.py turns them into profiles/*.json."""
import argparse
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402

from bench import WORKLOADS  # noqa: E402  (name -> key type, value bytes, n, distribution, description)

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
kt, vb, n, dist, _desc = WORKLOADS[a.workload]
kb = 4 if kt in (0, 2) else 8
G = 1 << 30
src = torch.empty(G, dtype=torch.uint8, device="cuda")
dst = torch.empty(G, dtype=torch.uint8, device="cuda")
TU.fill_keys(0, src, G // 4)
for w16 in (1, 0):
    for _ in range(2):
        TU.copy(dst, src, G, bool(w16))
torch.cuda.synchronize()
del src, dst
cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32, 8: T.ValueType.U64,
                                                                   16: T.ValueType.U128}[vb])
rs = T.RadixSort([], cfg)
d = rs.getTemporaryBufferBytes(n)
tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs() if vb else d.getTemporaryBufferBytesForSortKeys(),
                  dtype=torch.uint8, device="cuda")
keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
for s in range(a.steps + 1):
    if dist == "uniform":
        TU.fill_keys(kt, keys, n, start=s * n)
    else:
        TU.fill_dist(kt, keys, n, dist, start=s * n)
    if vb:
        TU.iota(vb, vals, n)
        rs.sortPairs(keys, vals, n, tmp, 0, kb * 8)
    else:
        rs.sortKeys(keys, n, tmp, 0, kb * 8)
torch.cuda.synchronize()
assert TU.count_unsorted(kt, keys, n, 0, kb * 8) == 0
print("profile_run ok", a.workload, n)
