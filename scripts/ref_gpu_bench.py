#!/usr/bin/env python3
"""Time the REFERENCE's own kernels (oracle/_ref: kernel.cu via hipRTC, its
pass loop) on MI355X next to libthrs, same inputs (splitmix64, fresh per run).
usage: python scripts/ref_gpu_bench.py --n 16777216 [--kt 0] [--vb 0] [--runs 3]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 24)
ap.add_argument("--kt", type=int, default=0)
ap.add_argument("--vb", type=int, default=0)
ap.add_argument("--runs", type=int, default=3)
a = ap.parse_args()

import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from oracle import ref as R  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402

torch.cuda.set_device(0)
kb = 4 if a.kt in (0, 2) else 8
vt = {0: 0, 4: 0, 8: 1, 16: 2}[a.vb]
n = a.n
keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
vals = torch.empty(max(1, n * a.vb), dtype=torch.uint8, device="cuda")
tmp = torch.empty(sum(R.temp_bytes(a.kt, vt, n)), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()
res = {"n": n, "key_type": a.kt, "value_bytes": a.vb}
for who in ("reference", "libthrs"):
    times = []
    if who == "libthrs":
        rs = T.RadixSort([], T.RadixSort.Config(keyType=T.KeyType(a.kt), valueType=T.ValueType(vt)))
        d = rs.getTemporaryBufferBytes(n)
        tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
    for r in range(a.runs + 1):
        TU.fill_keys(a.kt, keys, n, start=r * n)
        if a.vb:
            TU.iota(a.vb, vals, n)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if who == "reference":
            R.sort(a.kt, vt, False, keys, vals if a.vb else None, n, tmp, 0, kb * 8, stream)
        elif a.vb:
            rs.sortPairs(keys, vals, n, tmp, 0, kb * 8, stream)
        else:
            rs.sortKeys(keys, n, tmp, 0, kb * 8, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
        assert TU.count_unsorted(a.kt, keys, n, 0, kb * 8) == 0, who
    ms = statistics.median(times)
    res[who] = {"ms": round(ms, 4), "Gkeys_s": round(n / ms / 1e6, 3)}
    print(who, res[who], flush=True)
print(json.dumps(res))
