#!/usr/bin/env python3
"""What the per-launch HIP events (thrs_profile_enable) add to a sort: the
same workload timed with and without them, interleaved, fresh inputs.
usage: python scripts/prof_overhead.py [--workload ref160m] [--rounds 8]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ref160m")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    kt, vb, n, _, _ = WORKLOADS[a.workload]
    kb = 4 if kt in (0, 2) else 8
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                8: T.ValueType.U64, 16: T.ValueType.U128}[vb])
    rs = T.RadixSort([], cfg)
    d = rs.getTemporaryBufferBytes(n)
    tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs() if vb else d.getTemporaryBufferBytesForSortKeys(),
                      dtype=torch.uint8, device="cuda")
    keys = [torch.empty(n * kb, dtype=torch.uint8, device="cuda") for _ in range(a.steps)]
    vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
    res = {False: [], True: []}
    for r in range(a.rounds + 1):
        for prof in (False, True):
            for i in range(a.steps):
                TU.fill_keys(kt, keys[i], n, start=(r * a.steps + i) * n)
            torch.cuda.synchronize()
            T.profile_enable(prof)
            t0 = time.perf_counter()
            for i in range(a.steps):
                if vb:
                    rs.sortPairs(keys[i], vals, n, tmp, 0, kb * 8)
                else:
                    rs.sortKeys(keys[i], n, tmp, 0, kb * 8)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            T.profile_enable(False)
            if r > 0:
                res[prof].append((t1 - t0) / a.steps * 1e3)
    print(json.dumps({"workload": a.workload, "ms_no_events": round(statistics.median(res[False]), 4),
                      "ms_with_events": round(statistics.median(res[True]), 4)}))


if __name__ == "__main__":
    main()
