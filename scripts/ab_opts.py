#!/usr/bin/env python3
"""Interleaved A/B of thrs_options settings (one process, one library, the
same fresh input per round for every setting): ms per sort and per-launch
times of the device passes / local sort, output checked (sortedness +
multiset fingerprint).

usage: python scripts/ab_opts.py [--workload c2] [--rounds 6] "offsets=lookback" "offsets=reserve" ...
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--lib", default=None, help="another libthrs build (exp/variants/libthrs_<name>.so)")
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    if a.lib:
        T.LIB_PATH = os.path.join(ROOT, "exp", "variants", f"libthrs_{a.lib}.so")
    kt, vb, n, dist, _ = WORKLOADS[a.workload]
    kb = 4 if kt in (0, 2) else 8
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                8: T.ValueType.U64, 16: T.ValueType.U128}[vb])
    sorters = []
    for st in a.settings:
        kw = dict(x.split("=") for x in st.split(",") if x)
        sorters.append((st, T.RadixSort([], cfg, T.Options(**kw))))
    d = sorters[0][1].getTemporaryBufferBytes(n)
    tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs() if vb else d.getTemporaryBufferBytesForSortKeys(),
                      dtype=torch.uint8, device="cuda")
    keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
    vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
    res = {st: {"ms": [], "launch": []} for st, _ in sorters}
    for r in range(a.rounds + 1):
        for st, rs in sorters:
            if dist == "uniform":
                TU.fill_keys(kt, keys, n, start=r * n)
            else:
                TU.fill_dist(kt, keys, n, dist, start=r * n)
            if vb:
                TU.iota(vb, vals, n)
            fp = TU.fingerprint(kt, keys, n)
            torch.cuda.synchronize()
            T.profile_enable(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if vb:
                rs.sortPairs(keys, vals, n, tmp, 0, kb * 8)
            else:
                rs.sortKeys(keys, n, tmp, 0, kb * 8)
            e1.record()
            torch.cuda.synchronize()
            launches = [round(x, 4) for k in (1, 2) for x in T.profile_launches(k) if x > 0.02]
            T.profile_enable(False)
            rs.checkDeviceError(tmp)
            assert TU.count_unsorted(kt, keys, n, 0, kb * 8) == 0, st
            if not vb:
                assert TU.fingerprint(kt, keys, n) == fp, (st, "keys lost or duplicated")
            if r > 0:
                res[st]["ms"].append(e0.elapsed_time(e1))
                res[st]["launch"].append(launches)
    for st, v in res.items():
        cols = list(zip(*v["launch"]))
        print(json.dumps({"setting": st, "ms_med": round(statistics.median(v["ms"]), 4),
                          "ms_min": round(min(v["ms"]), 4),
                          "launch_med": [round(statistics.median(c), 4) for c in cols]}), flush=True)


if __name__ == "__main__":
    main()
