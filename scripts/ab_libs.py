#!/usr/bin/env python3
"""Interleaved A/B of libthrs builds (one process, same fresh input per round
for every library): ms per sort and per-launch times of the device passes and
the local sort.  Libraries: 'main' (tinyhipradixsort_amd/libthrs.so) or
exp/variants/libthrs_<name>.so.  --nocheck NAME: experiment builds whose
output is knowingly wrong.

usage: python scripts/ab_libs.py [--workload c2] [--rounds 6] [--nocheck a,b] main vec ...
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402
from bench import WORKLOADS  # noqa: E402
from sweep import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--nocheck", default="")
    ap.add_argument("--n", type=int, default=None, help="keys (default: the workload's)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    kt, vb, n, dist, _ = WORKLOADS[a.workload]
    n = a.n or n
    kb = 4 if kt in (0, 2) else 8
    libs = []
    for name in a.libs:
        path = T.LIB_PATH if name == "main" else os.path.join(ROOT, "exp", "variants", f"libthrs_{name}.so")
        L = load(path)
        L.thrs_profile_read_launches.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int)]
        libs.append((name, L))
    cfg = T._CConfig(1, kt, {0: 0, 4: 0, 8: 1, 16: 2}[vb], 0)
    tb = 0
    for _, L in libs:
        d = T._CTempDef()
        L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
        tb = max(tb, d.pSumBuffer + d.keyOutBuffer + (d.valueOutBuffer if vb else 0))
    tmp = torch.empty(tb, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
    vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {name: {"ms": [], "launch": []} for name, _ in libs}
    nochk = set(filter(None, a.nocheck.split(",")))
    for r in range(a.rounds + 1):
        for name, L in libs:
            if dist == "uniform":
                TU.fill_keys(kt, keys, n, start=r * n)
            else:
                TU.fill_dist(kt, keys, n, dist, start=r * n)
            if vb:
                TU.iota(vb, vals, n)
            fp = TU.fingerprint(kt, keys, n) if name not in nochk else None
            torch.cuda.synchronize()
            L.thrs_profile_enable(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if vb:
                rc = L.thrs_sort_pairs(ctypes.byref(cfg), keys.data_ptr(), vals.data_ptr(), n, tmp.data_ptr(), 0,
                                       kb * 8, s.cuda_stream)
            else:
                rc = L.thrs_sort_keys(ctypes.byref(cfg), keys.data_ptr(), n, tmp.data_ptr(), 0, kb * 8, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            assert rc == 0, (name, rc)
            launches = []
            for kind in (1, 2):
                ms = (ctypes.c_double * 32)()
                cnt = ctypes.c_int()
                L.thrs_profile_read_launches(kind, ms, 32, ctypes.byref(cnt))
                launches += [round(ms[i], 4) for i in range(min(cnt.value, 32)) if ms[i] > 0.02]
            L.thrs_profile_enable(0)
            if name not in nochk:
                assert L.thrs_check_device_error(tmp.data_ptr(), s.cuda_stream) == 0, name
                assert TU.count_unsorted(kt, keys, n, 0, kb * 8) == 0, name
                if not vb:
                    assert TU.fingerprint(kt, keys, n) == fp, (name, "keys lost or duplicated")
            if r > 0:
                res[name]["ms"].append(e0.elapsed_time(e1))
                res[name]["launch"].append(launches)
    for name, v in res.items():
        cols = list(zip(*v["launch"]))
        print(json.dumps({"lib": name, "ms_med": round(statistics.median(v["ms"]), 4),
                          "ms_min": round(min(v["ms"]), 4),
                          "launch_med": [round(statistics.median(c), 4) for c in cols]}), flush=True)


if __name__ == "__main__":
    main()
