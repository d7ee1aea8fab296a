#!/usr/bin/env python3
"""A/B timing of libthrs builds through the stable part of the C-ABI
(thrs_get_temporary_buffer_bytes / thrs_sort_keys / thrs_sort_pairs /
thrs_profile_*), so builds of different ABI versions (e.g. the round-1
library) run on the same box, same inputs (splitmix64, fresh per step).
usage: python scripts/ab_sort.py LIB [LIB ...] [--kt 0] [--vb 0] [--n 1073741824] [--steps 5] [--rounds 2]"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--kt", type=int, default=0)
ap.add_argument("--vb", type=int, default=0)
ap.add_argument("--n", type=int, default=1 << 30)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--rounds", type=int, default=2)
a = ap.parse_args()
import torch  # noqa: E402

from tinyhipradixsort_amd import testutil as TU  # noqa: E402

torch.cuda.set_device(0)


class Cfg(ctypes.Structure):
    _fields_ = [("a", ctypes.c_int32), ("k", ctypes.c_int32), ("v", ctypes.c_int32), ("o", ctypes.c_int32)]


class Def(ctypes.Structure):
    _fields_ = [("p", ctypes.c_uint64), ("k", ctypes.c_uint64), ("v", ctypes.c_uint64)]


kb = 4 if a.kt in (0, 2) else 8
vt = {0: 0, 4: 0, 8: 1, 16: 2}[a.vb]
n = a.n
stream = torch.cuda.current_stream()
keys = [torch.empty(n * kb, dtype=torch.uint8, device="cuda") for _ in range(a.steps)]
vals = [torch.empty(max(1, n * a.vb), dtype=torch.uint8, device="cuda") for _ in range(a.steps)] if a.vb else None
libs = []
for p in a.libs:
    L = ctypes.CDLL(os.path.abspath(p))
    L.thrs_get_temporary_buffer_bytes.argtypes = [ctypes.POINTER(Cfg), ctypes.c_uint32, ctypes.POINTER(Def)]
    L.thrs_sort_keys.argtypes = [ctypes.POINTER(Cfg), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
    L.thrs_sort_pairs.argtypes = [ctypes.POINTER(Cfg), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    libs.append((p, L))
cfg = Cfg(1, a.kt, vt, 0)
res = {}
for rnd in range(a.rounds):
    for p, L in libs:
        d = Def()
        L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
        tmp = torch.empty(d.p + d.k + d.v, dtype=torch.uint8, device="cuda")
        for i in range(a.steps):
            TU.fill_keys(a.kt, keys[i], n, start=(i + 7 * rnd) * n)
            if a.vb:
                TU.iota(a.vb, vals[i], n)
        torch.cuda.synchronize()
        # one warm-up on buffer 0, then refill it
        rc = (L.thrs_sort_pairs(ctypes.byref(cfg), keys[0].data_ptr(), vals[0].data_ptr(), n, tmp.data_ptr(), 0, kb * 8,
                                stream.cuda_stream) if a.vb else
              L.thrs_sort_keys(ctypes.byref(cfg), keys[0].data_ptr(), n, tmp.data_ptr(), 0, kb * 8, stream.cuda_stream))
        assert rc == 0, rc
        TU.fill_keys(a.kt, keys[0], n, start=(99 + rnd) * n)
        if a.vb:
            TU.iota(a.vb, vals[0], n)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(a.steps):
            if a.vb:
                L.thrs_sort_pairs(ctypes.byref(cfg), keys[i].data_ptr(), vals[i].data_ptr(), n, tmp.data_ptr(), 0,
                                  kb * 8, stream.cuda_stream)
            else:
                L.thrs_sort_keys(ctypes.byref(cfg), keys[i].data_ptr(), n, tmp.data_ptr(), 0, kb * 8,
                                 stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        if TU.count_unsorted(a.kt, keys[a.steps - 1], n, 0, kb * 8):
            print(f"{os.path.basename(p)}: OUTPUT NOT SORTED (ablation builds only)", flush=True)
        res.setdefault(p, []).append(ms)
        print(f"{os.path.basename(p):24s} round {rnd}: {ms:.4f} ms/sort  {n / ms / 1e6:.2f} Gkeys/s", flush=True)
        del tmp
print(json.dumps({os.path.basename(p): round(statistics.median(v), 4) for p, v in res.items()}))
