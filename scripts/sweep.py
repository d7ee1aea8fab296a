#!/usr/bin/env python3
"""Interleaved A/B timing of libthrs variants (build/variants/libthrs_*.so) on
one GPU, in ONE process (methodology: MI355X guide s5.4 rule 24).

Each round, every variant sorts a freshly generated input (same inputs for
all variants within a round); reports median/min ms per sort and the per-pass
kernel time from thrs_profile_*.  Correctness of each output is checked with
the testutil sortedness + fingerprint kernels.

usage: python scripts/sweep.py [--workload c2] [--n N] [--rounds R] [variant ...]
"""
import argparse
import ctypes
import glob
import json
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import tinyhipradixsort_amd as T  # noqa: E402
from tinyhipradixsort_amd import testutil as TU  # noqa: E402

WL = {"c2": (0, 0, 1 << 30), "c3": (0, 4, 1 << 30), "c4": (2, 0, 1 << 28), "c5": (1, 8, 1 << 28),
      "k64": (1, 0, 1 << 29), "kf32v32": (2, 4, 1 << 30), "f32k": (2, 0, 1 << 30), "ref160m": (0, 0, 160000000)}


def load(path):
    L = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.thrs_get_temporary_buffer_bytes.argtypes = [ctypes.POINTER(T._CConfig), u32, ctypes.POINTER(T._CTempDef)]
    L.thrs_sort_keys.argtypes = [ctypes.POINTER(T._CConfig), vp, u32, vp, i32, i32, vp]
    L.thrs_sort_pairs.argtypes = [ctypes.POINTER(T._CConfig), vp, vp, u32, vp, i32, i32, vp]
    L.thrs_profile_enable.argtypes = [i32]
    L.thrs_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    L.thrs_check_device_error.argtypes = [vp, vp]
    if hasattr(L, "thrs_profile_read_kind"):
        L.thrs_profile_read_kind.argtypes = [i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2", choices=sorted(WL))
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--vendor", action="store_true", help="also time hipcub::DeviceRadixSort")
    ap.add_argument("--iota", action="store_true",
                    help="keys = 0..n-1 (u32): every pass sees exactly T/256 keys per digit per tile")
    ap.add_argument("--nocheck", default="", help="comma list of EXPERIMENT variants whose output is knowingly wrong")
    ap.add_argument("--no-main", action="store_true", help="time only the named variants (per-library rocprof runs)")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    kt, vb, n = WL[a.workload]
    n = a.n or n
    kb = 4 if kt in (0, 2) else 8
    paths = [os.path.join(ROOT, "exp", "variants", f"libthrs_{v}.so") for v in a.variants] if a.variants else \
        sorted(glob.glob(os.path.join(ROOT, "exp", "variants", "libthrs_*.so")))
    paths = ([] if a.no_main else [T.LIB_PATH]) + [p for p in paths if os.path.exists(p)]
    libs = [(os.path.basename(p)[len("libthrs"):-3].lstrip("_") or "main", load(p)) for p in paths]
    cfg = T._CConfig(1, kt, {0: 0, 4: 0, 8: 1, 16: 2}[vb], 0)
    tmp_bytes = 0
    for _, L in libs:
        d = T._CTempDef()
        L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
        tmp_bytes = max(tmp_bytes, d.pSumBuffer + d.keyOutBuffer + (d.valueOutBuffer if vb else 0))
    tmp = torch.empty(tmp_bytes, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
    vals = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {name: {"ms": [], "pass_ms": [], "hist_ms": [], "local_ms": []} for name, _ in libs}
    vend = None
    vpath = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_vendor.so")
    if a.vendor and os.path.exists(vpath) and kt in (0, 1) and vb in (0, kb):
        V = ctypes.CDLL(vpath)
        V.thrsv_temp_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
        V.thrsv_sort.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [
            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        vt = ctypes.c_uint64()
        assert V.thrsv_temp_bytes(kb, vb, n, ctypes.byref(vt)) == 0
        vtmp = torch.empty(vt.value, dtype=torch.uint8, device="cuda")
        kb2 = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
        vb2 = torch.empty(max(1, n * vb), dtype=torch.uint8, device="cuda")
        vend = (V, vtmp, kb2, vb2)
        res["hipcub"] = {"ms": [], "pass_ms": [], "hist_ms": [], "local_ms": []}
    for r in range(a.rounds + 1):
        for name, L in libs:
            if a.iota:
                TU.iota(kb, keys, n)
            else:
                TU.fill_keys(kt, keys, n, start=r * n)
            if vb:
                TU.iota(vb, vals, n)
            fp = TU.fingerprint(kt, keys, n) if r == 1 else None
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
            h, p = ctypes.c_double(), ctypes.c_double()
            nh, np_ = ctypes.c_int(), ctypes.c_int()
            L.thrs_profile_read(ctypes.byref(h), ctypes.byref(nh), ctypes.byref(p), ctypes.byref(np_))
            lm, nl = ctypes.c_double(), ctypes.c_int()
            if hasattr(L, "thrs_profile_read_kind"):
                L.thrs_profile_read_kind(2, ctypes.byref(lm), ctypes.byref(nl))
            L.thrs_profile_enable(0)
            if name not in a.nocheck.split(","):
                assert L.thrs_check_device_error(tmp.data_ptr(), s.cuda_stream) == 0, name
            if r == 1 and name not in a.nocheck.split(","):
                bad = TU.count_unsorted(kt, keys, n, 0, kb * 8)
                assert bad == 0 and TU.fingerprint(kt, keys, n) == fp, (name, "WRONG OUTPUT", bad)
            if r > 0:   # round 0 is warm-up
                res[name]["ms"].append(e0.elapsed_time(e1))
                res[name]["pass_ms"].append(p.value / max(1, np_.value))
                res[name]["hist_ms"].append(h.value / max(1, nh.value))
                res[name]["local_ms"].append(lm.value / max(1, nl.value))
        if vend is not None:
            V, vtmp, kb2, vb2 = vend
            TU.fill_keys(kt, keys, n, start=r * n)
            if vb:
                TU.iota(vb, vals, n)
            torch.cuda.synchronize()
            sel = ctypes.c_int()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = V.thrsv_sort(kb, vb, keys.data_ptr(), kb2.data_ptr(), vals.data_ptr(), vb2.data_ptr(), n,
                              vtmp.data_ptr(), vtmp.numel(), ctypes.byref(sel), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            assert rc == 0
            if r == 1:
                out = kb2 if sel.value else keys
                assert TU.count_unsorted(kt, out, n, 0, kb * 8) == 0
            if r > 0:
                res["hipcub"]["ms"].append(e0.elapsed_time(e1))
                res["hipcub"]["pass_ms"].append(float("nan"))
                res["hipcub"]["hist_ms"].append(float("nan"))
                res["hipcub"]["local_ms"].append(float("nan"))
    out = []
    for name, d in res.items():
        med = statistics.median(d["ms"])
        pm = statistics.median(d["pass_ms"])
        alg = 2 * n * (kb + vb)
        out.append({"variant": name, "ms_med": round(med, 3), "ms_min": round(min(d["ms"]), 3),
                    "Gkeys_s": round(n / med / 1e6, 2), "pass_ms": round(pm, 4),
                    "pass_GBps": round(alg / pm / 1e6, 1), "hist_ms": round(statistics.median(d["hist_ms"]), 4),
                    "local_ms": round(statistics.median(d["local_ms"]), 4)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
