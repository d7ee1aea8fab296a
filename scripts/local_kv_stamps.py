#!/usr/bin/env python3
"""Per-chunk phase timeline of thrs_local_kv (8-byte keys, no values) from a
-DTHRS_STAMPS build (exp/variants/libthrs_stamps.so).  Stamps are
s_memrealtime (100 MHz = 10 ns): 0 entry, 1 keys loaded (+ items and low
words in LDS), 2 two rounds done, 3 tie fix-up done (+barrier), 4 sorted
items read back, 5 write-out issued, 6 stores drained; 7 = HW_ID.
With --kt / --vb: other 8-byte key types, and pairs (ValueType by --vb).
usage: python scripts/local_kv_stamps.py [--n N] [--kt 1] [--vb 0] [--lib PATH]"""
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

NAMES = ["load", "rounds", "fixup", "readback", "writeout_issue", "drain"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kt", type=int, default=1, help="key type: 1 u64, 3 f64")
    ap.add_argument("--vb", type=int, default=0, help="value bytes: 0, 4, 8, 16")
    ap.add_argument("--lib", default=os.path.join(ROOT, "exp", "variants", "libthrs_stamps.so"))
    a = ap.parse_args()
    L = load(a.lib)
    L.thrs_debug_set_local_stamps.argtypes = [ctypes.c_void_p]
    n = a.n
    vt = {0: 0, 4: 0, 8: 1, 16: 2}[a.vb]
    cfg = T._CConfig(0, a.kt, vt, 0)
    d = T._CTempDef()
    L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
    tmp = torch.empty(d.pSumBuffer + d.keyOutBuffer + (d.valueOutBuffer if a.vb else 0), dtype=torch.uint8,
                      device="cuda")
    keys = torch.empty(8 * n, dtype=torch.uint8, device="cuda")
    vals = torch.empty(max(1, a.vb * n), dtype=torch.uint8, device="cuda")
    st = torch.zeros(65536 * 8, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    for it in range(2):
        TU.fill_keys(a.kt, keys, n, start=it * n)
        if a.vb:
            TU.iota(a.vb, vals, n)
        torch.cuda.synchronize()
        L.thrs_debug_set_local_stamps(st.data_ptr() if it == 1 else None)
        if a.vb:
            assert L.thrs_sort_pairs(ctypes.byref(cfg), keys.data_ptr(), vals.data_ptr(), n, tmp.data_ptr(), 0, 64,
                                     s.cuda_stream) == 0
        else:
            assert L.thrs_sort_keys(ctypes.byref(cfg), keys.data_ptr(), n, tmp.data_ptr(), 0, 64, s.cuda_stream) == 0
        torch.cuda.synchronize()
    L.thrs_debug_set_local_stamps(None)
    assert TU.count_unsorted(a.kt, keys, n, 0, 64) == 0
    x = st.cpu().numpy().reshape(65536, 8)
    x = x[(x[:, 0] > 0) & (x[:, 6] > 0)]
    t0 = x[:, 0].min()
    rep = {"chunks": int(x.shape[0]), "span_us": float((x[:, 6].max() - t0) / 100.0)}
    for i, k in enumerate(NAMES):
        v = (x[:, i + 1] - x[:, i]) / 100.0
        rep[k] = {"med_us": round(float(np.median(v)), 2), "p10": round(float(np.percentile(v, 10)), 2),
                  "p90": round(float(np.percentile(v, 90)), 2), "mean": round(float(v.mean()), 2)}
    v = (x[:, 6] - x[:, 0]) / 100.0
    rep["life"] = {"med_us": round(float(np.median(v)), 2), "mean": round(float(v.mean()), 2)}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
