#!/usr/bin/env python3
"""Per-chunk phase timeline of the local bucket sort (thrs_local) from a
-DTHRS_STAMPS build (build/variants/libthrs_stamps.so).  Stamps are
s_memrealtime (100 MHz = 10 ns): 0 entry, 1 keys loaded (vmcnt drained),
2 round 0 done, 3 round 1 done, 4 write-out issued, 5 stores drained;
6 = HW_ID, 7 = XCC id.
usage: python scripts/local_stamps.py [--n N]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "variants", "libthrs_stamps.so"))
    a = ap.parse_args()
    L = load(a.lib)
    L.thrs_debug_set_local_stamps.argtypes = [ctypes.c_void_p]
    n = a.n
    cfg = T._CConfig(1, 0, 0, 0)
    d = T._CTempDef()
    L.thrs_get_temporary_buffer_bytes(ctypes.byref(cfg), n, ctypes.byref(d))
    tmp = torch.empty(d.pSumBuffer + d.keyOutBuffer, dtype=torch.uint8, device="cuda")
    keys = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(65536 * 8, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    for it in range(2):
        TU.fill_keys(0, keys, n, start=it * n)
        torch.cuda.synchronize()
        L.thrs_debug_set_local_stamps(st.data_ptr() if it == 1 else None)
        assert L.thrs_sort_keys(ctypes.byref(cfg), keys.data_ptr(), n, tmp.data_ptr(), 0, 32, s.cuda_stream) == 0
        torch.cuda.synchronize()
    L.thrs_debug_set_local_stamps(None)
    assert TU.count_unsorted(0, keys, n, 0, 32) == 0
    x = st.cpu().numpy().reshape(65536, 8)
    x = x[x[:, 0] > 0]
    t0 = x[:, 0].min()
    ph = {"load": x[:, 1] - x[:, 0], "round0": x[:, 2] - x[:, 1], "round1": x[:, 3] - x[:, 2],
          "writeout_issue": x[:, 4] - x[:, 3], "drain": x[:, 5] - x[:, 4], "life": x[:, 5] - x[:, 0]}
    rep = {"chunks": int(x.shape[0]), "span_us": float((x[:, 5].max() - t0) / 100.0)}
    for k, v in ph.items():
        v = v / 100.0
        rep[k] = {"med_us": round(float(np.median(v)), 2), "p10": round(float(np.percentile(v, 10)), 2),
                  "p90": round(float(np.percentile(v, 90)), 2), "mean": round(float(v.mean()), 2)}
    # concurrency: how many workgroups are in each phase, sampled every 2 us
    T_ = np.arange(t0, x[:, 5].max(), 200)
    conc = {}
    for name, (a0, a1) in {"load": (0, 1), "rounds": (1, 3), "writeout": (3, 5), "alive": (0, 5)}.items():
        c = [int(((x[:, a0] <= t) & (x[:, a1] > t)).sum()) for t in T_]
        conc[name] = {"mean": round(float(np.mean(c)), 1), "max": int(np.max(c))}
    rep["concurrency"] = conc
    # same-CU pairs: start-time offset between the two workgroups sharing a CU slot
    hw = x[:, 6]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    key = (x[:, 7] << 8) | (se << 5) | (sh << 4) | cu
    rep["distinct_cus"] = int(len(np.unique(key)))
    print(json.dumps(rep, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "local_stamps.npy"), x)


if __name__ == "__main__":
    main()
