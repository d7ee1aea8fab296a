"""Debug: f32 pairs in [1, 2) on the bucket path without a key range (squeezed):
first mismatches against the oracle."""
import os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch
from oracle import oracle as O
from test_gpu_parity import make_sorter, _mode_after
n = 1 << 21
raw = O.randomize_np(O.F32, O.splitmix64_stream(4444 + 4, n)).astype(np.uint32)
keys = ((raw & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)).astype(np.uint32)
vals = (np.arange(n, dtype=np.uint32) * np.uint32(2654435761)).astype(np.uint32)
ek, ev = O.lsd_sort(O.F32, keys, vals, 0, 32, False)
rs = make_sorter(O.F32, 4, False, path="bucket")
(mode, big), k, v = _mode_after(torch, rs, keys, vals, O.F32, 4)
k = k.view(np.uint32); ek = ek.view(np.uint32)
bad = np.nonzero(k != ek)[0]
print("mode", mode, big, "bad", len(bad), "vals bad", int((v != ev).sum()))
for i in bad[:12]:
    print(i, hex(int(k[i])), hex(int(ek[i])), hex(int(k[i]) ^ int(ek[i])))
