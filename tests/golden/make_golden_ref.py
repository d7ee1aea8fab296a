"""Regenerate the golden digests with the REFERENCE's own kernels (GPU box).

Inputs come from the reference's own splitmix64 (oracle/_ref/libfpkey_ref.so,
unittest.cpp:24-35) through randomizeValues (unittest.cpp:96-116); outputs from
its kernels (kernel.cu via hipRTC, oracle/_ref/refk_*.co) with its pass loop.
Writes gpurun_out/golden_ref.json; tests/golden/pin_golden.py then checks it
digest-for-digest against tests/golden/golden.json (made by the CPU oracle)
and records the pin in golden.json.

usage (on the GPU box): python tests/golden/make_golden_ref.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import cases as C  # noqa: E402
from oracle import ref as R  # noqa: E402


class RefRng:
    """The reference's splitmix64 (compiled), state 0 per test."""

    def __init__(self):
        self.buf = R.splitmix64(1 << 24)
        self.i = 0

    def next(self) -> int:
        v = int(self.buf[self.i])
        self.i += 1
        return v

    def draws(self, n: int) -> np.ndarray:
        v = self.buf[self.i:self.i + n]
        self.i += n
        return v


def keys_of(kt, d):
    from oracle import oracle as O
    return O.randomize_np(kt, d)


def stream(name, kind, kt, vb):
    rng = RefRng()
    for _ in range(C.TEST_ITERATION):
        n = 1 + rng.next() % (C.TEST_MAX_ARRAY_SIZE - 1)
        if name == "SortKeys.extremeCase":
            k = np.zeros(n, np.uint32)
            k[rng.next() % n] = 1
            k[rng.next() % n] = 42
            yield {"n": n, "keys": k}
        elif kind == "window":
            s = rng.next() % 64
            item = {"n": n, "start": s, "keys": keys_of(kt, rng.draws(n))}
            if vb:
                item["values"] = C._values(n, vb)
            yield item
        else:
            item = {"n": n, "keys": keys_of(kt, rng.draws(n))}
            if vb:
                item["values"] = C._values(n, vb)
            yield item


def main():
    import torch
    torch.cuda.set_device(0)
    vt = {4: 0, 8: 1, 16: 2}
    out = {"generator": "tests/golden/make_golden_ref.py",
           "source": "reference kernels (kernel.cu via hipRTC for gfx950) + reference splitmix64, on MI355X",
           "cases": {}}
    for name, (kind, kt, vb, desc, _f) in C.CASES.items():
        rows = []
        for item in stream(name, kind, kt, vb):
            keys, vals = item["keys"], item.get("values")
            n = keys.shape[0]
            s, e = (int(item["start"]), int(item["start"]) + 8) if kind == "window" else (0, keys.itemsize * 8)
            kd = torch.from_numpy(keys.view(np.uint8).copy()).cuda()
            vd = torch.from_numpy(np.ascontiguousarray(vals).view(np.uint8).reshape(-1).copy()).cuda() if vb else None
            tmp = torch.empty(sum(R.temp_bytes(kt, vt.get(vb, 0), n)), dtype=torch.uint8, device="cuda")
            R.sort(kt, vt.get(vb, 0), desc, kd, vd, n, tmp, s, e, torch.cuda.current_stream())
            torch.cuda.synchronize()
            row = {"n": int(n), "keys": C.digest(kd.cpu().numpy().view(keys.dtype))}
            if "start" in item:
                row["start"] = int(item["start"])
            if vb:
                row["values"] = C.digest(vd.cpu().numpy().view(vals.dtype).reshape(vals.shape))
            rows.append(row)
        out["cases"][name] = rows
        print(f"{name}: {len(rows)} iterations", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "golden_ref.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
