"""Bindings of the REFERENCE build (oracle/_ref/, made by oracle/ref/Makefile
from the sources under /root/reference) -- TEST INFRASTRUCTURE ONLY.

* libfpkey_ref.so: the reference's own host getKeyBits (fpKey.hpp:15-38) and
  splitmix64 (unittest.cpp:24-35), compiled as they are.  Pins the oracle's
  transform and streams (tests/test_oracle_ref.py).
* liboracle_refk.so + refk_*.co: the reference's own kernels (kernel.cu via
  hipRTC, one code object per Config) launched with its pass loop
  (tinyhipradixsort.hpp:854-944).  Pins libthrs and the oracle on the GPU
  (tests/test_gpu_ref.py) and times the reference on MI355X (bench.py
  --ref-gpu).

Only tests/, smoke() and bench.py's baseline legs import this, as checker or
baseline -- never as the thing measured for `value`.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
FPKEY_LIB = os.path.join(REF_DIR, "libfpkey_ref.so")
REFK_LIB = os.path.join(REF_DIR, "liboracle_refk.so")

_fp = None
_rk = None


def available() -> bool:
    return os.path.exists(FPKEY_LIB)


def kernels_available() -> bool:
    return os.path.exists(REFK_LIB) and os.path.exists(os.path.join(REF_DIR, "refk_k0_v0_d0_a0.co"))


def fplib():
    global _fp
    if _fp is None:
        L = ctypes.CDLL(FPKEY_LIB)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        for f in ("ref_key_bits_u32", "ref_key_bits_u64", "ref_key_bits_f32", "ref_key_bits_f64"):
            getattr(L, f).argtypes = [vp, vp, u64]
        L.ref_splitmix64_fill.argtypes = [ctypes.POINTER(ctypes.c_uint64), vp, u64]
        _fp = L
    return _fp


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def key_bits(key_type: int, keys: np.ndarray) -> np.ndarray:
    """getKeyBits of the reference's fpKey.hpp (no ORDER_MASK), widened to u64.
    key_type as thrs::KeyType; keys as raw bit patterns."""
    keys = np.ascontiguousarray(keys)
    n = keys.shape[0]
    if key_type in (0, 2):
        out = np.empty(n, np.uint32)
        f = fplib().ref_key_bits_u32 if key_type == 0 else fplib().ref_key_bits_f32
    else:
        out = np.empty(n, np.uint64)
        f = fplib().ref_key_bits_u64 if key_type == 1 else fplib().ref_key_bits_f64
    f(_p(keys), _p(out), n)
    return out.astype(np.uint64)


def splitmix64(n: int, state: int = 0) -> np.ndarray:
    """n draws of the reference's splitmix64 from `state`."""
    x = ctypes.c_uint64(state)
    out = np.empty(n, np.uint64)
    fplib().ref_splitmix64_fill(ctypes.byref(x), _p(out), n)
    return out


def rklib():
    global _rk
    if _rk is None:
        L = ctypes.CDLL(REFK_LIB)
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.refk_temp_bytes.argtypes = [i32, i32, u32, ctypes.POINTER(ctypes.c_uint64)]
        L.refk_sort.argtypes = [i32, i32, i32, i32, vp, vp, u32, vp, i32, i32, vp]
        L.refk_sort.restype = i32
        _rk = L
    return _rk


def temp_bytes(key_type: int, value_type: int, n: int) -> tuple[int, int, int]:
    """TemporaryBufferDef of the reference (tinyhipradixsort.hpp:833-843)."""
    out = (ctypes.c_uint64 * 3)()
    rklib().refk_temp_bytes(key_type, value_type, n, out)
    return int(out[0]), int(out[1]), int(out[2])


def sort(key_type: int, value_type: int, descending: bool, keys, values, n: int, tmp, start_bits: int,
         end_bits: int, stream, aligned16: bool = True):
    """The reference's sortKeys (values None) / sortPairs on device buffers
    (torch tensors or integer addresses); stream a torch stream or handle."""
    def ptr(x):
        return None if x is None else (x if isinstance(x, int) else x.data_ptr())
    s = stream if isinstance(stream, int) or stream is None else stream.cuda_stream
    rc = rklib().refk_sort(key_type, value_type, int(descending), int(aligned16), ptr(keys), ptr(values), n,
                           ptr(tmp), start_bits, end_bits, s)
    if rc:
        raise RuntimeError(f"refk_sort failed: {rc}")
