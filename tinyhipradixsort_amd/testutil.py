"""ctypes bindings for libthrs_testutil.so -- GPU generators and property
checkers used by tests/ and bench.py only (never by the sort path)."""
from __future__ import annotations

import ctypes
import os

from . import TESTUTIL_PATH, _ptr, _stream, _check

_tl = None


def tlib() -> ctypes.CDLL:
    global _tl
    if _tl is None:
        if not os.path.exists(TESTUTIL_PATH):
            raise ImportError(f"{TESTUTIL_PATH} is missing: run `make`")
        L = ctypes.CDLL(TESTUTIL_PATH)
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        ull_p = ctypes.POINTER(ctypes.c_ulonglong)
        L.thrsu_fill_keys.argtypes = [i32, vp, u64, u64, u64, vp]
        L.thrsu_fill_dist.argtypes = [i32, vp, u64, u64, u64, i32, vp]
        L.thrsu_iota.argtypes = [i32, vp, u64, u64, vp]
        L.thrsu_check_sorted.argtypes = [i32, i32, vp, u64, i32, i32, ull_p, vp]
        L.thrsu_fingerprint.argtypes = [i32, vp, u64, ull_p, vp]
        L.thrsu_check_pairs.argtypes = [i32, i32, i32, vp, vp, vp, u64, i32, i32, ull_p, vp]
        L.thrsu_copy.argtypes = [vp, vp, u64, i32, vp]
        L.thrsu_probe_lds_order_partial.argtypes = [i32, ctypes.POINTER(ctypes.c_uint)]
        for f in ("thrsu_probe_lds_order_partial", "thrsu_copy", "thrsu_fill_keys", "thrsu_fill_dist", "thrsu_iota", "thrsu_check_sorted", "thrsu_fingerprint", "thrsu_check_pairs"):
            getattr(L, f).restype = i32
        _tl = L
    return _tl


def fill_keys(key_type: int, out, n: int, start: int = 0, state: int = 0, stream=None):
    """Keys = randomizeValues over splitmix64 draws start+1..start+n (unittest.cpp:96-116)."""
    _check(tlib().thrsu_fill_keys(int(key_type), _ptr(out), n, start, state, _stream(stream)))


DISTS = {"uniform": 0, "sorted": 1, "reverse": 2, "extreme": 3, "fewuniq": 4}


def fill_dist(key_type: int, out, n: int, dist: str, start: int = 0, state: int = 0, stream=None):
    """Keys of a named distribution (thrs_testutil.hip k_fill_dist): uniform
    (= fill_keys), sorted / reverse (stratified sorted uniform sample),
    extreme (unittest.cpp:191-225's all-zero array with two set keys),
    fewuniq (16 distinct uniform keys)."""
    _check(tlib().thrsu_fill_dist(int(key_type), _ptr(out), n, start, state, DISTS[dist], _stream(stream)))


def iota(value_bytes: int, out, n: int, start: int = 0, stream=None):
    _check(tlib().thrsu_iota(value_bytes, _ptr(out), n, start, _stream(stream)))


def count_unsorted(key_type: int, keys, n: int, start_bits: int, end_bits: int, descending=False, stream=None) -> int:
    r = (ctypes.c_ulonglong * 1)()
    _check(tlib().thrsu_check_sorted(int(key_type), int(descending), _ptr(keys), n, start_bits, end_bits, r,
                                     _stream(stream)))
    return int(r[0])


def fingerprint(key_type: int, keys, n: int, stream=None) -> tuple[int, int]:
    r = (ctypes.c_ulonglong * 2)()
    _check(tlib().thrsu_fingerprint(int(key_type), _ptr(keys), n, r, _stream(stream)))
    return int(r[0]), int(r[1])


def check_pairs(key_type: int, value_bytes: int, keys_in, keys_out, vals, n: int, start_bits: int, end_bits: int,
                descending=False, stream=None) -> dict:
    r = (ctypes.c_ulonglong * 5)()
    _check(tlib().thrsu_check_pairs(int(key_type), int(descending), value_bytes, _ptr(keys_in), _ptr(keys_out),
                                    _ptr(vals), n, start_bits, end_bits, r, _stream(stream)))
    return {"gather_mismatch": int(r[0]), "unstable": int(r[1]), "index_sum": int(r[2]), "index_xor": int(r[3]),
            "u128_halves": int(r[4])}


def expected_index_fingerprint(n: int) -> tuple[int, int]:
    """sum and xor-of-mix of 0..n-1, for check_pairs (computed in numpy)."""
    import numpy as np
    s = (n * (n - 1) // 2) % (1 << 64)
    x = 0
    step = 1 << 24
    for a in range(0, n, step):
        i = np.arange(a, min(n, a + step), dtype=np.uint64)
        with np.errstate(over="ignore"):
            z = i
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
        x ^= int(np.bitwise_xor.reduce(z)) if z.size else 0
    return s, x


def copy(dst, src, nbytes: int, width16: bool = True, stream=None):
    """Streaming copy with 16-B (or 4-B) lanes: rocprofv3 byte-counter calibration."""
    _check(tlib().thrsu_copy(_ptr(dst), _ptr(src), nbytes, int(width16), _stream(stream)))


def probe_lds_order_partial(iters: int = 64) -> int:
    """Lanes whose LDS-atomic return broke lane order under a partial exec mask
    (thrs_testutil.hip k_probe_partial); 0 = ordered on this device."""
    bad = ctypes.c_uint(0)
    _check(tlib().thrsu_probe_lds_order_partial(iters, ctypes.byref(bad)))
    return int(bad.value)
