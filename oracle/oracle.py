"""Python side of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module, and only as the checker.  The product path
(``libthrs.so`` behind ``include/thrs/tinyhipradixsort.hpp`` and the Python
mirror in ``tinyhipradixsort_amd``) never imports it.

Two restatements live here, and the tests check them against each other:

* ``liboracle.so`` (``oracle.cpp``): splitmix64 (unittest.cpp:24-35), the
  generators (unittest.cpp:96-125), getKeyBits (fpKey.hpp:15-38 plus the
  ORDER_MASK of tinyhipradixsort.hpp:64-115) and the 8-bit-digit pass loop
  (tinyhipradixsort.hpp:854-944); plus the reference tests' own oracles
  std::sort / std::stable_sort (unittest.cpp:154-161, 283-291, 343-348,
  358-377).
* numpy: a vectorised splitmix64 stream (counter form, output i from state s
  is mix(s + gamma*(i+1))) and the sort contract
  ``stable_sort(keys, by=digits of getKeyBits(k)^ORDER_MASK in [start,end))``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lock = threading.Lock()
_lib = None

U32, U64, F32, F64 = 0, 1, 2, 3           # == thrs::KeyType (tinyhipradixsort.hpp:638-644)
KEY_BYTES = {U32: 4, U64: 8, F32: 4, F64: 8}
KEY_DTYPE = {U32: np.uint32, U64: np.uint64, F32: np.uint32, F64: np.uint64}  # raw bit patterns
GAMMA = np.uint64(0x9E3779B97F4A7C15)


def lib():
    """Load (building on first use if needed) liboracle.so."""
    global _lib
    with _lock:
        if _lib is None:
            src = os.path.join(_HERE, "oracle.cpp")
            if (not os.path.exists(_LIB)) or os.path.getmtime(_LIB) < os.path.getmtime(src):
                subprocess.check_call(["make", "-s", "-C", _HERE])
            L = ctypes.CDLL(_LIB)
            vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
            L.orc_splitmix64_next.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
            L.orc_splitmix64_next.restype = u64
            L.orc_splitmix64_fill.argtypes = [ctypes.POINTER(ctypes.c_uint64), vp, u64]
            L.orc_randomize_keys.argtypes = [i32, ctypes.POINTER(ctypes.c_uint64), vp, u64]
            L.orc_key_bits.argtypes = [i32, vp, vp, u64, i32]
            L.orc_lsd_sort.argtypes = [i32, i32, vp, vp, u64, i32, i32, i32]
            L.orc_lsd_sort.restype = i32
            L.orc_std_sort_keys.argtypes = [i32, vp, u64, i32]
            L.orc_parallel_sort_u32.argtypes = [vp, u64]
            L.orc_parallel_sort_u64.argtypes = [vp, u64]
            L.orc_std_stable_sort_pairs.argtypes = [i32, i32, vp, vp, u64]
            L.orc_parallel_stable_sort_pairs.argtypes = [i32, i32, vp, vp, u64]
            L.orc_parallel_sort_keys.argtypes = [i32, vp, u64]
            L.orc_std_stable_sort_window_u64.argtypes = [vp, vp, u64, i32, i32]
            _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


# ---------------------------------------------------------------- splitmix64
class SplitMix64:
    """unittest.cpp:24-35 -- state starts at 0 and is recreated per test."""

    def __init__(self, x: int = 0):
        self.x = ctypes.c_uint64(x)

    def next(self) -> int:
        return int(lib().orc_splitmix64_next(ctypes.byref(self.x)))

    def fill(self, n: int) -> np.ndarray:
        out = np.empty(n, np.uint64)
        lib().orc_splitmix64_fill(ctypes.byref(self.x), _p(out), n)
        return out

    def randomize_keys(self, key_type: int, n: int) -> np.ndarray:
        """randomizeValues<T> (unittest.cpp:96-116); raw bit patterns."""
        out = np.empty(n, KEY_DTYPE[key_type])
        lib().orc_randomize_keys(key_type, ctypes.byref(self.x), _p(out), n)
        return out


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def splitmix64_stream(start: int, n: int, state: int = 0) -> np.ndarray:
    """Draws start+1 .. start+n of splitmix64 seeded with `state` (numpy form)."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        return _mix(np.uint64(state) + GAMMA * i)


def randomize_np(key_type: int, draws: np.ndarray) -> np.ndarray:
    """randomizeValues<T> applied to already-drawn splitmix64 outputs."""
    if key_type == U32:
        return draws.astype(np.uint32)
    if key_type == F32:
        return (draws & np.uint64(0xFF7FFFFF)).astype(np.uint32)
    if key_type == U64:
        return draws.copy()
    return draws & np.uint64(0xFFEFFFFFFFFFFFFF)


# ---------------------------------------------------------------- transforms
def key_bits(key_type: int, keys: np.ndarray, descending: bool = False) -> np.ndarray:
    """getKeyBits(k) ^ ORDER_MASK widened to u64 (C restatement)."""
    keys = np.ascontiguousarray(keys)
    out = np.empty(keys.shape[0], np.uint64)
    lib().orc_key_bits(key_type, _p(keys), _p(out), keys.shape[0], int(descending))
    return out


def key_bits_np(key_type: int, keys: np.ndarray, descending: bool = False) -> np.ndarray:
    """numpy restatement of the same transform (fpKey.hpp:23-38)."""
    if key_type in (U32, U64):
        b = keys.astype(np.uint64)
    elif key_type == F32:
        b = keys.astype(np.uint64)
        b = np.where((b & np.uint64(0x7FFFFFFF)) == 0, np.uint64(0), b)
        flip = np.where(b >> np.uint64(31) != 0, np.uint64(0xFFFFFFFF), np.uint64(0x80000000))
        b = b ^ flip
    else:
        b = keys.astype(np.uint64)
        b = np.where((b & np.uint64(0x7FFFFFFFFFFFFFFF)) == 0, np.uint64(0), b)
        flip = np.where(b >> np.uint64(63) != 0, np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0x8000000000000000))
        b = b ^ flip
    if descending:
        b = b ^ np.uint64(0xFFFFFFFF if KEY_BYTES[key_type] == 4 else 0xFFFFFFFFFFFFFFFF)
    return b


# ---------------------------------------------------------------- sorts
def lsd_sort(key_type: int, keys: np.ndarray, values: np.ndarray | None = None,
             start_bits: int = 0, end_bits: int | None = None, descending: bool = False):
    """Pass-by-pass restatement of RadixSort::sort (tinyhipradixsort.hpp:854-944).

    Returns new (keys, values) arrays; inputs are not modified.  values may be
    any contiguous array whose row is 4, 8 or 16 bytes.
    """
    if end_bits is None:
        end_bits = KEY_BYTES[key_type] * 8
    k = np.ascontiguousarray(keys).copy()
    v = None
    vb = 0
    if values is not None:
        v = np.ascontiguousarray(values).copy()
        vb = v.nbytes // max(1, k.shape[0]) if k.shape[0] else v.dtype.itemsize
    rc = lib().orc_lsd_sort(key_type, vb, _p(k), _p(v), k.shape[0], start_bits, end_bits, int(descending))
    if rc < 0:
        raise ValueError("(endBits - startBits) % 8 != 0 (tinyhipradixsort.hpp:856)")
    return k, v


def contract_sort_order(key_type: int, keys: np.ndarray, start_bits: int = 0,
                        end_bits: int | None = None, descending: bool = False) -> np.ndarray:
    """numpy form of the contract: stable argsort by the [start,end) window of
    getKeyBits(k)^ORDER_MASK, read as 8-bit digits (bits past the key width are 0)."""
    if end_bits is None:
        end_bits = KEY_BYTES[key_type] * 8
    width = KEY_BYTES[key_type] * 8
    b = key_bits_np(key_type, keys, descending)
    order = np.arange(keys.shape[0])
    bit = start_bits
    while bit < end_bits:                      # LSD: one stable pass per digit
        if bit >= width:
            d = np.zeros(keys.shape[0], np.uint64)
        else:
            d = (b[order] >> np.uint64(bit)) & np.uint64(0xFF)
        order = order[np.argsort(d, kind="stable")]
        bit += 8
    return order


def std_sort_keys(key_type: int, keys: np.ndarray, descending: bool = False) -> np.ndarray:
    k = np.ascontiguousarray(keys).copy()
    lib().orc_std_sort_keys(key_type, _p(k), k.shape[0], int(descending))
    return k


def parallel_sort(keys: np.ndarray, key_type: int | None = None) -> np.ndarray:
    """__gnu_parallel::sort with operator< of the key type (floats as floats)."""
    k = np.ascontiguousarray(keys).copy()
    if key_type is None:
        key_type = U32 if k.dtype.itemsize == 4 else U64
    lib().orc_parallel_sort_keys(key_type, _p(k), k.shape[0])
    return k


def parallel_stable_sort_pairs(key_type: int, keys: np.ndarray, values: np.ndarray):
    k = np.ascontiguousarray(keys).copy()
    v = np.ascontiguousarray(values).copy()
    vb = v.nbytes // max(1, k.shape[0])
    lib().orc_parallel_stable_sort_pairs(key_type, vb, _p(k), _p(v), k.shape[0])
    return k, v


def std_stable_sort_pairs(key_type: int, keys: np.ndarray, values: np.ndarray):
    k = np.ascontiguousarray(keys).copy()
    v = np.ascontiguousarray(values).copy()
    vb = v.nbytes // max(1, k.shape[0])
    lib().orc_std_stable_sort_pairs(key_type, vb, _p(k), _p(v), k.shape[0])
    return k, v


def std_stable_sort_window_u64(keys: np.ndarray, values: np.ndarray | None, start_bit: int,
                               descending: bool = False):
    k = np.ascontiguousarray(keys, dtype=np.uint64).copy()
    v = None if values is None else np.ascontiguousarray(values, dtype=np.uint32).copy()
    lib().orc_std_stable_sort_window_u64(_p(k), _p(v), k.shape[0], start_bit, int(descending))
    return k, v
