"""The reference's test streams, regenerated bit-exactly.

Each generator yields the inputs one iteration of the matching UTEST in
/root/reference/unittest.cpp would feed to sortKeys/sortPairs: splitmix64 with
state 0 recreated per test (unittest.cpp:24-35, 135, 198, 261, 305, 386),
n = 1 + next() % 99999 (:138), randomizeValues (:96-116), values = index
(:315-318, 394-397), u128 = {i, i} (:471-481).

Test infrastructure only (imports the oracle's splitmix64).
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from oracle import oracle as O  # noqa: E402

TEST_ITERATION = 128      # unittest.cpp:20
TEST_MAX_ARRAY_SIZE = 100000

KEY_NAMES = {"u32": O.U32, "u64": O.U64, "f32": O.F32, "f64": O.F64}


def _values(n: int, vbytes: int) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    if vbytes == 4:
        return i.astype(np.uint32)
    if vbytes == 8:
        return i
    return np.stack([i, i], axis=1).copy()     # u128{x, x}


def sort_keys_stream(key_type: int, iterations: int = TEST_ITERATION):
    """testSortKeys<K> (unittest.cpp:127-168)."""
    rng = O.SplitMix64()
    for _ in range(iterations):
        n = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1)
        yield {"n": n, "keys": rng.randomize_keys(key_type, n)}


def extreme_stream(iterations: int = TEST_ITERATION):
    """SortKeys.extremeCase (unittest.cpp:191-225)."""
    rng = O.SplitMix64()
    for _ in range(iterations):
        n = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1)
        k = np.zeros(n, np.uint32)
        k[rng.next() % n] = 1
        k[rng.next() % n] = 42
        yield {"n": n, "keys": k}


def start_bits_keys_stream(iterations: int = TEST_ITERATION):
    """StartBits.u64, sortKeys half (unittest.cpp:261-297); same stream for asc and desc."""
    rng = O.SplitMix64()
    for _ in range(iterations):
        n = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1)
        s = rng.next() % 64
        yield {"n": n, "start": s, "keys": rng.randomize_keys(O.U64, n)}


def start_bits_pairs_stream(iterations: int = TEST_ITERATION):
    """StartBits.u64, sortPairs half (unittest.cpp:305-354), u32 values."""
    rng = O.SplitMix64()
    for _ in range(iterations):
        n = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1)
        s = rng.next() % 64
        yield {"n": n, "start": s, "keys": rng.randomize_keys(O.U64, n), "values": _values(n, 4)}


def sort_pairs_stream(key_type: int, vbytes: int, iterations: int = TEST_ITERATION):
    """testSortPairs<K,V> (unittest.cpp:379-424)."""
    rng = O.SplitMix64()
    for _ in range(iterations):
        n = 1 + rng.next() % (TEST_MAX_ARRAY_SIZE - 1)
        yield {"n": n, "keys": rng.randomize_keys(key_type, n), "values": _values(n, vbytes)}


# name -> (kind, key_type, value_bytes, descending, stream factory)
CASES = {
    "SortKeys.u32": ("keys", O.U32, 0, False, lambda it=TEST_ITERATION: sort_keys_stream(O.U32, it)),
    "SortKeysDescending.u32": ("keys", O.U32, 0, True, lambda it=TEST_ITERATION: sort_keys_stream(O.U32, it)),
    "SortKeys.f32": ("keys", O.F32, 0, False, lambda it=TEST_ITERATION: sort_keys_stream(O.F32, it)),
    "SortKeys.extremeCase": ("keys", O.U32, 0, False, lambda it=TEST_ITERATION: extreme_stream(it)),
    "SortKeys.u64": ("keys", O.U64, 0, False, lambda it=TEST_ITERATION: sort_keys_stream(O.U64, it)),
    "SortKeys.f64": ("keys", O.F64, 0, False, lambda it=TEST_ITERATION: sort_keys_stream(O.F64, it)),
    "SortKeysDescending.f64": ("keys", O.F64, 0, True, lambda it=TEST_ITERATION: sort_keys_stream(O.F64, it)),
    "StartBits.u64.keys": ("window", O.U64, 0, False, lambda it=TEST_ITERATION: start_bits_keys_stream(it)),
    "StartBits.u64.keysDescending": ("window", O.U64, 0, True, lambda it=TEST_ITERATION: start_bits_keys_stream(it)),
    "StartBits.u64.pairs": ("window", O.U64, 4, False, lambda it=TEST_ITERATION: start_bits_pairs_stream(it)),
    "SortPairs.K32V32": ("pairs", O.U32, 4, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.U32, 4, it)),
    "SortPairs.KF32V32": ("pairs", O.F32, 4, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.F32, 4, it)),
    "SortPairs.K64V32": ("pairs", O.U64, 4, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.U64, 4, it)),
    "SortPairs.KF64V32": ("pairs", O.F64, 4, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.F64, 4, it)),
    "SortPairs.K32V64": ("pairs", O.U32, 8, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.U32, 8, it)),
    "SortPairs.K64V64": ("pairs", O.U64, 8, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.U64, 8, it)),
    "SortPairs.K64V128": ("pairs", O.U64, 16, False, lambda it=TEST_ITERATION: sort_pairs_stream(O.U64, 16, it)),
}


def oracle_result(name: str, item: dict):
    """Expected (keys, values) of one iteration, from the LSD restatement."""
    kind, kt, vb, desc, _ = CASES[name]
    keys = item["keys"]
    vals = item.get("values")
    if kind == "window":
        s = int(item["start"])
        return O.lsd_sort(kt, keys, vals, s, s + 8, desc)
    return O.lsd_sort(kt, keys, vals, 0, O.KEY_BYTES[kt] * 8, desc)


def digest(a: np.ndarray | None) -> str | None:
    import hashlib
    if a is None:
        return None
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


# Explicit float vectors: every class of f32 the bit transform orders
# (fpKey.hpp:23-30): -NaN < -Inf < -normal < -denorm < -0 == +0 < +denorm <
# +normal < +Inf < +NaN.  Listed in input order; expected order computed by
# hand below and asserted against the oracle in tests.
F32_SPECIALS = [
    0x7FC00000,  # +qNaN
    0x00000000,  # +0
    0xFF800000,  # -Inf
    0x80000000,  # -0
    0x00000001,  # +min denorm
    0x3F800000,  # +1
    0xFFC00000,  # -qNaN
    0x807FFFFF,  # -max denorm
    0x7F800000,  # +Inf
    0xBF800000,  # -1
    0x80000001,  # -min denorm
    0x007FFFFF,  # +max denorm
    0x7F7FFFFF,  # +FLT_MAX
    0xFF7FFFFF,  # -FLT_MAX
    0x7F800001,  # +sNaN
    0xFFFFFFFF,  # -NaN (all ones)
]
# ascending, stable (+0 at input 1 precedes -0 at input 3)
F32_SPECIALS_ASC = [
    0xFFFFFFFF, 0xFFC00000, 0xFF800000, 0xFF7FFFFF, 0xBF800000, 0x807FFFFF, 0x80000001,
    0x00000000, 0x80000000,
    0x00000001, 0x007FFFFF, 0x3F800000, 0x7F7FFFFF, 0x7F800000, 0x7F800001, 0x7FC00000,
]
# descending, stable: the ORDER_MASK flips the transformed key, ties keep input order
F32_SPECIALS_DESC = [
    0x7FC00000, 0x7F800001, 0x7F800000, 0x7F7FFFFF, 0x3F800000, 0x007FFFFF, 0x00000001,
    0x00000000, 0x80000000,
    0x80000001, 0x807FFFFF, 0xBF800000, 0xFF7FFFFF, 0xFF800000, 0xFFC00000, 0xFFFFFFFF,
]
