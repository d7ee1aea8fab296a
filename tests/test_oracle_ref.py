"""CPU: pin the oracle (oracle/oracle.cpp + numpy forms) against the
REFERENCE's own host code, built from /root/reference by oracle/ref/Makefile
into oracle/_ref/libfpkey_ref.so:
  getKeyBits(u32/u64/float/double)   fpKey.hpp:15-38 (compiled as-is)
  splitmix64                         unittest.cpp:24-35 (extracted verbatim)
and reproduce the reference's host-only KAT FPKeys.float (unittest.cpp:81-94)
with the reference's transform.  The oracle adds ORDER_MASK (kernel.cu:18-24)
on top, which the reference applies only on the device (pinned on the GPU by
tests/test_gpu_ref.py against the reference's own kernels)."""
import numpy as np
import pytest

import cases as C
from oracle import oracle as O
from oracle import ref as R

pytestmark = pytest.mark.skipif(not R.available(), reason="oracle/_ref not built (needs /root/reference)")


def f32_sweep():
    """Every sign x exponent with the edge and random mantissas, plus the
    SURVEY's special vectors: NaN/Inf/denormals/+-0 all included."""
    rng = np.random.default_rng(1234)
    sign = np.arange(2, dtype=np.uint32)[:, None, None] << 31
    exp = np.arange(256, dtype=np.uint32)[None, :, None] << 23
    mant = np.concatenate([np.array([0, 1, 2, 0x3FFFFF, 0x400000, 0x7FFFFE, 0x7FFFFF], np.uint32),
                           rng.integers(0, 1 << 23, 250, dtype=np.uint32)])[None, None, :]
    bits = (sign | exp | mant).reshape(-1)
    return np.concatenate([bits, np.array(C.F32_SPECIALS, np.uint32)])


def f64_sweep():
    rng = np.random.default_rng(4321)
    sign = np.arange(2, dtype=np.uint64)[:, None, None] << np.uint64(63)
    exp = np.arange(2048, dtype=np.uint64)[None, :, None] << np.uint64(52)
    mant = np.concatenate([np.array([0, 1, (1 << 51), (1 << 52) - 1], np.uint64),
                           rng.integers(0, 1 << 52, 60, dtype=np.uint64)])[None, None, :]
    return (sign | exp | mant).reshape(-1)


def test_splitmix64_is_the_reference_stream():
    ref = R.splitmix64(1 << 20)
    assert [hex(int(x)) for x in ref[:3]] == ["0xe220a8397b1dcdaf", "0x6e789e6aa1b965f4", "0x6c45d188009454f"]
    assert np.array_equal(ref, O.splitmix64_stream(0, 1 << 20))          # numpy counter form
    assert np.array_equal(ref, O.SplitMix64().fill(1 << 20))             # oracle.cpp
    assert np.array_equal(R.splitmix64(1000, state=12345), O.splitmix64_stream(0, 1000, state=12345))


@pytest.mark.parametrize("kt", [O.U32, O.U64, O.F32, O.F64])
def test_key_bits_is_the_reference_transform(kt):
    if kt == O.F32:
        keys = np.concatenate([f32_sweep(), (O.splitmix64_stream(99, 1 << 20) >> np.uint64(7)).astype(np.uint32)])
    elif kt == O.F64:
        keys = np.concatenate([f64_sweep(), O.splitmix64_stream(77, 1 << 20)])
    elif kt == O.U32:
        keys = O.splitmix64_stream(5, 1 << 20).astype(np.uint32)
    else:
        keys = O.splitmix64_stream(6, 1 << 20)
    ref = R.key_bits(kt, keys)
    assert np.array_equal(O.key_bits(kt, keys), ref)            # oracle.cpp
    assert np.array_equal(O.key_bits_np(kt, keys), ref)         # numpy form
    # the device form adds ORDER_MASK (kernel.cu:18-24): descending = the complement
    mask = np.uint64(0xFFFFFFFF if O.KEY_BYTES[kt] == 4 else 0xFFFFFFFFFFFFFFFF)
    assert np.array_equal(O.key_bits(kt, keys, descending=True), ref ^ mask)


def test_reference_stream_generators():
    """randomizeValues (unittest.cpp:96-116) over the reference's splitmix64."""
    draws = R.splitmix64(5000, state=0)
    r = O.SplitMix64()
    for kt in (O.U32, O.F32, O.U64, O.F64):
        r = O.SplitMix64()
        assert np.array_equal(r.randomize_keys(kt, 5000), O.randomize_np(kt, draws))


def test_fpkeys_float_kat_with_reference_transform():
    """FPKeys.float (unittest.cpp:81-94) with the reference's own getKeyBits:
    -0 and +0 share a key, FLT_MAX < +Inf, and a < b <=> key(a) < key(b) on
    random pairs -- and the oracle agrees on every one."""
    f = np.array([-0.0, 0.0, np.finfo(np.float32).max, np.inf], np.float32).view(np.uint32)
    kb = R.key_bits(O.F32, f)
    assert kb[0] == kb[1] and kb[2] < kb[3]
    rng = np.random.default_rng(7)
    n = 1_000_000
    a = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    b = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    ka, kb2 = R.key_bits(O.F32, a.view(np.uint32)), R.key_bits(O.F32, b.view(np.uint32))
    assert np.array_equal(a < b, ka < kb2)
    assert np.array_equal(O.key_bits(O.F32, a.view(np.uint32)), ka)
