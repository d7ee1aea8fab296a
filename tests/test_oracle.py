"""CPU: pin the oracle against the golden fixtures and the reference's own test
oracles (no GPU)."""
import json
import os

import numpy as np
import pytest

import cases as C
from oracle import oracle as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
FAST_ITERS = 12   # the full 128 are checked by tests/golden/make_golden.py and the GPU suite


def test_splitmix64_anchors():
    # SURVEY.md s4 (computed independently in the survey session)
    r = O.SplitMix64()
    got = [r.next() for _ in range(3)]
    assert got == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]
    assert [hex(x) for x in got] == GOLDEN["anchors"]["splitmix64_first3"]
    assert np.array_equal(O.splitmix64_stream(0, 3), np.array(got, dtype=np.uint64))
    # counter form at an offset == sequential draws
    r = O.SplitMix64()
    seq = r.fill(1000)
    assert np.array_equal(O.splitmix64_stream(500, 500), seq[500:])


def test_sortkeys_u32_anchor():
    r = O.SplitMix64()
    n = 1 + r.next() % 99999
    k = r.randomize_keys(O.U32, n)
    assert n == 11258 and int(k[0]) == 0xA1B965F4
    s, _ = O.lsd_sort(O.U32, k)
    assert int(s[0]) == 0x000B41DE and int(s[-1]) == 0xFFFF8DA9
    assert C.digest(s) == "9481ce9aac4311b7" == GOLDEN["anchors"]["SortKeys.u32.iter0"]["sha256_16"]


@pytest.mark.parametrize("name", list(C.CASES))
def test_oracle_matches_golden(name):
    rows = GOLDEN["cases"][name]
    assert len(rows) == C.TEST_ITERATION
    for i, item in enumerate(C.CASES[name][4](FAST_ITERS)):
        k, v = C.oracle_result(name, item)
        assert rows[i]["n"] == item["n"]
        assert rows[i]["keys"] == C.digest(k), (name, i)
        if v is not None:
            assert rows[i]["values"] == C.digest(v), (name, i)


def test_f32_specials_order():
    keys = np.array(C.F32_SPECIALS, np.uint32)
    asc, _ = O.lsd_sort(O.F32, keys)
    desc, _ = O.lsd_sort(O.F32, keys, descending=True)
    assert asc.tolist() == C.F32_SPECIALS_ASC
    assert desc.tolist() == C.F32_SPECIALS_DESC


@pytest.mark.parametrize("kt", [O.U32, O.U64, O.F32, O.F64])
@pytest.mark.parametrize("desc", [False, True])
def test_transform_c_vs_numpy(kt, desc):
    raw = O.splitmix64_stream(0, 20000)
    keys = O.randomize_np(kt, raw) if kt in (O.U32, O.U64) else raw.astype(O.KEY_DTYPE[kt])
    keys = np.concatenate([keys, np.array([0, 1, 0x80000000, 0x7F800000, 0xFF800000, 0xFFFFFFFF],
                                          O.KEY_DTYPE[kt])])
    assert np.array_equal(O.key_bits(kt, keys, desc), O.key_bits_np(kt, keys, desc))


def test_float_transform_orders_like_float_compare():
    # FPKeys.float (unittest.cpp:81-94) on 10^6 vectorised pairs drawn the same way
    # (the reference's evaluation order of its two next() calls per operand is
    # unsequenced; the property, not the exact pairs, is what it pins)
    draws = O.splitmix64_stream(0, 4_000_000).reshape(-1, 4)
    def mk(sign, mag):
        return (np.where(sign % np.uint64(2) == 0, -1.0, 1.0) * mag.astype(np.float64) * 0.1).astype(np.float32)
    a = mk(draws[:, 0], draws[:, 1])
    b = mk(draws[:, 2], draws[:, 3])
    ka = O.key_bits(O.F32, a.view(np.uint32))
    kb = O.key_bits(O.F32, b.view(np.uint32))
    assert np.array_equal(a < b, ka < kb)
    assert O.key_bits(O.F32, np.array([0x80000000], np.uint32))[0] == O.key_bits(O.F32, np.array([0], np.uint32))[0]


@pytest.mark.parametrize("kt", [O.U32, O.U64, O.F32, O.F64])
def test_lsd_vs_contract_windows(kt):
    rng = np.random.default_rng(7)
    width = O.KEY_BYTES[kt] * 8
    raw = O.splitmix64_stream(77, 5000)
    keys = O.randomize_np(kt, raw)
    keys[::7] = keys[3]  # ties
    vals = np.arange(keys.shape[0], dtype=np.uint32)
    for _ in range(12):
        s = int(rng.integers(0, width))
        e = s + 8 * int(rng.integers(0, (width - s) // 8 + 2))
        for desc in (False, True):
            k, v = O.lsd_sort(kt, keys, vals, s, e, desc)
            order = O.contract_sort_order(kt, keys, s, e, desc)
            assert np.array_equal(keys[order], k)
            assert np.array_equal(vals[order], v)


def test_lsd_rejects_bad_bit_range():
    with pytest.raises(ValueError):
        O.lsd_sort(O.U32, np.zeros(4, np.uint32), None, 0, 31)


def test_lsd_empty_and_noop():
    k, _ = O.lsd_sort(O.U32, np.zeros(0, np.uint32))
    assert k.shape == (0,)
    x = np.array([5, 3, 9], np.uint32)
    k, _ = O.lsd_sort(O.U32, x, None, 16, 16)
    assert k.tolist() == [5, 3, 9]


def test_golden_is_pinned_by_the_reference():
    """tests/golden/pin_golden.py recorded that the reference's own kernels
    (make_golden_ref.py on MI355X) produce every committed digest."""
    p = GOLDEN.get("pinned_by")
    assert p and p["rows"] == sum(len(r) for r in GOLDEN["cases"].values()) == 17 * 128
    assert "reference kernels" in p["source"]
