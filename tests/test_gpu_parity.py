"""GPU parity: libthrs.so (through the C-ABI) against the oracle and the golden
fixtures on the reference's own test streams, plus size-independent property
checks at BASELINE.json's full sizes.  Integer/byte work: bit-exact throughout."""
import json
import os
import subprocess

import numpy as np
import pytest

import cases as C
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def to_dev(torch, a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to("cuda")


def from_dev(t, dtype, shape):
    return t.cpu().numpy().view(dtype).reshape(shape)


def make_sorter(kt, vb, desc, **options):
    import tinyhipradixsort_amd as T
    cfg = T.RadixSort.Config()
    cfg.keyType = T.KeyType(kt)
    cfg.valueType = {0: T.ValueType.U32, 4: T.ValueType.U32, 8: T.ValueType.U64, 16: T.ValueType.U128}[vb]
    cfg.sortOrder = T.SortOrder.Descending if desc else T.SortOrder.Ascending
    return T.RadixSort([], cfg, T.Options(**options))


def gpu_sort(torch, rs, item, kt, vb, start, end):
    keys = item["keys"]
    n = keys.shape[0]
    kd = to_dev(torch, keys)
    d = rs.getTemporaryBufferBytes(n)
    if vb:
        vd = to_dev(torch, item["values"])
        tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
        rs.sortPairs(kd, vd, n, tmp, start, end)
    else:
        vd = None
        tmp = torch.empty(d.getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
        rs.sortKeys(kd, n, tmp, start, end)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    k = from_dev(kd, O.KEY_DTYPE[kt], (n,))
    v = None if vd is None else from_dev(vd, item["values"].dtype, item["values"].shape)
    return k, v


@pytest.mark.parametrize("name", list(C.CASES))
def test_reference_streams_bit_exact(gpu, name):
    """Every iteration of the reference's UTEST streams: GPU output digest ==
    golden digest; the first iterations also compared element-wise to the oracle."""
    torch = gpu
    kind, kt, vb, desc, stream = C.CASES[name]
    rs = make_sorter(kt, vb, desc)
    rows = GOLDEN["cases"][name]
    for i, item in enumerate(stream()):
        if kind == "window":
            s = int(item["start"])
            start, end = s, s + 8
        else:
            start, end = 0, O.KEY_BYTES[kt] * 8
        k, v = gpu_sort(torch, rs, item, kt, vb, start, end)
        if i < 4:
            ek, ev = C.oracle_result(name, item)
            assert np.array_equal(k, ek), (name, i)
            if ev is not None:
                assert np.array_equal(v, ev), (name, i)
        assert C.digest(k) == rows[i]["keys"], (name, i, item["n"])
        if vb:
            assert C.digest(v) == rows[i]["values"], (name, i, item["n"])


@pytest.mark.parametrize("desc", [False, True])
def test_f32_special_values(gpu, desc):
    torch = gpu
    keys = np.array(C.F32_SPECIALS, np.uint32)
    rs = make_sorter(O.F32, 4, desc)
    item = {"keys": keys, "values": np.arange(keys.shape[0], dtype=np.uint32)}
    k, v = gpu_sort(torch, rs, item, O.F32, 4, 0, 32)
    assert k.tolist() == (C.F32_SPECIALS_DESC if desc else C.F32_SPECIALS_ASC)
    assert np.array_equal(keys[v], k)


@pytest.mark.parametrize("kt", [O.U32, O.U64, O.F32, O.F64])
@pytest.mark.parametrize("vb", [0, 4, 8, 16])
@pytest.mark.parametrize("desc", [False, True])
def test_matrix_vs_oracle(gpu, kt, vb, desc):
    """Every (key, value, order) combination, tile-boundary sizes, random windows."""
    torch = gpu
    rs = make_sorter(kt, vb, desc)
    width = O.KEY_BYTES[kt] * 8
    rng = np.random.default_rng(kt * 100 + vb * 2 + desc)
    sizes = [1, 2, 63, 64, 65, 255, 256, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 8193, 16385, 50000,
             123457]
    for j, n in enumerate(sizes):
        draws = O.splitmix64_stream(1000 * j, n)
        keys = O.randomize_np(kt, draws)
        if j % 3 == 1:
            keys = keys & np.array(0xF0F, keys.dtype)   # heavy ties: stability visible
        if j % 5 == 2:
            keys[:] = keys[0]                           # one bucket holds everything
        vals = C._values(n, vb) if vb else None
        if j % 4 == 3:
            s = int(rng.integers(0, width))
            e = s + 8 * int(rng.integers(1, 4))
        else:
            s, e = 0, width
        item = {"keys": keys, "values": vals}
        k, v = gpu_sort(torch, rs, item, kt, vb, s, e)
        ek, ev = O.lsd_sort(kt, keys, vals, s, e, desc)
        assert np.array_equal(k, ek), (n, s, e)
        if vb:
            assert np.array_equal(v, ev), (n, s, e)


def test_rank_probe_and_ballot_fallback(gpu):
    """The LDS-atomic rank path is used only where the lane-order probe passes;
    the ballot-match fallback must be bit-exact too (forced: Options.rank)."""
    import tinyhipradixsort_amd as T
    mode = T.lib().thrs_rank_mode()
    assert mode in (0, 1)
    print("rank mode:", "lds-atomic" if mode else "ballot")
    exe = os.path.join(ROOT, "tests", "cpp", "unittest_thrs")
    r = subprocess.run([exe, "--filter=SortPairs.K", "--rank=ballot"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]


def test_rank_order_partial_waves(gpu):
    """The atomic rank is only ever issued by fully active waves (padding
    items are ranked too), which is what thrs_probe_lds_order certifies.  This
    records whether the lane order also holds under partial exec masks, so a
    future partial-wave use is not relying on an unmeasured property."""
    from tinyhipradixsort_amd import testutil as TU
    import tinyhipradixsort_amd as T
    bad = TU.probe_lds_order_partial(64)
    print("partial-mask lane-order violations:", bad)
    if T.lib().thrs_rank_mode() == 1:
        assert bad == 0, f"{bad} lanes out of order under partial exec masks"


def test_cpp_port_of_reference_unittest(gpu):
    """The reference's UTEST matrix, ported to C++ against the drop-in header."""
    exe = os.path.join(ROOT, "tests", "cpp", "unittest_thrs")
    assert os.path.exists(exe), "build tests/cpp/unittest_thrs first (make)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=900)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


@pytest.mark.parametrize("claims", ["xcd", "ticket"])
def test_cpp_port_with_claim_mode_forced(gpu, claims):
    """The same UTEST matrix with the XCD-block tile claims (thrs_pass_xb)
    forced on for every configuration and size, and forced off (one-ticket
    tile ids): by default they only run for 4-byte keys at n >= 2^29."""
    exe = os.path.join(ROOT, "tests", "cpp", "unittest_thrs")
    r = subprocess.run([exe, f"--claims={claims}"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


@pytest.mark.parametrize("path", ["bucket", "lsd"])
def test_cpp_port_with_path_forced(gpu, path):
    """The UTEST matrix with the 3-HBM-pass path (bucket passes + local LDS
    sort, thrs_hybrid.hpp) forced on for every size (by default it runs from a
    measured bound per key / value type, thrs_host.hpp kBucketMin*) and off
    (plain LSD passes)."""
    exe = os.path.join(ROOT, "tests", "cpp", "unittest_thrs")
    r = subprocess.run([exe, f"--path={path}"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


@pytest.mark.parametrize("geom,seg", [("big", "1"), ("small", "1"), ("big", "0"), ("big", "top"), ("big32", "1"),
                                      ("big", "1-noplanes"), ("count16", "1"), ("count16", "1-noplanes"),
                                      ("count16", "0"), ("wide16", "1"), ("wide16", "1-noplanes"), ("tiny16", "1"),
                                      ("tiny16", "1-noplanes")])
@pytest.mark.parametrize("kt", [O.U32, O.F32])
@pytest.mark.parametrize("desc", [False, True])
def test_hybrid_paths_vs_oracle(gpu, kt, desc, geom, seg):
    """4-byte keys-only sorts with >= 3 digits take the hybrid path (forced
    here for every size; by default from 60M u32 / 40M f32 keys): chunked
    local sort (single- and multi-bucket chunks), and the gated fallback to
    plain LSD when one bucket exceeds the local capacity (18432 keys) --
    including an odd number of low passes (window of 3 digits: gated copy)."""
    torch = gpu
    # the two top-digit passes XCD-segmented (default), neither, or the top one
    # only; local-sort geometry: 18432- or 9216-key chunks; u32 keys over the
    # whole key sort 16-bit items in the big geometry unless "big32" -- by two
    # LSD rounds (default, "rank16") or by counting ("count16"), or in 34816-key
    # chunks ("wide16", the default above 2^30 + 2^26); with both top passes
    # segmented ("1") the 16-bit local sorts' keys travel as u16/u8 planes
    # through the top-digit passes (the temporary buffer holds the u8 plane at
    # every size) unless "noplanes" (thrs_options.planes)
    rs = make_sorter(kt, 0, desc, path="bucket",
                     segmented={"1": "auto", "0": "none", "top": "top_only"}[seg.split("-")[0]], localGeometry=geom,
                     planes="off" if seg.endswith("noplanes") else "auto")
    want_planes = seg == "1" and geom != "big32"
    assert rs.pathInfo(1 << 20, 0, 32, False)["planes"] == want_planes
    dists = {
        "uniform": lambda k: k,
        "low20": lambda k: k & np.array(0xFFFFF, k.dtype),        # 16 buckets -> fallback above 295k keys
        "top_skew": lambda k: k | np.array(0x7F000000, k.dtype),  # top digit fixed
        "ties": lambda k: k & np.array(0xFF00FF00, k.dtype),
        "const": lambda k: np.full_like(k, k[0]),
    }
    sizes = [1, 100, 18432, 18433, 70001, 300007, 1 << 20]
    windows = [(0, 32), (8, 32), (0, 24), (4, 28)]
    j = 0
    for name, f in dists.items():
        for n in sizes:
            for (s, e) in windows:
                j += 1
                if j % 2 and n >= 300007 and (s, e) != (0, 32):
                    continue  # keep the case count bounded
                keys = f(O.randomize_np(kt, O.splitmix64_stream(7777 * j, n)))
                k, _ = gpu_sort(torch, rs, {"keys": keys, "values": None}, kt, 0, s, e)
                ek, _ = O.lsd_sort(kt, keys, None, s, e, desc)
                assert np.array_equal(k, ek), (name, n, s, e)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("geom", ["big", "small", "tiny16"])
@pytest.mark.parametrize("kt", [O.U32, O.F32])
def test_hybrid_pairs_vs_oracle(gpu, kt, desc, geom):
    """sortPairs with 4-byte keys + u32 values over the whole key takes the
    hybrid path (single-bucket chunks, positions carried in the local sort's
    items); stability on ties, the gated LSD fallback, and partial windows
    (plain LSD).  f32 keys in every geometry too (a forced "tiny16" sends them
    through thrs_local_pairs<LocTiny>, whose keys are rebuilt from their
    images unless some key is -0: the "ties" stream holds +-0)."""
    torch = gpu
    rs = make_sorter(kt, 4, desc, path="bucket", localGeometry=geom)  # forced for every size
    dists = {
        "uniform": lambda k: k,
        "low20": lambda k: k & np.array(0xFFFFF, k.dtype),
        "ties": lambda k: k & np.array(0xFF00FF00, k.dtype),
        "few": lambda k: k & np.array(0x00030007, k.dtype),
        "const": lambda k: np.full_like(k, k[0]),
    }
    j = 0
    for name, f in dists.items():
        for n in [1, 100, 18432, 18433, 70001, 300007, 1 << 20]:
            for (s, e) in [(0, 32), (8, 32)]:
                j += 1
                keys = f(O.randomize_np(kt, O.splitmix64_stream(9191 * j, n)))
                if kt == O.F32 and name == "ties":                 # +0 and -0 among the ties
                    keys[3::11] = np.where(np.arange(keys[3::11].shape[0]) % 2, np.uint32(0x80000000), np.uint32(0))
                vals = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)
                k, v = gpu_sort(torch, rs, {"keys": keys, "values": vals}, kt, 4, s, e)
                ek, ev = O.lsd_sort(kt, keys, vals, s, e, desc)
                assert np.array_equal(k, ek), (name, n, s, e)
                assert np.array_equal(v, ev), (name, n, s, e)


@pytest.mark.parametrize("kt", [O.U64, O.F64])
@pytest.mark.parametrize("vb", [0, 8])
@pytest.mark.parametrize("desc", [False, True])
def test_bucket64_vs_oracle(gpu, kt, vb, desc):
    """8-byte keys (with or without 8-byte values) over the whole key take the
    bucket path (forced here for every size; by default n in [12M-20M, 2^30 +
    2^24]): two device passes on the top 16 bits, the in-LDS sort per bucket
    (thrs_local_kv), u64 keys rebuilt / f64 keys and values permuted by
    carried positions; a bucket above 17408 keys takes the LSD fallback."""
    torch = gpu
    rs = make_sorter(kt, vb, desc, path="bucket")
    mask48 = np.uint64(0xFFFF000000000000)
    dists = {
        "uniform": lambda k: k,
        "low40": lambda k: k & np.uint64(0xFFFFFFFFFF),                  # one bucket -> fallback above 17408
        "top_fixed": lambda k: (k & ~mask48) | np.uint64(0x3FF0000000000000),
        "ties": lambda k: k & np.uint64(0xFFFF0000FF00FF00),
        "const": lambda k: np.full_like(k, k[0]),
        "signed_zero": lambda k: np.where(k & np.uint64(1), np.uint64(0x8000000000000000), np.uint64(0)),
    }
    j = 0
    for name, f in dists.items():
        for n in [1, 100, 17408, 17409, 70001, 300007, 1 << 20]:
            j += 1
            keys = f(O.randomize_np(kt, O.splitmix64_stream(4242 * j, n))).astype(np.uint64)
            vals = np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) if vb else None
            k, v = gpu_sort(torch, rs, {"keys": keys, "values": vals}, kt, vb, 0, 64)
            ek, ev = O.lsd_sort(kt, keys, vals, 0, 64, desc)
            assert np.array_equal(k, ek), (name, n)
            if vb:
                assert np.array_equal(v, ev), (name, n)


def test_concurrent_sorts_on_distinct_temps(gpu):
    """Per-call state lives in the caller's temp buffer: two sorts on two
    streams at once (the reference's module-global g_iterator would race)."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    rs = make_sorter(O.U32, 0, False)
    n = 3_000_001
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
    b = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
    TU.fill_keys(O.U32, a, n, 0)
    TU.fill_keys(O.U32, b, n, 12345)
    torch.cuda.synchronize()
    fa, fb = TU.fingerprint(O.U32, a, n), TU.fingerprint(O.U32, b, n)
    d = rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys()
    ta = torch.empty(d, dtype=torch.uint8, device="cuda")
    tb = torch.empty(d, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        rs.sortKeys(a, n, ta, 0, 32, s1)
        rs.sortKeys(b, n, tb, 0, 32, s2)
    torch.cuda.synchronize()
    for buf, f in ((a, fa), (b, fb)):
        assert TU.count_unsorted(O.U32, buf, n, 0, 32) == 0
        assert TU.fingerprint(O.U32, buf, n) == f


# ------------------------------------------------------------ full sizes
def _big_keys(torch, kt, n, start=0):
    from tinyhipradixsort_amd import testutil as TU
    kb = O.KEY_BYTES[kt]
    keys = torch.empty(kb * n, dtype=torch.uint8, device="cuda")
    TU.fill_keys(kt, keys, n, start)
    return keys


@pytest.mark.large
@pytest.mark.parametrize("kt,n,desc", [(O.U32, 1 << 30, False),      # C2
                                       (O.F32, 1 << 28, False),      # C4
                                       (O.U32, 1 << 28, True),
                                       (O.U64, 1 << 28, False),
                                       (O.F64, 1 << 27, True)])
def test_full_size_keys_properties(gpu, kt, n, desc):
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    keys = _big_keys(torch, kt, n)
    torch.cuda.synchronize()
    fp = TU.fingerprint(kt, keys, n)
    rs = make_sorter(kt, 0, desc)
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8,
                      device="cuda")
    rs.sortKeys(keys, n, tmp, 0, O.KEY_BYTES[kt] * 8)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert TU.count_unsorted(kt, keys, n, 0, O.KEY_BYTES[kt] * 8, desc) == 0
    assert TU.fingerprint(kt, keys, n) == fp
    # spot-check a window of the output against the oracle's sort of the same stream
    if n <= (1 << 28):
        k = from_dev(keys[: O.KEY_BYTES[kt] * 4096], O.KEY_DTYPE[kt], (4096,))
        assert np.array_equal(O.key_bits(kt, k, desc), np.sort(O.key_bits(kt, k, desc)))


@pytest.mark.large
def test_f32_raw_bits_with_nan_inf_full_size(gpu):
    """C4's second variant: raw 32-bit patterns (NaN/Inf/denormals included)."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    n = 1 << 28
    keys = _big_keys(torch, O.U32, n, 777)       # raw bits, reinterpreted as f32 keys
    torch.cuda.synchronize()
    fp = TU.fingerprint(O.F32, keys, n)
    rs = make_sorter(O.F32, 0, False)
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8,
                      device="cuda")
    rs.sortKeys(keys, n, tmp, 0, 32)
    torch.cuda.synchronize()
    assert TU.count_unsorted(O.F32, keys, n, 0, 32) == 0
    assert TU.fingerprint(O.F32, keys, n) == fp


@pytest.mark.large
@pytest.mark.parametrize("kt,vb,n", [(O.U32, 4, 1 << 30),     # C3
                                     (O.U64, 8, 1 << 30),     # C5's per-GPU local shape
                                     (O.U64, 8, 1 << 28),
                                     (O.F64, 8, 1 << 29),
                                     (O.F32, 8, 1 << 27),
                                     (O.U64, 16, 1 << 26)])
def test_full_size_pairs_stability(gpu, kt, vb, n):
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    keys = _big_keys(torch, kt, n)
    orig = keys.clone()
    vals = torch.empty(vb * n, dtype=torch.uint8, device="cuda")
    TU.iota(vb, vals, n)
    rs = make_sorter(kt, vb, False)
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8,
                      device="cuda")
    rs.sortPairs(keys, vals, n, tmp, 0, O.KEY_BYTES[kt] * 8)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    width = O.KEY_BYTES[kt] * 8
    r = TU.check_pairs(kt, vb, orig, keys, vals, n, 0, width)
    assert r["gather_mismatch"] == 0 and r["unstable"] == 0 and r["u128_halves"] == 0
    assert TU.count_unsorted(kt, keys, n, 0, width) == 0
    assert (r["index_sum"], r["index_xor"]) == TU.expected_index_fingerprint(n)


@pytest.mark.large
def test_u32_large_2pow31_plus_100(gpu):
    """SortKeys.u32Large (unittest.cpp:688-717): N = 2^31+100, 64-bit look-back words."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    n = (1 << 31) + 100
    keys = _big_keys(torch, O.U32, n)
    torch.cuda.synchronize()
    fp = TU.fingerprint(O.U32, keys, n)
    rs = make_sorter(O.U32, 0, False)
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8,
                      device="cuda")
    rs.sortKeys(keys, n, tmp, 0, 32)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert TU.count_unsorted(O.U32, keys, n, 0, 32) == 0
    assert TU.fingerprint(O.U32, keys, n) == fp
    # the first and last values of the reference's stream, pinned on the host
    head = from_dev(keys[:4 * 8], np.uint32, (8,))
    assert head[0] <= head[-1]


@pytest.mark.large
@pytest.mark.parametrize("dist", ["sorted", "reverse", "extreme", "fewuniq"])
@pytest.mark.parametrize("kt,vb,n", [(O.U32, 0, 1 << 30),      # C2 shape (3-HBM-pass path / its fallback)
                                     (O.U32, 4, 1 << 30),      # C3 shape
                                     (O.F32, 0, 1 << 28),      # C4 shape
                                     (O.U64, 8, 1 << 26)])
def test_full_size_low_entropy(gpu, dist, kt, vb, n):
    """Already-sorted, reverse-sorted, extremeCase (unittest.cpp:191-225) and
    16-distinct-key inputs at full size: sortedness, multiset fingerprint and,
    for pairs with index payloads, gather consistency + stability."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    kb = O.KEY_BYTES[kt]
    keys = torch.empty(kb * n, dtype=torch.uint8, device="cuda")
    TU.fill_dist(kt, keys, n, dist)
    orig = keys.clone() if vb else None
    torch.cuda.synchronize()
    fp = TU.fingerprint(kt, keys, n)
    rs = make_sorter(kt, vb, False)
    d = rs.getTemporaryBufferBytes(n)
    if vb:
        vals = torch.empty(vb * n, dtype=torch.uint8, device="cuda")
        TU.iota(vb, vals, n)
        tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
        rs.sortPairs(keys, vals, n, tmp, 0, kb * 8)
    else:
        tmp = torch.empty(d.getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
        rs.sortKeys(keys, n, tmp, 0, kb * 8)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert TU.count_unsorted(kt, keys, n, 0, kb * 8) == 0
    assert TU.fingerprint(kt, keys, n) == fp
    if vb:
        r = TU.check_pairs(kt, vb, orig, keys, vals, n, 0, kb * 8)
        assert r["gather_mismatch"] == 0 and r["unstable"] == 0
        assert (r["index_sum"], r["index_xor"]) == TU.expected_index_fingerprint(n)


@pytest.mark.parametrize("kt,vb", [(O.U32, 8), (O.U32, 16), (O.F32, 4), (O.F32, 8), (O.F32, 16), (O.U64, 4),
                                   (O.U64, 16), (O.F64, 4), (O.F64, 8), (O.F64, 16)])
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("geom", ["auto", "small", "big"])
def test_bucket_wide_payloads_vs_oracle(gpu, kt, vb, desc, geom):
    """f1: sortPairs with 8/16-byte payloads (ValueType::U128,
    tinyhipradixsort.hpp:779; K64V128, unittest.cpp:469-487) and f32 pairs on
    the bucket path (forced for every size): thrs_local_kv / thrs_local_pairs
    carry chunk positions and permute values -- and float keys, whose +0 and
    -0 share one image -- through the LDS stage; 16-byte values move whole.
    Big buckets take the per-bucket fallback.  thrs_local_kv in each of its
    geometries (auto at these sizes = 4352-key chunks, small = 8704, big =
    17408: sizes around every capacity)."""
    torch = gpu
    rs = make_sorter(kt, vb, desc, path="bucket", localGeometry=geom)
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    sign = np.array(1 << (8 * kb - 1), dtype=kdt)
    dists = {
        "uniform": lambda k: k,
        "ties": lambda k: k & np.array(0xFF00FF00 if kb == 4 else 0xFFFF0000FF00FF00, dtype=kdt),
        "signed_zero": lambda k: np.where(k & np.array(1, kdt), sign, np.array(0, kdt)).astype(kdt),
        "lowbits": lambda k: k & np.array((1 << (8 * kb - 12)) - 1, dtype=kdt),   # 16 big buckets
        "const": lambda k: np.full_like(k, k[0]),
    }
    j = 0
    for name, f in dists.items():
        for n in [1, 100, 4352, 4353, 8704, 8705, 17408, 17409, 70001, 300007]:
            j += 1
            keys = f(O.randomize_np(kt, O.splitmix64_stream(5151 * j + vb, n))).astype(kdt)
            vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(
                {4: np.uint32, 8: np.uint64, 16: np.uint64}[vb])
            if vb == 16:
                vals = vals.reshape(n, 2)
            k, v = gpu_sort(torch, rs, {"keys": keys, "values": vals}, kt, vb, 0, 8 * kb)
            ek, ev = O.lsd_sort(kt, keys, vals, 0, 8 * kb, desc)
            assert np.array_equal(k.view(kdt), ek.view(kdt)), (name, n)
            assert np.array_equal(v, ev), (name, n)


@pytest.mark.parametrize("kt,vb", [(O.U64, 0), (O.U64, 8), (O.F64, 8), (O.U64, 16)])
@pytest.mark.parametrize("desc", [False, True])
def test_local_kv_tie_runs(gpu, kt, vb, desc):
    """thrs_local_kv on 8-byte keys sorts each chunk by the 16 bits below the
    bucket (two rounds), then insertion-sorts every run of items sharing those
    bits on the rest of the key and the position; a run longer than 32 items
    sends the chunk back to input order and six rounds.  Keys here fill 256
    buckets of ~16K keys (near the 17408-key chunk capacity) with those 16
    bits drawn from 4096 values (runs of ~4: the fix-up), from 64 values (runs
    of ~256: the six rounds), constant, or with whole keys repeated in runs
    (the 17408-key geometry, asked: by size this n takes 4352-key chunks)."""
    torch = gpu
    rs = make_sorter(kt, vb, desc, path="bucket", localGeometry="big")
    kdt = O.KEY_DTYPE[kt]
    n = 1 << 22
    r = O.splitmix64_stream(777 + vb + 2 * desc, 2 * n)
    # 256 buckets: the image's top 16 bits differ in bits 53..60 only (bit 52
    # clear: f64 keys are finite)
    top = (r[:n] >> np.uint64(56)) << np.uint64(53)
    low = r[n:] & np.uint64(0xFFFFFFFF)
    cases = {
        "runs4": top | ((r[n:] >> np.uint64(40)) & np.uint64(0xFFF)) << np.uint64(32) | low,
        "runs256": top | ((r[n:] >> np.uint64(40)) & np.uint64(0x3F)) << np.uint64(32) | low,
        "const16": top | np.uint64(0x1234) << np.uint64(32) | low,
        "dupkeys": top | ((r[n:] >> np.uint64(40)) & np.uint64(0xFFF)) << np.uint64(32) | (low & np.uint64(3)),
    }
    for name, keys in cases.items():
        keys = keys.astype(np.uint64).view(kdt)
        vals = None
        if vb:
            vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(
                {4: np.uint32, 8: np.uint64, 16: np.uint64}[vb])
            if vb == 16:
                vals = vals.reshape(n, 2)
        (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
        ek, ev = O.lsd_sort(kt, keys, vals, 0, 64, desc)
        assert mode == 0, (name, mode, big)     # every chunk sorted locally
        assert np.array_equal(k.view(kdt), ek.view(kdt)), name
        if vb:
            assert np.array_equal(v, ev), name


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("geom", ["auto", "small", "wide16", "tiny16"])
def test_f32_keys_only_zero_chunk(gpu, desc, geom):
    """f32 keys-only on the bucket path sort 16-bit items (thrs_local16): +0
    and -0 share one image, so the chunk holding it takes the zeros' bit
    patterns from the input in input order (fpKey.hpp:23-30: -0 -> +0, stable).
    Mixed with the denormals and tiny normals that share the zero's bucket."""
    torch = gpu
    rs = make_sorter(O.F32, 0, desc, path="bucket", localGeometry=geom)
    for j, n in enumerate([1, 64, 5000, 100003, 1 << 20]):
        raw = O.splitmix64_stream(8080 + j, n).astype(np.uint32)
        sel = raw % np.uint32(4)
        small = raw >> np.uint32(18)                       # denormals 1 .. 2^14, positive or negative
        keys = np.where(sel == 0, np.uint32(0x80000000), np.where(sel == 1, np.uint32(0),
                        np.where(sel == 2, small, small | np.uint32(0x80000000)))).astype(np.uint32)
        keys[::7] = O.randomize_np(O.F32, O.splitmix64_stream(99 + j, n))[::7]
        k, _ = gpu_sort(torch, rs, {"keys": keys, "values": None}, O.F32, 0, 0, 32)
        ek, _ = O.lsd_sort(O.F32, keys, None, 0, 32, desc)
        assert np.array_equal(k.view(np.uint32), ek.view(np.uint32)), (n, geom)


def _mode_after(torch, rs, keys, vals, kt, vb):
    n = keys.shape[0]
    kd = to_dev(torch, keys)
    d = rs.getTemporaryBufferBytes(n)
    tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
    if vb:
        vd = to_dev(torch, vals)
        rs.sortPairs(kd, vd, n, tmp, 0, 8 * O.KEY_BYTES[kt])
    else:
        vd = None
        rs.sortKeys(kd, n, tmp, 0, 8 * O.KEY_BYTES[kt])
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    mode = rs.debugBucketMode(tmp, n, bool(vb))
    k = from_dev(kd, O.KEY_DTYPE[kt], (n,))
    v = None if vd is None else from_dev(vd, vals.dtype, vals.shape)
    return mode, k, v


def _squeezed_images(img, W, cap):
    """numpy model of thrs_plan_rows's squeeze decision (thrs_hybrid.hpp
    plan_squeeze): if some bucket would overflow and not every key is in one
    bucket, in each image half holding big buckets drop the highest bucket bit
    (below the half bit) that all its non-empty buckets share."""
    img = img.astype(np.uint64)
    b = (img >> np.uint64(W - 16)).astype(np.int64)
    cnt = np.bincount(b, minlength=65536)
    if not ((cnt > cap).any() and cnt.max() < img.shape[0]):
        return img
    out = img.copy()
    any_sq = False
    for h in (0, 1):
        nz = np.nonzero(cnt[h << 15:(h + 1) << 15])[0] + (h << 15)
        big = int((cnt[h << 15:(h + 1) << 15] > cap).sum())
        if nz.size == 0 or big == 0:
            continue
        o1 = int(np.bitwise_or.reduce(nz))
        o0 = int(np.bitwise_or.reduce(~nz & 0xFFFF))
        cm = ~(o1 & o0) & 0x7FFF
        if not cm:
            continue
        bit = cm.bit_length() - 1 + W - 16
        hi = np.uint64(~((2 << bit) - 1) & ((1 << W) - 1))
        lo = np.uint64((1 << bit) - 1)
        sel = (img >> np.uint64(W - 1)) == np.uint64(h)
        out[sel] = (img[sel] & hi) | ((img[sel] & lo) << np.uint64(1))
        any_sq = True
    return out if any_sq else img


@pytest.mark.parametrize("kt,vb", [(O.U32, 0), (O.U32, 4), (O.F32, 0), (O.U64, 8), (O.U32, 16)])
def test_per_bucket_fallback(gpu, kt, vb):
    """Only buckets above the local capacity take device passes (thrs_fallback.hpp):
    a quarter of the keys in one bucket next to uniform ones (one big chunk,
    the others sorted locally), 16 distinct keys (both low passes are
    identities, skipped), keys confined to 2^20 values (16 big chunks, both low
    passes run).  Bit-exact vs the oracle, and the plan's mode says which ran."""
    torch = gpu
    rs = make_sorter(kt, vb, False, path="bucket")
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    n = 1 << 21
    base = O.randomize_np(kt, O.splitmix64_stream(777 + vb, n)).astype(kdt)
    few = O.randomize_np(kt, O.splitmix64_stream(31, 16)).astype(kdt)
    cases = {
        "one_big": np.where(np.arange(n) % 4 == 0, base[0], base).astype(kdt),
        "few_unique": few[np.arange(n) % 16],
        "low20": (base & np.array(0xFFFFF if kb == 4 else 0xFFFFFFFFFFFF, kdt)).astype(kdt),
    }
    cap = rs.pathInfo(n, 0, 8 * kb, bool(vb))["local_cap"]
    for name, keys in cases.items():
        # expected plan: buckets (top 16 image bits) above the local capacity
        # -- for float keys under the squeeze thrs_plan_rows may choose
        img = O.key_bits_np(kt, keys)
        if kt in (O.F32, O.F64):
            img = _squeezed_images(img, 8 * kb, cap)
        cnt = np.bincount((img >> np.uint64(8 * kb - 16)).astype(np.int64), minlength=65536)
        ebig = int((cnt > cap).sum())
        emode = 0 if ebig == 0 else (2 if int(cnt.max()) == n else 1)
        assert ebig >= 1, name
        vals = None
        if vb:
            vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(40503)).view(
                {4: np.uint32, 8: np.uint64, 16: np.uint64}[vb])
            if vb == 16:
                vals = vals.reshape(n, 2)
        (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
        ek, ev = O.lsd_sort(kt, keys, vals, 0, 8 * kb, False)
        assert np.array_equal(k.view(kdt), ek.view(kdt)), name
        if vb:
            assert np.array_equal(v, ev), name
        assert (mode, big) == (emode, ebig), (name, mode, big)


@pytest.mark.parametrize("kt,vb", [(O.U32, 0), (O.U32, 4), (O.U64, 0), (O.U64, 8), (O.F32, 4)])
@pytest.mark.parametrize("desc", [False, True])
def test_key_range_keeps_buckets_local(gpu, kt, vb, desc):
    """thrs_options.keyRange (the multi-GPU finish): keys confined to a narrow
    image range [lo, hi] fill all 65536 buckets once the sort orders by
    ((img - lo) << sh), so every bucket fits its local sort (mode 0) where
    without the range some buckets overflow; same bytes as the oracle either way.
    lo == hi (one key value) returns at once, leaving the input as it is."""
    torch = gpu
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    n = 1 << 21
    raw = O.randomize_np(kt, O.splitmix64_stream(4444 + vb, n)).astype(kdt)
    if kt == O.F32:   # floats in [1, 2): one exponent, 2^23 mantissas
        keys = ((raw & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)).astype(kdt)
    else:
        keys = (np.array(0x1234 << (8 * kb - 16), kdt) | (raw & np.array((1 << 20) - 1, kdt))).astype(kdt)
    img = O.key_bits_np(kt, keys, desc)
    lo, hi = int(img.min()), int(img.max())
    vals = None
    if vb:
        vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(
            {4: np.uint32, 8: np.uint64}[vb])
    ek, ev = O.lsd_sort(kt, keys, vals, 0, 8 * kb, desc)
    # without the range: 16 overflowing buckets for 4-byte integer keys (20
    # random low bits reach bits 16..19), one bucket holding every key for
    # 8-byte keys; f32 keys in [1, 2): 128 buckets, which the squeeze
    # (thrs_plan_rows) doubles -- enough here (the model says which)
    no_range_mode = 1 if kb == 4 else 2
    if kt == O.F32:
        cap = make_sorter(kt, vb, desc, path="bucket").pathInfo(n, 0, 32, bool(vb))["local_cap"]
        cnt = np.bincount((_squeezed_images(img, 32, cap) >> np.uint64(16)).astype(np.int64), minlength=65536)
        no_range_mode = 0 if int(cnt.max()) <= cap else 1
    for rng, want_mode in (((lo, hi), 0), (None, no_range_mode)):
        rs = make_sorter(kt, vb, desc, path="bucket", keyRange=rng)
        (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
        assert np.array_equal(k.view(kdt), ek.view(kdt)), (rng, mode)
        if vb:
            assert np.array_equal(v, ev), rng
        assert mode == want_mode, (rng, mode, big)
    one = np.full(1000, keys[0], kdt)
    rs = make_sorter(kt, vb, desc, keyRange=(int(img[0]), int(img[0])))
    k, _ = gpu_sort(torch, rs, {"keys": one, "values": None if not vb else vals[:1000]}, kt, vb, 0, 8 * kb)
    assert np.array_equal(k, one)


@pytest.mark.parametrize("kt,vb", [(O.F32, 0), (O.F64, 0), (O.F64, 8)])
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("where", ["straddles_zero", "excludes_zero"])
def test_key_range_float_zeros(gpu, kt, vb, desc, where):
    """keyRange on the float local sorts: f32 keys-only is
    thrs_local16's +-0 chunk (+0 and -0 share one image and must keep their
    input order and bits), f64 the permuted-key thrs_local_kv.  A range that
    straddles zero with mixed +0 / -0 keys, and one that excludes zero (the
    image of 0 then lies outside [lo, hi]); bit-exact with the oracle."""
    torch = gpu
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    fdt = np.float32 if kb == 4 else np.float64
    n = (1 << 20) + 4097
    rng = np.random.default_rng(1000 * kb + vb + (7 if desc else 0) + len(where))
    if where == "straddles_zero":
        f = rng.uniform(-1e-3, 1e-3, n).astype(fdt)
        z = rng.random(n)
        f[z < 0.1] = fdt(0.0)
        f[(z >= 0.1) & (z < 0.2)] = -fdt(0.0)
    else:
        f = rng.uniform(1.0, 2.0, n).astype(fdt)
    keys = f.view(kdt).copy()
    img = O.key_bits_np(kt, keys, desc)
    lo, hi = int(img.min()), int(img.max())
    vals = None
    if vb:
        vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(np.uint64)
    ek, ev = O.lsd_sort(kt, keys, vals, 0, 8 * kb, desc)
    rs = make_sorter(kt, vb, desc, path="bucket", keyRange=(lo, hi))
    (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
    assert np.array_equal(k.view(kdt), ek.view(kdt)), (where, mode, big)
    if vb:
        assert np.array_equal(v, ev), where


def _float_keys_from_images(kt, img, desc):
    """raw float bit patterns whose sort image (getKeyBits ^ descending mask,
    kernel.cu:18-24, 46-69) is img (img never the image of -0)."""
    kb = O.KEY_BYTES[kt]
    dt = O.KEY_DTYPE[kt]
    top = dt(1) << dt(8 * kb - 1)
    b = (img ^ dt(~dt(0) if desc else 0)).astype(dt)     # getKeyBits(raw)
    return np.where((b & top) != 0, b ^ top, ~b).astype(dt)


def _squeeze_case_keys(kt, n, desc, varying, seed):
    """Images whose 16 bucket bits are the half bit + `varying - 1` other
    varying bits; the rest of the bucket field is constant per half, with a
    different constant pattern in each half (some bits 1, some 0).  The bits
    below the bucket field are random.  So only 2^varying buckets hold keys
    until the squeeze drops one constant bit per half (thrs_plan_rows)."""
    kb = O.KEY_BYTES[kt]
    dt = O.KEY_DTYPE[kt]
    W = 8 * kb
    rng = np.random.default_rng(seed)
    img = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    h = (img >> dt(W - 1)) & dt(1)
    pos = [2, 5, 9, 11, 13][:varying - 1]            # varying bucket bits besides the half bit
    vmask = sum(1 << p for p in pos)
    cst = [0x5A31 & ~vmask & 0x7FFF, 0x26C4 & ~vmask & 0x7FFF]   # per half
    field = (img >> dt(W - 16)) & dt(0x7FFF)
    field = (field & dt(vmask)) | np.where(h == 1, dt(cst[1]), dt(cst[0])).astype(dt)
    img = (img & dt((1 << (W - 16)) - 1)) | (field << dt(W - 16)) | (h << dt(W - 1))
    return _float_keys_from_images(kt, img.astype(dt), desc)


@pytest.mark.parametrize("kt,vb", [(O.F32, 0), (O.F32, 4), (O.F32, 8), (O.F64, 0), (O.F64, 8)])
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("fits", [True, False])
def test_squeeze_vs_oracle(gpu, kt, vb, desc, fits):
    """The data-chosen bucket bits (float keys, thrs_plan_rows + KeyMap<U,
    true>): keys whose images share constant bits inside the bucket field
    overflow their buckets; the plan drops one constant bit per image half,
    histograms again under that map and the local sorts fit (fits=True, mode 0)
    -- or, with too few varying bits, the per-bucket fallback runs under the
    squeezed map (fits=False, mode 1).  Bit-exact with the oracle either way."""
    torch = gpu
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    n = (1 << 20) + 333
    kv = kb == 8 or vb >= 8          # 17408-key chunks (thrs_local_kv), else 9216 (both asked)
    varying = (5 if kv else 6) if fits else 3
    keys = _squeeze_case_keys(kt, n, desc, varying, 71 * kb + vb + (5 if desc else 0) + (3 if fits else 0))
    vals = None
    if vb:
        vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(
            {4: np.uint32, 8: np.uint64}[vb])
    ek, ev = O.lsd_sort(kt, keys, vals, 0, 8 * kb, desc)
    rs = make_sorter(kt, vb, desc, path="bucket", localGeometry="big" if kv else "small")
    (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
    assert np.array_equal(k.view(kdt), ek.view(kdt)), (mode, big)
    if vb:
        assert np.array_equal(v, ev)
    assert mode == (0 if fits else 1), (mode, big)


@pytest.mark.parametrize("kt,vb", [(O.F32, 0), (O.F32, 4), (O.F64, 0), (O.F64, 8)])
@pytest.mark.parametrize("desc", [False, True])
def test_squeeze_sample_violation(gpu, kt, vb, desc):
    """the SAMPLED squeeze guessed wrong.  thrs_squeeze_sample
    reads 32 evenly spaced runs of 256 keys (thrs_hybrid.hpp kSqBlocks); keys
    outside those runs flip the bucket bit the sample finds constant (the
    highest constant bit of each half), so the first histogram's check raises
    meta[kMetaSqViol], the plan drops the guess and the keys are histogrammed
    again under the PLAIN map.  Bit-exact with the oracle, and the plan's mode
    is the one the plain map implies (its overflowing buckets: mode 1)."""
    torch = gpu
    kb = O.KEY_BYTES[kt]
    kdt = O.KEY_DTYPE[kt]
    W = 8 * kb
    n = (1 << 20) + 333
    kv = kb == 8 or vb >= 8
    keys = _squeeze_case_keys(kt, n, desc, 5 if kv else 6, 97 * kb + vb + (5 if desc else 0))
    img = O.key_bits_np(kt, keys, desc).astype(kdt)
    # the sampled runs: [j n / 32, j n / 32 + 256), j < 32; one violator in
    # every gap, its field bit 14 (constant 0 or 1 per half in both
    # constructions) flipped
    pos = np.array([j * n // 32 + 4096 + 7 * j for j in range(32)])
    img[pos] ^= kdt(1) << kdt(W - 2)
    keys = _float_keys_from_images(kt, img, desc)
    assert np.array_equal(O.key_bits_np(kt, keys, desc).astype(kdt), img)
    vals = None
    if vb:
        vals = (np.arange(n * vb // 4, dtype=np.uint32) * np.uint32(2654435761)).view(
            {4: np.uint32, 8: np.uint64}[vb])
    ek, ev = O.lsd_sort(kt, keys, vals, 0, W, desc)
    rs = make_sorter(kt, vb, desc, path="bucket", **({"localGeometry": "big"} if kv else {}))
    cap = rs.pathInfo(n, 0, W, bool(vb))["local_cap"]
    cnt = np.bincount((img.astype(np.uint64) >> np.uint64(W - 16)).astype(np.int64), minlength=65536)
    ebig = int((cnt > cap).sum())
    assert ebig > 0
    (mode, big), k, v = _mode_after(torch, rs, keys, vals, kt, vb)
    assert np.array_equal(k.view(kdt), ek.view(kdt)), (mode, big)
    if vb:
        assert np.array_equal(v, ev)
    assert (mode, big) == (1, ebig), (mode, big, ebig)


@pytest.mark.large
@pytest.mark.parametrize("kt,vb,n", [(O.F32, 0, 1 << 30),    # f32 keys-only, the reference's generator
                                     (O.F32, 4, 1 << 30),    # SortPairs.KF32V32's distribution (unittest.cpp:433-439)
                                     (O.F64, 8, 1 << 29)])   # f64 pairs (randomizeValues clears bit 52)
def test_reference_float_generator_stays_local(gpu, kt, vb, n):
    """randomizeValues (unittest.cpp:96-116) clears the lowest exponent bit of
    every f32 / f64 key, so half of the 65536 top-16-bit buckets are empty and
    at these sizes every used bucket would overflow its local sort.  The
    squeeze keeps the whole sort on the bucket path: mode 0, no big chunks;
    sortedness, the multiset fingerprint and (pairs) gather + stability."""
    torch = gpu
    import tinyhipradixsort_amd as T
    from tinyhipradixsort_amd import testutil as TU
    kb = O.KEY_BYTES[kt]
    keys = _big_keys(torch, kt, n)
    orig = keys.clone() if vb else None
    torch.cuda.synchronize()
    fp = TU.fingerprint(kt, keys, n)
    rs = make_sorter(kt, vb, False)
    d = rs.getTemporaryBufferBytes(n)
    if vb:
        vals = torch.empty(vb * n, dtype=torch.uint8, device="cuda")
        TU.iota(vb, vals, n)
        tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
        rs.sortPairs(keys, vals, n, tmp, 0, kb * 8)
    else:
        tmp = torch.empty(d.getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
        rs.sortKeys(keys, n, tmp, 0, kb * 8)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert rs.debugBucketMode(tmp, n, bool(vb)) == (0, 0)
    assert T.debug_big_keys(tmp, kt, vb, n) == 0
    assert TU.count_unsorted(kt, keys, n, 0, kb * 8) == 0
    assert TU.fingerprint(kt, keys, n) == fp
    if vb:
        r = TU.check_pairs(kt, vb, orig, keys, vals, n, 0, kb * 8)
        assert r["gather_mismatch"] == 0 and r["unstable"] == 0
        assert (r["index_sum"], r["index_xor"]) == TU.expected_index_fingerprint(n)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("zeros", ["plus_only", "few_signed", "many_signed"])
def test_f32_planes_signed_zeros(gpu, zeros, desc):
    """f32 keys-only at 2^28 (the default bucket path with the image planes:
    the top-digit passes carry 3 + 2 bytes of each key's image, not the key).
    -0 and +0 share one image (kernel.cu:46-69's getKeyBits), so the planes
    lose the zeros' signs: the bucket histogram logs up to 1024 zero keys with
    their positions (thrs_local16 restores the signs in their stable order,
    mode 0), and with more zeros than that a -0 sends the sort through the
    whole-key passes (mode 3).  +0 only: nothing to restore (mode 0).
    Checked on the GPU: sortedness, the raw-bit multiset, and the zeros' raw
    bits in input order."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    n = 1 << 28
    keys = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
    TU.fill_keys(2, keys, n, start=77 + int(desc))
    k32 = keys.view(torch.int32)
    k32[(k32 & 0x7FFFFFFF) == 0] = 1                      # the generator's own zeros, if any
    # 700 zeros fit the zero log, 3000 do not; either way the zeros' bucket
    # (4096 keys on average at 2^28) stays within its local sort (9216 keys)
    step = n // (700 if zeros == "few_signed" else 3000) + 1
    idx = torch.arange(5, n, step, device="cuda")
    k32[idx] = 0
    if zeros != "plus_only":
        k32[idx[1::3]] = -(1 << 31)
    zin = k32[(k32 & 0x7FFFFFFF) == 0].clone()
    fp = TU.fingerprint(2, keys, n)
    rs = make_sorter(2, 0, desc)
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8,
                      device="cuda")
    rs.sortKeys(keys, n, tmp, 0, 32)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert rs.debugBucketMode(tmp, n, False) == ((3, 0) if zeros == "many_signed" else (0, 0))
    assert TU.count_unsorted(2, keys, n, 0, 32, descending=desc) == 0
    assert TU.fingerprint(2, keys, n) == fp
    zout = k32[(k32 & 0x7FFFFFFF) == 0]
    assert torch.equal(zout, zin)


@pytest.mark.parametrize("desc", [False, True])
def test_f32_planes_with_key_range(gpu, desc):
    """The multi-GPU finish's shape for f32 keys: 2^28 keys with a keyRange
    (thrs_options.keyRange, the split's [lo, hi]) on the image planes, with
    +0 / -0 keys inside the range (the zero log) -- the local sort then takes
    the general inverse map (the linear per-chunk rebuild needs no range).
    Checked on the GPU: mode 0, sortedness, the raw-bit multiset and the
    zeros' raw bits in input order."""
    torch = gpu
    from tinyhipradixsort_amd import testutil as TU
    n = 1 << 28
    g = torch.Generator(device="cuda")
    g.manual_seed(4242 + int(desc))
    # images uniform in [0x7F000000, 0x81000000): floats on both sides of zero
    # (down to the denormals), uniform in the range's image space as the
    # split of a uniform distribution is
    im = torch.randint(0, 1 << 25, (n,), device="cuda", generator=g, dtype=torch.int64) + 0x7F000000
    raw = torch.where(im >= 0x80000000, im ^ 0x80000000, im ^ 0xFFFFFFFF)
    k32 = torch.where(raw >= 0x80000000, raw - (1 << 32), raw).to(torch.int32)
    idx = torch.arange(11, n, n // 600 + 1, device="cuda")
    k32[idx] = 0
    k32[idx[::4]] = -(1 << 31)
    keys = k32.view(torch.uint8)
    zin = k32[(k32 & 0x7FFFFFFF) == 0].clone()
    b = k32.to(torch.int64) & 0xFFFFFFFF
    b = torch.where((b & 0x7FFFFFFF) == 0, torch.zeros_like(b), b)       # getKeyBits: -0 -> +0
    img = torch.where(b >= 0x80000000, b ^ 0xFFFFFFFF, b ^ 0x80000000)
    if desc:
        img = img ^ 0xFFFFFFFF
    lo, hi = int(img.min().item()), int(img.max().item())
    fp = TU.fingerprint(2, keys, n)
    rs = make_sorter(2, 0, desc, keyRange=(lo, hi))
    assert rs.pathInfo(n, 0, 32, False)["planes"]
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8,
                      device="cuda")
    rs.sortKeys(keys, n, tmp, 0, 32)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    assert rs.debugBucketMode(tmp, n, False) == (0, 0)
    assert TU.count_unsorted(2, keys, n, 0, 32, descending=desc) == 0
    assert TU.fingerprint(2, keys, n) == fp
    assert torch.equal(k32[(k32 & 0x7FFFFFFF) == 0], zin)
