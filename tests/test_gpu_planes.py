"""GPU parity of the key-plane codecs, element-wise against the oracle.

The bucket path for u32 / f32 keys without values carries each key's image
through the two top-digit passes as planes (thrs_kernels.hpp kCodecSplit /
kCodecPlanes: a u16 + u8 plane, then a u16 plane), and the top-digit pass
reads whole tiles inside one second-digit region with vector loads, which walk
the keys out of input order.  The headline (C2), C4, u32Large and the
reference's own timed shape (160M keys, unittest.cpp:490-571) all run these
codecs, so they are compared here with the oracle's pass-by-pass restatement
of RadixSort::sort (tinyhipradixsort.hpp:854-944), key for key:

* the DEFAULT path at the sizes where it runs them: u32 keys at 60,000,000 and
  160,000,000 (4096-key chunks, Loc16Tiny) and 2^28 (9216-key chunks), f32
  keys at 150,000,000 with raw NaN / Inf / denormal bits and signed zeros,
  u32 pairs at 160M (LocTiny; pairs carry whole keys);
* a FORCED bucket path at small n with a distribution that puts the keys in
  four second-digit regions, so nearly every top-pass tile is a vector tile.

u32 / f32 keys with u32 values carry the keys as the same planes (no vector
tiles: the values keep input order), so their keys AND values are compared
with the oracle's, which checks the stable order of equal keys through the
codecs.  f32 pairs take the zeros' signs from the zero log (mode 0) up to
1024 zeros, and run whole keys (mode 3) past that when a -0 is among them.

Each planes case asserts pathInfo()['planes'] and that the vector branch ran
(thrs_debug_vector_tiles, a counter the top-digit pass keeps)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sorter(kt, vb, desc, **options):
    import tinyhipradixsort_amd as T
    cfg = T.RadixSort.Config()
    cfg.keyType = T.KeyType(kt)
    cfg.valueType = T.ValueType.U32
    cfg.sortOrder = T.SortOrder.Descending if desc else T.SortOrder.Ascending
    return T.RadixSort([], cfg, T.Options(**options))


def _sort_on_gpu(torch, rs, kt, keys, vals=None):
    """(sorted keys, sorted values, tmp) through the C-ABI; keys/vals are host arrays."""
    n = keys.shape[0]
    kd = torch.from_numpy(keys.view(np.uint8)).to("cuda")
    d = rs.getTemporaryBufferBytes(n)
    if vals is not None:
        vd = torch.from_numpy(vals.view(np.uint8)).to("cuda")
        tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
        rs.sortPairs(kd, vd, n, tmp, 0, 32)
    else:
        vd = None
        tmp = torch.empty(d.getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
        rs.sortKeys(kd, n, tmp, 0, 32)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    k = kd.cpu().numpy().view(keys.dtype)
    v = None if vd is None else vd.cpu().numpy().view(vals.dtype)
    return k, v, tmp


def _u32_keys(n, seed):
    return O.randomize_np(O.U32, O.splitmix64_stream(seed, n))


def _f32_raw_keys(n, seed):
    """Uniform raw bit patterns as f32 keys (NaNs ~1/256, denormals ~1/256, both
    signs), plus +-Inf, +-NaN payloads and 600 signed zeros (under the zero
    log's 1024: the planes keep running, mode 0)."""
    k = _u32_keys(n, seed)
    k[k & np.uint32(0x7FFFFFFF) == 0] = 1                     # the stream's own zeros, if any
    rng = np.random.default_rng(seed)
    specials = np.array([0x7F800000, 0xFF800000, 0x7FC00000, 0xFFC00000, 0x7F800001, 0xFFFFFFFF,
                         0x00000001, 0x80000001, 0x007FFFFF, 0x807FFFFF], np.uint32)
    pos = rng.choice(n, 4000, replace=False)
    k[pos[:3400]] = specials[np.arange(3400) % specials.shape[0]]
    k[pos[3400:]] = np.where(np.arange(600) % 3 == 0, np.uint32(0x80000000), np.uint32(0))
    return k                                                   # raw f32 bits, as the oracle takes them


def _expect_planes(rs, T, tmp, kt, n, min_frac):
    assert rs.pathInfo(n, 0, 32, False)["planes"]
    assert rs.debugBucketMode(tmp, n, False)[0] == 0           # mode 0: the planes ran
    tiles = T.debug_vector_tiles(tmp, kt, n)
    total = -(-n // 32768)
    print(f"vector tiles {tiles} of ~{total}")
    assert tiles >= min_frac * total, (tiles, total)


@pytest.mark.large
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("n", [60_000_000, 160_000_000, 1 << 28])
def test_u32_keys_default_path_planes_vs_oracle(gpu, n, desc):
    """u32 keys-only on the DEFAULT path at the sizes where it takes the
    planes: 4096-key chunks (<= 3 x 2^26 keys; 160M is the reference's own
    bench size, unittest.cpp:490-571) and 9216-key chunks (2^28).  Uniform
    keys: every second-digit region spans many tiles, so most top-pass tiles
    take the vector loads."""
    import tinyhipradixsort_amd as T
    torch = gpu
    keys = _u32_keys(n, 6100 + int(desc))
    rs = _sorter(O.U32, 0, desc)
    info = rs.pathInfo(n, 0, 32, False)
    assert (info["path"], info["local"]) == ("bucket", "thrs_local16")
    assert info["local_cap"] == (4096 if n <= 3 << 26 else 9216)
    k, _, tmp = _sort_on_gpu(torch, rs, O.U32, keys)
    _expect_planes(rs, T, tmp, O.U32, n, 0.75)
    ek, _ = O.lsd_sort(O.U32, keys, None, 0, 32, desc)
    assert np.array_equal(k, ek)


@pytest.mark.large
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("n", [40_000_000, 150_000_000])
def test_f32_keys_default_path_planes_vs_oracle(gpu, n, desc):
    """f32 keys-only on the default path at its lower bound (40M) and at 150M
    (planes; the squeeze may go on): raw NaN / Inf / denormal bits and 600
    signed zeros, whose signs the zero log restores in input order
    (getKeyBits maps -0 to +0, kernel.cu:46-69).  Bit-exact against the
    oracle."""
    import tinyhipradixsort_amd as T
    torch = gpu
    assert _sorter(O.F32, 0, desc).pathInfo(n, 0, 32, False)["path"] == "bucket"
    keys = _f32_raw_keys(n, 6200 + int(desc) + n % 7)
    rs = _sorter(O.F32, 0, desc)
    k, _, tmp = _sort_on_gpu(torch, rs, O.F32, keys)
    _expect_planes(rs, T, tmp, O.F32, n, 0.75)
    ek, _ = O.lsd_sort(O.F32, keys, None, 0, 32, desc)
    assert np.array_equal(k, ek)


@pytest.mark.large
@pytest.mark.parametrize("desc", [False, True])
def test_u32_pairs_default_path_vs_oracle(gpu, desc):
    """u32 keys + u32 values at the reference's bench size, 160M (the default
    bucket path with 4096-key chunks, LocTiny): keys and values bit-exact
    against the oracle, so the stable order of equal keys is checked too."""
    torch = gpu
    n = 160_000_000
    keys = _u32_keys(n, 6300 + int(desc))
    keys[::7] &= np.uint32(0xFFFF00FF)                         # ties: stability visible
    vals = np.arange(n, dtype=np.uint32)
    rs = _sorter(O.U32, 4, desc)
    info = rs.pathInfo(n, 0, 32, True)
    assert (info["path"], info["local"], info["local_cap"], info["planes"]) == ("bucket", "thrs_local_pairs", 4096,
                                                                                True)
    assert rs.pathInfo(35_000_000, 0, 32, True)["path"] == "bucket"   # the lower bound (row 129)
    k, v, tmp = _sort_on_gpu(torch, rs, O.U32, keys, vals)
    assert rs.debugBucketMode(tmp, n, True)[0] == 0            # mode 0: the planes ran
    ek, ev = O.lsd_sort(O.U32, keys, vals, 0, 32, desc)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("geom", ["tiny16", "small", "big"])
@pytest.mark.parametrize("n", [1 << 20, 3 * (1 << 20) + 12345])
def test_forced_bucket_pairs_planes_vs_oracle(gpu, n, geom, desc):
    """u32 pairs on a forced bucket path (planes on, mode 0) in every pairs
    chunk geometry: ties in the low 16 bits every 5th key, so the values'
    stable order through the split / planes codecs and the plane-fed local
    sort is visible.  Keys and values bit-exact against the oracle."""
    torch = gpu
    keys = _u32_keys(n, 6600 + n % 89 + int(desc) + 3 * len(geom))
    keys[::5] &= np.uint32(0xFFFF0000)
    vals = np.arange(n, dtype=np.uint32) ^ np.uint32(0x5A5A5A5A)
    rs = _sorter(O.U32, 4, desc, path="bucket", localGeometry=geom)
    assert rs.pathInfo(n, 0, 32, True)["planes"]
    k, v, tmp = _sort_on_gpu(torch, rs, O.U32, keys, vals)
    assert rs.debugBucketMode(tmp, n, True)[0] == 0
    ek, ev = O.lsd_sort(O.U32, keys, vals, 0, 32, desc)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


@pytest.mark.parametrize("desc", [False, True])
def test_forced_bucket_pairs_planes_ranged_and_off(gpu, desc):
    """u32 pairs with a key range (the codecs carry the RANGED images,
    thrs_options.keyRange) and with the planes off: both equal the oracle."""
    torch = gpu
    n = (1 << 21) + 777
    lo = 0x01230000
    keys = (lo + (_u32_keys(n, 6700 + int(desc)) >> np.uint32(8))).astype(np.uint32)   # images in [lo, lo + 2^24)
    vals = np.arange(n, dtype=np.uint32)
    ek, ev = O.lsd_sort(O.U32, keys, vals, 0, 32, desc)
    img = keys ^ np.uint32(0xFFFFFFFF) if desc else keys
    rng = (int(img.min()), int(img.max()))
    for kw in ({"keyRange": rng}, {"planes": "off"}):
        rs = _sorter(O.U32, 4, desc, path="bucket", **kw)
        assert rs.pathInfo(n, 0, 32, True)["planes"] == ("planes" not in kw)
        k, v, _ = _sort_on_gpu(torch, rs, O.U32, keys, vals)
        assert np.array_equal(k, ek), kw
        assert np.array_equal(v, ev), kw


@pytest.mark.parametrize("desc", [False, True])
def test_forced_bucket_pairs_big_chunks_vs_oracle(gpu, desc):
    """u32 pairs where a few buckets exceed the local capacity (mode 1: the
    single top-digit launches run their whole-key bodies, with the values, and
    the per-bucket fallback sorts the big chunks): keys and values against the
    oracle."""
    torch = gpu
    n = 3 << 20
    keys = _u32_keys(n, 6800 + int(desc))
    keys[: n // 3] = (keys[: n // 3] & np.uint32(0x0000FFFF)) | np.uint32(0x77770000)   # one 1M-key bucket
    perm = np.random.default_rng(6800).permutation(n)
    keys = keys[perm]
    vals = np.arange(n, dtype=np.uint32)
    rs = _sorter(O.U32, 4, desc, path="bucket")
    k, v, tmp = _sort_on_gpu(torch, rs, O.U32, keys, vals)
    assert rs.debugBucketMode(tmp, n, True)[0] == 1
    ek, ev = O.lsd_sort(O.U32, keys, vals, 0, 32, desc)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("kt", [O.U32, O.F32])
@pytest.mark.parametrize("geom", ["tiny16", "small", "big"])
@pytest.mark.parametrize("n", [1 << 20, 3 * (1 << 20) + 12345])
def test_forced_bucket_vector_tiles_vs_oracle(gpu, n, geom, kt, desc):
    """A forced bucket path at sizes the oracle finishes at once, with the
    keys in four second-digit regions (raw bits 18-23 cleared): every region
    spans 8+ tiles, so nearly every top-pass tile takes the vector loads, and
    the 1024+ buckets stay within the local capacity (mode 0: planes on).
    f32 adds signed zeros and specials."""
    import tinyhipradixsort_amd as T
    torch = gpu
    seed = 6400 + n % 97 + 3 * int(desc) + 7 * kt
    keys = _u32_keys(n, seed) if kt == O.U32 else _f32_raw_keys(n, seed)
    keys &= np.uint32(0xFF03FFFF)
    rs = _sorter(kt, 0, desc, path="bucket", localGeometry=geom)
    k, _, tmp = _sort_on_gpu(torch, rs, kt, keys)
    _expect_planes(rs, T, tmp, kt, n, 0.5)
    ek, _ = O.lsd_sort(kt, keys, None, 0, 32, desc)
    assert np.array_equal(k, ek)


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("kt", [O.U32, O.F32])
def test_forced_bucket_planes_vs_noplanes(gpu, kt, desc):
    """The same forced-bucket sorts with the planes on and off
    (thrs_options.planes): both equal the oracle, and only the first takes the
    vector tiles."""
    import tinyhipradixsort_amd as T
    torch = gpu
    n = 1 << 21
    keys = _u32_keys(n, 6500 + kt + int(desc)) & np.uint32(0xFF07FFFF)
    ek, _ = O.lsd_sort(kt, keys, None, 0, 32, desc)
    for planes in ("auto", "off"):
        rs = _sorter(kt, 0, desc, path="bucket", planes=planes)
        k, _, tmp = _sort_on_gpu(torch, rs, kt, keys)
        assert np.array_equal(k, ek), planes
        assert rs.pathInfo(n, 0, 32, False)["planes"] == (planes == "auto")
        tiles = T.debug_vector_tiles(tmp, kt, n)
        assert (tiles > 0) == (planes == "auto"), (planes, tiles)


def _f32_pairs_keys(n, seed, zeros):
    """Raw f32 bits with NaN / Inf / denormal specials and signed zeros:
    "plus" (600 +0), "signed" (600 zeros, a third -0: within the zero log) or
    "many" (3000 zeros, a third -0: past the log's 1024, mode 3)."""
    k = _f32_raw_keys(n, seed)
    if zeros == "plus":
        k[k == np.uint32(0x80000000)] = 0
    elif zeros == "many":
        pos = np.random.default_rng(seed + 1).choice(n, 3000, replace=False)
        k[pos] = np.where(np.arange(3000) % 3 == 1, np.uint32(0x80000000), np.uint32(0))
    return k


_F32_PAIRS_MODE = {"plus": 0, "signed": 0, "many": 3}


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("zeros", ["plus", "signed", "many"])
@pytest.mark.parametrize("geom", ["tiny16", "small", "big"])
def test_forced_bucket_f32_pairs_planes_vs_oracle(gpu, geom, zeros, desc):
    """f32 pairs on a forced bucket path (every pairs geometry, tiny16
    included): planes (mode 0) with +0 only or up to 1024 signed zeros (the
    zero log restores their signs in the zeros' chunk), whole keys (mode 3)
    past that; keys (raw bits: NaN payloads, signed zeros) and values
    bit-exact against the oracle."""
    torch = gpu
    n = 3 * (1 << 20) + 4321
    keys = _f32_pairs_keys(n, 6900 + int(desc) + 2 * len(zeros) + len(geom), zeros)
    vals = np.arange(n, dtype=np.uint32)
    rs = _sorter(O.F32, 4, desc, path="bucket", localGeometry=geom)
    assert rs.pathInfo(n, 0, 32, True)["planes"]
    k, v, tmp = _sort_on_gpu(torch, rs, O.F32, keys, vals)
    assert rs.debugBucketMode(tmp, n, True)[0] == _F32_PAIRS_MODE[zeros]
    ek, ev = O.lsd_sort(O.F32, keys, vals, 0, 32, desc)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)


@pytest.mark.large
@pytest.mark.parametrize("zeros", ["plus", "signed", "many"])
def test_f32_pairs_default_path_vs_oracle(gpu, zeros):
    """f32 pairs at 32M, the default bucket path's lower bound (planes, the
    squeeze may go on): keys and values against the oracle."""
    torch = gpu
    n = 32_000_000
    keys = _f32_pairs_keys(n, 7000 + len(zeros), zeros)
    vals = np.arange(n, dtype=np.uint32)
    rs = _sorter(O.F32, 4, False)
    info = rs.pathInfo(n, 0, 32, True)
    assert (info["path"], info["local"], info["planes"]) == ("bucket", "thrs_local_pairs", True)
    k, v, tmp = _sort_on_gpu(torch, rs, O.F32, keys, vals)
    mode = rs.debugBucketMode(tmp, n, True)[0]
    # (3000 zeros overflow the zero's 4096-key chunk at this size: mode 1,
    # big chunks, which also runs whole keys)
    assert mode == _F32_PAIRS_MODE[zeros] or (zeros == "many" and mode == 1), mode
    ek, ev = O.lsd_sort(O.F32, keys, vals, 0, 32, False)
    assert np.array_equal(k, ek)
    assert np.array_equal(v, ev)
