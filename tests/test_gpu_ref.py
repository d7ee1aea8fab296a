"""GPU parity against the REFERENCE's own kernels (kernel.cu compiled by
hipRTC for gfx950, oracle/_ref/refk_*.co, launched with the reference's pass
loop by oracle/_ref/liboracle_refk.so): for every key type, value type, order,
window and tile-boundary size, libthrs (through the C-ABI), the reference's
kernels and the CPU oracle produce the same bytes; the reference's kernels also
reproduce the committed golden digests of the reference's test streams.
Sizes keep the reference's chained scan within co-resident workgroups."""
import json
import os

import numpy as np
import pytest

import cases as C
from oracle import oracle as O
from oracle import ref as R

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
VT = {4: 0, 8: 1, 16: 2}


@pytest.fixture(scope="module")
def refk(gpu):
    assert R.kernels_available(), "oracle/_ref is not built (make -C oracle/ref, needs /root/reference)"
    return R


def to_dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to("cuda")


def run_both(torch, kt, vb, desc, keys, vals, s, e):
    import tinyhipradixsort_amd as T
    n = keys.shape[0]
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType=T.ValueType(VT.get(vb, 0)),
                             sortOrder=T.SortOrder.Descending if desc else T.SortOrder.Ascending)
    rs = T.RadixSort([], cfg)
    kd, kr = to_dev(torch, keys), to_dev(torch, keys)
    vd = vr = None
    if vb:
        vd, vr = to_dev(torch, vals), to_dev(torch, vals)
    d = rs.getTemporaryBufferBytes(n)
    tmp = torch.empty(d.getTemporaryBufferBytesForSortPairs(), dtype=torch.uint8, device="cuda")
    if vb:
        rs.sortPairs(kd, vd, n, tmp, s, e)
    else:
        rs.sortKeys(kd, n, tmp, s, e)
    rt = R.temp_bytes(kt, VT.get(vb, 0), n)
    rtmp = torch.empty(sum(rt), dtype=torch.uint8, device="cuda")
    R.sort(kt, VT.get(vb, 0), desc, kr, vr, n, rtmp, s, e, torch.cuda.current_stream())
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    out = lambda t, like: None if t is None else t.cpu().numpy().view(like.dtype).reshape(like.shape)
    return out(kd, keys), out(vd, vals), out(kr, keys), out(vr, vals)


@pytest.mark.parametrize("kt", [O.U32, O.U64, O.F32, O.F64])
@pytest.mark.parametrize("vb", [0, 4, 8, 16])
@pytest.mark.parametrize("desc", [False, True])
def test_libthrs_equals_reference_kernels(refk, gpu, kt, vb, desc):
    torch = gpu
    width = O.KEY_BYTES[kt] * 8
    sizes = [1, 100, 2047, 2048, 2049, 10007, 65537, 300001]
    for j, n in enumerate(sizes):
        keys = O.randomize_np(kt, O.splitmix64_stream(31337 * (j + 1), n))
        if j % 3 == 1:
            keys = keys & np.array(0x0F0F, keys.dtype)         # ties: stability
        if kt == O.F32 and j % 4 == 2:                         # raw bits: NaN / Inf / denormals / -0
            keys = O.splitmix64_stream(999 + j, n).astype(np.uint32)
        vals = C._values(n, vb) if vb else None
        windows = [(0, width), (8, 24)] + ([(width - 8, width)] if width == 64 else [])
        for (s, e) in windows:
            k, v, rk, rv = run_both(torch, kt, vb, desc, keys, vals, s, e)
            ek, ev = O.lsd_sort(kt, keys, vals, s, e, desc)
            assert np.array_equal(rk, ek), ("reference kernels vs oracle", n, s, e)
            assert np.array_equal(k, rk), ("libthrs vs reference kernels", n, s, e)
            if vb:
                assert np.array_equal(rv, ev) and np.array_equal(v, rv), (n, s, e)


@pytest.mark.parametrize("name", list(C.CASES))
def test_reference_kernels_reproduce_golden(refk, gpu, name):
    """The committed golden digests (all 128 iterations of each UTEST stream)
    are what the reference's own kernels output."""
    torch = gpu
    kind, kt, vb, desc, stream = C.CASES[name]
    rows = GOLDEN["cases"][name]
    for i, item in enumerate(stream(128)):
        keys, vals = item["keys"], item.get("values")
        n = keys.shape[0]
        s, e = (int(item["start"]), int(item["start"]) + 8) if kind == "window" else (0, O.KEY_BYTES[kt] * 8)
        kr = to_dev(torch, keys)
        vr = to_dev(torch, vals) if vb else None
        rtmp = torch.empty(sum(R.temp_bytes(kt, VT.get(vb, 0), n)), dtype=torch.uint8, device="cuda")
        R.sort(kt, VT.get(vb, 0), desc, kr, vr, n, rtmp, s, e, torch.cuda.current_stream())
        torch.cuda.synchronize()
        k = kr.cpu().numpy().view(keys.dtype)
        assert C.digest(k) == rows[i]["keys"], (name, i)
        if vb:
            assert C.digest(vr.cpu().numpy().view(vals.dtype).reshape(vals.shape)) == rows[i]["values"], (name, i)
