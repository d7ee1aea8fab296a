"""Device-side failures reach the caller of the failing sort (thrs_capi.h
"Device-side failures"; the reference's THRS_ASSERT, tinyhipradixsort.hpp:14-15,
fails loudly), and only that caller.

libthrs_spin0.so is the library built with THRS_SPIN_MAX=0: every look-back
or tile-claim wait gives up at once, so a large sort fails on the device
while a one-tile sort (no wait) succeeds.  The failure must surface
  (a) through checkDeviceError on the failing sort's temporary buffer,
  (b) through sortKeys(..., checked=True) of the failing sort itself,
  (c) through accumulateDeviceError into a caller word (stream-ordered),
  (d) through take_device_error (device-wide sticky word),
and (e) an unrelated sort issued after the failure, on another temporary
buffer, must run and succeed.  The normal library reports nothing.  A first
sort issued inside a stream capture (the sticky word is not set up there)
must not disable later sorts (init retried after it is skipped)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
import tinyhipradixsort_amd as T
from tinyhipradixsort_amd import testutil as TU
T.LIB_PATH = {lib!r}
torch.cuda.set_device(0)
rs = T.RadixSort([], T.RadixSort.Config())
n = 1 << 24
keys = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
m = 1000
small = torch.empty(4 * m, dtype=torch.uint8, device="cuda")
tmp2 = torch.empty(rs.getTemporaryBufferBytes(m).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
acc = torch.zeros(1, dtype=torch.int32, device="cuda")
res = dict(check=0, checked=0, acc=0, take=0, other_ok=0, other_bad=0, attempts=6)
for attempt in range(res["attempts"]):
    TU.fill_keys(0, keys, n, start=attempt * n)
    try:
        rs.sortKeys(keys, n, tmp, 0, 32, checked=True)                # (b)
    except T.ThrsError as e:
        res["checked"] += e.status == -5
    try:
        rs.checkDeviceError(tmp)                                     # (a)
    except T.ThrsError as e:
        res["check"] += e.status == -5
    acc.zero_()
    rs.accumulateDeviceError(tmp, acc)                               # (c)
    torch.cuda.synchronize()
    res["acc"] += int(acc.item()) != 0
    try:
        T.take_device_error()                                        # (d)
    except T.ThrsError as e:
        res["take"] += e.status == -5
    TU.fill_keys(0, small, m, start=attempt)                         # (e) an unrelated sort still runs
    try:
        rs.sortKeys(small, m, tmp2, 0, 32, checked=True)
        res["other_ok"] += TU.count_unsorted(0, small, m, 0, 32) == 0
    except T.ThrsError:
        res["other_bad"] += 1
print(res)
"""

CAPTURE = r"""
import sys, torch
sys.path.insert(0, {root!r})
import tinyhipradixsort_amd as T
from tinyhipradixsort_amd import testutil as TU
torch.cuda.set_device(0)
rs = T.RadixSort([], T.RadixSort.Config())
n = 100003
keys = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
TU.fill_keys(0, keys, n, start=0)
torch.cuda.synchronize()
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):            # the library's FIRST call in this process is captured
    rs.sortKeys(keys, n, tmp, 0, 32, stream=s)
g.replay()
torch.cuda.synchronize()
ok_graph = TU.count_unsorted(0, keys, n, 0, 32) == 0
TU.fill_keys(0, keys, n, start=n)
rs.sortKeys(keys, n, tmp, 0, 32, checked=True)  # outside the capture: runs and publishes normally
ok_after = TU.count_unsorted(0, keys, n, 0, 32) == 0
T.take_device_error()
print(dict(graph=ok_graph, after=ok_after))
"""


def _run(code):
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return eval(r.stdout.strip().splitlines()[-1])


def test_forced_timeout_is_reported_to_its_own_caller():
    lib = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_spin0.so")
    assert os.path.exists(lib), "build it first (make)"
    res = _run(SCRIPT.format(root=ROOT, lib=lib))
    print(res)
    k = res["attempts"]
    # the 2^24-key sort fails with no spinning allowed (1024 tiles: in practice
    # every attempt); each failure is seen by all four reports of that sort
    assert res["checked"] >= 1, res
    assert res["check"] == res["checked"] == res["acc"] == res["take"], res
    assert res["other_ok"] == k and res["other_bad"] == 0, res


def test_normal_library_reports_nothing():
    res = _run(SCRIPT.format(root=ROOT, lib=os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs.so")))
    k = res["attempts"]
    assert res == dict(check=0, checked=0, acc=0, take=0, other_ok=k, other_bad=0, attempts=k), res


def test_first_sort_under_stream_capture():
    res = _run(CAPTURE.format(root=ROOT))
    assert res == {"graph": True, "after": True}, res


BUCKET = r"""
import sys, torch
sys.path.insert(0, {root!r})
import tinyhipradixsort_amd as T
from tinyhipradixsort_amd import testutil as TU
T.LIB_PATH = {lib!r}
torch.cuda.set_device(0)
GUARD = 1 << 20
def guarded(nbytes):
    buf = torch.full((nbytes + 2 * GUARD,), 0xA5, dtype=torch.uint8, device="cuda")
    return buf, buf[GUARD:GUARD + nbytes]
def guards_ok(buf):
    return bool((buf[:GUARD] == 0xA5).all().item()) and bool((buf[-GUARD:] == 0xA5).all().item())
res = dict(failed=0, reported=0, guards_ok=0, other_ok=0, sorts=0)
for kt, vb, dist in ((0, 0, "uniform"), (0, 0, "fewuniq"), (0, 4, "uniform"), (0, 4, "fewuniq"), (1, 8, "uniform"),
                     (1, 8, "fewuniq"), (2, 4, "uniform")):
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={{0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                 8: T.ValueType.U64}}[vb])
    rs = T.RadixSort([], cfg, T.Options(path="bucket"))
    n = 1 << 24
    kb = 8 if kt in (1, 3) else 4
    d = rs.getTemporaryBufferBytes(n)
    tbytes = d.getTemporaryBufferBytesForSortPairs() if vb else d.getTemporaryBufferBytesForSortKeys()
    kbuf, keys = guarded(kb * n)
    tbuf, tmp = guarded(tbytes)
    vbuf, vals = guarded(max(1, vb * n))
    if dist == "uniform":
        TU.fill_keys(kt, keys, n, start=7 * n)
    else:
        TU.fill_dist(kt, keys, n, dist)                 # few distinct keys: big chunks, the per-bucket fallback
    if vb:
        TU.iota(vb, vals, n)
    torch.cuda.synchronize()
    res["sorts"] += 1
    try:
        if vb:
            rs.sortPairs(keys, vals, n, tmp, 0, 8 * kb, checked=True)
        else:
            rs.sortKeys(keys, n, tmp, 0, 8 * kb, checked=True)
    except T.ThrsError as e:
        res["failed"] += 1
        res["reported"] += e.status == -5
    torch.cuda.synchronize()
    res["guards_ok"] += guards_ok(kbuf) and guards_ok(tbuf) and guards_ok(vbuf)
    try:
        T.take_device_error()
    except T.ThrsError:
        pass
m = 1000
small = torch.empty(4 * m, dtype=torch.uint8, device="cuda")
rs = T.RadixSort([], T.RadixSort.Config())
tmp2 = torch.empty(rs.getTemporaryBufferBytes(m).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
TU.fill_keys(0, small, m, start=3)
rs.sortKeys(small, m, tmp2, 0, 32, checked=True)
res["other_ok"] = TU.count_unsorted(0, small, m, 0, 32) == 0
print(res)
"""


def test_forced_timeout_on_the_bucket_path_stays_in_bounds():
    """the bucket path with every look-back giving up at
    once (libthrs_spin0.so): the segmented top-digit passes, the local sorts
    and -- for few-distinct-key inputs -- the per-bucket fallback's passes
    (thrs_pass_big) and copy-back (thrs_big_copy).  Every failing sort is
    reported to its caller, nothing outside the keys, values and temporary
    buffer is written (1 MiB canary bands on both sides of each, checked
    after every sort), and an unrelated sort afterwards succeeds."""
    lib = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_spin0.so")
    assert os.path.exists(lib), "build it first (make)"
    res = _run(BUCKET.format(root=ROOT, lib=lib))
    print(res)
    assert res["sorts"] == 7 and res["guards_ok"] == 7, res
    assert res["failed"] >= 1 and res["reported"] == res["failed"], res
    assert res["other_ok"], res


INJECT = r"""
import sys, ctypes, torch
import numpy as np
sys.path.insert(0, {root!r})
import tinyhipradixsort_amd as T
from tinyhipradixsort_amd import testutil as TU
T.LIB_PATH = {lib!r}
torch.cuda.set_device(0)
L = T.lib()
L.thrs_debug_inject.argtypes = [ctypes.c_int]
GUARD = 1 << 20
def guarded(nbytes):
    buf = torch.full((nbytes + 2 * GUARD,), 0xA5, dtype=torch.uint8, device="cuda")
    return buf, buf[GUARD:GUARD + nbytes]
def guards_ok(buf):
    return bool((buf[:GUARD] == 0xA5).all().item()) and bool((buf[-GUARD:] == 0xA5).all().item())
# two buckets of 15000 keys each (above the small local sort's 9216): the plan
# lists two big chunks; every tile chain is one tile long, so nothing spins
n = 30000
rng = np.random.default_rng(5)
host = ((np.arange(n, dtype=np.uint32) % 2) << 16) | rng.integers(0, 1 << 16, n, dtype=np.uint32)
rs = T.RadixSort([], T.RadixSort.Config(), T.Options(path="bucket"))
tbytes = rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys()
res = {{}}
for inject in (1, 0):
    L.thrs_debug_inject(inject)
    kbuf, keys = guarded(4 * n)
    tbuf, tmp = guarded(tbytes)
    keys.copy_(torch.from_numpy(host.view(np.uint8)).cuda())
    acc = torch.zeros(1, dtype=torch.int32, device="cuda")
    status = 0
    try:
        rs.sortKeys(keys, n, tmp, 0, 32, checked=True)
    except T.ThrsError as e:
        status = e.status
    rs.accumulateDeviceError(tmp, acc)
    torch.cuda.synchronize()
    out = keys.cpu().numpy().view(np.uint32)
    res[inject] = dict(status=status, word=int(acc.item()), guards=guards_ok(kbuf) and guards_ok(tbuf),
                       exact=bool(np.array_equal(out, np.sort(host))))
    try:
        T.take_device_error()
    except T.ThrsError:
        pass
print(res)
"""


def test_stale_big_chunk_entry_is_reported():
    """a stale entry in the plan's big-chunk list (the
    round-4 ordering bug's shape) is caught by thrs_plan_rows's check, never
    addresses past a table, and reaches the caller as THRS_ERROR_DEVICE_CHECK
    (error word bit 1, no timeout bit).  The same sort without the injection
    is exact.  (libthrs_spin0.so: built with THRS_FAULT_INJECT.)"""
    lib = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_spin0.so")
    assert os.path.exists(lib), "build it first (make)"
    res = _run(INJECT.format(root=ROOT, lib=lib))
    print(res)
    assert res[1]["status"] == -6 and res[1]["word"] == 2 and res[1]["guards"], res
    assert res[0] == dict(status=0, word=0, guards=True, exact=True), res


CLAIMS = r"""
import sys, torch
sys.path.insert(0, {root!r})
import tinyhipradixsort_amd as T
from tinyhipradixsort_amd import testutil as TU
T.LIB_PATH = {lib!r}
torch.cuda.set_device(0)
rs = T.RadixSort([], T.RadixSort.Config(), T.Options(tileClaims="xcd_blocks", path="lsd"))
n = 1 << 24
keys = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
tmp = torch.empty(rs.getTemporaryBufferBytes(n).getTemporaryBufferBytesForSortKeys(), dtype=torch.uint8, device="cuda")
res = dict(failed=0, timeout=0, other=0, attempts=6)
for attempt in range(res["attempts"]):
    TU.fill_keys(0, keys, n, start=attempt * n)
    try:
        rs.sortKeys(keys, n, tmp, 0, 8, checked=True)   # ONE pass (8-bit window), XCD-block tile claims
    except T.ThrsError as e:
        res["failed"] += 1
        res["timeout"] += e.status == -5
        res["other"] += e.status != -5
    try:
        T.take_device_error()
    except T.ThrsError:
        pass
print(res)
"""


def test_claim_timeout_reports_lookback_timeout():
    """a tile-claim wait that gives up on the XCD-block path
    (thrs_pass_xb's xb_claim) sets the spin bit of the error word, so the
    caller sees THRS_ERROR_LOOKBACK_TIMEOUT (-5), not THRS_ERROR_DEVICE_CHECK
    (-6, a clamped run).  One pass (8-bit window) with the XCD-block claims
    forced, built with THRS_SPIN_MAX=0 (libthrs_spin0.so): every failing sort
    must report -5."""
    lib = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_spin0.so")
    assert os.path.exists(lib), "build it first (make)"
    res = _run(CLAIMS.format(root=ROOT, lib=lib))
    print(res)
    assert res["failed"] >= 1 and res["timeout"] == res["failed"] and res["other"] == 0, res
