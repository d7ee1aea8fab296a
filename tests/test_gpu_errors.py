"""Device-side failures reach the caller (thrs_capi.h "Device-side failures";
the reference's THRS_ASSERT, tinyhipradixsort.hpp:14-15, fails loudly).

libthrs_spin0.so is the library built with THRS_SPIN_MAX=0: every look-back
or tile-claim wait gives up at once, so a large sort fails on the device.
The failure must surface (a) through checkDeviceError on its temporary
buffer, (b) as the error of the NEXT sort call on the device, without a
synchronisation, and (c) through take_device_error -- and the normal library
must report nothing."""
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
small = torch.zeros(4 * 1000, dtype=torch.uint8, device="cuda")
res = {{"check": 0, "next": 0, "take": 0, "clean_after": 1}}
for attempt in range(8):
    TU.fill_keys(0, keys, n, start=attempt * n)
    rs.sortKeys(keys, n, tmp, 0, 32)
    torch.cuda.synchronize()
    try:
        rs.sortKeys(small, 1000, tmp, 0, 32)   # must report the earlier failure
    except T.ThrsError as e:
        res["next"] += e.status == -5
        continue
    try:
        rs.checkDeviceError(tmp)
    except T.ThrsError as e:
        res["check"] += e.status == -5
# after a reported failure the sticky word is clear: a tiny sort (one tile, no wait) succeeds
try:
    rs.sortKeys(small, 1000, tmp, 0, 32)
    torch.cuda.synchronize()
    T.take_device_error()
except T.ThrsError:
    res["clean_after"] = 0
print(res)
"""


def _run(lib):
    code = SCRIPT.format(root=ROOT, lib=lib)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return eval(r.stdout.strip().splitlines()[-1])


def test_forced_timeout_is_reported():
    lib = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_spin0.so")
    assert os.path.exists(lib), "build it first (make)"
    res = _run(lib)
    print(res)
    assert res["next"] >= 1, res           # the next call on the device raised
    assert res["clean_after"] == 1, res


def test_normal_library_reports_nothing():
    res = _run(os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs.so"))
    assert res == {"check": 0, "next": 0, "take": 0, "clean_after": 1}, res
