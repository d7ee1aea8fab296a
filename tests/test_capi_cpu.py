"""CPU: the C-ABI libraries load and export every declared symbol; host-only
logic of the boundary (temp sizing, argument validation, enum mapping) works
without a device."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import tinyhipradixsort_amd as T

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "thrs", "thrs_capi.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(thrs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("thrs_sort_keys", "thrs_sort_pairs", "thrs_get_temporary_buffer_bytes", "thrs_malloc", "thrs_free"):
        assert s in syms


def test_libthrs_exports_every_declared_symbol():
    L = T.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert L.thrs_abi_version() == T.ABI_VERSION


def test_libthrs_is_gfx950_code():
    blob = open(T.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob    # the embedded code object targets gfx950


def test_testutil_exports():
    from tinyhipradixsort_amd import testutil
    L = testutil.tlib()
    for s in ("thrsu_fill_keys", "thrsu_iota", "thrsu_check_sorted", "thrsu_fingerprint", "thrsu_check_pairs"):
        assert hasattr(L, s)


def test_bytes_of_and_enums():
    assert T.bytesOf(T.KeyType.U32) == 4 and T.bytesOf(T.KeyType.F64) == 8
    assert T.bytesOf(T.ValueType.U128) == 16
    c = T.RadixSort.Config()
    c.configureWithKey(np.float32)
    assert c.keyType == T.KeyType.F32
    c.configureWithKeyPair(np.uint64, 16)
    assert c.keyType == T.KeyType.U64 and c.valueType == T.ValueType.U128
    c.configureWithKeyPair(np.float64, np.uint32)
    assert c.keyType == T.KeyType.F64 and c.valueType == T.ValueType.U32
    with pytest.raises(T.ThrsError):
        c.configureWithKeyPair(np.uint32, 2)


@pytest.mark.parametrize("kt,vt", [(T.KeyType.U32, T.ValueType.U32), (T.KeyType.U64, T.ValueType.U128),
                                   (T.KeyType.F32, T.ValueType.U64)])
@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 99999, 1 << 20, (1 << 31) + 100])
def test_temporary_buffer_layout(kt, vt, n):
    cfg = T.RadixSort.Config(keyType=kt, valueType=vt)
    d = T.RadixSort([], cfg).getTemporaryBufferBytes(n)
    kb, vb = T.bytesOf(kt), T.bytesOf(vt)
    assert d.keyOutBuffer == -(-kb * n // 16) * 16           # hpp:840
    assert d.valueOutBuffer == -(-vb * n // 16) * 16         # hpp:841
    assert d.pSumBuffer % 16 == 0 and d.pSumBuffer > 0
    assert d.getTemporaryBufferBytesForSortKeys() == d.pSumBuffer + d.keyOutBuffer
    assert d.getTemporaryBufferBytesForSortPairs() == d.pSumBuffer + d.keyOutBuffer + d.valueOutBuffer
    assert d.getOutputKeyBuffer(1000) == 1000 + d.pSumBuffer
    assert d.getOutputValueBuffer(1000) == 1000 + d.pSumBuffer + d.keyOutBuffer
    # scratch (look-back status words) stays a modest fraction of the payload
    # (the reference's pSum region is 4*256*ceil(n/2048) = n/2 bytes, hpp:839),
    # plus a fixed ~1.1 MiB: the 3-pass path's bucket histogram and chunk table
    # and the segmented pass's extra look-back rows; u32 / f32 keys: + the
    # bucket path's u8 plane (n bytes: its two u16 planes fill keyOut),
    # reserved for every n up to 2^31 + 2^25 (a forced bucket path carries
    # the planes too),
    # and room for a big chunk per 4097 keys (the 4096-key local geometry:
    # 3 KiB of fallback tables each, ~0.75 B per key below 2^28 keys) -- per
    # 4353 keys for thrs_local_kv's types (8-byte keys, 8/16-byte values: its
    # 4352-key chunks, 6 KiB each, ~1.4 B per key below 2^28 keys; row 130)
    plane = -(-n // 256) * 256 if kt in (T.KeyType.U32, T.KeyType.F32) and n <= (1 << 31) + (1 << 25) else 0
    kv = kb == 8 or vb >= 8
    if n >= (1 << 20):
        assert d.pSumBuffer < ((0.4 if kb == 4 else 0.3) * d.keyOutBuffer + plane + (3 << 20) // 2
                               + (1.5 * n if kv else 0))


def test_argument_validation_needs_no_device():
    L = T.lib()
    cfg = T._CConfig(1, 0, 0, 0)
    # (endBits - startBits) % 8 != 0 -> THRS_ERROR_BIT_RANGE (hpp:856), checked before any HIP call
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 10, None, 0, 31, None) == -2
    assert L.thrs_sort_pairs(ctypes.byref(cfg), None, None, 10, None, 3, 8, None) == -2
    # n == 0 and start >= end are no-ops
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 0, None, 0, 32, None) == 0
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 5, None, 16, 16, None) == 0
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 5, None, 40, 32, None) == 0
    # every digit past the key width: identity, no launch
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 5, None, 32, 64, None) == 0
    # invalid enums / null pointers / negative start
    bad = T._CConfig(1, 9, 0, 0)
    assert L.thrs_sort_keys(ctypes.byref(bad), None, 5, None, 0, 32, None) == -1
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 5, None, 0, 32, None) == -1
    assert L.thrs_sort_keys(ctypes.byref(cfg), None, 5, None, -8, 32, None) == -1
    assert L.thrs_sort_keys(None, None, 5, None, 0, 32, None) == -1
    assert L.thrs_status_string(-2).startswith(b"THRS_ERROR_BIT_RANGE")
    with pytest.raises(T.ThrsError) as e:
        T.RadixSort([], T.RadixSort.Config()).sortKeys(0, 10, 0, 0, 12, 0)
    assert e.value.status == -2


def test_header_compiles_without_hip_headers(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include <thrs/tinyhipradixsort.hpp>\n#include <thrs/fpKey.hpp>\n'
                   'int main(){ thrs::RadixSort::Config c; c.configureWithKeyPair<double, uint64_t>();'
                   ' return (int)c.keyType + (getKeyBits(-0.0f) == getKeyBits(0.0f) ? 0 : 1); }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "tinyhipradixsort_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text and "liboracle" not in text, f


def test_path_info_matches_the_configs():
    """thrs_get_path_info: the host's path choice per BASELINE.json config (no
    device work) and the HBM bytes that path must move."""
    def info(kt, vt, n, pairs, s=0, e=None, **opt):
        cfg = T.RadixSort.Config(keyType=kt, valueType=vt)
        rs = T.RadixSort([], cfg, T.Options(**opt))
        return rs.pathInfo(n, s, e if e is not None else 8 * T.bytesOf(kt), pairs)
    U32, U64, F32 = T.KeyType.U32, T.KeyType.U64, T.KeyType.F32
    c2 = info(U32, T.ValueType.U32, 1 << 30, False)
    assert (c2["path"], c2["local"], c2["planes"], c2["device_passes"]) == ("bucket", "thrs_local16", True, 2)
    assert c2["min_bytes"] == (4 + 7 + 5 + 6) * (1 << 30)           # hist 4, passes 4+3 and 3+2, local 2+4
    c3 = info(U32, T.ValueType.U32, 1 << 30, True)
    assert (c3["path"], c3["local"], c3["planes"]) == ("bucket", "thrs_local_pairs", True)
    # keys as planes, values as they are: hist 4, passes (4+4)+(3+4) and
    # (3+4)+(2+4), local (2+4)+(4+4)
    assert c3["min_bytes"] == (4 + 15 + 13 + 14) * (1 << 30)
    c3off = info(U32, T.ValueType.U32, 1 << 30, True, planes="off")
    assert not c3off["planes"] and c3off["min_bytes"] == (4 + 16 + 16 + 16) * (1 << 30)
    assert info(F32, T.ValueType.U32, 1 << 30, True)["planes"]            # f32 pairs too
    assert not info(U32, T.ValueType.U64, 1 << 30, True)["planes"]        # 8-byte values: whole keys
    c4 = info(F32, T.ValueType.U32, 1 << 28, False)
    assert (c4["path"], c4["local"], c4["planes"], c4["local_cap"]) == ("bucket", "thrs_local16", True, 9216)
    assert c4["min_bytes"] == (4 + 7 + 5 + 6) * (1 << 28)
    # the lower bounds of the default's bucket window (docs/EXPERIMENTS.md row 87)
    assert info(U32, T.ValueType.U32, 59999999, False)["path"] == "lsd"
    assert info(U32, T.ValueType.U32, 60000000, False)["path"] == "bucket"
    assert info(U32, T.ValueType.U32, 60000000, False)["planes"]
    assert info(F32, T.ValueType.U32, 39999999, False)["path"] == "lsd"
    assert info(F32, T.ValueType.U32, 40000000, False)["path"] == "bucket"
    # u32 keys-only up to 3 x 2^26: 4096-key chunks (docs/EXPERIMENTS.md row 112)
    assert info(U32, T.ValueType.U32, 160000000, False)["local_cap"] == 4096
    assert info(U32, T.ValueType.U32, 3 << 26, False)["local_cap"] == 4096
    assert info(U32, T.ValueType.U32, (3 << 26) + 1, False)["local_cap"] == 9216
    assert info(F32, T.ValueType.U32, 160000000, False)["local_cap"] == 9216
    assert info(U32, T.ValueType.U32, 160000000, True)["local_cap"] == 4096   # pairs too (row 115)
    assert info(F32, T.ValueType.U32, 160000000, True)["local_cap"] == 4096   # f32 pairs too (row 131)
    assert info(F32, T.ValueType.U32, 1 << 27, False)["local_cap"] == 4096      # f32 keys up to 2^27 (row 131)
    assert info(F32, T.ValueType.U32, (1 << 27) + 1, False)["local_cap"] == 9216
    assert info(U32, T.ValueType.U32, 34999999, True)["path"] == "lsd"
    assert info(U32, T.ValueType.U32, 35000000, True)["path"] == "bucket"
    assert info(F32, T.ValueType.U32, 31999999, True)["path"] == "lsd"
    assert info(F32, T.ValueType.U32, 32000000, True)["path"] == "bucket"
    # thrs_local_kv's types (row 130)
    assert info(U64, T.ValueType.U32, 19999999, False)["path"] == "lsd"
    assert info(U64, T.ValueType.U32, 20000000, False)["path"] == "bucket"
    assert info(U64, T.ValueType.U64, 11999999, True)["path"] == "lsd"
    assert info(U64, T.ValueType.U64, 12000000, True)["path"] == "bucket"
    assert info(T.KeyType.F64, T.ValueType.U64, 14999999, True)["path"] == "lsd"
    assert info(U64, T.ValueType.U128, 8000000, True)["path"] == "bucket"
    assert info(U32, T.ValueType.U64, 31999999, True)["path"] == "lsd"
    assert info(U32, T.ValueType.U128, 25000000, True)["path"] == "bucket"
    c5 = info(U64, T.ValueType.U64, 1 << 30, True)
    assert (c5["path"], c5["local"], c5["local_cap"]) == ("bucket", "thrs_local_kv", 17408)
    # thrs_local_kv geometries by size (docs/EXPERIMENTS.md row 130): 8704-key
    # chunks up to 2^29, 4352 up to 3 x 2^26; asked: big / small / tiny16
    assert info(U64, T.ValueType.U64, (1 << 29) + 1, True, path="bucket")["local_cap"] == 17408
    assert info(U64, T.ValueType.U64, 1 << 29, True)["local_cap"] == 8704
    assert info(T.KeyType.F64, T.ValueType.U64, 1 << 29, True)["local_cap"] == 8704
    assert info(U64, T.ValueType.U128, 1 << 29, True)["local_cap"] == 8704
    assert info(U64, T.ValueType.U64, 3 << 26, True, path="bucket")["local_cap"] == 4352
    assert info(U64, T.ValueType.U64, 1 << 20, True, path="bucket", localGeometry="big")["local_cap"] == 17408
    assert info(U64, T.ValueType.U64, 1 << 20, True, path="bucket", localGeometry="small")["local_cap"] == 8704
    assert info(U32, T.ValueType.U64, 1 << 30, True, path="bucket", localGeometry="tiny16")["local_cap"] == 4352
    wide = info(U32, T.ValueType.U128, 1 << 30, True)
    assert (wide["path"], wide["local"]) == ("bucket", "thrs_local_kv")
    assert info(U32, T.ValueType.U32, 1 << 20, False)["path"] == "lsd"
    assert info(U32, T.ValueType.U32, 1 << 20, False, path="bucket", s=0, e=24)["local"] == "thrs_local"
    lsd = info(U32, T.ValueType.U32, 1 << 20, False, path="lsd")
    assert lsd["min_bytes"] == 4 * (1 << 20) + 4 * 8 * (1 << 20)     # histogram + 4 passes of read + write


def test_kernel_argument_structs_are_determinate(tmp_path):
    """Every struct run_sort passes to a kernel by value has a default
    initialiser on each field and no implicit padding, so no field reaches a
    kernel indeterminate (docs/EXPERIMENTS.md row 106's class of bug).
    tests/cpp/struct_init.cpp default-initialises each over 0xAA- and
    0x55-filled memory and compares the bytes; compiled host-only."""
    exe = tmp_path / "struct_init"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "--offload-host-only", "-x", "hip",
                        "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tinyhipradixsort_amd", "csrc"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "struct_init.cpp")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
