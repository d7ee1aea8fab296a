"""tinyhipradixsort_amd -- MI355X-native LSD radix sort, Python host mirror.

Mirrors the reference's host API (/root/reference/tinyhipradixsort.hpp) name
for name, over the C-ABI of the in-tree ``libthrs.so`` (declared in
``include/thrs/thrs_capi.h``):

    KeyType / ValueType / SortOrder / bytesOf          (hpp:638-692)
    Buffer                                             (hpp:501-528)
    RadixSort.Config + configureWithKey(KeyT)
                     + configureWithKeyPair(KeyT, V)  (hpp:697-749)
    RadixSort(extraArgs, config)                       (hpp:751-804)
    TemporaryBufferDef / getTemporaryBufferBytes       (hpp:806-843)
    sortKeys / sortPairs                               (hpp:845-852)

Device buffers may be passed as torch tensors (``.data_ptr()`` is used) or as
integer device addresses; streams as ``torch.cuda.Stream``, an integer HIP
stream handle, or ``None`` for torch's current stream.  Errors raise
``ThrsError`` (the reference's THRS_ASSERT -> __debugbreak).

There is no CPU fallback: if ``libthrs.so`` is missing the import of the sort
entry points raises.  The CPU oracle under ``oracle/`` is test
infrastructure and is never imported from here.
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libthrs.so")
TESTUTIL_PATH = os.path.join(_HERE, "libthrs_testutil.so")
ABI_VERSION = 6

__all__ = ["KeyType", "ValueType", "SortOrder", "bytesOf", "div_round_up64", "next_multiple64", "Buffer",
           "RadixSort", "Options", "ThrsError", "lib", "LIB_PATH", "take_device_error"]


class ThrsError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{msg} (status {status})")
        self.status = status


_lib = None


def lib() -> ctypes.CDLL:
    """The in-tree libthrs.so.  Raises if it has not been built -- never
    substitutes anything else."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i32, i64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64
        L.thrs_abi_version.restype = i32
        L.thrs_status_string.argtypes = [i32]
        L.thrs_status_string.restype = ctypes.c_char_p
        L.thrs_key_bytes.argtypes = [i32]
        L.thrs_key_bytes.restype = u64
        L.thrs_value_bytes.argtypes = [i32]
        L.thrs_value_bytes.restype = u64
        L.thrs_get_temporary_buffer_bytes.argtypes = [ctypes.POINTER(_CConfig), u32, ctypes.POINTER(_CTempDef)]
        L.thrs_sort_keys.argtypes = [ctypes.POINTER(_CConfig), vp, u32, vp, i32, i32, vp]
        L.thrs_sort_pairs.argtypes = [ctypes.POINTER(_CConfig), vp, vp, u32, vp, i32, i32, vp]
        L.thrs_sort_keys_ex.argtypes = [ctypes.POINTER(_CConfig), ctypes.POINTER(_COptions), vp, u32, vp, i32, i32, vp]
        L.thrs_sort_pairs_ex.argtypes = [ctypes.POINTER(_CConfig), ctypes.POINTER(_COptions), vp, vp, u32, vp, i32,
                                         i32, vp]
        L.thrs_take_device_error.restype = i32
        L.thrs_digit_histogram.argtypes = [ctypes.POINTER(_CConfig), vp, u32, u64, u64, i32, vp, vp]
        L.thrs_digit_histogram.restype = i32
        L.thrs_digit_histogram_batch.argtypes = [ctypes.POINTER(_CConfig), vp, ctypes.POINTER(_CHistTarget), i32, i32,
                                                 vp, vp]
        L.thrs_digit_histogram_batch.restype = i32
        L.thrs_check_device_error.argtypes = [vp, vp]
        L.thrs_accumulate_device_error.argtypes = [vp, vp, vp]
        L.thrs_partition_pass.argtypes = [ctypes.POINTER(_CConfig), vp, vp, u32, vp, vp, vp, i32, vp, vp]
        L.thrs_malloc.argtypes = [ctypes.POINTER(vp), i64]
        L.thrs_free.argtypes = [vp]
        L.thrs_memcpy_htod_async.argtypes = [vp, vp, u64, vp]
        L.thrs_memcpy_dtoh.argtypes = [vp, vp, u64]
        L.thrs_memcpy_dtod_async.argtypes = [vp, vp, u64, vp]
        L.thrs_stream_create.argtypes = [ctypes.POINTER(vp)]
        L.thrs_stream_destroy.argtypes = [vp]
        L.thrs_stream_synchronize.argtypes = [vp]
        L.thrs_profile_enable.argtypes = [i32]
        L.thrs_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32),
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
        L.thrs_profile_read_kind.argtypes = [i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
        L.thrs_rank_mode.restype = i32
        L.thrs_profile_read_launches.argtypes = [i32, ctypes.POINTER(ctypes.c_double), i32, ctypes.POINTER(i32)]
        L.thrs_profile_read_launches.restype = i32
        L.thrs_profile_read_launch_kernels.argtypes = [i32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(u64), i32,
                                                       ctypes.POINTER(i32)]
        L.thrs_profile_read_launch_kernels.restype = i32
        L.thrs_profile_kernel_name.argtypes = [i32]
        L.thrs_profile_kernel_name.restype = ctypes.c_char_p
        L.thrs_debug_big_keys.argtypes = [vp, i32, i32, u32, vp, ctypes.POINTER(u64)]
        L.thrs_debug_big_keys.restype = i32
        L.thrs_get_path_info.argtypes = [ctypes.POINTER(_CConfig), ctypes.POINTER(_COptions), i32, u32, i32, i32,
                                     ctypes.POINTER(_CPathInfo)]
        L.thrs_get_path_info.restype = i32
        L.thrs_debug_bucket_mode.argtypes = [vp, i32, i32, u32, vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.thrs_debug_bucket_mode.restype = i32
        L.thrs_debug_vector_tiles.argtypes = [vp, i32, u32, vp, ctypes.POINTER(u32)]
        L.thrs_debug_vector_tiles.restype = i32
        for f in ("thrs_profile_enable", "thrs_profile_read", "thrs_profile_read_kind",
                  "thrs_get_temporary_buffer_bytes", "thrs_sort_keys", "thrs_sort_pairs", "thrs_sort_keys_ex",
                  "thrs_sort_pairs_ex", "thrs_check_device_error", "thrs_accumulate_device_error",
                  "thrs_partition_pass",
                  "thrs_malloc", "thrs_free", "thrs_memcpy_htod_async", "thrs_memcpy_dtoh", "thrs_memcpy_dtod_async",
                  "thrs_stream_create", "thrs_stream_destroy", "thrs_stream_synchronize"):
            getattr(L, f).restype = i32
        if L.thrs_abi_version() != ABI_VERSION:
            raise ImportError(f"libthrs ABI {L.thrs_abi_version()} != {ABI_VERSION}")
        _lib = L
    return _lib


def _check(rc: int):
    if rc != 0:
        raise ThrsError(rc, lib().thrs_status_string(rc).decode())


class _CConfig(ctypes.Structure):
    _fields_ = [("keyIs16byteAligned", ctypes.c_int32), ("keyType", ctypes.c_int32),
                ("valueType", ctypes.c_int32), ("sortOrder", ctypes.c_int32)]


class _COptions(ctypes.Structure):
    _fields_ = [("path", ctypes.c_int32), ("localGeometry", ctypes.c_int32), ("segmented", ctypes.c_int32),
                ("tileClaims", ctypes.c_int32), ("rank", ctypes.c_int32), ("planes", ctypes.c_int32),
                ("keyRange", ctypes.c_int32), ("squeeze", ctypes.c_int32), ("rangeLo", ctypes.c_uint64),
                ("rangeHi", ctypes.c_uint64)]


@dataclass
class Options:
    """thrs_options (thrs_capi.h): explicit path / tuning choices, no
    reference counterpart.  Every choice gives the same bit-exact result; the
    defaults are the library's own choice.  Values are the names below."""
    path: str = "auto"            # auto | lsd | bucket
    localGeometry: str = "auto"   # auto | big | small | big32 | count16 | rank16 | wide16 | tiny16
    segmented: str = "auto"       # auto | top_only | none
    tileClaims: str = "auto"      # auto | xcd_blocks | ticket
    rank: str = "auto"            # auto | atomic | ballot
    planes: str = "auto"          # auto | on | off
    squeeze: str = "auto"         # auto | off (float keys: data-chosen bucket bits)
    # key range promise (thrs_options.keyRange): every key's image
    # getKeyBits(k) ^ (descending ? ~0 : 0) lies in [rangeLo, rangeHi]; None = no promise
    keyRange: "tuple[int, int] | None" = None

    _ENUMS = {"path": ("auto", "lsd", "bucket"), "localGeometry": ("auto", "big", "small", "big32", "count16", "rank16", "wide16", "tiny16"),
              "segmented": ("auto", "top_only", "none"), "tileClaims": ("auto", "xcd_blocks", "ticket"),
              "rank": ("auto", "atomic", "ballot"), "planes": ("auto", "on", "off"), "squeeze": ("auto", "off")}

    def _c(self) -> "_COptions":
        o = _COptions()
        for f, names in self._ENUMS.items():
            v = getattr(self, f)
            if v not in names:
                raise ThrsError(-1, f"Options.{f}: {v!r} is not one of {names}")
            setattr(o, f, names.index(v))
        if self.keyRange is not None:
            lo, hi = (int(x) for x in self.keyRange)
            o.keyRange, o.rangeLo, o.rangeHi = 1, lo, hi
        return o


def take_device_error():
    """Raise (and clear) a device-side failure of any earlier sort on the
    current device that has finished, on any stream or thread
    (thrs_take_device_error; non-blocking, device-wide)."""
    _check(lib().thrs_take_device_error())


class _CPathInfo(ctypes.Structure):
    _fields_ = [("path", ctypes.c_int32), ("local", ctypes.c_int32), ("planes", ctypes.c_int32),
                ("devicePasses", ctypes.c_int32), ("minBytes", ctypes.c_uint64), ("localCap", ctypes.c_uint64)]


class _CHistTarget(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("count", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("prefixMask", ctypes.c_uint64), ("prefixValue", ctypes.c_uint64)]


class _CTempDef(ctypes.Structure):
    _fields_ = [("pSumBuffer", ctypes.c_uint64), ("keyOutBuffer", ctypes.c_uint64),
                ("valueOutBuffer", ctypes.c_uint64)]


class KeyType(enum.IntEnum):      # hpp:638-644
    U32 = 0
    U64 = 1
    F32 = 2
    F64 = 3


class ValueType(enum.IntEnum):    # hpp:645-650
    U32 = 0
    U64 = 1
    U128 = 2


class SortOrder(enum.IntEnum):    # hpp:679-683
    Ascending = 0
    Descending = 1


def bytesOf(t) -> int:            # hpp:651-678
    if isinstance(t, KeyType):
        return int(lib().thrs_key_bytes(int(t)))
    if isinstance(t, ValueType):
        return int(lib().thrs_value_bytes(int(t)))
    raise ThrsError(-1, "bytesOf: not a KeyType/ValueType")


def div_round_up64(val: int, divisor: int) -> int:
    return (val + divisor - 1) // divisor


def next_multiple64(val: int, divisor: int) -> int:
    return div_round_up64(val, divisor) * divisor


def _ptr(x) -> int | None:
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, Buffer):
        return x.data()
    raise TypeError(f"cannot take a device address of {type(x)}")


def _n(n) -> int:
    """numberOfInputs is uint32_t in the reference (hpp:845): refuse what a
    ctypes c_uint32 would silently truncate."""
    n = int(n)
    if not 0 <= n <= 0xFFFFFFFF:
        raise ThrsError(-1, f"numberOfInputs {n} does not fit uint32_t (tinyhipradixsort.hpp:845)")
    return n


def _stream(s) -> int | None:
    if s is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(s, int):
        return s
    if hasattr(s, "cuda_stream"):
        return s.cuda_stream
    raise TypeError(f"not a stream: {type(s)}")


class Buffer:
    """hpp:501-528 -- device allocation of max(bytes, 1) via thrs_malloc."""

    def __init__(self, bytes_: int):
        self._bytes = max(int(bytes_), 1)
        p = ctypes.c_void_p()
        _check(lib().thrs_malloc(ctypes.byref(p), self._bytes))
        self._ptr = p.value

    def bytes(self) -> int:
        return self._bytes

    def data(self) -> int:
        return self._ptr

    def __del__(self):
        if getattr(self, "_ptr", None) and _lib is not None:
            _lib.thrs_free(self._ptr)
            self._ptr = None


def _key_type_of(k) -> KeyType:
    import numpy as np
    try:
        import torch
        tmap = {torch.float32: KeyType.F32, torch.float64: KeyType.F64, torch.int32: KeyType.U32,
                torch.int64: KeyType.U64, torch.uint32: KeyType.U32, torch.uint64: KeyType.U64}
        if k in tmap:
            return tmap[k]
    except (ImportError, AttributeError):
        pass
    dt = np.dtype(k)
    if dt == np.float32:
        return KeyType.F32
    if dt == np.float64:
        return KeyType.F64
    if dt.itemsize == 4:
        return KeyType.U32
    if dt.itemsize == 8:
        return KeyType.U64
    raise ThrsError(-1, f"configureWithKey: unsupported key type {k}")   # hpp:710 static_assert


def _itemsize(v) -> int:
    import numpy as np
    if isinstance(v, int):
        return v
    try:
        import torch
        if isinstance(v, torch.dtype):
            return torch.empty((), dtype=v).element_size()
    except ImportError:
        pass
    return np.dtype(v).itemsize


class RadixSort:
    """hpp:694-948 over the C-ABI."""

    @dataclass
    class Config:                 # hpp:697-749
        keyIs16byteAligned: bool = True
        keyType: KeyType = KeyType.U32
        valueType: ValueType = ValueType.U32
        sortOrder: SortOrder = SortOrder.Ascending

        def configureWithKey(self, key):
            self.keyType = _key_type_of(key)

        def configureWithKeyPair(self, key, value):
            self.configureWithKey(key)
            vb = _itemsize(value)
            if vb not in (4, 8, 16):
                raise ThrsError(-1, "configureWithKeyPair: value must be 4, 8 or 16 bytes")  # hpp:734
            self.valueType = {4: ValueType.U32, 8: ValueType.U64, 16: ValueType.U128}[vb]

    @dataclass
    class TemporaryBufferDef:     # hpp:806-832
        pSumBuffer: int
        keyOutBuffer: int
        valueOutBuffer: int

        def getTemporaryBufferBytesForSortKeys(self) -> int:
            return self.pSumBuffer + self.keyOutBuffer

        def getTemporaryBufferBytesForSortPairs(self) -> int:
            return self.pSumBuffer + self.keyOutBuffer + self.valueOutBuffer

        def getPSumBuffer(self, p: int) -> int:
            return p

        def getOutputKeyBuffer(self, p: int) -> int:
            return p + self.pSumBuffer

        def getOutputValueBuffer(self, p: int) -> int:
            return p + self.pSumBuffer + self.keyOutBuffer

    def __init__(self, extraArgs=(), config: "RadixSort.Config | None" = None, options: Options | None = None):
        self.m_config = config if config is not None else RadixSort.Config()
        self.options = options if options is not None else Options()   # extension: thrs_options
        lib()   # fail loudly here, like the reference's compile-time THRS_ASSERT (hpp:591)

    def _c(self) -> _CConfig:
        c = self.m_config
        return _CConfig(int(bool(c.keyIs16byteAligned)), int(c.keyType), int(c.valueType), int(c.sortOrder))

    def getTemporaryBufferBytes(self, numberOfMaxInputs: int) -> "RadixSort.TemporaryBufferDef":
        d = _CTempDef()
        _check(lib().thrs_get_temporary_buffer_bytes(ctypes.byref(self._c()), _n(numberOfMaxInputs), ctypes.byref(d)))
        return RadixSort.TemporaryBufferDef(d.pSumBuffer, d.keyOutBuffer, d.valueOutBuffer)

    def sortKeys(self, inputKeyBuffer, numberOfInputs: int, temporaryBuffer, startBits: int, endBits: int,
                 stream=None, checked: bool = False):
        """hpp:845.  Asynchronous on `stream`; checked=True synchronises it and
        raises this sort's own device-side failure (THRS_CHECKED in the C++
        header)."""
        s = _stream(stream)
        _check(lib().thrs_sort_keys_ex(ctypes.byref(self._c()), ctypes.byref(self.options._c()),
                                       _ptr(inputKeyBuffer), _n(numberOfInputs), _ptr(temporaryBuffer),
                                       int(startBits), int(endBits), s))
        if checked:
            _check(lib().thrs_check_device_error(_ptr(temporaryBuffer), s))

    def sortPairs(self, inputKeyBuffer, inputValueBuffer, numberOfInputs: int, temporaryBuffer, startBits: int,
                  endBits: int, stream=None, checked: bool = False):
        """hpp:849.  As sortKeys."""
        s = _stream(stream)
        _check(lib().thrs_sort_pairs_ex(ctypes.byref(self._c()), ctypes.byref(self.options._c()),
                                        _ptr(inputKeyBuffer), _ptr(inputValueBuffer), _n(numberOfInputs),
                                        _ptr(temporaryBuffer), int(startBits), int(endBits), s))
        if checked:
            _check(lib().thrs_check_device_error(_ptr(temporaryBuffer), s))

    def partitionPass(self, inputKeyBuffer, inputValueBuffer, numberOfInputs: int, temporaryBuffer, outputKeyBuffer,
                      outputValueBuffer, bitLocation: int, counts, stream=None):
        """One stable out-of-place pass by the digit at bitLocation plus its 256
        bucket counts (device u32[256]); thrs_partition_pass, the bucket
        exchange's partition step (no reference counterpart)."""
        _check(lib().thrs_partition_pass(ctypes.byref(self._c()), _ptr(inputKeyBuffer), _ptr(inputValueBuffer),
                                         _n(numberOfInputs), _ptr(temporaryBuffer), _ptr(outputKeyBuffer),
                                         _ptr(outputValueBuffer), int(bitLocation), _ptr(counts), _stream(stream)))

    def digitHistogram(self, inputKeyBuffer, numberOfInputs: int, prefixMask: int, prefixValue: int,
                       bitLocation: int, counts, stream=None):
        """counts[d] (device u32[256], zeroed first) = keys whose transformed
        key t has t & prefixMask == prefixValue and digit d at bitLocation
        (thrs_digit_histogram, the multi-GPU split refinement)."""
        _check(lib().thrs_digit_histogram(ctypes.byref(self._c()), _ptr(inputKeyBuffer), _n(numberOfInputs),
                                          int(prefixMask) & (2**64 - 1), int(prefixValue) & (2**64 - 1),
                                          int(bitLocation), _ptr(counts), _stream(stream)))

    def digitHistograms(self, inputKeyBuffer, targets, bitLocation: int, counts, stream=None):
        """counts[i] (device u32[len(targets)][256], zeroed first) = the
        digitHistogram of keys [offset, offset + count) with prefix (mask,
        value), for every (offset, count, mask, value) in targets, in one
        launch (thrs_digit_histogram_batch: a refinement level of the
        multi-GPU split)."""
        arr = (_CHistTarget * max(1, len(targets)))()
        for i, (off, cnt, mask, value) in enumerate(targets):
            arr[i] = _CHistTarget(int(off), _n(cnt), 0, int(mask) & (2**64 - 1), int(value) & (2**64 - 1))
        _check(lib().thrs_digit_histogram_batch(ctypes.byref(self._c()), _ptr(inputKeyBuffer), arr, len(targets),
                                                int(bitLocation), _ptr(counts), _stream(stream)))

    def pathInfo(self, numberOfInputs: int, startBits: int, endBits: int, pairs: bool) -> dict:
        """The path such a sort takes and the HBM bytes it moves when no bucket
        overflows (thrs_get_path_info; a host decision, no device work)."""
        o = _CPathInfo()
        _check(lib().thrs_get_path_info(ctypes.byref(self._c()), ctypes.byref(self.options._c()), int(bool(pairs)),
                                    _n(numberOfInputs), int(startBits), int(endBits), ctypes.byref(o)))
        local = {0: None, 1: "thrs_local16", 2: "thrs_local", 3: "thrs_local_pairs", 4: "thrs_local_kv",
                 5: "thrs_local_count16"}[o.local]
        return {"path": "bucket" if o.path else "lsd", "local": local, "planes": bool(o.planes),
                "device_passes": o.devicePasses, "min_bytes": o.minBytes, "local_cap": o.localCap}

    def debugBucketMode(self, temporaryBuffer, numberOfInputs: int, pairs: bool, stream=None) -> tuple:
        """(mode, big chunks) the last bucket-path sort on temporaryBuffer found
        (thrs_debug_bucket_mode; synchronising, diagnostics only)."""
        m, b = ctypes.c_int(), ctypes.c_int()
        vb = int(lib().thrs_value_bytes(int(self.m_config.valueType))) if pairs else 0
        _check(lib().thrs_debug_bucket_mode(_ptr(temporaryBuffer), int(self.m_config.keyType), vb,
                                            _n(numberOfInputs), _stream(stream), ctypes.byref(m), ctypes.byref(b)))
        return m.value, b.value

    def checkDeviceError(self, temporaryBuffer, stream=None):
        """Synchronising: raises if a look-back spin bound was hit in the last
        sort on temporaryBuffer."""
        _check(lib().thrs_check_device_error(_ptr(temporaryBuffer), _stream(stream)))

    def accumulateDeviceError(self, temporaryBuffer, acc, stream=None):
        """Stream-ordered, no synchronisation: acc (device u32) |= the error
        word of the last sort on temporaryBuffer (thrs_accumulate_device_error)."""
        _check(lib().thrs_accumulate_device_error(_ptr(temporaryBuffer), _ptr(acc), _stream(stream)))


def profile_enable(on: bool = True):
    """Start (and reset) / stop HIP-event timing of the sort kernels (bench only)."""
    _check(lib().thrs_profile_enable(int(on)))


def profile_launches(kind: int) -> list:
    """Per-launch milliseconds of one kind since profile_enable, in issue order
    (thrs_profile_read_launches; synchronises the recorded events)."""
    cnt = ctypes.c_int()
    _check(lib().thrs_profile_read_launches(int(kind), None, 0, ctypes.byref(cnt)))
    buf = (ctypes.c_double * max(1, cnt.value))()
    _check(lib().thrs_profile_read_launches(int(kind), buf, cnt.value, ctypes.byref(cnt)))
    return [buf[i] for i in range(cnt.value)]


def profile_launch_kernels(kind: int) -> list:
    """(kernel name, algorithmic bytes) of every launch of one kind since
    profile_enable, in the order of profile_launches (bytes 0 = data-dependent:
    the per-bucket fallback's launches; see debug_big_keys)."""
    cnt = ctypes.c_int()
    _check(lib().thrs_profile_read_launch_kernels(int(kind), None, None, 0, ctypes.byref(cnt)))
    ids = (ctypes.c_int32 * max(1, cnt.value))()
    byt = (ctypes.c_uint64 * max(1, cnt.value))()
    _check(lib().thrs_profile_read_launch_kernels(int(kind), ids, byt, cnt.value, ctypes.byref(cnt)))
    return [(lib().thrs_profile_kernel_name(ids[i]).decode(), int(byt[i])) for i in range(cnt.value)]


def debug_big_keys(temporaryBuffer, keyType: int, valueBytes: int, n: int, stream=None) -> int:
    """Keys of the last bucket-path sort on this buffer that took the
    per-bucket fallback (thrs_debug_big_keys; synchronising)."""
    out = ctypes.c_uint64()
    _check(lib().thrs_debug_big_keys(_ptr(temporaryBuffer), int(keyType), int(valueBytes), int(n),
                                     _stream(stream), ctypes.byref(out)))
    return int(out.value)


def debug_vector_tiles(temporaryBuffer, keyType: int, n: int, stream=None) -> int:
    """Tiles of the last keys-only bucket-path sort on this buffer whose
    top-digit pass took the planes codec's vector loads
    (thrs_debug_vector_tiles; synchronising)."""
    out = ctypes.c_uint32()
    _check(lib().thrs_debug_vector_tiles(_ptr(temporaryBuffer), int(keyType), int(n), _stream(stream),
                                         ctypes.byref(out)))
    return int(out.value)


def profile_read() -> dict:
    """Synchronise recorded events; summed ms and launch counts since enable
    (hist = histogram + scan/plan, pass = device-wide digit passes, local =
    the 3-pass path's in-LDS bucket sort, fallback = the per-bucket
    fallback's launches)."""
    out = {}
    for kind, name in ((0, "hist"), (1, "pass"), (2, "local"), (3, "fallback")):
        ms, n = ctypes.c_double(), ctypes.c_int()
        _check(lib().thrs_profile_read_kind(kind, ctypes.byref(ms), ctypes.byref(n)))
        out[name + "_ms"] = ms.value
        out[name + "_launches"] = n.value
    return out
