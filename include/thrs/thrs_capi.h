/* thrs_capi.h -- the C-ABI drop-in boundary of libthrs.so (MI355X / gfx950).
 *
 * Plain pointers, sizes and ints only; no C++ or torch types.  Every entry
 * point replaces one piece of the reference's host API
 * (/root/reference/tinyhipradixsort.hpp), cited per function.  The header-only
 * C++ API in <thrs/tinyhipradixsort.hpp> is a thin wrapper over these, and the
 * Python mirror (tinyhipradixsort_amd) binds them with ctypes.
 *
 * Conventions
 *   - Return value: THRS_SUCCESS (0) or a negative thrs_status; never aborts.
 *   - Streams are HIP streams (hipStream_t, ABI-identical to the reference's
 *     oroStream on the HIP backend); 0 means the null stream.
 *   - Sorting is asynchronous on the stream; the caller synchronises.
 *   - All per-call scratch lives in the caller's temporary buffer, so two
 *     sorts on distinct temporary buffers may run concurrently.
 */
#ifndef THRS_CAPI_H
#define THRS_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef THRS_HIP_STREAM_DECLARED
#define THRS_HIP_STREAM_DECLARED
typedef struct ihipStream_t* hipStream_t; /* identical to HIP's own typedef */
#endif

#define THRS_ABI_VERSION 6

typedef enum thrs_status {
  THRS_SUCCESS = 0,
  THRS_ERROR_INVALID_VALUE = -1,   /* bad enum, null pointer, negative bits   */
  THRS_ERROR_BIT_RANGE = -2,       /* (endBits-startBits)%8 != 0 (hpp:856)    */
  THRS_ERROR_HIP = -3,             /* a HIP runtime call failed               */
  THRS_ERROR_OUT_OF_MEMORY = -4,   /* thrs_malloc failed                      */
  THRS_ERROR_LOOKBACK_TIMEOUT = -5, /* device look-back spin bound hit        */
  THRS_ERROR_DEVICE_CHECK = -6     /* a device-side range check failed: a
                                      digit run or bucket id past its table
                                      was clamped (output is wrong)         */
} thrs_status;

/* == thrs::KeyType / ValueType / SortOrder (tinyhipradixsort.hpp:638-683) */
enum { THRS_KEY_U32 = 0, THRS_KEY_U64 = 1, THRS_KEY_F32 = 2, THRS_KEY_F64 = 3 };
enum { THRS_VALUE_U32 = 0, THRS_VALUE_U64 = 1, THRS_VALUE_U128 = 2 };
enum { THRS_ORDER_ASCENDING = 0, THRS_ORDER_DESCENDING = 1 };

/* == RadixSort::Config (tinyhipradixsort.hpp:697-749) */
typedef struct thrs_config {
  int32_t keyIs16byteAligned; /* hint only: alignment is re-checked per call */
  int32_t keyType;            /* THRS_KEY_*   */
  int32_t valueType;          /* THRS_VALUE_* */
  int32_t sortOrder;          /* THRS_ORDER_* */
} thrs_config;

/* Explicit per-call path and tuning choices (no reference counterpart: the
 * reference has one path).  All-zero = THRS_*_AUTO everywhere = what
 * thrs_sort_keys / thrs_sort_pairs do.  Every choice produces the same,
 * bit-identical result; they exist for tests, A/B measurements and callers
 * that know their key distribution (e.g. the multi-GPU finish, whose buckets
 * never fit the local sort).  Nothing is read from the environment. */
enum { THRS_PATH_AUTO = 0, THRS_PATH_LSD = 1, THRS_PATH_BUCKET = 2 };
enum { THRS_LOCAL_AUTO = 0, THRS_LOCAL_BIG = 1, THRS_LOCAL_SMALL = 2, THRS_LOCAL_BIG32 = 3, THRS_LOCAL_COUNT16 = 4,
       THRS_LOCAL_RANK16 = 5, THRS_LOCAL_WIDE16 = 6, THRS_LOCAL_TINY16 = 7 };
enum { THRS_SEG_AUTO = 0, THRS_SEG_TOP_ONLY = 1, THRS_SEG_NONE = 2 };
enum { THRS_CLAIMS_AUTO = 0, THRS_CLAIMS_XCD_BLOCKS = 1, THRS_CLAIMS_TICKET = 2 };
enum { THRS_RANK_AUTO = 0, THRS_RANK_ATOMIC = 1, THRS_RANK_BALLOT = 2 };
enum { THRS_PLANES_AUTO = 0, THRS_PLANES_ON = 1, THRS_PLANES_OFF = 2 };
enum { THRS_SQUEEZE_AUTO = 0, THRS_SQUEEZE_OFF = 1 };
typedef struct thrs_options {
  int32_t path;          /* THRS_PATH_*: LSD = one device pass per digit; BUCKET = the
                            3-HBM-pass path wherever the key/value types and window
                            allow it, for any n (AUTO: n in [2^28, 2^30 + 2^26])   */
  int32_t localGeometry; /* THRS_LOCAL_*: the bucket path's in-LDS sort: 18432- (BIG) or
                            9216-key (SMALL) chunks; 4-byte keys-only over the whole
                            key sort 16-bit items, BIG32 = 32-bit items; u32 keys-only:
                            COUNT16 = counting sort of the 16-bit items, RANK16 = two
                            LSD rounds on them; WIDE16 = 34816-key chunks (AUTO above
                            2^30 + 2^26, to 2^31 + 2^25); TINY16 = 4096-key chunks
                            for 4-byte keys alone or with 4-byte values (AUTO for
                            u32 up to 3 x 2^26).  Sorts with 8/16-byte values
                            or 8-byte keys use 17408-key chunks whatever is asked.    */
  int32_t segmented;     /* THRS_SEG_*: XCD-segmented top-digit passes (AUTO: both)   */
  int32_t tileClaims;    /* THRS_CLAIMS_*: XCD-block tile claims in the digit passes
                            (AUTO: 4-byte keys without values, n >= 2^29)            */
  int32_t rank;          /* THRS_RANK_*: in-tile rank by lane-ordered LDS atomics
                            (AUTO: where the per-device probe confirms the order) or
                            by the 8-ballot match                                    */
  int32_t planes;        /* THRS_PLANES_*: u32 / f32 keys on the bucket path, without
                            values or with 4-byte values: the top-digit passes carry
                            the keys as a u16 + a u8 plane (12 instead of 16 bytes
                            per key over the two passes, 6 instead of 8 in the local
                            sort; values as they are).  AUTO = ON where it applies;
                            OFF = full keys                                         */
  int32_t keyRange;      /* 1: the caller promises rangeLo <= img(k) <= rangeHi for every
                            key, img(k) = getKeyBits(k) ^ (descending ? ~0 : 0) (fpKey.hpp
                            and kernel.cu:18-24), and a full-window sort orders by
                            ((img - rangeLo) << sh), sh = the leading zero bits of
                            rangeHi - rangeLo: monotone on the range, so the output is
                            the same bytes, while keys confined to a narrow range fill
                            the bucket path's 16-bit buckets evenly (the multi-GPU
                            finish, tinyhipradixsort_amd/dist.py).  rangeLo == rangeHi:
                            every key is equal, the sort returns at once.  Ignored
                            where it does not apply (windows; 4-byte keys-only sorts
                            on the 32-bit local sort), but always validated:
                            rangeLo > rangeHi, or rangeHi above the key width's
                            largest image, is THRS_ERROR_INVALID_VALUE on every
                            sort.  A false promise gives unspecified output.
                            0 = no range.                                          */
  int32_t squeeze;       /* THRS_SQUEEZE_*: float keys on the bucket path may drop a
                            bucket bit that every key of an image half shares (the
                            reference's float generator clears one, unittest.cpp:103,
                            108); AUTO = when the buckets would overflow, OFF = never.
                            Same bytes either way.                                   */
  uint64_t rangeLo;
  uint64_t rangeHi;
} thrs_options;

/* == RadixSort::TemporaryBufferDef (tinyhipradixsort.hpp:806-832).
 * Layout of the caller's temporary buffer: [pSumBuffer][keyOut][valueOut].
 * pSumBuffer is this implementation's scratch (histograms, digit bases, tile
 * counters, look-back status words); keyOut/valueOut are the ping-pong
 * partners of the caller's key/value buffers. */
typedef struct thrs_temp_def {
  uint64_t pSumBuffer;
  uint64_t keyOutBuffer;
  uint64_t valueOutBuffer;
} thrs_temp_def;

/* ABI version of the loaded library (== THRS_ABI_VERSION). */
int thrs_abi_version(void);

/* Human-readable name of a thrs_status. */
const char* thrs_status_string(int status);

/* == bytesOf(KeyType) / bytesOf(ValueType) (tinyhipradixsort.hpp:651-678);
 * 0 for an invalid enum. */
uint64_t thrs_key_bytes(int keyType);
uint64_t thrs_value_bytes(int valueType);

/* == RadixSort::getTemporaryBufferBytes (tinyhipradixsort.hpp:833-843). */
int thrs_get_temporary_buffer_bytes(const thrs_config* config, uint32_t numberOfMaxInputs, thrs_temp_def* out);

/* == RadixSort::sortKeys (tinyhipradixsort.hpp:845-848).  Sorts the 8-bit
 * digits of getKeyBits(key) (XOR all-ones when descending) covering
 * [startBits, endBits), least significant first; result in inputKeyBuffer.
 * startBits >= endBits is a no-op; numberOfInputs == 0 is a no-op. */
int thrs_sort_keys(const thrs_config* config, void* inputKeyBuffer, uint32_t numberOfInputs, void* temporaryBuffer,
                   int startBits, int endBits, hipStream_t stream);

/* == RadixSort::sortPairs (tinyhipradixsort.hpp:849-852).  Stable: equal keys
 * keep their input order, so values follow their keys bit-exactly. */
int thrs_sort_pairs(const thrs_config* config, void* inputKeyBuffer, void* inputValueBuffer, uint32_t numberOfInputs,
                    void* temporaryBuffer, int startBits, int endBits, hipStream_t stream);

/* thrs_sort_keys / thrs_sort_pairs with explicit options (NULL = defaults). */
int thrs_sort_keys_ex(const thrs_config* config, const thrs_options* options, void* inputKeyBuffer,
                      uint32_t numberOfInputs, void* temporaryBuffer, int startBits, int endBits, hipStream_t stream);
int thrs_sort_pairs_ex(const thrs_config* config, const thrs_options* options, void* inputKeyBuffer,
                       void* inputValueBuffer, uint32_t numberOfInputs, void* temporaryBuffer, int startBits,
                       int endBits, hipStream_t stream);

/* Multi-GPU building block (no reference counterpart -- the reference is
 * single-GPU): ONE stable LSD pass by the 8-bit digit at
 * bitLocation (the reference's per-pass digit, tinyhipradixsort.hpp:862-867,
 * kernel.cu:56-77 transform and descending flip), OUT OF PLACE keysIn ->
 * keysOut (valuesIn -> valuesOut when valuesIn != NULL), plus the digit's 256
 * bucket counts, in output order, written to the device array counts[256].
 * After it, bucket d occupies keysOut[sum(counts[0..d)) .. +counts[d]), in
 * input order -- the send segments of the bucket exchange.  temporaryBuffer
 * needs the pSumBuffer bytes of thrs_get_temporary_buffer_bytes(n). */
int thrs_partition_pass(const thrs_config* config, const void* keysIn, const void* valuesIn, uint32_t numberOfInputs,
                        void* temporaryBuffer, void* keysOut, void* valuesOut, int bitLocation, uint32_t* counts,
                        hipStream_t stream);

/* Multi-GPU building block (no reference counterpart): the exact-split
 * refinement of the bucket exchange.  counts[256] (device u32, zeroed first)
 * receives, by d, the number of keys in keys[0, n) whose transformed key t =
 * getKeyBits(key) ^ ORDER_MASK (kernel.cu:18-24, 46-69) satisfies
 * (t & prefixMask) == prefixValue and ((t >> bitLocation) & 0xFF) == d.
 * Masks are 64-bit; for 4-byte keys only their low 32 bits are used.  keys
 * needs no particular alignment (any sub-range of a key buffer). */
int thrs_digit_histogram(const thrs_config* config, const void* keys, uint32_t numberOfInputs, uint64_t prefixMask,
                         uint64_t prefixValue, int bitLocation, uint32_t* counts, hipStream_t stream);
/* The same for nTargets key ranges of one buffer at once (one memset and one
 * launch per 16 ranges: every boundary still being refined at one level of
 * the multi-GPU split): counts[i][256] for keys[offset_i, offset_i + count_i)
 * with prefix (prefixMask_i, prefixValue_i).  targets is a host array. */
typedef struct thrs_hist_target {
  uint64_t offset;       /* first key of the range (keys, not bytes) */
  uint32_t count;        /* keys in the range                        */
  uint32_t reserved;     /* zero                                     */
  uint64_t prefixMask;
  uint64_t prefixValue;
} thrs_hist_target;
int thrs_digit_histogram_batch(const thrs_config* config, const void* keys, const thrs_hist_target* targets,
                               int nTargets, int bitLocation, uint32_t* counts, hipStream_t stream);

/* Device-side failures (no reference counterpart; the reference would hang
 * where these give up).  A look-back or tile-claim wait is bounded; when the
 * bound is hit the sort's output is wrong and the failure is recorded in the
 * sort's own `temporaryBuffer` (until the next sort that uses it), and ORed
 * into a per-device sticky word in host memory.  A sort never fails because
 * of an EARLIER sort: each caller checks its own sort, either way below.  A
 * sort with nothing to do (n > 0 but an empty or identity bit window, or a
 * keyRange holding one key) launches no kernel and clears the word, so its
 * check reports success.
 *   thrs_check_device_error         synchronises `stream`; returns
 *                                   THRS_ERROR_LOOKBACK_TIMEOUT (a wait gave up)
 *                                   or THRS_ERROR_DEVICE_CHECK (a range check
 *                                   clamped a run) if the last sort on
 *                                   `temporaryBuffer` failed;
 *   thrs_accumulate_device_error    stream-ordered, no synchronisation:
 *                                   *acc |= that sort's error word (device
 *                                   memory, u32), so a sequence of sorts on one
 *                                   temporary buffer (the multi-GPU exchange)
 *                                   is checked once at its end;
 *   thrs_take_device_error          reads and clears the DEVICE-WIDE sticky
 *                                   word (non-blocking: it sees failures of
 *                                   sorts that have finished, on any stream or
 *                                   thread -- including ones already reported
 *                                   through their temporary buffer). */
int thrs_check_device_error(void* temporaryBuffer, hipStream_t stream);
int thrs_accumulate_device_error(const void* temporaryBuffer, uint32_t* acc, hipStream_t stream);
int thrs_take_device_error(void);

/* Kernel timing for benchmarks (no reference counterpart; the reference's
 * per-kernel stopwatches are commented out at tinyhipradixsort.hpp:881-928).
 * While enabled, every sort records hipEvents on ITS stream around the
 * histogram+scan launches and around each per-digit pass launch.
 * thrs_profile_read synchronises those events and returns the summed
 * milliseconds and launch counts since the last enable.  Off by default; not
 * for use under stream capture. */
int thrs_profile_enable(int enable);
int thrs_profile_read(double* histMs, int* histLaunches, double* passMs, int* passLaunches);
/* Same, for one launch kind: 0 = histogram + scan/plan, 1 = device-wide digit
 * pass, 2 = local (in-LDS) bucket sort of the 3-pass path, 3 = the 3-pass
 * path's fallback-only passes (they exit at once unless a bucket overflowed). */
int thrs_profile_read_kind(int kind, double* ms, int* launches);
/* Same, launch by launch in issue order: ms[i] for the first min(cap, *count)
 * launches of `kind`, *count = all of them.  A gated launch that had nothing
 * to do (the per-bucket fallback's launches when no bucket overflowed, the
 * key-codec variants of the top passes when the planes ran) takes a few
 * microseconds. */
int thrs_profile_read_launches(int kind, double* ms, int cap, int* count);
/* The kernel of each of those launches (THRS_PK_*) and its algorithmic bytes
 * (one read + one write of every key and value it permutes, a read of every
 * key it counts; 0 = data-dependent: the per-bucket fallback's launches, whose
 * bytes follow from thrs_debug_big_keys), in the same order as
 * thrs_profile_read_launches. */
enum { THRS_PK_ZERO = 0, THRS_PK_HIST = 1, THRS_PK_SCAN = 2, THRS_PK_HIST_JOINT = 3, THRS_PK_PLAN = 4,
       THRS_PK_PASS = 5, THRS_PK_PASS_XB = 6, THRS_PK_PASS_SEG = 7, THRS_PK_LOCAL16 = 8, THRS_PK_LOCAL = 9,
       THRS_PK_LOCAL_PAIRS = 10, THRS_PK_LOCAL_KV = 11, THRS_PK_LOCAL_COUNT16 = 12, THRS_PK_BIG_PLAN = 13,
       THRS_PK_BIG_HIST = 14, THRS_PK_PASS_BIG = 15, THRS_PK_BIG_COPY = 16, THRS_PK_COPY = 17,
       THRS_PK_SQUEEZE_SAMPLE = 18, THRS_PK_HIST_REDUCE = 19 };
int thrs_profile_read_launch_kernels(int kind, int32_t* kernel, uint64_t* bytes, int cap, int* count);
/* The kernel function's name for a THRS_PK_* id ("" for an unknown id). */
const char* thrs_profile_kernel_name(int kernel);

/* The path a sort with these arguments takes -- a host decision, no device
 * work -- and the bytes it reads and writes in HBM when no bucket overflows
 * (benchmark diagnostics; no reference counterpart). */
enum { THRS_LOCALK_NONE = 0, THRS_LOCALK_16 = 1, THRS_LOCALK_32 = 2, THRS_LOCALK_PAIRS = 3, THRS_LOCALK_KV = 4,
       THRS_LOCALK_COUNT16 = 5 };
typedef struct thrs_path_info {
  int32_t path;          /* 0 = one device pass per digit (LSD), 1 = bucket path          */
  int32_t local;         /* the bucket path's local sort: THRS_LOCALK_*                     */
  int32_t planes;        /* 1: 4-byte keys cross the top-digit passes as u16 + u8 planes   */
  int32_t devicePasses;  /* device-wide digit passes of one sort                           */
  uint64_t minBytes;     /* HBM bytes read + written by one sort, histogram included      */
  uint64_t localCap;     /* keys per local-sort chunk (a bigger bucket takes the fallback) */
} thrs_path_info;
int thrs_get_path_info(const thrs_config* config, const thrs_options* options, int pairs, uint32_t n, int startBits,
                   int endBits, thrs_path_info* out);

/* Rank path of the current device: 1 = one LDS atomic per key (gfx950
 * services conflicting lanes of a fully active wave in lane order; checked by
 * a one-time probe kernel per device), 0 = ballot match (always stable).
 * No reference counterpart. */
int thrs_rank_mode(void);

/* Diagnostic (tests, benchmarks): synchronises `stream` and reports what the
 * LAST bucket-path sort on `temporaryBuffer` found: *mode = 0 every bucket fit
 * its local sort, 1 some big chunks took the per-bucket fallback, 2 one bucket
 * held every key; *bigChunks = the number of big chunks.  Meaningless after
 * an LSD-path sort.  keyType / valueBytes / n: as that sort's. */
int thrs_debug_bucket_mode(const void* temporaryBuffer, int keyType, int valueBytes, uint32_t n, hipStream_t stream,
                           int* mode, int* bigChunks);

/* Diagnostic: synchronises `stream`; *keys = the keys of the LAST bucket-path
 * sort on `temporaryBuffer` that sat in big chunks (the per-bucket fallback's
 * work), 0 when every bucket fit its local sort.  Arguments as
 * thrs_debug_bucket_mode. */
int thrs_debug_big_keys(const void* temporaryBuffer, int keyType, int valueBytes, uint32_t n, hipStream_t stream,
                        uint64_t* keys);

/* Diagnostic: synchronises `stream`; *tiles = the tiles of the LAST
 * keys-only bucket-path sort on `temporaryBuffer` whose top-digit pass read the
 * key planes with vector loads (whole tiles inside one second-digit region;
 * 0 when the planes did not run).  Tests use it to prove that branch ran. */
int thrs_debug_vector_tiles(const void* temporaryBuffer, int keyType, uint32_t n, hipStream_t stream,
                            uint32_t* tiles);

/* Diagnostic: resident workgroups per CU of the 3-pass path's local bucket
 * sort kernel (4-byte keys), from the runtime's occupancy calculator. */
int thrs_debug_local_occupancy(void);

/* Diagnostic: in -DTHRS_STAMPS builds only, the local bucket sort writes 8
 * s_memrealtime stamps per chunk to buf[chunk*8 .. +7] (NULL = off). */
int thrs_debug_set_local_stamps(void* buf);

/* == thrs::Buffer (tinyhipradixsort.hpp:501-528): hipMalloc(max(bytes,1)). */
int thrs_malloc(void** ptr, int64_t bytes);
int thrs_free(void* ptr);

/* Helpers the header-only API and ported tests use in place of the
 * reference's Orochi calls (oroMemcpyHtoDAsync / oroMemcpyDtoH /
 * oroStreamSynchronize / oroStreamCreate, unittest.cpp:55, 143-152). */
int thrs_memcpy_htod_async(void* dst, const void* src, uint64_t bytes, hipStream_t stream);
int thrs_memcpy_dtoh(void* dst, const void* src, uint64_t bytes);
int thrs_memcpy_dtod_async(void* dst, const void* src, uint64_t bytes, hipStream_t stream);
int thrs_stream_create(hipStream_t* stream);
int thrs_stream_destroy(hipStream_t stream);
int thrs_stream_synchronize(hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* THRS_CAPI_H */
