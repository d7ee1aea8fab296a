"""Multi-GPU bucket-exchange sort over torch.distributed (RCCL on ROCm).

The reference is single-GPU (no collectives anywhere); this is
the new row s8(e).  One process per GPU; rank r holds a contiguous slice of the
global input, and rank order is the global order for stability.  The result
is bit-exact with ONE stable single-GPU sort (tinyhipradixsort.hpp:854-944) of
the concatenation rank 0 || rank 1 || ... : rank g ends up holding a
contiguous slice of that sorted sequence.

One sort = five steps:

  1. partition  thrs_partition_pass: ONE stable LSD pass by the digit the
                reference's LAST pass uses (bit location startBits + 8(P-1),
                the top digit of the effective window), out of place, which
                also yields that digit's 256 bucket counts.
  2. counts     all_gather of the 256 counts of every rank (1 KiB each) and
                one device->host copy: all_to_all needs split sizes on the host.
  3. plan       contiguous digit ranges [b_g, b_g+1) per destination, chosen
                on the global counts so every rank receives ~total/G keys.
  4. exchange   all_to_all_single of keys (then values); rank g receives the
                segments in source-rank order and each segment in source order.
  5. finish     a full local sort of the received keys over the same window.

Why this is exact: for two keys with equal sort bits the top digit is equal,
so both go to the same destination; they arrive ordered by (source rank,
source position) -- their global order -- and the local sort is stable.  For
unequal keys the top digit decides the destination first, and the local
sort orders within one.  Balance is to a granularity of one top-digit bucket;
a single-bucket-heavy input (unittest.cpp:191-225's extremeCase) lands on one
rank, which is correct but unbalanced ("multi-GPU").

The local steps are pluggable (`ops`) only so the host logic -- planning,
split sizes, exchange order -- can be tested on CPU ranks over gloo with the
oracle standing in; the default, and the only product path, is HipLocalOps
over libthrs.so, which raises if the library is missing.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from . import KeyType, Options, RadixSort, SortOrder, ValueType, bytesOf

BINS = 256


# ----------------------------------------------------------------- host logic
def pass_locations(key_bytes: int, start_bits: int, end_bits: int) -> list[int]:
    """Bit locations of the passes that read key bits (thrs_capi.hip sort_impl:
    the reference's loop at tinyhipradixsort.hpp:862, minus identity passes
    at or past the key width)."""
    if (end_bits - start_bits) % 8:
        raise ValueError("(endBits - startBits) % 8 != 0 (tinyhipradixsort.hpp:856)")
    return [b for b in range(start_bits, end_bits, 8) if b < key_bytes * 8]


def assign_ranges(global_counts, world: int) -> list[int]:
    """Digit bounds b_0=0 <= b_1 <= ... <= b_G=256: destination g receives
    buckets [b_g, b_g+1).  b_g is the bucket boundary whose exclusive prefix
    count is closest to g*total/G (ties to the lower boundary), never below
    b_g-1."""
    c = np.asarray(global_counts, dtype=np.int64).reshape(BINS)
    excl = np.concatenate([[0], np.cumsum(c)])           # excl[b] = keys in buckets < b
    total = int(excl[-1])
    bounds = [0]
    for g in range(1, world):
        target = total * g / world
        lo = bounds[-1]
        b = lo + int(np.argmin(np.abs(excl[lo:] - target)))
        bounds.append(b)
    bounds.append(BINS)
    return bounds


@dataclass
class ExchangePlan:
    bounds: list[int]
    send: list[int]          # keys this rank sends to each destination
    recv: list[int]          # keys this rank receives from each source
    n_out: int = field(init=False)

    def __post_init__(self):
        self.n_out = int(sum(self.recv))


def exchange_plan(all_counts, rank: int) -> ExchangePlan:
    """all_counts[src][d] = keys of source rank src in bucket d."""
    a = np.asarray(all_counts, dtype=np.int64)
    world = a.shape[0]
    bounds = assign_ranges(a.sum(axis=0), world)
    send = [int(a[rank, bounds[g]:bounds[g + 1]].sum()) for g in range(world)]
    recv = [int(a[src, bounds[rank]:bounds[rank + 1]].sum()) for src in range(world)]
    return ExchangePlan(bounds, send, recv)


# ----------------------------------------------------------------- local ops
class HipLocalOps:
    """The product's local steps: libthrs.so on the tensors' GPU."""

    def __init__(self, config: RadixSort.Config):
        self.rs = RadixSort([], config)
        self.rs_lsd = RadixSort([], config, Options(path="lsd"))
        self._tmp = None
        self.lsd_finish = False  # set by DistributedRadixSort for world > 1 (see sort)

    def temp(self, n: int, like):
        import torch
        d = self.rs.getTemporaryBufferBytes(max(1, n))
        need = d.getTemporaryBufferBytesForSortPairs()
        if self._tmp is None or self._tmp.numel() < need or self._tmp.device != like.device:
            self._tmp = torch.empty(need, dtype=torch.uint8, device=like.device)
        return self._tmp

    def partition(self, keys, vals, n: int, bit: int):
        """-> (keys', vals', counts) with counts a device int32[256] tensor."""
        import torch
        pk = torch.empty_like(keys)
        pv = torch.empty_like(vals) if vals is not None else None
        counts = torch.empty(BINS, dtype=torch.int32, device=keys.device)
        self.rs.partitionPass(keys, vals, n, self.temp(n, keys), pk, pv, bit, counts)
        return pk, pv, counts

    def sort(self, keys, vals, n: int, start_bits: int, end_bits: int):
        if n == 0:
            return
        tmp = self.temp(n, keys)
        # A rank's keys share 256/world top digits, so the 3-HBM-pass path's
        # 16-bit buckets would hold ~world * 2^14 keys each: always over the
        # local sort's capacity, i.e. its fallback plus a wasted bucket
        # histogram.  For world > 1 the finish asks for the plain LSD path
        # (an explicit per-call option: DESIGN.md s4).
        rs = self.rs_lsd if self.lsd_finish else self.rs
        if vals is None:
            rs.sortKeys(keys, n, tmp, start_bits, end_bits)
        else:
            rs.sortPairs(keys, vals, n, tmp, start_bits, end_bits)


# ----------------------------------------------------------------- the sorter
class DistributedRadixSort:
    """Bucket-exchange sort of the concatenation of every rank's keys (and
    values).  Collective: every rank of `group` calls sort() together."""

    def __init__(self, key_type=KeyType.U32, value_type=None, sort_order=SortOrder.Ascending, group=None,
                 ops=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.key_type = KeyType(key_type)
        self.kb = bytesOf(self.key_type)
        self.value_type = None if value_type is None else ValueType(value_type)
        self.vb = 0 if value_type is None else bytesOf(self.value_type)
        cfg = RadixSort.Config(keyType=self.key_type, valueType=self.value_type or ValueType.U32,
                               sortOrder=SortOrder(sort_order))
        self.ops = ops if ops is not None else HipLocalOps(cfg)
        if hasattr(self.ops, "lsd_finish"):
            self.ops.lsd_finish = self.world > 1
        self.backend = dist.get_backend(group)
        self.last_plan: ExchangePlan | None = None

    # keys/values travel as flat byte tensors
    @staticmethod
    def _bytes(t):
        return t.contiguous().view(-1).view(__import__("torch").uint8)

    def _a2a(self, out, inp, out_splits, in_splits):
        """all_to_all_single on byte tensors; a gloo group (CPU tests) with
        device tensors stages through host memory."""
        import torch
        if self.backend == "gloo" and inp.device.type != "cpu":
            o = torch.empty(out.numel(), dtype=torch.uint8)
            self.dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
            return
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _all_counts(self, counts):
        import torch
        c = counts.to(torch.int64)
        if self.backend == "gloo" and c.device.type != "cpu":
            c = c.cpu()
        parts = [torch.empty_like(c) for _ in range(self.world)]
        self.dist.all_gather(parts, c, group=self.group)
        return torch.stack(parts).cpu().numpy()         # the one host sync of the sort

    def sort(self, keys, n: int | None = None, values=None, start_bits: int = 0, end_bits: int | None = None,
             timings: dict | None = None):
        """keys: this rank's slice (any dtype of the key's width, contiguous).
        Returns (keys_out, values_out, n_out) as new byte-viewable tensors of
        the same dtypes.  `timings`, if given, accumulates per-phase seconds
        (synchronising at phase boundaries: bench diagnostics only)."""
        import torch
        kb, vb = self.kb, self.vb
        if (values is None) != (vb == 0):
            raise ValueError("values must be given exactly when the sorter has a value type")
        if end_bits is None:
            end_bits = kb * 8
        kflat = self._bytes(keys)
        n = kflat.numel() // kb if n is None else int(n)
        vflat = self._bytes(values) if values is not None else None
        locs = pass_locations(kb, start_bits, end_bits)
        if not locs:        # every pass is an identity: nothing moves between ranks either
            return keys, values, n
        dev = kflat.device
        clock = _Clock(timings, dev)

        k_in, v_in = kflat[:n * kb], (vflat[:n * vb] if vflat is not None else None)
        pk, pv, counts = self.ops.partition(k_in, v_in, n, locs[-1])
        clock.mark("partition")
        plan = exchange_plan(self._all_counts(counts), self.rank)
        self.last_plan = plan
        clock.mark("counts")
        rk = torch.empty(plan.n_out * kb, dtype=torch.uint8, device=dev)
        self._a2a(rk, pk, [c * kb for c in plan.recv], [c * kb for c in plan.send])
        rv = None
        if vb:
            rv = torch.empty(plan.n_out * vb, dtype=torch.uint8, device=dev)
            self._a2a(rv, pv, [c * vb for c in plan.recv], [c * vb for c in plan.send])
        del pk, pv
        clock.mark("exchange")
        self.ops.sort(rk, rv, plan.n_out, start_bits, end_bits)
        clock.mark("finish")
        ko = rk.view(keys.dtype) if keys.dtype != torch.uint8 else rk
        vo = None
        if rv is not None:
            vo = rv.view(values.dtype) if values.dtype != torch.uint8 else rv
        return ko, vo, plan.n_out


class _Clock:
    """Per-phase wall time (synchronising) -- only when a timings dict is given."""

    def __init__(self, timings, device):
        self.t = timings
        self.dev = device
        if self.t is not None:
            self._sync()
            self.last = time.perf_counter()

    def _sync(self):
        if self.dev.type == "cuda":
            import torch
            torch.cuda.synchronize(self.dev)

    def mark(self, name):
        if self.t is None:
            return
        self._sync()
        now = time.perf_counter()
        self.t[name] = self.t.get(name, 0.0) + (now - self.last)
        self.last = now
