"""Multi-GPU bucket-exchange sort over torch.distributed (RCCL on ROCm).

The reference is single-GPU (no collectives anywhere); this is
the new row s8(e).  One process per GPU; rank r holds a contiguous slice of the
global input, and rank order is the global order for stability.  The result
is bit-exact with ONE stable single-GPU sort (tinyhipradixsort.hpp:854-944) of
the concatenation rank 0 || rank 1 || ... : rank g ends up holding global
sorted positions [floor(gN/G), floor((g+1)N/G)) -- exactly balanced, whatever
the key distribution (SURVEY.md s7 hard part 7, s8(e).3).

One sort:

  1. partition  thrs_partition_pass: ONE stable pass by the window's TOP digit
                (bit location of the reference's last pass), out of place; it
                also yields that digit's 256 bucket counts.
  2. counts     all_gather of every rank's 256 counts (host copy: all_to_all
                needs host split sizes).
  3. split      target g = floor(gN/G) falls in some top-digit bucket b_g at
                offset o_g.  If o_g > 0 the boundary is refined digit by digit
                (thrs_digit_histogram_batch: the keys of every b_g still being
                refined, matching the digits fixed so far, in one launch; one
                all_gather per level; pick the digit that holds o_g) until
                the full sort key v_g is known; the keys equal to v_g are then
                split in global (source rank, source position) order.  Every
                rank computes every rank's cut points from the gathered counts.
                Buckets holding a boundary are sorted locally (stable, same
                window) so each cut is one position.
  4. exchange   ONE grouped point-to-point exchange (batch_isend_irecv: one
                RCCL group) of keys and values together; rank g receives the
                segments in source-rank order, each in source order, straight
                into its output buffers (its own segment is a device copy).
  5. finish     a local stable sort of the received keys over the window.  The
                split fixes the image range [lo_g, hi_g] every key of rank g
                lies in (key_range below); the finish passes it to the library
                (thrs_options.keyRange), which orders by ((img - lo_g) << sh) --
                the same order -- so the bucket path's 16-bit buckets stay
                balanced although the rank holds ~1/G of the key space.
  6. check      every libthrs step ORs its temporary buffer's device-error
                word into one device word; it is read once at the end and a
                look-back / claim timeout in any step raises (thrs_capi.h
                "Device-side failures").

Why this is exact: rank g receives exactly the keys of global ranks
[T_g, T_g+1) (keys below v_g, plus the first equal ones by (rank, position)).
Equal keys arrive ordered by (source rank, source position): the partition is
stable, a split bucket's local sort is stable, segments arrive in source
order, and the finish is stable -- so the concatenation over ranks is the
global stable sort.

The local steps are pluggable (`ops`) only so the host logic -- splitting,
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


@dataclass
class Target:
    """Global sorted position `pos` = the first key of rank g's output."""
    pos: int
    bucket: int              # top-digit bucket holding position pos
    offset: int              # pos - keys in lower buckets (then: within the fixed prefix); 0 = cut at the start
    mask: int = 0            # transformed-key digits fixed so far
    value: int = 0
    lt: np.ndarray | None = None   # per rank: keys of the bucket below the fixed prefix
    eq: np.ndarray | None = None   # per rank: keys of the bucket equal to the fixed prefix
    inside: bool = False     # the cut lies inside the bucket (its keys must be ordered locally)

    @property
    def refining(self) -> bool:
        """still inside a group of keys sharing the fixed prefix"""
        return self.offset > 0


def make_targets(counts: np.ndarray, world: int, top_loc: int) -> list[Target]:
    """counts[r][b] = keys of rank r in top-digit bucket b.  Targets
    T_g = floor(g N / world), g = 1 .. world-1."""
    counts = np.asarray(counts, dtype=np.int64)
    tot = counts.sum(axis=0)
    excl = np.concatenate([[0], np.cumsum(tot)])
    n_all = int(excl[-1])
    out = []
    for g in range(1, world):
        pos = g * n_all // world
        b = int(np.searchsorted(excl, pos, side="right")) - 1
        b = min(max(b, 0), BINS - 1)
        t = Target(pos, b, pos - int(excl[b]), mask=0xFF << top_loc, value=b << top_loc)
        t.inside = t.offset > 0
        t.lt = np.zeros(counts.shape[0], np.int64)
        t.eq = counts[:, b].copy()
        out.append(t)
    return out


def refine(targets: list[Target], hist: np.ndarray, loc: int):
    """One refinement level.  hist[r][i][d] = keys of rank r in the bucket of
    the i-th still-refining target matching its prefix, by the digit at bit
    `loc`.  Fixes that digit for each of them."""
    active = [t for t in targets if t.refining]
    for i, t in enumerate(active):
        h = np.asarray(hist[:, i, :], dtype=np.int64)
        tot = h.sum(axis=0)
        cum = np.cumsum(tot)
        d = int(np.searchsorted(cum, t.offset, side="right"))   # first digit whose prefix sum exceeds offset
        t.offset -= int(cum[d] - tot[d])
        t.lt = t.lt + h[:, :d].sum(axis=1)
        t.eq = h[:, d].copy()
        t.mask |= 0xFF << loc
        t.value |= d << loc


def key_range(targets: list[Target], rank: int, key_bytes: int) -> tuple[int, int]:
    """[lo, hi] of the images (getKeyBits ^ descending mask) of the keys rank
    `rank` receives, from the split of a FULL-window sort.  Boundary g (the
    first key of rank g) has its digits fixed down to some level: every key of
    rank g is >= t.value (fixed digits, zeros below); the keys of rank g-1 are
    < t.value when the cut lies at the start of that prefix group (offset 0),
    and <= t.value when it lies inside it (refined to the full key, equal keys
    split by (rank, position))."""
    lo, hi = 0, (1 << (8 * key_bytes)) - 1
    if rank >= 1:
        lo = targets[rank - 1].value
    if rank + 1 <= len(targets):
        t = targets[rank]
        hi = t.value if t.offset > 0 else t.value - 1
    return lo, max(lo, hi)


def cut_points(counts: np.ndarray, targets: list[Target]) -> np.ndarray:
    """cuts[r][g], g = 0 .. world: rank r sends positions [cuts[r][g],
    cuts[r][g+1]) of its partitioned (and split-bucket sorted) keys to rank g.
    Keys equal to a refined target's full key are split by (rank, position)."""
    counts = np.asarray(counts, dtype=np.int64)
    world = counts.shape[0]
    off = np.concatenate([np.zeros((world, 1), np.int64), np.cumsum(counts, axis=1)], axis=1)  # off[r][b]
    cuts = np.zeros((world, world + 1), np.int64)
    cuts[:, world] = counts.sum(axis=1)
    for g, t in enumerate(targets, start=1):
        c = off[:, t.bucket].copy()
        if t.inside:
            # keys below the final prefix group, + rank r's keys of the group
            # below the cut (the group split in (rank, position) order)
            eq_before = np.concatenate([[0], np.cumsum(t.eq)[:-1]])
            c += t.lt + np.clip(t.offset - eq_before, 0, t.eq)
        cuts[:, g] = c
    return cuts


@dataclass
class ExchangePlan:
    cuts: np.ndarray         # [world][world+1]
    rank: int
    send: list[int] = field(init=False)
    recv: list[int] = field(init=False)
    n_out: int = field(init=False)

    def __post_init__(self):
        c = self.cuts
        self.send = [int(c[self.rank, g + 1] - c[self.rank, g]) for g in range(c.shape[0])]
        self.recv = [int(c[src, self.rank + 1] - c[src, self.rank]) for src in range(c.shape[0])]
        self.n_out = int(sum(self.recv))


# ----------------------------------------------------------------- local ops
class HipLocalOps:
    """The product's local steps: libthrs.so on the tensors' GPU."""

    def __init__(self, config: RadixSort.Config):
        self.config = config
        self.rs = RadixSort([], config)
        self._tmp = None
        self._acc = None   # device u32: OR of every step's device-error word

    def temp(self, n: int, like):
        import torch
        d = self.rs.getTemporaryBufferBytes(max(1, n))
        need = d.getTemporaryBufferBytesForSortPairs()
        if self._tmp is None or self._tmp.numel() < need or self._tmp.device != like.device:
            self._tmp = torch.empty(need, dtype=torch.uint8, device=like.device)
        if self._acc is None or self._acc.device != like.device:
            self._acc = torch.zeros(1, dtype=torch.int32, device=like.device)
        return self._tmp

    def _note(self, tmp):
        """stream-ordered: acc |= the error word of the step that just ran on tmp"""
        self.rs.accumulateDeviceError(tmp, self._acc)

    def reset_errors(self):
        """Stream-ordered: forget what an earlier, failed sort accumulated
        (a step that raised before check_errors ran), so a later healthy sort
        never reports it."""
        if self._acc is not None:
            self._acc.zero_()

    def check_errors(self):
        """Synchronising: raise if any step since the last check hit a device
        look-back / claim timeout (its output would be wrong)."""
        if self._acc is None:
            return
        bad = int(self._acc.item())
        self._acc.zero_()
        if bad:
            from . import ThrsError
            raise ThrsError(-5, "THRS_ERROR_LOOKBACK_TIMEOUT in a step of the distributed sort")

    def partition(self, keys, vals, n: int, bit: int):
        """-> (keys', vals', counts) with counts a device int32[256] tensor."""
        import torch
        pk = torch.empty_like(keys)
        pv = torch.empty_like(vals) if vals is not None else None
        counts = torch.empty(BINS, dtype=torch.int32, device=keys.device)
        tmp = self.temp(n, keys)
        self.rs.partitionPass(keys, vals, n, tmp, pk, pv, bit, counts)
        self._note(tmp)
        return pk, pv, counts

    def histograms(self, keys, ranges, bit: int):
        """device int32[len(ranges)][256]: for each (first key, count, mask,
        value) range, the digit histogram of its keys matching the prefix --
        one launch for the whole refinement level."""
        import torch
        h = torch.empty((len(ranges), BINS), dtype=torch.int32, device=keys.device)
        self.rs.digitHistograms(keys, ranges, bit, h)
        return h

    def sort(self, keys, vals, n: int, start_bits: int, end_bits: int, finish: bool = True, key_range=None):
        """key_range: (lo, hi) images every key lies in (the finish of a
        full-window sort) -> thrs_options.keyRange."""
        if n == 0:
            return
        tmp = self.temp(n, keys)
        rs = self.rs if key_range is None else RadixSort([], self.config, Options(keyRange=key_range))
        if vals is None:
            rs.sortKeys(keys, n, tmp, start_bits, end_bits)
        else:
            rs.sortPairs(keys, vals, n, tmp, start_bits, end_bits)
        self._note(tmp)


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
        self.backend = dist.get_backend(group)
        self.last_plan: ExchangePlan | None = None
        self.last_targets: list[Target] = []
        self.last_range: tuple[int, int] | None = None

    # keys/values travel as flat byte tensors
    @staticmethod
    def _bytes(t):
        return t.contiguous().view(-1).view(__import__("torch").uint8)

    def _exchange(self, rk, rv, pk, pv, plan: "ExchangePlan"):
        """Keys and values of every segment in ONE grouped point-to-point
        exchange (batch_isend_irecv: one RCCL group), received in source-rank
        order straight into rk / rv; this rank's own segment is a local copy.
        A gloo group (CPU tests) with device tensors stages through host
        memory."""
        import torch
        kb, vb = self.kb, self.vb
        send_off = np.concatenate([[0], np.cumsum(plan.send)])
        recv_off = np.concatenate([[0], np.cumsum(plan.recv)])
        staged = self.backend == "gloo" and pk.device.type != "cpu"
        srcs = [(pk, kb)] + ([(pv, vb)] if vb else [])
        dsts = [(rk, kb)] + ([(rv, vb)] if vb else [])
        if staged:
            srcs = [(t.cpu(), w) for t, w in srcs]
            hdst = [(torch.empty(t.numel(), dtype=torch.uint8), w) for t, w in dsts]
        else:
            hdst = dsts
        ops = []
        for peer in range(self.world):
            for (src, w), (dst, _) in zip(srcs, hdst):
                a, b = int(send_off[peer]) * w, int(send_off[peer + 1]) * w
                c, d = int(recv_off[peer]) * w, int(recv_off[peer + 1]) * w
                if peer == self.rank:
                    if d > c:
                        dst[c:d].copy_(src[a:b])
                    continue
                # peer is a rank of self.group: pass it as group_peer (P2POp's
                # `peer` is a GLOBAL rank, which differs inside a subgroup)
                if b > a:
                    ops.append(self.dist.P2POp(self.dist.isend, src[a:b], group=self.group, group_peer=peer))
                if d > c:
                    ops.append(self.dist.P2POp(self.dist.irecv, dst[c:d], group=self.group, group_peer=peer))
        if ops:
            for r in self.dist.batch_isend_irecv(ops):
                r.wait()
        if staged:
            for (dst, _), (h, _) in zip(dsts, hdst):
                dst.copy_(h)

    def _gather(self, t):
        """all_gather of a small int tensor -> host numpy [world, *t.shape]
        (a host synchronisation).  Device counts are u32 (thrs_capi.h): read
        as int32, they are widened without sign extension."""
        import torch
        c = t.to(torch.int64)
        if t.dtype == torch.int32:
            c &= 0xFFFFFFFF
        if self.backend == "gloo" and c.device.type != "cpu":
            c = c.cpu()
        parts = [torch.empty_like(c) for _ in range(self.world)]
        self.dist.all_gather(parts, c, group=self.group)
        return torch.stack(parts).cpu().numpy()

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

        if hasattr(self.ops, "reset_errors"):
            self.ops.reset_errors()
        k_in, v_in = kflat[:n * kb], (vflat[:n * vb] if vflat is not None else None)
        pk, pv, counts = self.ops.partition(k_in, v_in, n, locs[-1])
        clock.mark("partition")
        all_counts = self._gather(counts)                       # [world][256]
        clock.mark("counts")
        targets = make_targets(all_counts, self.world, locs[-1])
        self.last_targets = targets
        mine = all_counts[self.rank]
        off = np.concatenate([[0], np.cumsum(mine)])
        # refinement: one level per lower digit while a boundary lies inside a bucket
        for loc in reversed(locs[:-1]):
            active = [t for t in targets if t.refining]
            if not active:
                break
            ranges = [(int(off[t.bucket]), int(mine[t.bucket]), t.mask, t.value) for t in active]
            refine(targets, self._gather(self.ops.histograms(pk, ranges, loc)), loc)
        # buckets holding a refined boundary: stable local sort, so each cut is one position
        if len(locs) > 1:
            for b in sorted({t.bucket for t in targets if t.inside}):
                lo, cnt = int(off[b]), int(mine[b])
                if cnt > 1:
                    self.ops.sort(pk[lo * kb:(lo + cnt) * kb], pv[lo * vb:(lo + cnt) * vb] if vb else None, cnt,
                                  start_bits, end_bits, finish=False)
        plan = ExchangePlan(cut_points(all_counts, targets), self.rank)
        self.last_plan = plan
        clock.mark("split")
        if self.world == 1:
            # every key stays on this rank: the exchange would copy pk into a
            # buffer of its own size -- finish pk in place
            rk, rv = pk[:plan.n_out * kb], (pv[:plan.n_out * vb] if vb else None)
        else:
            rk = torch.empty(plan.n_out * kb, dtype=torch.uint8, device=dev)
            rv = torch.empty(plan.n_out * vb, dtype=torch.uint8, device=dev) if vb else None
            self._exchange(rk, rv, pk, pv, plan)
        del pk, pv
        clock.mark("exchange")
        full = start_bits == 0 and end_bits >= kb * 8
        rng = key_range(targets, self.rank, kb) if full else None
        self.last_range = rng
        self.ops.sort(rk, rv, plan.n_out, start_bits, end_bits, key_range=rng)
        clock.mark("finish")
        if hasattr(self.ops, "check_errors"):
            self.ops.check_errors()
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
