"""Bucket-exchange host logic (tinyhipradixsort_amd/dist.py) on CPU ranks over
gloo: planning, split sizes, exchange order and stability.  The two local GPU
steps (partition pass, local sort) are played by the oracle here -- the GPU
versions of those steps are covered by tests/test_gpu_parity.py and
tests/test_gpu_dist.py.  Expected result: ONE oracle LSD sort
(tinyhipradixsort.hpp:854-944 restated) of the concatenation of all ranks'
inputs, with the global index as payload so stability is checked exactly."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tinyhipradixsort_amd import dist as D  # noqa: E402

NP_KEY = {O.U32: np.uint32, O.U64: np.uint64, O.F32: np.uint32, O.F64: np.uint64}


class OracleOps:
    """Stand-in for HipLocalOps (test infrastructure only)."""

    def __init__(self, kt, vb, desc):
        self.kt, self.vb, self.desc = kt, vb, desc
        self.dt = NP_KEY[kt]
        self.ranges = 0

    def partition(self, keys, vals, n, bit):
        k = keys.numpy().view(self.dt)[:n]
        d = ((O.key_bits_np(self.kt, k, self.desc) >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64)
        order = np.argsort(d, kind="stable")
        pk = torch.from_numpy(np.ascontiguousarray(k[order]).view(np.uint8).copy())
        pv = None
        if vals is not None:
            pv = torch.from_numpy(np.ascontiguousarray(vals.numpy().reshape(n, self.vb)[order]).reshape(-1).copy())
        return pk, pv, torch.from_numpy(np.bincount(d, minlength=256).astype(np.int32))

    def histograms(self, keys, ranges, bit):
        allk = keys.numpy().view(self.dt)
        out = []
        for lo, n, mask, value in ranges:
            t = O.key_bits_np(self.kt, allk[lo:lo + n], self.desc)
            sel = (t & np.uint64(mask)) == np.uint64(value)
            d = ((t[sel] >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64)
            out.append(np.bincount(d, minlength=256).astype(np.int32))
        return torch.from_numpy(np.stack(out))

    def sort(self, keys, vals, n, s, e, finish=True, key_range=None):
        if n == 0:
            return
        k = keys.numpy().view(self.dt)[:n]
        if key_range is not None:   # the split's range promise (thrs_options.keyRange) must hold
            t = O.key_bits_np(self.kt, k, self.desc)
            lo, hi = key_range
            assert int(t.min()) >= lo and int(t.max()) <= hi, ("key range promise broken", lo, hi)
            self.ranges += 1
        v = vals.numpy().reshape(n, self.vb) if vals is not None else None
        k2, v2 = O.lsd_sort(self.kt, k, v, s, e, self.desc)
        keys.copy_(torch.from_numpy(k2.view(np.uint8).reshape(-1)))
        if vals is not None:
            vals.copy_(torch.from_numpy(v2.reshape(-1)))


# (key type, value bytes, sizes per rank, start, end, descending, generator)
CASES = [
    (O.U32, 4, [5000, 7001], 0, 32, False, "random"),
    (O.U32, 0, [3000, 0], 0, 32, False, "random"),            # an empty rank
    (O.U32, 4, [4000, 4000], 0, 32, False, "extreme"),        # unittest.cpp:191-225: one bucket holds all
    (O.F32, 4, [2500, 3100], 0, 32, False, "random"),
    (O.F32, 4, [2500, 3100], 0, 32, True, "random"),
    (O.U64, 8, [3000, 2000], 8, 40, False, "random"),         # window: top pass at bit 32
    (O.U32, 4, [3000, 3000], 8, 24, False, "fewbits"),        # many ties -> stability across ranks
    (O.F64, 16, [1500, 1700], 0, 64, True, "random"),
    (O.U32, 4, [2000, 2000], 32, 40, False, "random"),        # all passes are identities
    (O.U64, 8, [3000, 2500], 0, 64, False, "extreme"),        # one key value: split by (rank, position)
    (O.U32, 4, [4000, 100], 0, 32, False, "fewbits"),         # skewed sizes and few distinct keys
    (O.U32, 4, [3000, 3000], 16, 24, False, "extreme"),       # one digit: no refinement level
]


def gen(kind, kt, n, start):
    draws = O.splitmix64_stream(start, n)
    k = O.randomize_np(kt, draws)
    if kind == "extreme":
        k = np.zeros(n, NP_KEY[kt])
        if n > 7:
            k[7], k[n // 2] = 1, 42
    elif kind == "fewbits":
        k = (k & NP_KEY[kt](0x00030300)).astype(NP_KEY[kt])
    return k


def _worker(rank, world, port, cases):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        for ci, (kt, vb, sizes, s, e, desc, kind) in enumerate(cases):
            sizes = list(sizes) + [sizes[-1] + 17 * r for r in range(len(sizes), world)]
            glob = np.concatenate([gen(kind, kt, sizes[r], 1000 * ci + sum(sizes[:r])) for r in range(world)])
            gidx = np.arange(glob.shape[0], dtype=np.uint64)
            lo = sum(sizes[:rank])
            mine = glob[lo:lo + sizes[rank]]
            keys = torch.from_numpy(np.ascontiguousarray(mine).view(np.uint8).copy())
            vals = None
            if vb:
                v = np.zeros((sizes[rank], vb), np.uint8)
                v[:, :8 if vb >= 8 else 4] = gidx[lo:lo + sizes[rank]].astype(
                    np.uint64 if vb >= 8 else np.uint32).view(np.uint8).reshape(sizes[rank], -1)
                vals = torch.from_numpy(v.reshape(-1).copy())
            vt = {0: None, 4: 0, 8: 1, 16: 2}[vb]
            sorter = D.DistributedRadixSort(kt, vt, int(desc), ops=OracleOps(kt, vb, desc))
            ko, vo, n_out = sorter.sort(keys, sizes[rank], vals, s, e)
            if s == 0 and e >= 8 * O.KEY_BYTES[kt] and n_out:   # the finish got (and kept) a key range
                assert sorter.ops.ranges == 1 and sorter.last_range is not None, ci
            # expected: one stable sort of the concatenation
            ev = None
            if vb:
                ev = np.zeros((glob.shape[0], vb), np.uint8)
                ev[:, :8 if vb >= 8 else 4] = gidx.astype(np.uint64 if vb >= 8 else np.uint32).view(
                    np.uint8).reshape(glob.shape[0], -1)
            ek, ev = O.lsd_sort(kt, glob, ev, s, e, desc)
            counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(counts, torch.tensor([n_out], dtype=torch.int64))
            off = int(sum(int(c) for c in counts[:rank]))
            assert sum(int(c) for c in counts) == glob.shape[0], ci
            got_k = ko.numpy().view(NP_KEY[kt])[:n_out]
            assert np.array_equal(got_k, ek[off:off + n_out]), (ci, rank, "keys")
            if vb:
                assert np.array_equal(vo.numpy().reshape(n_out, vb), ev[off:off + n_out]), (ci, rank, "values")
            if pass_reads_bits(kt, s, e):   # exact balance: global positions [rN/G, (r+1)N/G)
                total = glob.shape[0]
                assert n_out == (rank + 1) * total // world - rank * total // world, (ci, rank, n_out)
    finally:
        dist.destroy_process_group()


def pass_reads_bits(kt, s, e):
    return bool(D.pass_locations(O.KEY_BYTES[kt], s, e))


def free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bucket_exchange_gloo(world):
    cases = CASES if world < 8 else [c for c in CASES if c[6] != "random"] + CASES[:2]
    mp.spawn(_worker, args=(world, free_port(), cases), nprocs=world, join=True)


def _subgroup_worker(rank, world, port):
    """Two concurrent sorts on subgroups whose group ranks differ from the
    global ranks ({0, 2} and {1, 3} of a world of 4): every segment must reach
    the right process (P2POp group_peer)."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        groups = [dist.new_group([0, 2]), dist.new_group([1, 3])]
        mine = groups[rank % 2]
        members = [0, 2] if rank % 2 == 0 else [1, 3]
        sizes = [3001, 2500]
        glob = np.concatenate([gen("random", O.U32, sizes[i], 91 * members[0] + 7 * i) for i in range(2)])
        gidx = np.arange(glob.shape[0], dtype=np.uint32)
        me = members.index(rank)
        lo = sum(sizes[:me])
        keys = torch.from_numpy(np.ascontiguousarray(glob[lo:lo + sizes[me]]).view(np.uint8).copy())
        vals = torch.from_numpy(gidx[lo:lo + sizes[me]].view(np.uint8).copy())
        sorter = D.DistributedRadixSort(O.U32, 0, 0, group=mine, ops=OracleOps(O.U32, 4, False))
        assert sorter.rank == me and sorter.world == 2
        ko, vo, n_out = sorter.sort(keys, sizes[me], vals, 0, 32)
        ek, ev = O.lsd_sort(O.U32, glob, gidx.view(np.uint8).reshape(-1, 4).copy(), 0, 32, False)
        total = glob.shape[0]
        off = me * total // 2
        assert n_out == (me + 1) * total // 2 - off
        assert np.array_equal(ko.numpy().view(np.uint32)[:n_out], ek[off:off + n_out])
        assert np.array_equal(vo.numpy().reshape(n_out, 4), ev[off:off + n_out])
    finally:
        dist.destroy_process_group()


def test_bucket_exchange_on_subgroups():
    mp.spawn(_subgroup_worker, args=(4, free_port()), nprocs=4, join=True)


def _simulate(ranks, kt, s, e, desc=False):
    """The host split logic on in-memory ranks (numpy histograms): returns
    each rank's received keys after the finish, to compare with one stable sort."""
    world = len(ranks)
    locs = D.pass_locations(O.KEY_BYTES[kt], s, e)
    parts, counts = [], []
    for k in ranks:
        t = O.key_bits_np(kt, k, desc)
        d = ((t >> np.uint64(locs[-1])) & np.uint64(0xFF)).astype(np.int64)
        o = np.argsort(d, kind="stable")
        parts.append(k[o])
        counts.append(np.bincount(d, minlength=256))
    counts = np.array(counts)
    targets = D.make_targets(counts, world, locs[-1])
    for loc in reversed(locs[:-1]):
        act = [tg for tg in targets if tg.refining]
        if not act:
            break
        hist = np.zeros((world, len(act), 256), np.int64)
        for r in range(world):
            off = np.concatenate([[0], np.cumsum(counts[r])])
            for i, tg in enumerate(act):
                kk = parts[r][off[tg.bucket]:off[tg.bucket + 1]]
                t = O.key_bits_np(kt, kk, desc)
                sel = (t & np.uint64(tg.mask)) == np.uint64(tg.value)
                hist[r, i] = np.bincount(((t[sel] >> np.uint64(loc)) & np.uint64(0xFF)).astype(np.int64),
                                         minlength=256)
        D.refine(targets, hist, loc)
    for r in range(world):          # sort split buckets locally
        off = np.concatenate([[0], np.cumsum(counts[r])])
        for b in {tg.bucket for tg in targets if tg.inside}:
            seg = parts[r][off[b]:off[b + 1]]
            parts[r][off[b]:off[b + 1]] = O.lsd_sort(kt, seg, None, s, e, desc)[0]
    cuts = D.cut_points(counts, targets)
    out = []
    for g in range(world):
        recv = np.concatenate([parts[r][cuts[r, g]:cuts[r, g + 1]] for r in range(world)])
        out.append(O.lsd_sort(kt, recv, None, s, e, desc)[0])
    return out


@pytest.mark.parametrize("world", [2, 5, 8])
@pytest.mark.parametrize("kind", ["random", "extreme", "fewbits", "onebucket"])
def test_exact_split_host_logic(world, kind):
    rng = np.random.default_rng(world * 10 + len(kind))
    sizes = [int(x) for x in rng.integers(0, 3000, world)]
    ranks = []
    for r, n in enumerate(sizes):
        k = O.randomize_np(O.U32, O.splitmix64_stream(777 * r, n))
        if kind == "extreme":
            k = np.zeros(n, np.uint32)
        elif kind == "fewbits":
            k = (k & np.uint32(0x01000103)).astype(np.uint32)
        elif kind == "onebucket":
            k = (k & np.uint32(0x00FFFFFF)).astype(np.uint32)   # one top digit, many keys
        ranks.append(k)
    out = _simulate(ranks, O.U32, 0, 32)
    glob = np.concatenate(ranks)
    exp = O.lsd_sort(O.U32, glob, None, 0, 32)[0]
    total = glob.shape[0]
    got = np.concatenate(out)
    assert np.array_equal(got, exp)
    for g in range(world):
        assert out[g].shape[0] == (g + 1) * total // world - g * total // world


def test_exact_split_stability_of_equal_keys():
    """All keys equal: the split follows (rank, position) -- checked through
    the cut points directly."""
    counts = np.zeros((3, 256), np.int64)
    counts[:, 7] = [5, 0, 7]
    targets = D.make_targets(counts, 3, 24)
    for loc in (16, 8, 0):
        act = [t for t in targets if t.refining]
        hist = np.zeros((3, len(act), 256), np.int64)
        hist[:, :, 0] = counts[:, 7][:, None]
        D.refine(targets, hist, loc)
    cuts = D.cut_points(counts, targets)
    # 12 keys, 4 per rank: rank0 takes r0[0:4]; rank1 takes r0[4], r2[0:3]; rank2 takes r2[3:7]
    assert cuts.tolist() == [[0, 4, 5, 5], [0, 0, 0, 0], [0, 0, 3, 7]]


def test_pass_locations():
    assert D.pass_locations(4, 0, 32) == [0, 8, 16, 24]
    assert D.pass_locations(4, 8, 48) == [8, 16, 24]
    assert D.pass_locations(8, 60, 68) == [60]
    with pytest.raises(ValueError):
        D.pass_locations(4, 0, 12)
