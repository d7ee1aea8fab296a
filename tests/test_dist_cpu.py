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

    def partition(self, keys, vals, n, bit):
        k = keys.numpy().view(self.dt)[:n]
        d = ((O.key_bits_np(self.kt, k, self.desc) >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64)
        order = np.argsort(d, kind="stable")
        pk = torch.from_numpy(np.ascontiguousarray(k[order]).view(np.uint8).copy())
        pv = None
        if vals is not None:
            pv = torch.from_numpy(np.ascontiguousarray(vals.numpy().reshape(n, self.vb)[order]).reshape(-1).copy())
        return pk, pv, torch.from_numpy(np.bincount(d, minlength=256).astype(np.int32))

    def sort(self, keys, vals, n, s, e):
        if n == 0:
            return
        k = keys.numpy().view(self.dt)[:n]
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
            if kind == "random" and s < e and pass_reads_bits(kt, s, e):
                total = glob.shape[0]
                assert abs(n_out - total / world) <= total / world * 0.25 + 64, (ci, rank, n_out)
    finally:
        dist.destroy_process_group()


def pass_reads_bits(kt, s, e):
    return bool(D.pass_locations(O.KEY_BYTES[kt], s, e))


def free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_exchange_gloo(world):
    mp.spawn(_worker, args=(world, free_port(), CASES), nprocs=world, join=True)


def test_assign_ranges_balanced_uniform():
    c = np.full(256, 1000)
    for g in (1, 2, 4, 8):
        b = D.assign_ranges(c, g)
        assert b[0] == 0 and b[-1] == 256 and len(b) == g + 1
        assert all(b[i + 1] - b[i] == 256 // g for i in range(g))


def test_assign_ranges_skew_and_empty():
    c = np.zeros(256, np.int64)
    c[0] = 10
    c[42] = 1_000_000
    b = D.assign_ranges(c, 4)
    assert b == sorted(b) and b[0] == 0 and b[-1] == 256
    assert D.assign_ranges(np.zeros(256), 3) == [0, 0, 0, 256]


def test_exchange_plan_conserves():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 500, size=(4, 256))
    plans = [D.exchange_plan(a, r) for r in range(4)]
    send = np.array([p.send for p in plans])
    recv = np.array([p.recv for p in plans])
    assert (send == recv.T).all()
    assert send.sum() == a.sum() and all(p.bounds == plans[0].bounds for p in plans)


def test_pass_locations():
    assert D.pass_locations(4, 0, 32) == [0, 8, 16, 24]
    assert D.pass_locations(4, 8, 48) == [8, 16, 24]
    assert D.pass_locations(8, 60, 68) == [60]
    with pytest.raises(ValueError):
        D.pass_locations(4, 0, 12)
