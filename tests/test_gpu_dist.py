"""GPU side of the bucket exchange (tinyhipradixsort_amd/dist.py):

* thrs_partition_pass (the partition step) against the oracle: output ==
  a stable argsort by the digit, counts == the digit's bincount;
* a 2-rank exchange with the real HIP local steps, both ranks on cuda:0 (the
  one-GPU box): gloo carries the collectives through host memory, the
  partition and the local sort run in libthrs.so; expected = ONE oracle LSD
  sort of the concatenation (global index payload -> stability checked).
RCCL itself is exercised by bench.py --gpus N (torch.distributed.run)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

NP_KEY = {O.U32: np.uint32, O.U64: np.uint64, O.F32: np.uint32, O.F64: np.uint64}


@pytest.mark.parametrize("kt,vb,desc,bit,n", [
    (O.U32, 0, False, 24, 100003), (O.U32, 4, False, 0, 70001), (O.F32, 4, True, 24, 65536 + 3),
    (O.U64, 8, False, 56, 50000), (O.F64, 16, False, 40, 33333), (O.U32, 4, False, 8, 1),
    # digits at bit 8 and above take the segmented pass over the bucket
    # histogram's position segments (thrs_partition_plan): many tiles per segment
    (O.U32, 0, False, 24, (1 << 24) + 7), (O.U64, 8, True, 56, (1 << 22) + 5), (O.U32, 4, False, 16, 3 << 20),
    (O.F32, 0, True, 24, 1 << 23), (O.F64, 8, False, 8, (1 << 21) + 1),
])
def test_partition_pass_vs_oracle(gpu, kt, vb, desc, bit, n):
    import tinyhipradixsort_amd as T
    torch = gpu
    k = O.randomize_np(kt, O.splitmix64_stream(7, n))
    v = np.arange(n * max(vb, 1), dtype=np.uint8).reshape(n, max(vb, 1))[:, :vb] if vb else None
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt),
                             valueType={0: T.ValueType.U32, 4: T.ValueType.U32, 8: T.ValueType.U64,
                                        16: T.ValueType.U128}[vb],
                             sortOrder=T.SortOrder.Descending if desc else T.SortOrder.Ascending)
    rs = T.RadixSort([], cfg)
    kd = torch.from_numpy(k.view(np.uint8).copy()).cuda()
    vd = torch.from_numpy(np.ascontiguousarray(v).reshape(-1).copy()).cuda() if vb else None
    ko, vo = torch.empty_like(kd), (torch.empty_like(vd) if vb else None)
    counts = torch.empty(256, dtype=torch.int32, device="cuda")
    tmp = torch.empty(rs.getTemporaryBufferBytes(n).pSumBuffer, dtype=torch.uint8, device="cuda")
    rs.partitionPass(kd, vd, n, tmp, ko, vo, bit, counts)
    torch.cuda.synchronize()
    rs.checkDeviceError(tmp)
    d = ((O.key_bits_np(kt, k, desc) >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64)
    order = np.argsort(d, kind="stable")
    assert np.array_equal(counts.cpu().numpy().astype(np.int64), np.bincount(d, minlength=256))
    assert np.array_equal(ko.cpu().numpy().view(NP_KEY[kt]), k[order])
    if vb:
        assert np.array_equal(vo.cpu().numpy().reshape(n, vb), v[order])
    # the input is untouched (out of place)
    assert np.array_equal(kd.cpu().numpy().view(NP_KEY[kt]), k)


def test_partition_pass_rejects(gpu):
    import tinyhipradixsort_amd as T
    torch = gpu
    rs = T.RadixSort([], T.RadixSort.Config())
    kd = torch.zeros(64, dtype=torch.uint8, device="cuda")
    counts = torch.empty(256, dtype=torch.int32, device="cuda")
    tmp = torch.empty(rs.getTemporaryBufferBytes(16).pSumBuffer, dtype=torch.uint8, device="cuda")
    with pytest.raises(T.ThrsError):
        rs.partitionPass(kd, None, 16, tmp, kd, None, 0, counts)       # in place
    with pytest.raises(T.ThrsError):
        rs.partitionPass(kd, None, 16, tmp, torch.empty_like(kd), None, 32, counts)   # past the key width


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from tinyhipradixsort_amd import dist as D
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        for ci, (kt, vb, sizes, s, e, desc) in enumerate(CASES):
            glob = _keys(ci, kt, sum(sizes))
            lo = sum(sizes[:rank])
            kd = torch.from_numpy(glob[lo:lo + sizes[rank]].view(np.uint8).copy()).cuda()
            vd = None
            if vb:
                idx = np.arange(lo, lo + sizes[rank], dtype=np.uint32 if vb == 4 else np.uint64)
                vd = torch.from_numpy(idx.view(np.uint8).copy()).cuda()
            sorter = D.DistributedRadixSort(kt, None if not vb else {4: 0, 8: 1}[vb], int(desc))
            ko, vo, n_out = sorter.sort(kd, sizes[rank], vd, s, e)
            torch.cuda.synchronize()
            np.save(os.path.join(out_dir, f"c{ci}_r{rank}_k.npy"), ko.cpu().numpy()[:n_out * O.KEY_BYTES[kt]])
            if vb:
                np.save(os.path.join(out_dir, f"c{ci}_r{rank}_v.npy"), vo.cpu().numpy()[:n_out * vb])
    finally:
        dist.destroy_process_group()


CASES = [(O.U32, 4, [300001, 250007], 0, 32, False), (O.F32, 0, [65536 * 3, 1000], 0, 32, True),
         (O.U64, 8, [120000, 90001], 16, 48, False),
         (O.U32, 4, [200000, 150001], 0, 32, False),      # extremeCase-shaped: all zero but two keys
         (O.U64, 8, [100000, 100000], 0, 64, False)]      # one top-digit bucket, many keys


def _keys(ci, kt, n):
    k = O.randomize_np(kt, O.splitmix64_stream(ci * 10 ** 6, n))
    if ci == 3:
        k = np.zeros(n, np.uint32)
        k[n // 3], k[2 * n // 3] = 1, 42
    if ci == 4:
        k = k & np.uint64(0x00FFFFFFFFFFFFFF)
    return k


def test_two_ranks_one_gpu(gpu, tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for ci, (kt, vb, sizes, s, e, desc) in enumerate(CASES):
        glob = _keys(ci, kt, sum(sizes))
        idx = np.arange(sum(sizes), dtype=np.uint32 if vb == 4 else np.uint64) if vb else None
        ek, ev = O.lsd_sort(kt, glob, idx, s, e, desc)
        gk = np.concatenate([np.load(tmp_path / f"c{ci}_r{r}_k.npy") for r in range(2)]).view(NP_KEY[kt])
        assert np.array_equal(gk, ek), ci
        if vb:
            gv = np.concatenate([np.load(tmp_path / f"c{ci}_r{r}_v.npy") for r in range(2)]).view(idx.dtype)
            assert np.array_equal(gv, ev), ci
        # exact balance: rank 0 holds global positions [0, N/2)
        n0 = np.load(tmp_path / f"c{ci}_r0_k.npy").size // O.KEY_BYTES[kt]
        assert n0 == sum(sizes) // 2, (ci, n0)


@pytest.mark.parametrize("kt,desc", [(O.U32, False), (O.F32, True), (O.U64, False), (O.F64, True)])
def test_digit_histogram_vs_numpy(gpu, kt, desc):
    """thrs_digit_histogram (the exact split's refinement) on an unaligned
    sub-range, with a prefix mask."""
    import tinyhipradixsort_amd as T
    torch = gpu
    n = 200003
    k = O.randomize_np(kt, O.splitmix64_stream(42, n))
    k[: n // 2] &= np.array(0xFF0000FF if O.KEY_BYTES[kt] == 4 else 0xFF000000000000FF, k.dtype)
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), sortOrder=T.SortOrder.Descending if desc else T.SortOrder.Ascending)
    rs = T.RadixSort([], cfg)
    kd = torch.from_numpy(k.view(np.uint8).copy()).cuda()
    kb = O.KEY_BYTES[kt]
    t = O.key_bits_np(kt, k, desc)
    h = torch.empty(256, dtype=torch.int32, device="cuda")
    for (mask, value, bit) in [(0, 0, 0), (0xFF << (kb * 8 - 8), int(t[7]) & (0xFF << (kb * 8 - 8)), 8),
                               ((0xFF << (kb * 8 - 8)) | 0xFF, int(t[3]) & ((0xFF << (kb * 8 - 8)) | 0xFF), 16)]:
        lo, hi = 3, n - 5                                # a sub-range at an unaligned offset
        rs.digitHistogram(kd[lo * kb:hi * kb], hi - lo, mask, value, bit, h)
        torch.cuda.synchronize()
        tt = t[lo:hi]
        sel = (tt & np.uint64(mask)) == np.uint64(value)
        exp = np.bincount(((tt[sel] >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64), minlength=256)
        assert np.array_equal(h.cpu().numpy().astype(np.int64), exp), (mask, value, bit)


@pytest.mark.parametrize("kt,desc", [(O.U32, False), (O.F64, True)])
def test_digit_histogram_batch_vs_numpy(gpu, kt, desc):
    """thrs_digit_histogram_batch: several ranges of one buffer (unaligned,
    overlapping, empty, and more than one launch's 16) with their own prefixes
    in one call -- a whole refinement level of the multi-GPU split."""
    import tinyhipradixsort_amd as T
    torch = gpu
    n = 300007
    k = O.randomize_np(kt, O.splitmix64_stream(43, n))
    kb = O.KEY_BYTES[kt]
    k[::3] &= np.array(0xFF00FFFF if kb == 4 else 0xFF00FFFFFFFFFFFF, k.dtype)
    cfg = T.RadixSort.Config(keyType=T.KeyType(kt), sortOrder=T.SortOrder.Descending if desc else T.SortOrder.Ascending)
    rs = T.RadixSort([], cfg)
    kd = torch.from_numpy(k.view(np.uint8).copy()).cuda()
    t = O.key_bits_np(kt, k, desc)
    top = 0xFF << (kb * 8 - 8)
    rng = np.random.default_rng(5)
    ranges = []
    for i in range(19):
        lo = int(rng.integers(0, n - 1))
        cnt = 0 if i == 4 else int(rng.integers(1, n - lo))
        mask = 0 if i % 3 == 0 else top
        ranges.append((lo, cnt, mask, int(t[lo]) & mask if cnt else 0))
    bit = kb * 8 - 16
    h = torch.empty((len(ranges), 256), dtype=torch.int32, device="cuda")
    rs.digitHistograms(kd, ranges, bit, h)
    torch.cuda.synchronize()
    got = h.cpu().numpy().astype(np.int64)
    for i, (lo, cnt, mask, value) in enumerate(ranges):
        tt = t[lo:lo + cnt]
        sel = (tt & np.uint64(mask)) == np.uint64(value)
        exp = np.bincount(((tt[sel] >> np.uint64(bit)) & np.uint64(0xFF)).astype(np.int64), minlength=256)
        assert np.array_equal(got[i], exp), i


def test_bench_force_dist_runs_rccl_at_world_1(gpu):
    """bench.py --force-dist: the bucket exchange through the nccl (= RCCL)
    backend at world size 1 -- the code path of the N-GPU bench lines."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist", "--n", str(1 << 22),
                        "--steps", "2", "--warmup", "1", "--cpu-baseline", "off"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    # stdout is the ONE JSON line the driver reads: RCCL's version banner
    # (printed to fd 1 at communicator set-up) must not reach it
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["value"] > 0 and "bucket-exchange" in line["config"]["parallelism"]


def _worker_big(rank, world, port, out_dir, kt, vb, n):
    import json
    import torch
    import torch.distributed as dist
    import tinyhipradixsort_amd as T
    from tinyhipradixsort_amd import dist as D
    from tinyhipradixsort_amd import testutil as TU
    torch.cuda.set_device(0)
    backend = "gloo" if world > 1 else "nccl"
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world, **kw)
    try:
        kb = O.KEY_BYTES[kt]
        kd = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
        TU.fill_keys(kt, kd, n, start=rank * n)
        vd = None
        if vb:
            vd = torch.empty(n * vb, dtype=torch.uint8, device="cuda")
            TU.iota(vb, vd, n, start=rank * n)
        sorter = D.DistributedRadixSort(kt, None if not vb else {4: 0, 8: 1}[vb])
        # a first (cold) sort loads every kernel: its gated no-op launches
        # would time above the 20-us threshold below
        k0 = kd.clone()
        v0 = None if vd is None else vd.clone()
        sorter.sort(k0, n, v0, 0, 8 * kb)
        torch.cuda.synchronize()
        del k0, v0
        T.profile_enable(True)
        ko, vo, n_out = sorter.sort(kd, n, vd, 0, 8 * kb)
        torch.cuda.synchronize()
        local = [x for x in T.profile_launches(2) if x >= 0.02]
        T.profile_enable(False)
        # what the finish's bucket path found (the finish is the last sort on
        # the sorter's temp buffer): big chunks would have taken the fallback.
        # (Not the fallback launches' times: two ranks share this one GPU, so
        # a gated no-op launch can time above any threshold.)
        mode, big = sorter.ops.rs.debugBucketMode(sorter.ops._tmp, n_out, bool(vb))
        bad = TU.count_unsorted(kt, ko, n_out, 0, 8 * kb)
        first = last = None
        if n_out:
            kk = ko.view(torch.int32 if kb == 4 else torch.int64)
            first, last = int(kk[0].item()) & ((1 << (8 * kb)) - 1), int(kk[n_out - 1].item()) & ((1 << (8 * kb)) - 1)
        res = {"n_out": n_out, "unsorted": bad, "first": first, "last": last, "local_launches": len(local),
               "mode": mode, "big_chunks": big, "range": sorter.last_range}
        if vb:   # the payload is the global index: every one arrives once (one rank: all of them)
            vkt = 1 if vb == 8 else 0
            res["fp_in"], res["fp_out"] = TU.fingerprint(vkt, vd, n), TU.fingerprint(vkt, vo, n_out)
        json.dump(res, open(os.path.join(out_dir, f"r{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kt,vb,n", [(2, O.U32, 0, 1 << 28), (1, O.U64, 8, 1 << 28),
                                           (2, O.U32, 0, 1 << 27), (1, O.U32, 0, 1 << 27),
                                           (2, O.U64, 8, 1 << 27), (2, O.U32, 0, 1 << 29)])
def test_bucket_finish_with_key_range(gpu, tmp_path, world, kt, vb, n):
    """The exchange's finish runs the bucket path (VERDICT r02
    next-step 3): each rank passes the key range the exact split fixed
    (dist.key_range -> thrs_options.keyRange), so its 16-bit buckets stay
    balanced and the local sort -- not the per-bucket fallback -- finishes
    the sort.  World 2 over gloo with real HIP steps (u32 keys, 2^27 .. 2^29
    per rank: 2^27 is C2's per-rank share at 8 GPUs, VERDICT r03 item 6;
    u64 + u64 at 2^27 too: its measured bound is 12M keys, row 130),
    world 1 over RCCL (u32 at 2^27; the C5 shape at 2^28: u64 keys + u64
    index payload)."""
    import json
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_worker_big, args=(world, port, str(tmp_path), kt, vb, n), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    assert sum(r["n_out"] for r in res) == world * n
    # the ranged finish's bucket-path bound is 2^27 for 4-byte keys without
    # values (the measured C2 shape); other types keep their own
    # (u64 + u64: 12M keys, docs/EXPERIMENTS.md row 130)
    bucket = (O.KEY_BYTES[kt] == 4 and vb == 0) or n >= 12_000_000
    for r in res:
        assert r["unsorted"] == 0, r
        if bucket:
            assert r["local_launches"] >= 1 and r["mode"] == 0 and r["big_chunks"] == 0, r
        else:
            assert r["local_launches"] == 0, r
    for a, b in zip(res, res[1:]):
        assert a["last"] <= b["first"], (a, b)
    if world > 1:
        # rank 0's range is a strict part of the key space
        assert res[0]["range"][1] < (1 << (8 * O.KEY_BYTES[kt])) - 1, res[0]
    if vb and world == 1:
        assert res[0]["fp_in"] == res[0]["fp_out"], res[0]
