#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X.

metric: "Gkeys/s and achieved HBM GB/s (% of peak), u32 keys N=2^30, 1/2/4/8 GPU"

* N=1 (default): workload C2 = sortKeys of 2^30 u32 keys, bits [0,32), the
  reference bench's input distribution (splitmix64 from state 0,
  unittest.cpp:544-548), generated on the GPU and resident in HBM before the
  timed region.  One step = one full sort of a FRESH input buffer (the sort is
  in place, so every step gets its own pre-generated buffer; see --pool).  For
  4-byte keys-only sorts the library takes its 3-HBM-pass path: bucket
  histogram + plan, two device-wide passes for the top two digits, and one
  in-LDS local sort of every 16-bit bucket; other workloads run
  histogram + one pass per digit.
* N>1: launched by torch.distributed.run, one rank per GPU; each rank holds
  2^30 u32 keys (weak scaling) and one step is the bucket-exchange sort of all
  N*2^30 keys (local digit histogram -> RCCL all-gather of counts -> local
  partition -> RCCL all-to-all -> local LSD finish).

Timing: W warm-up steps, then barrier + synchronize, K steps, synchronize +
barrier; the max over ranks.  rank 0 prints ONE JSON line.  `roofline` uses the
dominant kernel (thrs_pass) timed with HIP events on the sort's own stream
inside the timed region; `cpu_baseline` times the reference's CPU path
(std::sort, unittest.cpp:156) on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Gkeys/s and achieved HBM GB/s (% of peak), u32 keys N=2^30, 1/2/4/8 GPU"

WORKLOADS = {
    # name: (key type, value bytes, n per GPU, description)
    "c2": (0, 0, 1 << 30, "C2: sortKeys u32, N=2^30 uniform (splitmix64), bits [0,32), 1xMI355X"),
    "c3": (0, 4, 1 << 30, "C3: sortPairs u32 key + u32 index payload (stable), N=2^30"),
    "c4": (2, 0, 1 << 28, "C4: sortKeys f32 via fpKey transform, N=2^28 (bits & 0xFF7FFFFF)"),
    "c5": (1, 8, 1 << 30, "C5: sortPairs u64 key + u64 index payload, 2^30 per GPU"),
}
KEY_BYTES = {0: 4, 1: 8, 2: 4, 3: 8}
DTYPE = {0: "u32", 1: "u64", 2: "f32", 3: "f64"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", default=None, choices=sorted(WORKLOADS))
    p.add_argument("--n", type=int, default=None, help="keys per GPU (default: the workload's)")
    p.add_argument("--pool", type=int, default=12, help="max distinct pre-generated input buffers")
    p.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--force-dist", action="store_true",
                   help="run the bucket-exchange path even at world size 1 (RCCL smoke test)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(n_target_s: float) -> dict:
    """std::sort of u32 keys (unittest.cpp:156), 1 thread, on a bounded sample
    of the same splitmix64 stream; the oracle library is the timer's subject."""
    import numpy as np
    from oracle import oracle as O
    n = 1 << 24
    keys = O.randomize_np(O.U32, O.splitmix64_stream(0, n))
    t0 = time.perf_counter()
    O.std_sort_keys(O.U32, keys)
    t1 = time.perf_counter() - t0
    # scale the sample so one sort takes ~ n_target_s / 4
    scale = max(1, min(8, int((n_target_s / 4) / max(t1, 1e-3))))
    n = n * (1 << (scale.bit_length() - 1))
    keys = O.randomize_np(O.U32, O.splitmix64_stream(0, n))
    times = []
    t_start = time.perf_counter()
    while len(times) < 3 or (time.perf_counter() - t_start < n_target_s and len(times) < 8):
        t0 = time.perf_counter()
        O.std_sort_keys(O.U32, keys)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(n / med / 1e9, 5), "unit": "Gkeys/s", "cores": 1, "kind": "port",
            "sample": f"std::sort (unittest.cpp:156) of {n} splitmix64 u32 keys, 1 thread, median of {len(times)} "
                      f"runs on {os.cpu_count()} visible host CPUs ({cpu_model()})"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(workload: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(workload, {}).get("thrs_pass_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    dist = None
    use_dist = world > 1 or args.force_dist
    if use_dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import tinyhipradixsort_amd as T
    from tinyhipradixsort_amd import testutil as TU

    wl = args.workload or "c2"
    kt, vb, n_default, desc = WORKLOADS[wl]
    n = args.n or n_default
    kb = KEY_BYTES[kt]
    steps, warmup = args.steps, args.warmup
    stream = torch.cuda.current_stream()

    def barrier():
        if dist is not None:
            dist.barrier()

    if not use_dist:
        cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                   8: T.ValueType.U64, 16: T.ValueType.U128}[vb])
        rs = T.RadixSort([], cfg)
        tdef = rs.getTemporaryBufferBytes(n)
        tmp_bytes = tdef.getTemporaryBufferBytesForSortPairs() if vb else tdef.getTemporaryBufferBytesForSortKeys()
        tmp = torch.empty(tmp_bytes, dtype=torch.uint8, device="cuda")
        # distinct fresh inputs for every step (bounded by --pool and memory)
        free, _total = torch.cuda.mem_get_info()
        per = n * (kb + vb)
        pool = max(1, min(args.pool, steps + warmup, int((free - tmp_bytes - (4 << 30)) // max(per, 1))))
        keys, vals = [], []
        for i in range(pool):
            kbuf = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
            TU.fill_keys(kt, kbuf, n, start=i * n)      # run r consumes stream draws r*N+1 .. (r+1)*N
            keys.append(kbuf)
            if vb:
                vbuf = torch.empty(n * vb, dtype=torch.uint8, device="cuda")
                TU.iota(vb, vbuf, n)
                vals.append(vbuf)
        torch.cuda.synchronize()

        def step(i):
            j = i % pool
            if vb:
                rs.sortPairs(keys[j], vals[j], n, tmp, 0, kb * 8, stream)
            else:
                rs.sortKeys(keys[j], n, tmp, 0, kb * 8, stream)

        for i in range(warmup):
            step(i)
        # warm-up buffers get regenerated so every timed step sorts fresh data
        for i in range(min(warmup, pool)):
            TU.fill_keys(kt, keys[i], n, start=(pool + i) * n)
        torch.cuda.synchronize()
        T.profile_enable(True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(warmup + i)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        prof = T.profile_read()
        T.profile_enable(False)
        rs.checkDeviceError(tmp)
        # correctness of the last timed step (outside the timed region)
        last = (warmup + steps - 1) % pool
        bad = TU.count_unsorted(kt, keys[last], n, 0, kb * 8)
        if bad:
            raise SystemExit(f"bench: output of the last step is not sorted ({bad} inversions)")
        recycled = steps + warmup > pool
        elapsed = t1 - t0
        scaling = "weak"
        global_keys = n
        parallelism = "single"
        phase = None
    else:
        from tinyhipradixsort_amd import dist as D
        vt = None if not vb else {4: T.ValueType.U32, 8: T.ValueType.U64, 16: T.ValueType.U128}[vb]
        sorter = D.DistributedRadixSort(key_type=kt, value_type=vt)
        # inputs: rank r of step i holds draws (i*world + r)*n + 1 .. of the
        # splitmix64 stream; values = global index.  The exchange sort is out
        # of place (inputs are never modified), so a pool of 2 stays fresh.
        pool = max(1, min(2, args.pool))
        keys, vals = [], []
        for i in range(pool):
            kbuf = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
            TU.fill_keys(kt, kbuf, n, start=(i * world + rank) * n)
            keys.append(kbuf)
            if vb:
                vbuf = torch.empty(n * vb, dtype=torch.uint8, device="cuda")
                TU.iota(vb, vbuf, n, start=rank * n)
                vals.append(vbuf)
        torch.cuda.synchronize()
        out = None

        def step(i, timings=None):
            j = i % pool
            return sorter.sort(keys[j], n, vals[j] if vb else None, 0, kb * 8, timings=timings)

        for i in range(warmup):
            out = step(i)
        phase_s = {}
        out = step(0, phase_s)                     # untimed per-phase breakdown (synchronising)
        del out
        torch.cuda.synchronize()
        T.profile_enable(True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            out = step(warmup + i)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        prof = T.profile_read()
        T.profile_enable(False)
        ko, _vo, n_out = out
        bad = TU.count_unsorted(kt, ko, n_out, 0, kb * 8)
        if bad:
            raise SystemExit(f"bench: rank {rank} output is not sorted ({bad} inversions)")
        recycled = False
        elapsed = t1 - t0
        scaling = "weak"
        global_keys = n * world
        parallelism = f"bucket-exchange x{world} (RCCL all_gather + all_to_all)"
        phase = {k: round(v * 1e3, 3) for k, v in phase_s.items()}
        phase["n_out_rank0"] = n_out if rank == 0 else None

    # max over ranks
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_per_step = elapsed / steps * 1e3
    value = global_keys / (elapsed / steps) / 1e9

    # roofline of the dominant kernel: one per-digit pass reads and writes every
    # key (+ value) once -> algorithmic bytes per launch = 2 * n * (K + V)
    roof = None
    if prof and prof.get("pass_launches"):
        avg_pass_ms = prof["pass_ms"] / prof["pass_launches"]
        alg_bytes = 2 * n * (kb + vb)
        achieved = alg_bytes / (avg_pass_ms / 1e3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": load_pmc_traffic(wl),
                # 3-HBM-pass path: the two top-digit passes are thrs_pass_seg
                "kernel": "thrs_pass_seg" if prof.get("local_launches") else "thrs_pass",
                "avg_launch_ms": round(avg_pass_ms, 4),
                "alg_bytes_per_launch": alg_bytes,
                "hist_avg_ms": round(prof["hist_ms"] / max(1, prof["hist_launches"]), 4)}
        # whole-sort algorithmic rate (B_alg = P*2*N*(K+V) for P 8-bit digits,
        # SURVEY.md s8(d)) -- the work of P LSD passes, whatever path ran
        passes = kb * 8 // 8
        roof["sort_alg_GBps"] = round(passes * alg_bytes * global_keys / n / (elapsed / steps) / 1e9, 1)
        roof["sort_frac_of_peak"] = round(roof["sort_alg_GBps"] / PEAK_HBM_GBS / max(1, world), 4)
        roof["pass_launches_per_sort"] = round(prof["pass_launches"] / steps, 2)
        if prof.get("local_launches"):
            # the 3-HBM-pass path's local bucket sort: reads and writes every key once
            lm = prof["local_ms"] / prof["local_launches"]
            la = alg_bytes / (lm / 1e3) / 1e9
            # (u32 keys over the whole key above 2^29: 16-bit items; u32 pairs: items carry positions)
            lk = ("thrs_local_pairs" if vb else
                  "thrs_local16" if (kt == 0 and n > (1 << 29))
                  else "thrs_local")
            roof["local"] = {"kernel": lk, "avg_launch_ms": round(lm, 4), "achieved": round(la, 1),
                             "frac": round(la / PEAK_HBM_GBS, 4), "alg_bytes_per_launch": alg_bytes}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 3), "unit": "Gkeys/s", "n_gpus": world, "steps": steps,
               "warmup": warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
               "scaling": scaling, "vs_baseline": None, "dtype": DTYPE[kt], "data": "synthetic",
               "config": {"workload": WORKLOADS[wl][3] if not use_dist else
                          f"{DTYPE[kt]} keys, {n} per GPU x {world} GPUs, bucket-exchange sort",
                          "keys_per_gpu": n, "global_keys": global_keys, "key": DTYPE[kt],
                          "value": None if not vb else f"{vb}B index payload", "bits": [0, kb * 8],
                          "parallelism": parallelism,
                          "inputs": "fresh per step" if not recycled else "pool recycled (some steps re-sort)"},
               "roofline": roof, "cpu_baseline": cpu}
        if phase:
            out["phases_ms"] = phase
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
