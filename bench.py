#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X.

metric: "Gkeys/s and achieved HBM GB/s (% of peak), u32 keys N=2^30, 1/2/4/8 GPU"

* N=1 (default): workload C2 = sortKeys of 2^30 u32 keys, bits [0,32), the
  reference bench's input distribution (splitmix64 from state 0,
  unittest.cpp:544-548), generated on the GPU and resident in HBM before the
  timed region.  One step = one full sort of a FRESH input buffer (the sort is
  in place, so every timed step gets its own pre-generated buffer).  For
  4-byte keys-only sorts the library takes its 3-HBM-pass path: bucket
  histogram + plan, two device-wide passes for the top two digits, and one
  in-LDS local sort of every 16-bit bucket; other workloads run
  histogram + one pass per digit.
* N>1: launched by torch.distributed.run, one rank per GPU.  Default
  (SURVEY.md s8(d)): STRONG scaling -- C2's 2^30 keys split over the N ranks
  (--scaling weak: the workload's n per rank; C5 is weak by definition, 2^30
  per GPU).  One step is the bucket-exchange sort of all keys (stable
  top-digit partition -> RCCL all-gather of counts -> exact global-rank split
  (digit refinement over small all-gathers, split buckets sorted locally) ->
  one grouped RCCL point-to-point exchange of keys and values -> local finish
  with the rank's key range, tinyhipradixsort_amd/dist.py): every rank ends
  with exactly its share of the global order, whatever the distribution.

Timing: W warm-up steps, then barrier + synchronize, K steps, synchronize +
barrier; the max over ranks.  rank 0 prints ONE JSON line.  `roofline` prices
the DOMINANT kernel -- the kernel with the most time per sort -- at its own
algorithmic bytes per launch, from per-launch HIP events on the sort's own
stream inside the timed region (gated launches that found nothing to do,
< 20 us, are not launches of the kernel's work); `cpu_baseline`
times the reference's CPU path (std::sort, unittest.cpp:156) on bounded
samples on this host, with the C1 size (2^20 keys) as its own legs.
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
    # name: (key type, value bytes, n per GPU, key distribution, description)
    "c2": (0, 0, 1 << 30, "uniform", "C2: sortKeys u32, N=2^30 uniform (splitmix64), bits [0,32), 1xMI355X"),
    "c3": (0, 4, 1 << 30, "uniform", "C3: sortPairs u32 key + u32 index payload (stable), N=2^30"),
    "c4": (2, 0, 1 << 28, "uniform", "C4: sortKeys f32 via fpKey transform, N=2^28 (bits & 0xFF7FFFFF)"),
    "c5": (1, 8, 1 << 30, "uniform", "C5: sortPairs u64 key + u64 index payload, 2^30 per GPU"),
    "u64k": (1, 0, 1 << 30, "uniform", "sortKeys u64, N=2^30 uniform (64-bit keys without payload)"),
    # f1: wide payloads (unittest.cpp:433-487: K32V64 / K32V128 / K64V128 / KF32V32)
    "k32v128": (0, 16, 1 << 30, "uniform", "sortPairs u32 key + 16-B payload (ValueType::U128), N=2^30"),
    "k64v128": (1, 16, 1 << 29, "uniform", "sortPairs u64 key + 16-B payload (K64V128), N=2^29"),
    "k32v64": (0, 8, 1 << 30, "uniform", "sortPairs u32 key + u64 payload, N=2^30"),
    "kf32v32": (2, 4, 1 << 30, "uniform", "sortPairs f32 key + u32 payload, N=2^30"),
    # the reference's float generator (randomizeValues clears the lowest exponent bit, unittest.cpp:103/108)
    "f32k": (2, 0, 1 << 30, "uniform", "sortKeys f32, N=2^30 (bits & 0xFF7FFFFF)"),
    "kf64v64": (3, 8, 1 << 29, "uniform", "sortPairs f64 key (bits & 0xFFEFFFFFFFFFFFFF) + u64 payload, N=2^29"),
    # the reference's own bench size: OrochiRadixSort.bench / benchKeyPair sort 160,000,000 u32 keys
    # (unittest.cpp:490-494, 574-578)
    "ref160m": (0, 0, 160_000_000, "uniform", "OrochiRadixSort.bench: sortKeys u32, N=160,000,000 (unittest.cpp:490-571)"),
    "ref160m_pairs": (0, 4, 160_000_000, "uniform",
                      "OrochiRadixSort.benchKeyPair: sortPairs u32 key + u32 payload, N=160,000,000 (unittest.cpp:574-)"),
    "u32large": (0, 0, (1 << 31) + 100, "uniform", "u32Large: sortKeys u32, N=2^31+100 uniform (unittest.cpp:688-717)"),
    # low-entropy inputs of C2's shape (not bench lines of BASELINE.json: robustness)
    "c2_sorted": (0, 0, 1 << 30, "sorted", "C2 shape, already-sorted input (stratified sorted uniform sample)"),
    "c2_reverse": (0, 0, 1 << 30, "reverse", "C2 shape, reverse-sorted input"),
    "c2_extreme": (0, 0, 1 << 30, "extreme", "C2 shape, extremeCase input: all zero but two keys (unittest.cpp:191-225)"),
    "c2_fewuniq": (0, 0, 1 << 30, "fewuniq", "C2 shape, 16 distinct uniform keys"),
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
    p.add_argument("--vendor", default="auto", choices=["auto", "off"],
                   help="time hipcub::DeviceRadixSort on the same inputs (N=1 only)")
    p.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    p.add_argument("--ref-gpu", default="auto", choices=["auto", "off"],
                   help="time the reference's own kernels (oracle/_ref) on the same inputs (N=1 only)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--lib", default=None, help="experiments: a variant build of libthrs.so (make variants)")
    p.add_argument("--opt", default="", help="experiments: thrs_options fields, e.g. planes=off,path=lsd")
    p.add_argument("--unchecked", action="store_true",
                   help="experiments only: skip the output check (timing a deliberately incomplete variant build)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the bucket-exchange path even at world size 1 (RCCL smoke test)")
    p.add_argument("--scaling", default="auto", choices=["auto", "strong", "weak"],
                   help="N>1: strong = the workload's n split over the ranks (default; C5: weak), "
                        "weak = the workload's n per rank")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _time_leg(fn, make, n_target_s: float, min_runs: int = 2, max_runs: int = 5):
    """median seconds of fn(make()) over a few runs within ~n_target_s"""
    times = []
    t_start = time.perf_counter()
    while len(times) < min_runs or (time.perf_counter() - t_start < n_target_s and len(times) < max_runs):
        a = make()
        t0 = time.perf_counter()
        fn(a)
        times.append(time.perf_counter() - t0)
    return statistics.median(times), len(times)


def cpu_baseline(kt: int, vb: int, n_target_s: float) -> dict:
    """The reference's CPU paths on this host, on bounded samples of the same
    splitmix64 stream (the oracle library is the timer's subject, never the
    GPU result's source):
      * std::sort, 1 thread (unittest.cpp:156) -- or std::stable_sort of pairs
        (stableSortPairs, unittest.cpp:358-377) for sortPairs workloads;
      * __gnu_parallel::sort / stable_sort on all of this process's CPU share,
        standing in for concurrency::parallel_radixsort / parallel_sort
        (unittest.cpp:563, 711; MSVC PPL is not on Linux).
    `value` is the all-core leg (the stronger baseline); `legs` lists both."""
    import numpy as np
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    kdt = O.KEY_DTYPE[kt]

    def keys_of(n):
        return O.randomize_np(kt, O.splitmix64_stream(0, n)).astype(kdt)

    legs = []
    per = n_target_s / 3
    # C1 as configured (BASELINE.json configs[0]: 2^20 keys, unittest.cpp
    # harness size): std::sort / stable_sort on 1 thread and on all threads
    n0 = 1 << 20
    ks0 = keys_of(n0)
    if vb:
        vs0 = np.arange(n0, dtype={4: np.uint32, 8: np.uint64}.get(vb, np.uint64))
        med, runs = _time_leg(lambda a: O.std_stable_sort_pairs(kt, a, vs0), lambda: ks0, per / 2, 3, 9)
        legs.append({"name": "C1 size: std::stable_sort pairs", "threads": 1, "n": n0,
                     "value": round(n0 / med / 1e9, 5), "runs": runs})
        med, runs = _time_leg(lambda a: O.parallel_stable_sort_pairs(kt, a, vs0), lambda: ks0, per / 2, 3, 9)
    else:
        med, runs = _time_leg(lambda a: O.std_sort_keys(kt, a), lambda: ks0, per / 2, 3, 9)
        legs.append({"name": "C1 size: std::sort (unittest.cpp:156)", "threads": 1, "n": n0,
                     "value": round(n0 / med / 1e9, 5), "runs": runs})
        med, runs = _time_leg(lambda a: O.parallel_sort(a, kt), lambda: ks0, per / 2, 3, 9)
    legs.append({"name": "C1 size: __gnu_parallel sort", "threads": threads, "n": n0,
                 "value": round(n0 / med / 1e9, 5), "runs": runs})
    # 1 thread: 2^24 keys (std::sort) / 2^22 pairs (stable_sort of pairs)
    if vb:
        n1 = 1 << 22
        ks = keys_of(n1)
        vs = np.arange(n1, dtype={4: np.uint32, 8: np.uint64}.get(vb, np.uint64))
        med, runs = _time_leg(lambda a: O.std_stable_sort_pairs(kt, a, vs), lambda: ks, per)
        legs.append({"name": "std::stable_sort pairs (unittest.cpp:369)", "threads": 1, "n": n1,
                     "value": round(n1 / med / 1e9, 5), "runs": runs})
    else:
        n1 = 1 << 24
        ks = keys_of(n1)
        med, runs = _time_leg(lambda a: O.std_sort_keys(kt, a), lambda: ks, per)
        legs.append({"name": "std::sort (unittest.cpp:156)", "threads": 1, "n": n1,
                     "value": round(n1 / med / 1e9, 5), "runs": runs})
    # all cores: 2^26 keys / 2^24 pairs
    nP = (1 << 24) if vb else (1 << 26)
    ks = keys_of(nP)
    if vb:
        vs = np.arange(nP, dtype={4: np.uint32, 8: np.uint64}.get(vb, np.uint64))
        med, runs = _time_leg(lambda a: O.parallel_stable_sort_pairs(kt, a, vs), lambda: ks, per)
        name = "__gnu_parallel::stable_sort pairs (stand-in for PPL parallel sort)"
    else:
        med, runs = _time_leg(lambda a: O.parallel_sort(a, kt), lambda: ks, per)
        name = "__gnu_parallel::sort (stand-in for PPL parallel_radixsort, unittest.cpp:563)"
    legs.append({"name": name, "threads": threads, "n": nP, "value": round(nP / med / 1e9, 5), "runs": runs})
    best = legs[-1]
    return {"value": best["value"], "unit": "Gkeys/s", "cores": threads, "kind": "port",
            "sample": f"{best['name']} of {best['n']} splitmix64 {DTYPE[kt]} keys, median of {best['runs']} runs, "
                      f"{threads} threads ({cpu_model()}); 1-thread leg in `legs`",
            "legs": legs}


def reference_gpu_bench(TU, kt, kb, vb, n, keys, vals, gen, stream, runs: int = 2):
    """The REFERENCE's own kernels on this MI355X (oracle/_ref: kernel.cu via
    hipRTC, launched with its pass loop, tinyhipradixsort.hpp:854-944) on the
    same inputs, event-timed per run on fresh input.  A baseline, never `value`."""
    import torch
    try:
        from oracle import ref as R
    except ImportError:
        return None
    if not R.kernels_available():
        return None
    vt = {0: 0, 4: 0, 8: 1, 16: 2}[vb]
    tmp = torch.empty(sum(R.temp_bytes(kt, vt, n)), dtype=torch.uint8, device="cuda")
    times = []
    for r in range(runs):
        j = r % len(keys)
        gen(keys[j], j)
        if vb:
            TU.iota(vb, vals[j], n)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        R.sort(kt, vt, False, keys[j], vals[j] if vb else None, n, tmp, 0, kb * 8, stream)
        b.record(stream)
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b))
        if TU.count_unsorted(kt, keys[j], n, 0, kb * 8):
            return None
    ms = statistics.median(times)
    return {"name": "reference kernels (kernel.cu via hipRTC, gfx950) + its pass loop", "value": round(n / ms / 1e6, 3),
            "unit": "Gkeys/s", "ms_per_sort": round(ms, 3), "runs": runs, "inputs": "same generator, fresh per run"}


def vendor_bench(T, TU, kt, kb, vb, n, keys, vals, gen, stream, runs: int = 3):
    """hipcub::DeviceRadixSort (rocPRIM) on the same inputs -- the MI355X
    analogue of the reference's CUB comparator (cudaEnv.cu:95-116) and of
    Oro::RadixSort (unittest.cpp:490-531).  Event-timed per run on fresh input
    (regenerated outside the timing)."""
    import ctypes
    import torch
    path = os.path.join(ROOT, "tinyhipradixsort_amd", "libthrs_vendor.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.thrsv_temp_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    L.thrsv_sort.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [
        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
    tb = ctypes.c_uint64()
    if L.thrsv_temp_bytes(kt, vb, n, ctypes.byref(tb)) != 0:
        return None
    vtmp = torch.empty(max(1, tb.value), dtype=torch.uint8, device="cuda")
    kalt = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
    valt = torch.empty(n * vb, dtype=torch.uint8, device="cuda") if vb else None
    sel = ctypes.c_int()
    times = []
    for r in range(runs + 1):               # run 0 is a warm-up
        j = r % len(keys)
        gen(keys[j], j)
        if vb:
            TU.iota(vb, vals[j], n)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        rc = L.thrsv_sort(kt, vb, keys[j].data_ptr(), kalt.data_ptr(), vals[j].data_ptr() if vb else None,
                          valt.data_ptr() if vb else None, n, vtmp.data_ptr(), tb.value, ctypes.byref(sel),
                          stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        if rc != 0:
            return None
        if r:
            times.append(a.elapsed_time(b))
    ms = statistics.median(times)
    out = keys[j] if sel.value == 0 else kalt
    if TU.count_unsorted(kt, out, n, 0, kb * 8):
        return None
    return {"name": "hipcub::DeviceRadixSort::" + ("SortPairs" if vb else "SortKeys") + " (rocPRIM)",
            "value": round(n / (ms / 1e3) / 1e9, 3), "unit": "Gkeys/s", "ms_per_sort": round(ms, 4),
            "runs": runs, "inputs": "same generator, fresh per run"}


GATED_NOOP_MS = 0.02   # a gated launch with nothing to do takes ~4-6 us; real launches at bench sizes > 0.2 ms
KIND_NAMES = {0: "hist", 1: "pass", 2: "local", 3: "fallback"}


def build_roofline(prof, kern, steps, n, kb, vb, pinfo, elapsed, global_keys, world, wl, big_keys=0):
    """`roofline` of the bench line from per-launch HIP-event times.  Every
    launch carries its kernel (thrs_profile_read_launch_kernels) and
    algorithmic bytes: 2 * keys * (K + V) for a launch that permutes keys
    (SURVEY.md s8(d)), keys * K for one that only counts them; the per-bucket
    fallback's launches move the big chunks' keys only (big_keys, read from
    the last sort's plan).  The DOMINANT kernel is the one with the most time
    per sort; its `achieved` = its bytes per launch / its average launch time.
    Gated launches that found nothing to do (< GATED_NOOP_MS) are not launches
    of the kernel's work.  `kinds` keeps the per-kind summary (hist / pass /
    local / fallback)."""
    if not prof:
        return None
    step_s = elapsed / steps
    kinds, kernels = {}, {}
    for k, ms in prof.items():
        eff = [x for x in ms if x >= GATED_NOOP_MS]
        kinds[KIND_NAMES[k]] = {"ms_per_sort": round(sum(eff) / steps, 4), "launches_per_sort": round(len(eff) / steps, 2),
                                "avg_launch_ms": round(sum(eff) / len(eff), 4) if eff else None,
                                "gated_noops_per_sort": round((len(ms) - len(eff)) / steps, 2)}
        per = len(eff) // steps if eff and len(eff) % steps == 0 else 0
        if per > 1:   # the same launches every sort: each one's average, in launch order
            kinds[KIND_NAMES[k]]["by_launch_ms"] = [round(sum(eff[i::per]) / steps, 4) for i in range(per)]
        for x, (name, byts) in zip(ms, kern.get(k, [])):
            if x < GATED_NOOP_MS:
                continue
            if byts == 0:   # data-dependent: the per-bucket fallback's work on the big chunks
                byts = {"thrs_big_hist": big_keys * kb, "thrs_pass_big": 2 * big_keys * (kb + vb),
                        "thrs_big_copy": 2 * big_keys * (kb + vb)}.get(name, 0)
            e = kernels.setdefault(name, {"ms": 0.0, "launches": 0, "bytes": 0})
            e["ms"] += x
            e["launches"] += 1
            e["bytes"] += byts
    for name, e in kernels.items():
        e["ms_per_sort"] = round(e.pop("ms") / steps, 4)
        e["avg_launch_ms"] = round(e["ms_per_sort"] * steps / e["launches"], 4)
        e["alg_bytes_per_launch"] = e.pop("bytes") // e["launches"]
        e["launches_per_sort"] = round(e.pop("launches") / steps, 2)
        e["GBps"] = round(e["alg_bytes_per_launch"] / (e["avg_launch_ms"] / 1e3) / 1e9, 1)
    cand = {k: v for k, v in kernels.items() if v["alg_bytes_per_launch"] > 0}
    if not cand:
        return None
    dom = max(cand, key=lambda k: cand[k]["ms_per_sort"])
    avg = cand[dom]["avg_launch_ms"]
    alg = cand[dom]["alg_bytes_per_launch"]
    achieved = alg / (avg / 1e3) / 1e9
    frac = achieved / PEAK_HBM_GBS
    traffic, traffic_src = load_pmc_traffic(wl, dom)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(frac, 4), "traffic": traffic, "traffic_source": traffic_src,
            "kernel": dom, "avg_launch_ms": avg, "alg_bytes_per_launch": alg,
            "kernels": kernels, "kinds": kinds}
    # whole sort: B_alg = P*2*N*(K+V) for P 8-bit digits, the
    # work of P LSD passes whatever path ran ...
    passes = kb
    # (an LSD-equivalent rate: the bucket path moves fewer bytes than P LSD
    # passes, so it can exceed the HBM peak -- then it is no fraction of a
    # roofline and is withheld; sort_min_frac below is the roofline figure)
    roof["sort_alg_GBps"] = round(passes * 2 * global_keys * (kb + vb) / step_s / 1e9, 1)
    frac_alg = roof["sort_alg_GBps"] / PEAK_HBM_GBS / max(1, world)
    roof["sort_frac_of_peak"] = round(frac_alg, 4) if frac_alg <= 1.0 else None
    # ... and on the bytes the path that ran must move at least (thrs_path_info)
    if pinfo:
        roof["path"] = pinfo
        roof["sort_min_bytes"] = pinfo["min_bytes"]
        roof["sort_min_GBps"] = round(pinfo["min_bytes"] / step_s / 1e9, 1)
        roof["sort_min_frac"] = round(pinfo["min_bytes"] / step_s / 1e9 / PEAK_HBM_GBS, 4)
    return roof


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(workload: str, kernel: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    --pmc run (profiles/pmc_traffic.json: which run, counters and gfx950
    corrections are recorded there), when that run measured this kernel.  Not
    measured by this process: returned with its source so the line says so."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        e = d.get(workload, {})
        if kernel.startswith("thrs_pass"):
            v = e.get("thrs_pass_bytes_per_launch")
        elif kernel == e.get("local_kernel") or kernel.startswith("thrs_local"):
            v = e.get("local_bytes_per_launch") if kernel == e.get("local_kernel") else None
        else:
            v = e.get(f"{kernel}_bytes_per_launch")
        if v is None:
            return None, None
        return v, f"profiles/pmc_traffic.json[{workload}] from {e.get('source', '?')} (rocprofv3 --pmc, not this run)"
    except (OSError, ValueError):
        return None, None


def main():
    args = parse()
    # stdout carries exactly one JSON line (rank 0).  Native libraries print
    # to file descriptor 1 (RCCL's version banner at communicator set-up, on
    # every rank), so fd 1 points at stderr from here on and the JSON line is
    # written to the saved descriptor.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
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
    if args.lib:
        T.LIB_PATH = os.path.abspath(args.lib)

    wl = args.workload or "c2"
    kt, vb, n_default, dist_name, desc = WORKLOADS[wl]
    dist_kind = dist_name
    # the 1/2/4/8-GPU curve is C2's 2^30 keys split over the
    # GPUs (strong); C5 is 2^30 per GPU (weak).  --n = the workload's size
    # (the total for strong scaling, per GPU for weak).
    scaling = args.scaling if args.scaling != "auto" else ("weak" if wl == "c5" else "strong")
    n_work = args.n or n_default
    if scaling == "strong":
        n = n_work * (rank + 1) // world - n_work * rank // world
        global_keys = n_work
    else:
        n = n_work
        global_keys = n_work * world
    kb = KEY_BYTES[kt]
    steps, warmup = args.steps, args.warmup
    stream = torch.cuda.current_stream()

    def barrier():
        if dist is not None:
            dist.barrier()

    if not use_dist:
        cfg = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                   8: T.ValueType.U64, 16: T.ValueType.U128}[vb])
        opts = T.Options(**dict(kv.split("=", 1) for kv in args.opt.split(",") if kv))
        rs = T.RadixSort([], cfg, opts)
        tdef = rs.getTemporaryBufferBytes(n)
        tmp_bytes = tdef.getTemporaryBufferBytesForSortPairs() if vb else tdef.getTemporaryBufferBytesForSortKeys()
        tmp = torch.empty(tmp_bytes, dtype=torch.uint8, device="cuda")
        # Every TIMED step sorts its own fresh buffer (the reference draws a new
        # stream per run, unittest.cpp:544-549): `steps` distinct buffers must
        # fit in HBM, else fail loudly -- inputs are never recycled.
        free, _total = torch.cuda.mem_get_info()
        per = n * (kb + vb)
        fit = int((free - tmp_bytes - (6 << 30)) // max(per, 1))
        if fit < steps:
            raise SystemExit(f"bench: {steps} fresh inputs of {per / 2**30:.1f} GiB do not fit in HBM "
                             f"(room for {fit}); use fewer --steps")
        pool = steps

        def gen(buf, i):        # run r consumes stream draws r*N+1 .. (r+1)*N
            if dist_kind == "uniform":
                TU.fill_keys(kt, buf, n, start=i * n)
            else:
                TU.fill_dist(kt, buf, n, dist_kind, start=i * n)

        keys, vals = [], []
        for i in range(pool):
            kbuf = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
            gen(kbuf, i)
            keys.append(kbuf)
            if vb:
                vbuf = torch.empty(n * vb, dtype=torch.uint8, device="cuda")
                TU.iota(vb, vbuf, n)
                vals.append(vbuf)
        keys_in0 = None
        if vb:      # keep one input for the stability/gather check of the last step
            keys_in0 = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
            keys_in0.copy_(keys[pool - 1])
        torch.cuda.synchronize()

        def step(j):
            if vb:
                rs.sortPairs(keys[j], vals[j], n, tmp, 0, kb * 8, stream)
            else:
                rs.sortKeys(keys[j], n, tmp, 0, kb * 8, stream)

        # warm-up sorts buffers 0..W-1 (mod pool), which are then regenerated
        # with the same draws, so the timed steps all see fresh input
        for i in range(warmup):
            step(i % pool)
        for i in range(min(warmup, pool)):
            gen(keys[i], i)
            if vb:
                TU.iota(vb, vals[i], n)
        # keys-only: an order-independent fingerprint of every timed input
        # (checked against its output after the timed region: a dropped or
        # duplicated key cannot pass as sorted output)
        fps = [TU.fingerprint(kt, keys[i], n) for i in range(steps)] if not vb and not args.unchecked else None
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        big_keys = T.debug_big_keys(tmp, kt, vb, n, stream)   # the last sort's fallback work (0: none)
        rs.checkDeviceError(tmp)      # raises on a look-back / claim timeout in any timed step
        # correctness of the last timed step (outside the timed region)
        last = steps - 1
        bad = 0 if args.unchecked else TU.count_unsorted(kt, keys[last], n, 0, kb * 8)
        if bad:
            raise SystemExit(f"bench: output of the last step is not sorted ({bad} inversions)")
        if fps is not None:
            lost = [i for i in range(steps) if TU.fingerprint(kt, keys[i], n) != fps[i]]
            if lost:
                raise SystemExit(f"bench: steps {lost} lost or duplicated keys (multiset fingerprint differs)")
        if vb and not args.unchecked:
            chk = TU.check_pairs(kt, vb, keys_in0, keys[last], vals[last], n, 0, kb * 8)
            if chk["gather_mismatch"] or chk["unstable"]:
                raise SystemExit(f"bench: pairs output of the last step is wrong: {chk}")
        # per-launch kernel times for the roofline: the same K steps again, on
        # regenerated inputs, with HIP events around every launch on the sort's
        # stream.  Those events cost ~0.1 ms per sort (scripts/prof_overhead.py),
        # so they are kept out of the timed region above.
        for i in range(steps):
            gen(keys[i], i)
            if vb:
                TU.iota(vb, vals[i], n)
        torch.cuda.synchronize()
        T.profile_enable(True)
        t2 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        prof = {k: T.profile_launches(k) for k in range(4)}
        kern = {k: T.profile_launch_kernels(k) for k in range(4)}
        T.profile_enable(False)
        rs.checkDeviceError(tmp)
        ev_ms = (t3 - t2) / steps * 1e3
        vendor = ref_gpu = None
        if args.vendor == "auto" and world == 1:
            del keys_in0
            vendor = vendor_bench(T, TU, kt, kb, vb, n, keys, vals, gen, stream)
        # (the reference's kernels index with 32-bit ints: up to 2^30 keys here)
        if args.ref_gpu == "auto" and world == 1 and dist_kind == "uniform" and n <= (1 << 30):
            ref_gpu = reference_gpu_bench(TU, kt, kb, vb, n, keys, vals, gen, stream)
        inputs = "fresh per step"
        elapsed = t1 - t0
        parallelism = "single"
        phase = None
    else:
        from tinyhipradixsort_amd import dist as D
        vt = None if not vb else {4: T.ValueType.U32, 8: T.ValueType.U64, 16: T.ValueType.U128}[vb]
        sorter = D.DistributedRadixSort(key_type=kt, value_type=vt)
        # inputs: rank r of step i holds draws (i*world + r)*n + 1 .. of the
        # splitmix64 stream; values = global index.  The exchange sort is out
        # of place (inputs are never modified), so a pool of 2 stays fresh.
        pool = 2
        keys, vals = [], []
        first = n_work * rank // world if scaling == "strong" else n * rank   # this rank's first global index
        for i in range(pool):
            kbuf = torch.empty(n * kb, dtype=torch.uint8, device="cuda")
            if dist_kind == "uniform":
                TU.fill_keys(kt, kbuf, n, start=i * global_keys + first)
            else:
                TU.fill_dist(kt, kbuf, n, dist_kind, start=i * global_keys + first)
            keys.append(kbuf)
            if vb:
                vbuf = torch.empty(n * vb, dtype=torch.uint8, device="cuda")
                TU.iota(vb, vbuf, n, start=first)
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
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            out = step(warmup + i)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        # per-launch kernel times (HIP events around every launch): a second
        # pass of the same steps, outside the timed region (as single-GPU)
        T.profile_enable(True)
        t2 = time.perf_counter()
        for i in range(steps):
            out2 = step(warmup + i)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        prof = {k: T.profile_launches(k) for k in range(4)}
        kern = {k: T.profile_launch_kernels(k) for k in range(4)}
        big_keys = 0
        T.profile_enable(False)
        del out2
        ev_ms = (t3 - t2) / steps * 1e3
        ko, _vo, n_out = out
        bad = TU.count_unsorted(kt, ko, n_out, 0, kb * 8)
        if bad:
            raise SystemExit(f"bench: rank {rank} output is not sorted ({bad} inversions)")
        # across ranks: every key arrived somewhere, and rank r's last key <=
        # rank r+1's first (unsigned key types compare as stored)
        tot = torch.tensor([n_out], dtype=torch.int64, device="cuda")
        dist.all_reduce(tot)
        if int(tot.item()) != global_keys:
            raise SystemExit(f"bench: {int(tot.item())} keys after the exchange, expected {global_keys}")
        if kt in (T.KeyType.U32, T.KeyType.U64):
            kdt = torch.int32 if kb == 4 else torch.int64
            kv = ko.view(kdt)[:n_out].to(torch.int64)
            ends = torch.tensor([[n_out, kv[0].item(), kv[-1].item()] if n_out else [0, 0, 0]], dtype=torch.int64,
                                device="cuda")
            allends = [torch.empty_like(ends) for _ in range(world)]
            dist.all_gather(allends, ends)
            mask = (1 << (8 * kb)) - 1
            seq = [(int(e[0, 1]) & mask, int(e[0, 2]) & mask) for e in allends if int(e[0, 0]) > 0]
            for (_a0, a1), (b0, _b1) in zip(seq, seq[1:]):
                if a1 > b0:
                    raise SystemExit("bench: ranks' key ranges overlap after the exchange")
        inputs = ("2 input buffers per rank, alternated: the exchange sort is out of place, so every step "
                  "sorts an unmodified input (the same two inputs repeat)")
        vendor = ref_gpu = None
        elapsed = t1 - t0
        parallelism = f"bucket-exchange x{world} (RCCL all_gather + grouped point-to-point exchange)"
        phase = {k: round(v * 1e3, 3) for k, v in phase_s.items()}
        phase["n_out_rank0"] = n_out if rank == 0 else None

    # max over ranks
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_per_step = elapsed / steps * 1e3
    value = global_keys / (elapsed / steps) / 1e9

    # roofline of the DOMINANT kernel kind (device passes, local sort or the
    # per-bucket fallback's passes: the most time inside the timed region);
    # algorithmic bytes per launch = 2 * n * (K + V) (one read and one write of
    # every key and value); gated launches that found nothing
    # to do (< GATED_NOOP_MS) are not launches of the kernel's work
    cfg_info = T.RadixSort.Config(keyType=T.KeyType(kt), valueType={0: T.ValueType.U32, 4: T.ValueType.U32,
                                                                     8: T.ValueType.U64, 16: T.ValueType.U128}[vb])
    pinfo = T.RadixSort([], cfg_info, T.Options(**dict(kv.split("=", 1) for kv in args.opt.split(",") if kv))).pathInfo(
        n, 0, kb * 8, bool(vb)) if not use_dist else None
    roof = build_roofline(prof, kern, steps, n, kb, vb, pinfo, elapsed, global_keys, world, wl, big_keys)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(kt, vb, args.cpu_seconds)

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 3), "unit": "Gkeys/s", "n_gpus": world, "steps": steps,
               "warmup": warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
               "scaling": scaling, "vs_baseline": None, "dtype": DTYPE[kt], "data": "synthetic",
               "config": {"workload": WORKLOADS[wl][4] if not use_dist else
                          f"{WORKLOADS[wl][4]} -- {global_keys} keys over {world} GPUs ({scaling} scaling), "
                          f"bucket-exchange sort",
                          "keys_per_gpu": n, "global_keys": global_keys, "key": DTYPE[kt],
                          "value": None if not vb else f"{vb}B index payload", "bits": [0, kb * 8],
                          "parallelism": parallelism,
                          "distribution": dist_name,
                          "inputs": inputs},
               "roofline": roof, "cpu_baseline": cpu, "vendor": vendor, "reference_gpu": ref_gpu,
               "timing": {"ms_per_step_with_launch_events": round(ev_ms, 4),
                          "note": "value / ms_per_step: K sorts between a barrier + synchronize on both sides, "
                                  "no per-launch events; roofline per-launch times: a second pass of the same K "
                                  "steps with HIP events around every launch (their cost is the difference)"}}
        if phase:
            out["phases_ms"] = phase
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
