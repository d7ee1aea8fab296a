// thrs_pipe.hpp -- the bucket path's top-digit pass, software-pipelined
// (gfx950; experiment THRS_SEG_PIPE, docs/EXPERIMENTS.md).
//
// thrs_pass_seg runs one tile at a time per CU: load + count (~5 us), scan,
// rank + stage, look-back walk (~3 us), write-out -- ~14 us per 32768-key
// tile, with the CU's memory idle during the walk and its LDS idle during
// the loads (scripts/seg_stamps.py).  Here a workgroup holds two tiles at
// once and splits its waves by role:
//   waves 0-3   WALKERS: hold no keys; thread d < 256 scans digit d and walks
//               the decoupled look-back for it (GroupWalk, thrs_kernels.hpp)
//   waves 4-15  KEY WAVES: 12 x 64 x KPT keys per tile, ranked in registers
// Per iteration (tile i current, i+1 next):
//   1  walkers: scan of tile i's counts -> per-wave running offsets; thread 0
//      claims tile i+1 (just before it is loaded: a tile is never claimed long
//      before its aggregate can be published)
//   2  key waves: rank tile i into the LDS stage, then load tile i+1 and
//      count it into the same (now free) per-wave rows;
//      walkers, at the same time: walk tile i
//   3  tile i+1's aggregate published; every wave writes tile i out
// so tile i+1's loads and counting run under tile i's walk.  Results are the
// bytes of thrs_pass_seg: the same stable order (item j of lane l of key wave
// kw is key kw*64*KPT + 64j + l), the same segments, tables and clamps.
#pragma once
#include "thrs_kernels.hpp"

namespace thrs_dev {
namespace {

struct PipeGeom {
  static constexpr int WAVES = 16, WALK_WAVES = 4, KEY_WAVES = 12;
#ifndef THRS_PIPE_DBG
#define THRS_PIPE_DBG 0  // register-pressure diagnostics only: 1 no walk, 2 no write-out, 3 no next-tile load
#endif
#ifndef THRS_PIPE_KPT
#define THRS_PIPE_KPT 36
#endif
  static constexpr int KPT = THRS_PIPE_KPT;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr uint32_t TILE = 64u * KEY_WAVES * KPT;
  // the write-out: all 16 waves, or (THRS_PIPE_WALKER_WO 0) the key waves
  // only -- a walker's stores would sit in its vmcnt ahead of its next walk's
  // loads (gfx9: one counter for loads and stores)
#ifndef THRS_PIPE_WALKER_WO
#define THRS_PIPE_WALKER_WO 1
#endif
  static constexpr int WO_THREADS = THRS_PIPE_WALKER_WO ? THREADS : 64 * KEY_WAVES;
  static constexpr int NS = (int)(TILE / WO_THREADS);  // stage slots per thread in the write-out
  // stage (4-byte keys / plane images) | s_cnt[KEY_WAVES][256] | s_gofs[256] | s_misc[32]
  static constexpr uint32_t LDS_BYTES = TILE * 4 + (KEY_WAVES + 1) * kBins * 4 + 32 * 4;
  static_assert(TILE % WO_THREADS == 0, "whole write-out rounds");
  static_assert(TILE < kArrival / kGroup, "group counts fit below the arrival bits");
};

template <int KT, typename ST, bool ATOMIC_RANK, int CODEC>
__global__ __launch_bounds__(PipeGeom::THREADS) __attribute__((amdgpu_waves_per_eu(4))) void thrs_pass_seg_pipe(
    const typename KeyTraits<KT>::U* __restrict__ keysIn, typename KeyTraits<KT>::U* __restrict__ keysOut,
    KeyMap<typename KeyTraits<KT>::U> km, int shift, uint32_t* __restrict__ segInfo,
    const uint32_t* __restrict__ segBase, ST* __restrict__ status, uint32_t* __restrict__ errFlag,
    GroupTables<ST> grp, const uint32_t* __restrict__ gate, uint32_t gateMask, uint8_t* __restrict__ hiPlane,
    const SqueezeWords* __restrict__ sq) {
  using U = typename KeyTraits<KT>::U;
  using P = PipeGeom;
  static_assert(sizeof(U) == 4, "4-byte keys without values");
  constexpr int KPT = P::KPT;
  constexpr uint32_t T = P::TILE, CHUNK = 64u * KPT;
  if (gate && !((gateMask >> *gate) & 1u)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  U* stage = reinterpret_cast<U*>(smem);
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + T * 4);  // [KEY_WAVES][256]
  uint32_t* s_gofs = s_cnt + P::KEY_WAVES * kBins;
  uint32_t* s_misc = s_gofs + kBins;  // [4..7] walker scan, [8] seg, [9] ticket
  __shared__ uint32_t segPos[kSegs + 1], segTiles[kSegs + 1];
  uint32_t* tickets = segInfo + 64;
  uint32_t tid0 = threadIdx.x;
  pin(tid0);
  // per-lane indices: re-pinned every iteration of the tile loop, so that no
  // lane-dependent address is hoisted out of it into a long-lived VGPR
  uint32_t tid = tid0, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool walker = w < (uint32_t)P::WALK_WAVES;
  const uint32_t kw = walker ? 0u : w - P::WALK_WAVES;  // key wave
  uint32_t d = tid & 255u;                               // walkers: the digit
  if (tid < 2 * (kSegs + 1)) (tid <= (uint32_t)kSegs ? segPos[tid] : segTiles[tid - kSegs - 1]) = segInfo[tid];
  __syncthreads();
  const uint32_t home = xcc_id() & (kSegs - 1);
  const uint32_t outEnd = segPos[kSegs];

  with_map<KT>(km, sq, [&](auto kmx) __attribute__((always_inline)) {
    uint32_t done = 0;  // thread 0: segments found exhausted
    auto claim = [&]() {  // thread 0: the next tile (seg = kSegs: none left)
      uint32_t seg = kSegs, t = 0;
      for (int q = 0; q < kSegs; ++q) {
        const uint32_t s = (home + q) & (kSegs - 1);
        if (done & (1u << s)) continue;
        const uint32_t nT = seg_tiles(segPos[s], segPos[s + 1], T);
        const uint32_t x = nT ? atomicAdd(&tickets[s], 1u) : nT;
        if (x < nT) {
          seg = s;
          t = x;
          break;
        }
        done |= 1u << s;
      }
      s_misc[8] = seg;
      s_misc[9] = t;
    };
    struct Tile {
      uint32_t seg, chain, id, valid;
      uint64_t keyStart;
    };
    auto describe = [&]() -> Tile {  // the tile in s_misc[8..9] (uniform)
      Tile x;
      x.seg = __builtin_amdgcn_readfirstlane(s_misc[8]);
      const uint32_t t = __builtin_amdgcn_readfirstlane(s_misc[9]);
      if (x.seg >= (uint32_t)kSegs) {
        x.chain = x.id = x.valid = 0;
        x.keyStart = 0;
        return x;
      }
      const uint32_t s0 = segPos[x.seg], s1 = segPos[x.seg + 1];
      const uint64_t t0 = seg_tile_base(s0, T) + (uint64_t)t * T;
      x.keyStart = max((uint64_t)s0, t0);
      x.valid = (uint32_t)(min((uint64_t)s1, t0 + T) - x.keyStart);
      x.chain = segTiles[x.seg];
      x.id = x.chain + t;
      return x;
    };
    auto digit_of = [&](U key) -> uint32_t { return (uint32_t)(kimg<KT>(kmx, key) >> shift) & 0xFFu; };

    uint32_t* cnt = s_cnt + kw * kBins;
    bool allU = false;  // key waves: every item of the wave has digit d0 (sorted input)
    uint32_t d0 = 0;
    // key waves: load tile x into k and count it into this wave's row (zeroed here)
    auto load_count = [&](const Tile& x, U (&k)[KPT]) {
      const uint64_t base = x.keyStart + (uint64_t)kw * CHUNK;
      int32_t lim = (int32_t)x.valid - (int32_t)(kw * CHUNK + lane);
      pin(reinterpret_cast<uint32_t&>(lim));
      const bool full = x.valid == T;
      if constexpr (CODEC == kCodecPlanes) {
        const uint16_t* lo = reinterpret_cast<const uint16_t*>(keysIn);
        if (full) {
#pragma unroll
          for (int j = 0; j < KPT; ++j) {
            const uint64_t i = base + j * 64 + lane;
            k[j] = ((uint32_t)hiPlane[i] << 16) | (uint32_t)lo[i];
          }
        } else {
#pragma unroll
          for (int j = 0; j < KPT; ++j) {
            const uint64_t i = base + j * 64 + lane;
            k[j] = (j * 64 < lim) ? (((uint32_t)hiPlane[i] << 16) | (uint32_t)lo[i]) : 0u;
          }
        }
      } else {
        if (full) {
#pragma unroll
          for (int j = 0; j < KPT; ++j) k[j] = keysIn[base + j * 64 + lane];
        } else {
#pragma unroll
          for (int j = 0; j < KPT; ++j) k[j] = (j * 64 < lim) ? keysIn[base + j * 64 + lane] : (U)0;
        }
      }
#pragma unroll
      for (int i = 0; i < kBins / 64; ++i) cnt[i * 64 + lane] = 0;
      auto dig = [&](int j) -> uint32_t {
        const uint32_t dd = digit_of(k[j]);
        return (full || j * 64 < lim) ? dd : 0xFFu;  // padding sorts after every real key
      };
      d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dig(0));
      const bool hint = full && __ballot(dig(0) != d0 || dig(KPT - 1) != d0) == 0;
      allU = false;
      if (hint) {
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < KPT; ++j) diff |= dig(j) ^ d0;
        allU = __ballot(diff != 0) == 0;
      }
      // no digit stays live from the check into the count (64 live values)
#pragma unroll
      for (int j = 0; j < KPT; ++j) pin(k[j]);
      if (allU) {
        if (lane == 0) __hip_atomic_fetch_add(&cnt[d0], 64u * KPT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j)
          __hip_atomic_fetch_add(&cnt[dig(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    };
    // key waves 0-3 (threads 256..511): publish tile x's aggregate (its counts in s_cnt)
    auto publish = [&](const Tile& x) {
      if (tid >= 256u && tid < 512u) {
        const uint32_t dp = tid - 256u;
        uint32_t t2 = 0;
#pragma unroll
        for (int ww = 0; ww < P::KEY_WAVES; ++ww) t2 += s_cnt[ww * kBins + dp];
        const uint32_t real2 = (dp == 255u) ? t2 - (T - x.valid) : t2;
        ST* pub = status + (uint64_t)x.id * kBins + dp;
        if (x.id != x.chain) store_agent(pub, Status<ST>::agg(real2));
        else store_agent(pub, Status<ST>::pre(real2));
        __hip_atomic_fetch_add(&grp.ga[(uint64_t)(x.id / kGroup) * kBins + dp], real2 + kArrival, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
    };

    auto put = [&](U key, uint32_t dst) __attribute__((always_inline)) {
      if constexpr (CODEC == kCodecSplit) {
        const uint32_t img = (uint32_t)kimg<KT>(kmx, key);
        reinterpret_cast<uint16_t*>(keysOut)[dst] = (uint16_t)img;
        hiPlane[dst] = (uint8_t)(img >> 24);
      } else if constexpr (CODEC == kCodecPlanes) {
        reinterpret_cast<uint16_t*>(keysOut)[dst] = (uint16_t)key;
      } else {
        keysOut[dst] = key;
      }
    };
    // write tile x out of the stage (every writer wave)
    auto write_out = [&](const Tile& x) {
      const bool writer = THRS_PIPE_WALKER_WO || !walker;
      const uint32_t wt = THRS_PIPE_WALKER_WO ? tid : tid - 64u * P::WALK_WAVES;  // writer index
      if (!writer || THRS_PIPE_DBG == 2) return;
      if (x.valid == T) {
        constexpr int NS = P::NS, WB = THRS_WO_BATCH;
#pragma unroll
        for (int j0 = 0; j0 < NS; j0 += WB) {
          U key[WB];
          uint32_t off[WB];
#pragma unroll
          for (int b = 0; b < WB; ++b)
            if (j0 + b < NS) key[b] = stage[(j0 + b) * P::WO_THREADS + wt];
#pragma unroll
          for (int b = 0; b < WB; ++b)
            if (j0 + b < NS) off[b] = s_gofs[digit_of(key[b])];
#pragma unroll
          for (int b = 0; b < WB; ++b)
            if (j0 + b < NS) put(key[b], off[b] + (j0 + b) * P::WO_THREADS + wt);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < P::NS; ++j) {
          const uint32_t i = j * P::WO_THREADS + wt;
          if (i < x.valid) {
            const U key = stage[i];
            put(key, s_gofs[digit_of(key)] + i);
          }
          if ((j % THRS_WO_BATCH) == THRS_WO_BATCH - 1) __builtin_amdgcn_sched_barrier(0);
        }
      }
    };

    // Loop over tiles X (claimed one step ahead); prev = X's predecessor on
    // this workgroup, ranked into the stage, its walk and write-out pending.
    //   1  key waves: load + count X      | walkers: walk prev
    //   2  X's aggregate published; every wave writes prev out
    //   3  walkers: scan X; thread 0 claims the next tile
    //   4  key waves: rank X into the stage
    // (k is live from 1 to 4 only; X's aggregate is out before X walks)
    if (tid == 0) claim();
    lds_barrier();
    Tile cur = describe(), prev{};
    bool havePrev = false;
    uint32_t realTot = 0, localStart = 0;  // walkers: prev's, for its walk
    for (;;) {
      const bool haveCur = cur.seg < (uint32_t)kSegs;
      if (!haveCur && !havePrev) break;
      pin(tid);
      pin(lane);
      pin(d);
      // k: declared per iteration, so that no path carries keys across the
      // walk or the next load (liveness is path-insensitive)
      U k[KPT];
      // ---- 1
      if (!walker) {
#if THRS_PIPE_DBG != 3
        if (haveCur) load_count(cur, k);
#endif
      } else if (havePrev) {
#if THRS_PIPE_DBG != 1
        GroupTables<ST> g = grp;
        g.nTiles = prev.chain + seg_tiles(segPos[prev.seg], segPos[prev.seg + 1], T);
        g.gmin = prev.chain / kGroup;
        g.gaNext = nullptr;
        g.gpNext = nullptr;
        GroupWalk<ST> gw(status, g, prev.id, d);
        gw.finish(realTot, segBase[prev.seg * kBins + d], outEnd, localStart, s_gofs, s_misc, errFlag, nullptr);
#endif
      }
      lds_barrier();
      // ---- 2
      if (haveCur) publish(cur);
      if (havePrev) write_out(prev);
      if (!haveCur) break;
      // ---- 3
      uint32_t tot = 0, incl = 0;
      if (walker) {
#pragma unroll
        for (int ww = 0; ww < P::KEY_WAVES; ++ww) tot += s_cnt[ww * kBins + d];
        realTot = (d == 255u) ? tot - (T - cur.valid) : tot;
        incl = wave_incl_scan(tot, lane);
        if (lane == 63) s_misc[4 + w] = incl;
      }
      lds_barrier();  // (also: prev's stage reads are done)
      if (tid == 0) claim();
      if (walker) {
        const uint32_t w0 = s_misc[4], w1 = s_misc[5], w2 = s_misc[6];
        localStart = incl - tot + (w > 0 ? w0 : 0u) + (w > 1 ? w1 : 0u) + (w > 2 ? w2 : 0u);
        uint32_t run = localStart;
#pragma unroll
        for (int ww = 0; ww < P::KEY_WAVES; ++ww) {
          const uint32_t c = s_cnt[ww * kBins + d];
          s_cnt[ww * kBins + d] = run;
          run += c;
        }
      }
      lds_barrier();
      // ---- 4
      if (!walker) {
        if (allU) {
          const uint32_t ubase = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt[d0]);
#pragma unroll
          for (int j = 0; j < KPT; ++j) stage[ubase + 64u * j + lane] = k[j];
        } else {
          const bool full = cur.valid == T;
          int32_t lim = (int32_t)cur.valid - (int32_t)(kw * CHUNK + lane);
          pin(reinterpret_cast<uint32_t&>(lim));
          auto dig = [&](int j) -> uint32_t {
            const uint32_t dd = digit_of(k[j]);
            return (full || j * 64 < lim) ? dd : 0xFFu;
          };
          if constexpr (ATOMIC_RANK) {
            constexpr int RP = THRS_RANK_PIPE;
            uint32_t rq[RP];
#pragma unroll
            for (int j = 0; j < RP && j < KPT; ++j) {
              pin(k[j]);
              rq[j] = __hip_atomic_fetch_add(&cnt[dig(j)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
              const uint32_t slot = rq[j % RP];
              if (j + RP < KPT) {
                pin(k[j + RP]);
                rq[j % RP] =
                    __hip_atomic_fetch_add(&cnt[dig(j + RP)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              }
              stage[slot] = k[j];
              __builtin_amdgcn_sched_barrier(0);
            }
          } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
              pin(k[j]);
              stage[wave_rank<false>(cnt, dig(j), lane, false)] = k[j];
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      }
      prev = cur;
      havePrev = true;
      cur = describe();  // the tile thread 0 claimed in 3 (s_misc[8..9])
      // (prev's stage writes and the rows' running offsets are consumed
      // before anyone touches them again: barrier after 1)
    }
  });
}

}  // namespace
}  // namespace thrs_dev
