// apg_maze.hpp — FloorMapDatasetMaze.get_data_point (ap_gym/envs/floor_map/floor_map_dataset_maze.py:24-55)
// on device, bit-exact: numpy's PCG64 stream of default_rng(idx), rng.permutation(directions) per carved
// cell, rng.random() for every eligible non-first direction, the recursive carve() as an explicit DFS.
//
// One lane per maze; the whole DFS works out of LDS and registers, global memory is touched only in a
// wave-wide memory phase every MZ_PERIOD iterations (so no load in the DFS ever waits behind a store):
//  * vis     visited bits of the odd cells, u64 [ncy][cw] per lane (lanes interleaved).  An odd cell is
//            cleared only when it is carved into, so `maze[next_pos] == 1` (maze.py:38) is "not visited";
//  * ring    the top MZ_RING stack frames, one byte each: the frame's permutation index (5 bits) and the
//            direction it was entered by (2 bits).  A frame's loop position k is not stored: a frame is
//            only ever returned to from the child it carved, whose entry direction names the position;
//            `first` is false in every frame below the top.  Older frames are spilled to global memory
//            in MZ_CHUNK-frame chunks; the chunk just below the ring is kept in registers (or prefetched
//            one memory phase ahead), so backtracking does not wait on a load;
//  * log     one u16 per carve (cell x | y << 7 | direction << 14), buffered in LDS and appended to a
//            global per-maze log in the memory phase.  After the DFS the wave paints each maze's
//            occupancy rows from its log in an LDS bitmap and writes them out coalesced.
// One iteration either carves (the first eligible direction from position k on, after its rng.random()
// draw when it is not the frame's first carve) or returns to the parent frame: 2 * cells - 1 iterations
// for a perfect maze, each with one LDS round trip (the current cell's three neighbour rows).
#pragma once
#include "apg_device.hpp"

namespace apg {

constexpr int MZ_RING = 64;    // frames held in LDS (a multiple of MZ_CHUNK)
constexpr int MZ_CHUNK = 32;   // frames per spill / reload
constexpr int MZ_PERIOD = 16;  // DFS iterations between memory phases (<= MZ_LOGBUF; ring headroom below)
constexpr int MZ_LOGBUF = 16;  // log entries buffered in LDS per lane
constexpr uint32_t MZ_LOG_PAD = 0xFFFFu;  // padding entry (x = 127 is never a cell: ncx <= 127)
static_assert(MZ_RING - MZ_PERIOD - MZ_CHUNK >= 0 && MZ_RING - MZ_PERIOD > MZ_CHUNK - 1, "ring headroom");

// Generator.permutation of the 4 directions is numpy's shuffle: swap(3, j3), swap(2, j2), swap(1, j1) with
// j3 = random_interval(3), j2 = random_interval(2), j1 = random_interval(1).  Index j3 * 6 + j2 * 2 + j1 ->
// the permuted directions, 2 bits each (direction of position k in bits 2k..2k+1).
constexpr uint64_t MZ_PERM_TAB0 = 0x4e4b272d1b1e3639ULL, MZ_PERM_TAB1 = 0x9c93878d6c637872ULL,
                   MZ_PERM_TAB2 = 0xe4e1d8d2c6c9b4b1ULL;

APG_DEV uint32_t mz_perm_of(uint32_t pidx) {
  const uint64_t t = pidx < 8u ? MZ_PERM_TAB0 : (pidx < 16u ? MZ_PERM_TAB1 : MZ_PERM_TAB2);
  return (uint32_t)(t >> ((pidx & 7u) * 8u)) & 255u;
}

// The maze's numpy stream (PCG64 + next_uint32's buffered half word), with the PCG64 outputs generated
// ahead into a small register FIFO: the DFS loop produces up to MZ_FILL outputs per iteration in uniform
// control flow, and the draw sites (rng.random(), the permutation's next_uint32 calls) only pop from the
// FIFO.  Without it a wave executed the 128-bit LCG step once per draw site any of its lanes reached
// (up to five per iteration).  The outputs are consumed in the same order, so the draws are unchanged.
// A DFS iteration consumes 0.88 outputs on average but up to ~3 on a forward run (a carve draws the new
// cell's permutation, 3+ next_uint32, after its own rng.random()): one fill per iteration leaves lanes short
// on 26 % of the iterations of a 127 x 127 maze, two fills into 6 slots on none (tools' FIFO simulation);
// a short lane steps the LCG inline.
constexpr int MZ_FIFO = 6, MZ_FILL = 2;
struct MzRng {
  uint64_t s_hi, s_lo, i_hi, i_lo;
  uint32_t f[2 * MZ_FIFO];  // queued outputs, front first: f[2i] low, f[2i + 1] high word
  int cnt;
  uint32_t has32, u32;
};

APG_DEV void mz_step(MzRng &R, uint32_t &lo, uint32_t &hi) {
  pcg_step(R.s_hi, R.s_lo, R.i_hi, R.i_lo);
  const uint64_t x = R.s_hi ^ R.s_lo;
  const unsigned rot = (unsigned)(R.s_hi >> 58);
  const uint64_t o = (x >> rot) | (x << ((64u - rot) & 63u));
  lo = (uint32_t)o;
  hi = (uint32_t)(o >> 32);
}

// one output into the FIFO when there is room (state advanced only then)
APG_DEV void mz_fill(MzRng &R) {
  const uint64_t sh = R.s_hi, sl = R.s_lo;
  uint32_t lo, hi;
  mz_step(R, lo, hi);
  const bool room = R.cnt < MZ_FIFO;
  if (!room) {
    R.s_hi = sh;
    R.s_lo = sl;
  }
#pragma unroll
  for (int i = 0; i < MZ_FIFO; i++) {
    const bool here = room && R.cnt == i;
    R.f[2 * i] = here ? lo : R.f[2 * i];
    R.f[2 * i + 1] = here ? hi : R.f[2 * i + 1];
  }
  R.cnt += room ? 1 : 0;
}

APG_DEV void mz_pop64(MzRng &R, uint32_t &lo, uint32_t &hi) {
  if (R.cnt == 0) {  // rare: a burst of draws outran the one-per-iteration refill
    mz_step(R, lo, hi);
    return;
  }
  lo = R.f[0];
  hi = R.f[1];
#pragma unroll
  for (int i = 0; i + 2 < 2 * MZ_FIFO; i++) R.f[i] = R.f[i + 2];
  R.cnt--;
}

APG_DEV uint32_t mz_next32(MzRng &R) {  // numpy next_uint32
  if (R.has32) {
    R.has32 = 0;
    return R.u32;
  }
  uint32_t lo, hi;
  mz_pop64(R, lo, hi);
  R.has32 = 1;
  R.u32 = hi;
  return lo;
}

APG_DEV double mz_next_double(MzRng &R) {  // numpy next_double: a whole output, the half-word buffer untouched
  uint32_t lo, hi;
  mz_pop64(R, lo, hi);
  return (double)((((uint64_t)hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0);
}

// rng.permutation(directions) (maze.py:33): random_interval's masked rejection on next_uint32
APG_DEV uint32_t mz_draw_perm(MzRng &R) {
  const uint32_t j3 = mz_next32(R) & 3u;
  uint32_t j2;
  do {
    j2 = mz_next32(R) & 3u;
  } while (j2 > 2u);
  const uint32_t j1 = mz_next32(R) & 1u;
  return j3 * 6u + j2 * 2u + j1;
}

struct MazeGeom {
  int h, w, ncx, ncy, cw;  // map rows / columns, odd cells per row / column, vis words per row
};

__host__ __device__ inline MazeGeom maze_geom(int h, int w) {
  MazeGeom m;
  m.h = h;
  m.w = w;
  m.ncx = (w - 1) / 2;
  m.ncy = (h - 1) / 2;
  m.cw = (m.ncx + 63) / 64;
  return m;
}

// Global scratch per maze: the carve log (<= one entry per carve plus one pad per memory phase that
// flushed, i.e. <= 2 * cells, rounded to whole 16-byte rows for the painter's loads), then the spilled
// frames (<= cells, whole chunks).
__host__ __device__ inline size_t maze_log_bytes(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (4 * cells + 64 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t maze_scratch_bytes(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (maze_log_bytes(h, w) + cells + MZ_CHUNK + 63) & ~(size_t)63;
}
// LDS per lane: vis rows, ring, log buffer
__host__ __device__ inline size_t maze_lane_lds_bytes(int h, int w) {
  const MazeGeom m = maze_geom(h, w);
  return (size_t)m.ncy * m.cw * 8 + MZ_RING + MZ_LOGBUF * 2;
}

struct MazeLane {
  uint64_t *vis;   // this lane's vis word 0 (stride L words)
  uint32_t *ring;  // this lane's ring word 0 (stride L words)
  uint32_t *logb;  // this lane's log-buffer word 0 (stride L words)
  int L;           // lanes of the workgroup (element stride)
};

APG_DEV MazeLane maze_lane_at(void *base, const MazeGeom &m, int L, int lane) {
  uint64_t *vis = reinterpret_cast<uint64_t *>(base);
  uint32_t *ring = reinterpret_cast<uint32_t *>(vis + (size_t)m.ncy * m.cw * L);
  uint32_t *logb = ring + (size_t)(MZ_RING / 4) * L;
  return MazeLane{vis + lane, ring + lane, logb + lane, L};
}

// L1-bypassing load (agent scope): a reloaded chunk may have been read before, then re-spilled
APG_DEV uint64_t mz_load_coherent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The DFS of one maze per lane.  Every lane of the wave must call it (wave-uniform memory phases);
// lanes with active == false only take part in them.  `spill` / `logg` are this maze's global scratch.
// Returns the log length in entries (pads included, even).
template <bool ONEW>
APG_DEV int maze_dfs(const Pcg64 &r0, bool active, const MazeGeom &m, double bp, const MazeLane &Z, uint8_t *spill,
                     uint32_t *logg) {
  MzRng R;
  R.s_hi = r0.s_hi;
  R.s_lo = r0.s_lo;
  R.i_hi = r0.i_hi;
  R.i_lo = r0.i_lo;
  R.has32 = r0.has32;
  R.u32 = r0.u32;
  R.cnt = 0;
#pragma unroll
  for (int i = 0; i < 2 * MZ_FIFO; i++) R.f[i] = 0u;
  const int L = Z.L;
  for (int i = 0; i < m.ncy * m.cw; i++) Z.vis[(size_t)i * L] = (active && i == 0) ? 1ULL : 0ULL;  // cell (1, 1)
  auto vis_row = [&](int cy, int k) -> uint64_t & { return Z.vis[(size_t)(cy * m.cw + k) * L]; };
  uint8_t *ring8 = reinterpret_cast<uint8_t *>(Z.ring);
  uint16_t *log16 = reinterpret_cast<uint16_t *>(Z.logb);
  // frame s lives in byte s & 3 of ring word (s >> 2) % (MZ_RING / 4); log entry n in half n & 1 of word n >> 1
  auto ring_byte = [&](int s) -> uint8_t & { return ring8[(size_t)(((s >> 2) & (MZ_RING / 4 - 1)) * L) * 4 + (s & 3)]; };
  auto log_half = [&](int n) -> uint16_t & { return log16[(size_t)((n >> 1) * L) * 2 + (n & 1)]; };

  int cx = 0, cy = 0, sp = 0, lo = 0, k = 0, lg = 0, logpos = 0;
  uint32_t from = 0, pidx = 0, perm = 0;
  bool first = true, done = !active, pend = false;
  uint32_t pd[MZ_CHUNK / 4];
#pragma unroll
  for (int i = 0; i < MZ_CHUNK / 4; i++) pd[i] = 0u;
  if (active) {
    pidx = mz_draw_perm(R);
    perm = mz_perm_of(pidx);
  }
  for (;;) {
    for (int it = 0; it < MZ_PERIOD; it++) {
      if (done) continue;
#pragma unroll
      for (int q = 0; q < MZ_FILL; q++) mz_fill(R);
      // eligible directions of the current cell: in bounds (0 < next < dims - 1) and not visited
      uint64_t rc0, rc1, ru, rd;
      const int xr = cx + 1, xl = cx - 1;
      const int yu = cy + 1 < m.ncy ? cy + 1 : cy, yd = cy > 0 ? cy - 1 : cy;
      if constexpr (ONEW) {
        rc0 = vis_row(cy, 0);
        rc1 = rc0;
        ru = vis_row(yu, 0);
        rd = vis_row(yd, 0);
      } else {
        rc0 = vis_row(cy, (xr < m.ncx ? xr : cx) >> 6);
        rc1 = vis_row(cy, (xl >= 0 ? xl : cx) >> 6);
        ru = vis_row(yu, cx >> 6);
        rd = vis_row(yd, cx >> 6);
      }
      uint32_t E = 0;
      if (xr < m.ncx && !((rc0 >> (xr & 63)) & 1ULL)) E |= 1u;
      if (xl >= 0 && !((rc1 >> (xl & 63)) & 1ULL)) E |= 2u;
      if (cy + 1 < m.ncy && !((ru >> (cx & 63)) & 1ULL)) E |= 4u;
      if (cy > 0 && !((rd >> (cx & 63)) & 1ULL)) E |= 8u;
      // the same set in permutation order, positions >= k
      uint32_t pm = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) pm |= ((E >> ((perm >> (2 * j)) & 3u)) & 1u) << j;
      pm &= (0xFu << k) & 0xFu;
      if (pm) {
        const int j = __builtin_ctz(pm);
        const uint32_t d = (perm >> (2 * j)) & 3u;
        k = j + 1;
        // first eligible branch always; later ones only if rng.random() < branching_prob (maze.py:42)
        const bool take = first || mz_next_double(R) < bp;
        if (take) {
          const int nx = cx + (d == 0u) - (d == 1u), ny = cy + (d == 2u) - (d == 3u);
          __hip_atomic_fetch_or(&vis_row(ny, nx >> 6), 1ULL << (nx & 63), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WAVEFRONT);
          log_half(lg) = (uint16_t)((uint32_t)nx | ((uint32_t)ny << 7) | (d << 14));
          lg++;
          ring_byte(sp) = (uint8_t)(pidx | (from << 5));
          sp++;
          cx = nx;
          cy = ny;
          from = d;
          first = true;
          k = 0;
          pidx = mz_draw_perm(R);
          perm = mz_perm_of(pidx);
        }
      } else if (sp == 0) {
        done = true;  // carve(starting_pos) returned
      } else if (sp > lo) {  // return to the parent frame (sp == lo: its chunk arrives at the next phase)
        sp--;
        const uint32_t fb = ring_byte(sp);
        cx -= (from == 0u) - (from == 1u);
        cy -= (from == 2u) - (from == 3u);
        pidx = fb & 31u;
        perm = mz_perm_of(pidx);
        uint32_t eq = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) eq |= (((perm >> (2 * j)) & 3u) == from ? 1u : 0u) << j;
        k = __builtin_ctz(eq) + 1;
        first = false;
        from = fb >> 5;
      }
    }
    // ---- memory phase (wave-uniform).  Everything this lane stored in the previous phase is complete
    // before any reload is issued below (vmcnt(0): issued MZ_PERIOD iterations ago, so it costs nothing).
    const bool more = __ballot(!done) != 0ULL;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const int cnt = sp - lo;
    // (a) the chunk below the ring back into it, once there is room for it and a period of pushes
    if (pend && cnt <= MZ_RING - MZ_PERIOD - MZ_CHUNK) {
      const int w0 = ((lo - MZ_CHUNK) >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 4; i++) Z.ring[(size_t)(w0 + i) * L] = pd[i];
      lo -= MZ_CHUNK;
      pend = false;
    } else if (cnt > MZ_RING - MZ_PERIOD) {
      // (b) spill the oldest chunk; it stays in registers as the chunk below the ring
      const int w0 = (lo >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 4; i++) pd[i] = Z.ring[(size_t)(w0 + i) * L];
      uint4 *dst = reinterpret_cast<uint4 *>(spill + lo);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 16; i++) dst[i] = make_uint4(pd[4 * i], pd[4 * i + 1], pd[4 * i + 2], pd[4 * i + 3]);
      lo += MZ_CHUNK;
      pend = true;
    }
    // (c) the log buffer out (dwords; an odd count is padded)
    if (lg > 0) {
      const int nw = (lg + 1) >> 1;
      if (lg & 1) log_half(lg) = (uint16_t)MZ_LOG_PAD;
#pragma unroll
      for (int i = 0; i < MZ_LOGBUF / 2; i++)
        if (i < nw) logg[(logpos >> 1) + i] = Z.logb[(size_t)i * L];
      logpos += 2 * nw;
      lg = 0;
    }
    // (d) prefetch the chunk below the ring (used at a later phase; the wait for it is the vmcnt(0) above)
    if (!pend && lo > 0) {
      const uint64_t *src = reinterpret_cast<const uint64_t *>(spill + lo - MZ_CHUNK);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 8; i++) {
        const uint64_t v = mz_load_coherent(src + i);
        pd[2 * i] = (uint32_t)v;
        pd[2 * i + 1] = (uint32_t)(v >> 32);
      }
      pend = true;
    }
    if (!more) break;
  }
  return logpos;
}

// Paint maze j's occupancy rows from its log into the wave's LDS bitmap bm[h][wpr] (all walls, then the
// start cell (1, 1), every carved cell and the passage it was entered through), wave-cooperatively.
APG_DEV void maze_paint(const MazeGeom &m, int wpr, const uint32_t *logg, int nlog, uint64_t *bm, int lane) {
  for (int i = lane; i < m.h * wpr; i += 64) {
    const int y = i / wpr, kk = i - y * wpr, lo = 64 * kk;
    uint64_t v = 0;
    if (m.w > lo) v = (m.w - lo >= 64) ? ~0ULL : ((1ULL << (m.w - lo)) - 1ULL);
    if (y == 1 && kk == 0) v &= ~2ULL;  // maze[1, 1] = 0 (maze.py:51)
    bm[i] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nq = (nlog + 7) >> 3;  // 16-byte rows of 8 entries
  const uint4 *src = reinterpret_cast<const uint4 *>(logg);
  for (int q = lane; q < nq; q += 64) {
    const uint4 v = src[q];
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint32_t e = (wv[t >> 1] >> (16 * (t & 1))) & 0xFFFFu;
      if (8 * q + t >= nlog || e == MZ_LOG_PAD) continue;
      const int x = 2 * (int)(e & 127u) + 1, y = 2 * (int)((e >> 7) & 127u) + 1;
      const uint32_t d = e >> 14;
      const int px = x - ((d == 0u) - (d == 1u)), py = y - ((d == 2u) - (d == 3u));  // passage cell
      if (py == y) {  // same row: one or two words
        const int k0 = x >> 6, k1 = px >> 6;
        if (k0 == k1) {
          __hip_atomic_fetch_and(&bm[y * wpr + k0], ~((1ULL << (x & 63)) | (1ULL << (px & 63))), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
          __hip_atomic_fetch_and(&bm[y * wpr + k0], ~(1ULL << (x & 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
          __hip_atomic_fetch_and(&bm[y * wpr + k1], ~(1ULL << (px & 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
      } else {
        __hip_atomic_fetch_and(&bm[y * wpr + (x >> 6)], ~(1ULL << (x & 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_and(&bm[py * wpr + (px >> 6)], ~(1ULL << (px & 63)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace apg
