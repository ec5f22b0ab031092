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
//            global per-maze log in whole 16-byte groups in the memory phase.  After the DFS the wave
//            paints each maze's occupancy rows from its log in an LDS bitmap and writes them out coalesced.
// One iteration checks the current frame: it carves (the first eligible direction from position k on,
// after its rng.random() draw when it is not the frame's first carve) or returns to the parent frame, both
// as one "move" (a return is a move against the entry direction): 2 * cells - 1 iterations for a perfect
// maze, each with one LDS round trip for the current cell's three neighbour rows.
//
// The kernel is VALU-issue bound at one wave per SIMD (the LDS state of 256 mazes fills a CU): every
// iteration executes the union of the carve and the return paths for its 64 lanes, so the paths are kept
// branch-light (the permutation draw is a window over the queued random words, not a rejection loop).
#pragma once
#include "apg_device.hpp"

namespace apg {

constexpr int MZ_RING = 64;    // frames held in LDS (a multiple of MZ_CHUNK)
constexpr int MZ_CHUNK = 32;   // frames per spill / reload
constexpr int MZ_PERIOD = 16;  // DFS iterations between memory phases (ring headroom below)
constexpr int MZ_LOGBUF = 24;  // log entries buffered in LDS per lane (< 8 left over + MZ_PERIOD new)
constexpr uint32_t MZ_LOG_PAD = 0xFFFFu;  // padding entry (x = 127 is never a cell: ncx <= 127)
static_assert(MZ_RING - MZ_PERIOD - MZ_CHUNK >= 0, "ring headroom");
static_assert(MZ_LOGBUF >= 7 + MZ_PERIOD && MZ_LOGBUF % 8 == 0, "log buffer: leftover group + one period");

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
// ahead into a small register FIFO: the DFS loop produces MZ_FILL outputs per iteration in uniform control
// flow, and the draw sites (rng.random(), the permutation's next_uint32 calls) only take from the FIFO.
// Without it a wave executed the 128-bit LCG step once per draw site any of its lanes reached (up to five
// per iteration).  The outputs are consumed in the same order, so the draws are unchanged.  A DFS iteration
// consumes 0.88 outputs on average but up to ~3 on a forward run: one fill per iteration leaves lanes short
// on 26 % of the iterations of a 127 x 127 maze, two fills into 4 slots on 0.03 % (tools/maze_fifo_sim.py);
// a short lane steps the LCG inline.
constexpr int MZ_FIFO = 4, MZ_FILL = 2;
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

// drop the front p (0..MZ_FIFO) outputs: two conditional shifts
APG_DEV void mz_drop(MzRng &R, int p) {
  if (p & 2) {
#pragma unroll
    for (int i = 0; i < 2 * MZ_FIFO - 4; i++) R.f[i] = R.f[i + 4];
  }
  if (p & 1) {
#pragma unroll
    for (int i = 0; i < 2 * MZ_FIFO - 2; i++) R.f[i] = R.f[i + 2];
  }
  R.cnt -= p;
}

APG_DEV void mz_pop64(MzRng &R, uint32_t &lo, uint32_t &hi) {
  if (R.cnt == 0) {  // rare: a burst of draws outran the refill
    mz_step(R, lo, hi);
    return;
  }
  lo = R.f[0];
  hi = R.f[1];
  mz_drop(R, 1);
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

// rng.permutation(directions) (maze.py:33): random_interval's masked rejection on next_uint32, reference form
APG_DEV uint32_t mz_draw_perm_loop(MzRng &R) {
  const uint32_t j3 = mz_next32(R) & 3u;
  uint32_t j2;
  do {
    j2 = mz_next32(R) & 3u;
  } while (j2 > 2u);
  const uint32_t j1 = mz_next32(R) & 1u;
  return j3 * 6u + j2 * 2u + j1;
}

// The same draw read off the window of queued next_uint32 values S = [buffered half?] f0lo f0hi f1lo ...
// without a loop: j3 = S0, j2 = the first of S1.. whose two low bits are not 3, j1 = the value after it.
// Falls back to the loop when the window does not hold the draw (> 5 rejections, or a short FIFO).
APG_DEV uint32_t mz_draw_perm(MzRng &R) {
  uint32_t S[2 * MZ_FIFO + 1];
  S[0] = R.has32 ? R.u32 : R.f[0];
#pragma unroll
  for (int i = 1; i < 2 * MZ_FIFO + 1; i++) S[i] = R.has32 ? R.f[i - 1] : (i < 2 * MZ_FIFO ? R.f[i] : 0u);
  const int avail = (int)R.has32 + 2 * R.cnt;
  uint32_t rej = 0;  // bit i - 1: S_i rejected (low bits 3), i = 1..6
#pragma unroll
  for (int i = 1; i <= 6; i++) rej |= ((S[i] & 3u) == 3u ? 1u : 0u) << (i - 1);
  const int i2 = 1 + __builtin_ctz(~rej);  // position of j2
  const int t = i2 + 2;                    // next_uint32 values consumed
  if (i2 > 6 || t > avail) return mz_draw_perm_loop(R);
  uint32_t s2 = S[1], s1 = S[2];
#pragma unroll
  for (int i = 2; i <= 6; i++) {
    s2 = i2 == i ? S[i] : s2;
    s1 = i2 == i ? S[i + 1] : s1;
  }
  const uint32_t j3 = S[0] & 3u, j2 = s2 & 3u, j1 = s1 & 1u;
  // consume t values: the buffered half first, then outputs (an output whose high half is left over is
  // buffered)
  const int q = t - (int)R.has32, p = (q + 1) >> 1;
  uint32_t hi_last = R.f[1];
#pragma unroll
  for (int i = 2; i <= MZ_FIFO; i++) hi_last = p == i ? R.f[2 * i - 1] : hi_last;
  R.has32 = (uint32_t)(q & 1);
  R.u32 = hi_last;
  mz_drop(R, p);
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

// Global scratch per maze: the carve log (one entry per carve, padded to whole 16-byte groups at the end),
// then the spilled frames (<= cells, whole chunks).
__host__ __device__ inline size_t maze_log_bytes(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (2 * cells + 16 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t maze_scratch_bytes(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (maze_log_bytes(h, w) + cells + MZ_CHUNK + 63) & ~(size_t)63;
}

// LDS of one k_maze workgroup (always laid out for 64 lanes, so every stride is a compile-time immediate):
//   [0, 512)        the permutation table: per index 16 B = the map "eligible directions (4 bits, by
//                   direction) -> eligible positions (4 bits, by permutation position)" as 16 nibbles, then
//                   the permutation (2 bits per position) | its inverse << 8
//   MZ_V            visited rows, u64 [ncy][cw][64 lanes], with the bits of columns >= ncx set (the
//                   column bounds cost nothing; the row bounds are two compares)
//   ring, log       u32 [MZ_RING / 4][64], u32 [MZ_LOGBUF / 2][64]
constexpr int MZ_LANES = 64, MZ_V = 512;
__host__ __device__ inline int maze_row_bytes(const MazeGeom &m) { return m.cw * 8 * MZ_LANES; }
__host__ __device__ inline int maze_ring_off(const MazeGeom &m) { return MZ_V + m.ncy * maze_row_bytes(m); }
__host__ __device__ inline int maze_log_off(const MazeGeom &m) { return maze_ring_off(m) + MZ_RING * MZ_LANES; }
__host__ __device__ inline size_t maze_wg_lds_bytes(int h, int w) {
  const MazeGeom m = maze_geom(h, w);
  return (size_t)maze_log_off(m) + MZ_LOGBUF * 2 * MZ_LANES;
}

// the permutation table (thread t < 24 writes entry t; the caller synchronizes)
APG_DEV void maze_table_init(char *lds, int t) {
  if (t >= 24) return;
  const uint32_t perm = mz_perm_of((uint32_t)t);
  uint32_t inv = 0;
  uint64_t pm = 0;
  for (int j = 0; j < 4; j++) inv |= (uint32_t)j << (2 * ((perm >> (2 * j)) & 3u));
  for (uint32_t E = 0; E < 16; E++) {
    uint32_t v = 0;
    for (int j = 0; j < 4; j++) v |= ((E >> ((perm >> (2 * j)) & 3u)) & 1u) << j;
    pm |= (uint64_t)v << (4 * E);
  }
  uint4 *e = reinterpret_cast<uint4 *>(lds) + t;
  *e = make_uint4((uint32_t)pm, (uint32_t)(pm >> 32), perm | (inv << 8), 0u);
}

// L1-bypassing load (agent scope): a reloaded chunk may have been read before, then re-spilled
APG_DEV uint64_t mz_load_coherent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The DFS of one maze per lane.  Every lane of the wave must call it (wave-uniform memory phases); lanes
// with active == false only take part in them.  `lds` is the workgroup's dynamic LDS (table initialized),
// `spill` / `logg` this maze's global scratch (16-byte aligned).  ONEW: ncx <= 63 (one vis word per row,
// the left neighbour of column 0 reads the pad bit 63).  Returns the log length in entries (a multiple of
// 8, the tail padded).
template <bool ONEW>
APG_DEV int maze_dfs(const Pcg64 &r0, bool active, const MazeGeom &m, double bp, char *lds, int lane, uint8_t *spill,
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
  const int CW = ONEW ? 1 : m.cw;
  const int RB = CW * 8 * MZ_LANES;  // bytes per vis row (all lanes)
  char *vis = lds + MZ_V + lane * 8;
  char *ring = lds + maze_ring_off(m) + lane * 4;
  char *logb = lds + maze_log_off(m) + lane * 4;
  uint32_t *logw = reinterpret_cast<uint32_t *>(logb);  // log dword i at logw[i * MZ_LANES]
  // visited rows: pad bits of the columns >= ncx, cell (1, 1) visited
  for (int r = 0; r < m.ncy; r++)
    for (int kk = 0; kk < CW; kk++) {
      const int lo = 64 * kk;
      uint64_t v = ~0ULL;
      if (m.ncx > lo) v = m.ncx - lo >= 64 ? 0ULL : ~((1ULL << (m.ncx - lo)) - 1ULL);
      if (r == 0 && kk == 0) v |= 1ULL;
      *reinterpret_cast<uint64_t *>(vis + r * RB + kk * 8 * MZ_LANES) = v;
    }
  const uint4 *tab = reinterpret_cast<const uint4 *>(lds);

  int cx = 0, cy = 0, sp = 0, lo = 0, k = 0, lg = 0, logpos = 0;
  int arow = 0;  // byte offset of the current cell's vis row
  uint32_t from = 0, pidx = 0, pinfo = 0;
  uint64_t pmt = 0;
  bool first = true, done = !active, pend = false;
  uint32_t pd[MZ_CHUNK / 4];
#pragma unroll
  for (int i = 0; i < MZ_CHUNK / 4; i++) pd[i] = 0u;
  auto load_perm = [&](uint32_t p) {
    const uint4 t = tab[p];
    pmt = (uint64_t)t.x | ((uint64_t)t.y << 32);
    pinfo = t.z;
  };
  if (active) {
    pidx = mz_draw_perm_loop(R);
    load_perm(pidx);
  }
  for (;;) {
    for (int it = 0; it < MZ_PERIOD; it++) {
      if (done) continue;
#pragma unroll
      for (int q = 0; q < MZ_FILL; q++) mz_fill(R);
      // eligible directions of the current cell: in bounds (pad bits, row compares) and not visited
      const uint64_t *vr = reinterpret_cast<const uint64_t *>(vis + arow);
      uint32_t E;
      if constexpr (ONEW) {
        // rows -1 and ncy read other LDS (the table / the ring): masked by the compares
        const uint64_t rc = ~vr[0], ru = ~vr[MZ_LANES], rd = ~vr[-MZ_LANES];
        E = (uint32_t)((rc >> ((cx + 1) & 63)) & 1ULL) | ((uint32_t)((rc >> ((cx - 1) & 63)) & 1ULL) << 1) |
            ((uint32_t)(cy + 1 < m.ncy && ((ru >> cx) & 1ULL)) << 2) | ((uint32_t)(cy > 0 && ((rd >> cx) & 1ULL)) << 3);
      } else {
        const int wc = CW * MZ_LANES, kx = cx >> 6, kr = (cx + 1) >> 6, kl = (cx - 1) >> 6;
        const uint64_t ru = ~vr[(cy + 1 < m.ncy ? wc : 0) + kx * MZ_LANES], rd = ~vr[(cy > 0 ? -wc : 0) + kx * MZ_LANES];
        const uint64_t rr = ~vr[(kr < CW ? kr : kx) * MZ_LANES], rl = ~vr[(cx > 0 ? kl : kx) * MZ_LANES];
        E = (uint32_t)(kr < CW && ((rr >> ((cx + 1) & 63)) & 1ULL)) |
            ((uint32_t)(cx > 0 && ((rl >> ((cx - 1) & 63)) & 1ULL)) << 1) |
            ((uint32_t)(cy + 1 < m.ncy && ((ru >> (cx & 63)) & 1ULL)) << 2) |
            ((uint32_t)(cy > 0 && ((rd >> (cx & 63)) & 1ULL)) << 3);
      }
      // the eligible permutation positions >= k
      const uint32_t pm = (uint32_t)(pmt >> (4 * E)) & (0xFu << k) & 0xFu;
      const int j = __builtin_ctz(pm | 0x10u);
      const uint32_t d = (pinfo >> (2 * j)) & 3u;
      // first eligible branch always; later ones only if rng.random() < branching_prob (maze.py:42)
      bool carve = pm != 0u;
      if (carve && !first) carve = mz_next_double(R) < bp;
      if (pm != 0u) k = j + 1;
      const bool back = pm == 0u && sp > lo;  // sp == lo > 0: the parent's chunk arrives at the next phase
      if (pm == 0u && sp == 0) done = true;   // carve(starting_pos) returned
      if (carve || back) {
        // one move: into d, or back against the entry direction
        const uint32_t mv = carve ? d : (from ^ 1u);
        const int dx = (mv == 0u) - (mv == 1u), dy = (mv == 2u) - (mv == 3u);
        cx += dx;
        cy += dy;
        arow += dy * RB;
        const int slot = carve ? sp : sp - 1;
        char *rb = ring + ((slot >> 2) & (MZ_RING / 4 - 1)) * (4 * MZ_LANES) + (slot & 3);
        uint32_t np, nfrom;
        if (carve) {
          *rb = (char)(pidx | (from << 5));
          __hip_atomic_fetch_or(reinterpret_cast<uint64_t *>(vis + arow + (cx >> 6) * 8 * MZ_LANES), 1ULL << (cx & 63),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
          *reinterpret_cast<uint16_t *>(logb + (lg >> 1) * (4 * MZ_LANES) + (lg & 1) * 2) =
              (uint16_t)((uint32_t)cx | ((uint32_t)cy << 7) | (d << 14));
          lg++;
          np = mz_draw_perm(R);
          nfrom = d;
        } else {
          const uint32_t fb = (uint8_t)*rb;
          np = fb & 31u;
          nfrom = fb >> 5;
        }
        sp += carve ? 1 : -1;
        const uint32_t child = from;
        pidx = np;
        from = nfrom;
        first = carve;
        load_perm(np);
        k = carve ? 0 : (int)((pinfo >> (8 + 2 * child)) & 3u) + 1;  // the child's position + 1
      }
    }
    // ---- memory phase (wave-uniform).  Everything this lane stored in the previous phase is complete
    // before any reload is issued below (vmcnt(0): issued MZ_PERIOD iterations ago).
    const bool more = __ballot(!done) != 0ULL;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const int cnt = sp - lo;
    uint32_t *ringw = reinterpret_cast<uint32_t *>(ring);
    // (a) the chunk below the ring back into it, once there is room for it and a period of pushes
    if (pend && cnt <= MZ_RING - MZ_PERIOD - MZ_CHUNK) {
      const int w0 = ((lo - MZ_CHUNK) >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 4; i++) ringw[(w0 + i) * MZ_LANES] = pd[i];
      lo -= MZ_CHUNK;
      pend = false;
    } else if (cnt > MZ_RING - MZ_PERIOD) {
      // (b) spill the oldest chunk; it stays in registers as the chunk below the ring
      const int w0 = (lo >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 4; i++) pd[i] = ringw[(w0 + i) * MZ_LANES];
      uint4 *dst = reinterpret_cast<uint4 *>(spill + lo);
#pragma unroll
      for (int i = 0; i < MZ_CHUNK / 16; i++) dst[i] = make_uint4(pd[4 * i], pd[4 * i + 1], pd[4 * i + 2], pd[4 * i + 3]);
      lo += MZ_CHUNK;
      pend = true;
    }
    // (c) the log buffer out in whole groups of 8 entries (16-byte stores); the rest moves to the front.
    // After the last period the tail is padded to a whole group.
    if (!more && (lg & 7)) {
      for (int e = lg; e < ((lg + 7) & ~7); e++)
        *reinterpret_cast<uint16_t *>(logb + (e >> 1) * (4 * MZ_LANES) + (e & 1) * 2) = (uint16_t)MZ_LOG_PAD;
      lg = (lg + 7) & ~7;
    }
    if (lg >= 8) {
      const int g = lg >> 3;  // groups: 1..3
      uint4 *dst = reinterpret_cast<uint4 *>(logg) + (logpos >> 3);
      dst[0] = make_uint4(logw[0], logw[MZ_LANES], logw[2 * MZ_LANES], logw[3 * MZ_LANES]);
      if (g > 1) dst[1] = make_uint4(logw[4 * MZ_LANES], logw[5 * MZ_LANES], logw[6 * MZ_LANES], logw[7 * MZ_LANES]);
      if (g > 2) dst[2] = make_uint4(logw[8 * MZ_LANES], logw[9 * MZ_LANES], logw[10 * MZ_LANES], logw[11 * MZ_LANES]);
      // the leftover (< 8 entries = 4 dwords) to the front
      const int w0 = 4 * g;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t v = logw[(w0 + i < MZ_LOGBUF / 2 ? w0 + i : 0) * MZ_LANES];
        if (w0 + i < MZ_LOGBUF / 2) logw[i * MZ_LANES] = v;
      }
      logpos += 8 * g;
      lg -= 8 * g;
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
#pragma unroll 4
  for (int q = lane; q < nq; q += 64) {  // unrolled: four rows' loads in flight before their atomics
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

// The f32 map observation of a painted bitmap (bool map / 255, lidar_localization2d.py:299) into dst[h * w],
// wave-cooperatively: 16-byte non-temporal stores over the 16-byte-aligned body of the map's floats (a
// wave-store of dwords per row left the kernel store-issue bound), scalar stores for the unaligned head and
// tail.  Cell c = y * w + x of float4 q is found once per store and then stepped (row wrap).
APG_DEV void bitmap_map_obs(const uint64_t *bm, int h, int w, int wpr, float *dst, int lane) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const float wall = 1.0f / 255.0f;
  const int cells = h * w;
  const int head = (int)(((16u - ((unsigned)(uintptr_t)dst & 15u)) & 15u) >> 2);  // floats before a 16-B boundary
  const int nbody = (cells - head) >> 2;
  const float invw = 1.0f / (float)w;
  auto cell_of = [&](int c, int &y, int &x) {
    y = (int)((float)c * invw);
    if (y * w > c) y--;
    if ((y + 1) * w <= c) y++;
    x = c - y * w;
  };
  auto bit = [&](int y, int x) { return (uint32_t)(bm[y * wpr + (x >> 6)] >> (x & 63)) & 1u; };
  for (int q = lane; q < nbody; q += 64) {
    int y, x;
    cell_of(head + 4 * q, y, x);
    f4 v;
    float *vv = reinterpret_cast<float *>(&v);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      vv[i] = bit(y, x) ? wall : 0.0f;
      x++;
      const bool wrap = x >= w;
      x = wrap ? 0 : x;
      y += wrap ? 1 : 0;
    }
    __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(dst + head) + q);
  }
  const int tail0 = head + 4 * nbody;
  if (lane < head || (lane >= 4 && lane - 4 < cells - tail0)) {
    const int c = lane < head ? lane : tail0 + lane - 4;
    int y, x;
    cell_of(c, y, x);
    dst[c] = bit(y, x) ? wall : 0.0f;
  }
}

}  // namespace apg
