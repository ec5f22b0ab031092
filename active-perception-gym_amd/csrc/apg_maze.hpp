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
// The DFS is VALU-issue bound at one wave per SIMD (the LDS state of 256 mazes fills a CU): every iteration
// executes the union of the carve and the return paths for its 64 lanes.  So the random numbers are not made
// there: k_maze_stream (full occupancy, one LCG jump per 256 outputs) writes each maze's PCG64 outputs ahead
// as the only bits the DFS reads of them — the two low bits of each 32-bit half (random_interval's masks
// are 3, 3, 1) and next_double() < branching_prob — 5 bits per output, and the DFS keeps the next 32 outputs
// in registers (topped up in the memory phase), reading every draw of an iteration off that window with a
// few bit operations: the permutation's rejection loop is a count of leading rejected halves.
#pragma once
#include "apg_device.hpp"
#include "apg_rng.hpp"

namespace apg {

constexpr int MZ_RING = 64;    // frames held in LDS (a multiple of MZ_CHUNK)
constexpr int MZ_CHUNK = 32;   // frames per spill / reload
constexpr int MZ_PERIOD = 16;  // DFS iterations between memory phases (ring headroom below)
constexpr int MZ_LOGBUF = 24;  // log entries buffered in LDS per lane (< 8 left over + MZ_PERIOD new)
constexpr uint32_t MZ_LOG_PAD = 0xFFFFu;  // padding entry (x = 127, resp. 63 in the ncx <= 63 format: never a cell)
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

// ---- the precomputed stream.  Group g of a maze's stream = its outputs 32g .. 32g+31:
//   H[g]  128 bits: output k's low half's two low bits at bits 4k, 4k+1, its high half's at 4k+2, 4k+3
//   D[g]  32 bits:  bit k = (output k >> 11) * 2^-53 < branching_prob (numpy next_double)
// laid out per maze as H[ng] (16 B each), D[ng], then the generator state after the ng * 32 outputs (s_hi, s_lo:
// a maze that needs more — about 1.77 outputs per cell are drawn, ng * 32 >= 1.8 per cell + 64 — steps the LCG
// from there in the memory phase).
constexpr int MZ_GROUP = 32;       // outputs per stream group
constexpr int MZ_ITEM_GROUPS = 8;  // groups per k_maze_stream item (one jump)
constexpr int MZ_MAX_ITEMS = 191;  // items per maze (+ 1 for the end state): k_maze_stream's 192 jump threads (255 x 255: 114)

__host__ __device__ inline int maze_stream_groups(int h, int w) {
  const int cells = ((w - 1) / 2) * ((h - 1) / 2);
  const int outputs = (9 * cells) / 5 + 64;
  const int per_item = MZ_GROUP * MZ_ITEM_GROUPS;
  return (outputs + per_item - 1) / per_item * MZ_ITEM_GROUPS;
}
__host__ __device__ inline size_t maze_stream_state_off(int ng) { return ((size_t)ng * 20 + 15) & ~(size_t)15; }
__host__ __device__ inline size_t maze_stream_bytes(int ng) { return maze_stream_state_off(ng) + 32; }  // + nlog

// (A, G): the state d LCG steps on is A * s + G * inc (mod 2^128), A = MUL^d, G = 1 + MUL + ... + MUL^(d-1)
struct MzJump {
  U128 A, G;
};
APG_DEV MzJump mz_jump(uint64_t d) {
  U128 am{0, 1}, ap{0, 0}, cm{PCG_MUL_HI, PCG_MUL_LO}, cp{0, 1};
  while (d) {
    if (d & 1ULL) {
      am = mul128(am, cm);
      ap = add128(mul128(ap, cm), cp);
    }
    cp = mul128(add128(cm, U128{0, 1}), cp);
    cm = mul128(cm, cm);
    d >>= 1;
  }
  return MzJump{am, ap};
}
APG_DEV void mz_jump_state(const MzJump &j, uint64_t &s_hi, uint64_t &s_lo, uint64_t i_hi, uint64_t i_lo) {
  const U128 s = add128(mul128(j.A, U128{s_hi, s_lo}), mul128(j.G, U128{i_hi, i_lo}));
  s_hi = s.hi;
  s_lo = s.lo;
}

// numpy next64 (XSL-RR of the stepped state) and its 5 stream bits
APG_DEV uint64_t mz_next64(uint64_t &s_hi, uint64_t &s_lo, uint64_t i_hi, uint64_t i_lo) {
  pcg_step(s_hi, s_lo, i_hi, i_lo);
  const uint64_t x = s_hi ^ s_lo;
  const unsigned rot = (unsigned)(s_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
APG_DEV uint32_t mz_nibble(uint64_t o) { return (uint32_t)(o & 3u) | ((uint32_t)(o >> 30) & 0xCu); }
APG_DEV uint32_t mz_dbit(uint64_t o, double bp) {
  return (double)(o >> 11) * (1.0 / 9007199254740992.0) < bp ? 1u : 0u;
}

// Item c of a maze: its groups c * MZ_ITEM_GROUPS .. + MZ_ITEM_GROUPS - 1, from the seeded state (s, inc) and
// the jump to output c * MZ_ITEM_GROUPS * MZ_GROUP.
APG_DEV void maze_stream_item(uint64_t s_hi, uint64_t s_lo, uint64_t i_hi, uint64_t i_lo, const MzJump &j, double bp,
                              int c, uint8_t *stream, int ng) {
  mz_jump_state(j, s_hi, s_lo, i_hi, i_lo);
  uint4 *H = reinterpret_cast<uint4 *>(stream) + (size_t)c * MZ_ITEM_GROUPS;
  uint32_t *D = reinterpret_cast<uint32_t *>(stream + (size_t)ng * 16) + (size_t)c * MZ_ITEM_GROUPS;
  for (int gi = 0; gi < MZ_ITEM_GROUPS; gi++) {
    uint32_t hw[4] = {0u, 0u, 0u, 0u}, dw = 0u;
#pragma unroll
    for (int k = 0; k < MZ_GROUP; k++) {
      const uint64_t o = mz_next64(s_hi, s_lo, i_hi, i_lo);
      hw[k >> 3] |= mz_nibble(o) << (4 * (k & 7));
      dw |= mz_dbit(o, bp) << k;
    }
    H[gi] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    D[gi] = dw;
  }
}

// The DFS's window: the next `avail` (<= 32) outputs of the stream, output k at bits 4k.. of h1:h0 and bit k of
// d; numpy's buffered high half (has_uint32) and its two low bits; e = stream index after the window; the two
// staged groups (e >> 5, +1) loaded one memory phase ahead; past the precomputed outputs, the generator.
struct MzWin {
  uint64_t h0, h1;
  uint32_t d;
  int avail, e;
  uint32_t has32, b2;
  uint64_t s[4];
  uint32_t sd[2];
  uint64_t ov_hi, ov_lo;
  int ov;
};

// h1:h0 >> 4p, d >> p (p in [0, 32])
APG_DEV void mz_win_shift(MzWin &W, int p) {
  const uint32_t s = 4u * (uint32_t)p, sm = s & 63u;
  const uint64_t a = W.h0 >> sm, b = W.h1 >> sm, c = (W.h1 << 1) << (63u - sm);
  W.h0 = s < 64u ? (a | c) : (s < 128u ? b : 0ULL);
  W.h1 = s < 64u ? b : 0ULL;
  W.d = p >= 32 ? 0u : W.d >> p;
  W.avail -= p;
}

// groups gq, gq + 1 of the stream into the staging registers (zeros past its end)
APG_DEV void mz_win_stage(MzWin &W, const uint8_t *stream, int ng, int gq) {
  const uint4 *H = reinterpret_cast<const uint4 *>(stream);
  const uint32_t *D = reinterpret_cast<const uint32_t *>(stream + (size_t)ng * 16);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    uint32_t dv = 0u;
    if (gq + i < ng) {
      v = H[gq + i];
      dv = D[gq + i];
    }
    W.s[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    W.s[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    W.sd[i] = dv;
  }
}

// The window topped up to 32 outputs: the staged outputs e .. (those below the precomputed end N = 32 ng),
// then outputs >= N from the generator (its state at N loaded on first use).
APG_DEV void mz_win_refill(MzWin &W, const uint8_t *stream, int ng, uint64_t i_hi, uint64_t i_lo, double bp) {
  const int need = 32 - W.avail;
  if (need <= 0) return;
  const int N = ng * MZ_GROUP;
  const uint32_t off = (uint32_t)(W.e & 31), bo = 4u * off, q = bo >> 6, r = bo & 63u;
  const uint64_t w0 = q ? W.s[1] : W.s[0], w1 = q ? W.s[2] : W.s[1], w2 = q ? W.s[3] : W.s[2];
  uint64_t t0 = (w0 >> r) | ((w1 << 1) << (63u - r)), t1 = (w1 >> r) | ((w2 << 1) << (63u - r));
  uint32_t td = (uint32_t)((((uint64_t)W.sd[1] << 32) | W.sd[0]) >> off);
  int ok = N - W.e;
  ok = ok < 0 ? 0 : (ok > need ? need : ok);
  if (ok < 32) {  // keep the staged outputs below N only
    const uint32_t kb = 4u * (uint32_t)ok;
    t0 = kb >= 64u ? t0 : t0 & ((1ULL << kb) - 1ULL);
    t1 = kb >= 64u ? t1 & ((1ULL << (kb - 64u)) - 1ULL) : 0ULL;
    td &= (1u << ok) - 1u;
  }
  // append at output `avail`: (t1:t0) << 4 avail, td << avail
  const uint32_t a = 4u * (uint32_t)W.avail, am = a & 63u;
  W.h0 |= a < 64u ? t0 << am : 0ULL;
  W.h1 |= a < 64u ? ((t1 << am) | ((t0 >> 1) >> (63u - am))) : (a < 128u ? t0 << am : 0ULL);
  W.d |= W.avail < 32 ? td << W.avail : 0u;
  for (int k = ok; k < need; k++) {  // past the precomputed stream (rare)
    if (!W.ov) {
      const uint64_t *st = reinterpret_cast<const uint64_t *>(stream + maze_stream_state_off(ng));
      W.ov_hi = st[0];
      W.ov_lo = st[1];
      W.ov = 1;
    }
    const uint64_t o = mz_next64(W.ov_hi, W.ov_lo, i_hi, i_lo);
    const int pos = W.avail + k;
    const uint64_t nib = (uint64_t)mz_nibble(o);
    if (pos < 16) W.h0 |= nib << (4 * pos);
    else W.h1 |= nib << (4 * (pos - 16));
    W.d |= mz_dbit(o, bp) << pos;
  }
  W.e += need;
  W.avail = 32;
}

// rng.permutation(directions) (maze.py:33) read off the window after `u0` outputs (the double drawn before
// it): numpy's shuffle draws j3 = random_interval(3), j2 = random_interval(2) (rejecting 3), j1 =
// random_interval(1), each from next_uint32 (the buffered half first) masked to 2 / 2 / 1 bits.
struct MzPerm {
  uint32_t pidx;
  int p;     // outputs consumed
  int q;     // halves taken from outputs (odd: the last output's high half is buffered)
  bool ok;   // the window holds the draw
};
APG_DEV MzPerm mz_perm_draw(const MzWin &W, uint64_t hs, int u0) {
  const uint64_t X = W.has32 ? ((hs << 2) | W.b2) : hs;  // half i (S_i) at bits 2i, 2i+1
  const uint64_t rejected = X & (X >> 1) & 0x5555555555555554ULL;  // bit 2i: S_i == 3 (i >= 1)
  const uint64_t kept = ~rejected & 0x5555555555555554ULL;
  const int i2 = (int)(__builtin_ctzll(kept | (1ULL << 62)) >> 1);  // first S_i != 3 (31: none up to 30)
  const int t = i2 + 2;                                             // halves drawn
  const int ic = i2 > 30 ? 30 : i2;
  MzPerm r;
  r.pidx = ((uint32_t)X & 3u) * 6u + ((uint32_t)(X >> (2 * ic)) & 3u) * 2u + ((uint32_t)(X >> (2 * ic + 2)) & 1u);
  r.q = t - (int)W.has32;
  r.p = (r.q + 1) >> 1;
  const int valid = 2 * (W.avail - u0) + (int)W.has32;  // halves of X from the window
  r.ok = t <= (valid < 32 ? valid : 32);
  return r;
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
// the spilled frames (<= cells, whole chunks), the precomputed stream (maze_stream_groups groups at most).
__host__ __device__ inline size_t maze_log_bytes(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (2 * cells + 16 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t maze_stream_off(int h, int w) {
  const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
  return (maze_log_bytes(h, w) + cells + MZ_CHUNK + 15) & ~(size_t)15;
}
// Mazes with more than 127 odd cells per row or column (maps wider or taller than 255; up to 511): their DFS state
// does not fit the LDS layout below, so k_maze_big carves them one thread per maze with the visited bits
// (u64 [ncy][cw]) and the frame stack (u32 per frame) in this scratch, writing the occupancy rows directly.
__host__ __device__ inline bool maze_big(int h, int w) { return (w - 1) / 2 > 127 || (h - 1) / 2 > 127; }
__host__ __device__ inline size_t maze_big_vis_bytes(int h, int w) {
  return ((size_t)((h - 1) / 2) * (size_t)(((w - 1) / 2 + 63) / 64) * 8 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t maze_scratch_bytes(int h, int w) {
  if (maze_big(h, w)) {
    const size_t cells = (size_t)((w - 1) / 2) * ((h - 1) / 2);
    return (maze_big_vis_bytes(h, w) + 4 * (cells + 1) + 63) & ~(size_t)63;
  }
  return (maze_stream_off(h, w) + maze_stream_bytes(maze_stream_groups(h, w)) + 63) & ~(size_t)63;
}

// LDS of one k_maze workgroup (always laid out for 64 lanes, so every stride is a compile-time immediate):
//   [0, 512)        the permutation table (maze_table_init)
//   MZ_V            visited rows, u64 [rows][cw][64 lanes], with the bits of columns >= ncx set (the column
//                   bounds cost nothing).  Mazes of ncx <= 63 (one word per row, maze_dfs_rows) also have an
//                   all-visited pad row below row 0 and above row ncy - 1, so the row bounds cost nothing
//                   either; wider mazes (maze_dfs_words) bound rows with two compares
//   ring, log       u32 [MZ_RING / 4][64], u32 [MZ_LOGBUF / 2][64]
// 127 x 127 (ncy = 63): 512 + 65 * 512 + 4096 + 3072 = 40960 B, four one-wave workgroups per CU.
constexpr int MZ_LANES = 64, MZ_V = 512;
__host__ __device__ inline bool maze_onew(const MazeGeom &m) { return m.ncx <= 63; }
__host__ __device__ inline int maze_row_bytes(const MazeGeom &m) { return m.cw * 8 * MZ_LANES; }
__host__ __device__ inline int maze_vis_off(const MazeGeom &m) {  // row 0
  return MZ_V + (maze_onew(m) ? maze_row_bytes(m) : 0);
}
__host__ __device__ inline int maze_ring_off(const MazeGeom &m) {
  return MZ_V + (m.ncy + (maze_onew(m) ? 2 : 0)) * maze_row_bytes(m);
}
__host__ __device__ inline int maze_log_off(const MazeGeom &m) { return maze_ring_off(m) + MZ_RING * MZ_LANES; }
__host__ __device__ inline size_t maze_wg_lds_bytes(int h, int w) {
  const MazeGeom m = maze_geom(h, w);
  return (size_t)maze_log_off(m) + MZ_LOGBUF * 2 * MZ_LANES;
}

// The permutation table (thread t < 32 writes entry t; the caller synchronizes).
// ONEW (maze_dfs_rows): entry c = j3 | j2 << 2 | j1 << 4 (the shuffle's three draws; j2 = 3 never occurs) holds
//   x, y  for each visited mask V (bit 0: column - 1, bit 1: row + 1, bit 2: column + 1, bit 3: row - 1) the
//         unvisited permutation positions, 4 bits at bits 4V..
//   z     the permutation (direction of position k at bits 2k)
//   w     for each direction r the positions after r's, (0xF << (position of r + 1)) & 0xF at bits 4r (where a
//         frame resumes when its child r returns)
// otherwise (maze_dfs_words): entry pidx = j3 * 6 + j2 * 2 + j1 holds the map "eligible directions (by
//   direction) -> eligible positions" as 16 nibbles, then the permutation | its inverse << 8.
template <bool ONEW>
APG_DEV void maze_table_init(char *lds, int t) {
  uint4 *e = reinterpret_cast<uint4 *>(lds) + t;
  if constexpr (ONEW) {
    if (t >= 32) return;
    const uint32_t j3 = t & 3, j2 = (t >> 2) & 3, j1 = t >> 4;
    if (j2 == 3) {
      *e = make_uint4(0u, 0u, 0u, 0u);
      return;
    }
    const uint32_t perm = mz_perm_of(j3 * 6 + j2 * 2 + j1);
    constexpr uint32_t vbit[4] = {2, 0, 1, 3};  // direction (+x, -x, +y, -y) -> bit of the visited mask
    uint64_t pm = 0;
    for (uint32_t V = 0; V < 16; V++) {
      uint32_t v = 0;
      for (int j = 0; j < 4; j++) v |= (((V >> vbit[(perm >> (2 * j)) & 3u]) & 1u) ^ 1u) << j;
      pm |= (uint64_t)v << (4 * V);
    }
    uint32_t after = 0;
    for (int j = 0; j < 4; j++) after |= ((0xFu << (j + 1)) & 0xFu) << (4 * ((perm >> (2 * j)) & 3u));
    *e = make_uint4((uint32_t)pm, (uint32_t)(pm >> 32), perm, after);
  } else {
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
    *e = make_uint4((uint32_t)pm, (uint32_t)(pm >> 32), perm | (inv << 8), 0u);
  }
}

// L1-bypassing load (agent scope): a reloaded chunk may have been read before, then re-spilled
APG_DEV uint64_t mz_load_coherent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The DFS's frame stack and carve log outside the iterations: frames sp - 1 .. lo in the LDS ring (older ones
// spilled, the chunk below the ring in pd when pend), lg entries in the LDS log buffer, logpos flushed.
struct MzStack {
  int sp, lo, lg, logpos;
  bool pend;
  uint32_t pd[MZ_CHUNK / 4];
};

// The wave-uniform memory phase between MZ_PERIOD iterations: window refill, ring spill / reload, log flush,
// prefetch of the chunk below the ring, the next stream groups staged.  Everything this lane stored in the previous
// phase is complete before any reload is issued (vmcnt(0): issued MZ_PERIOD iterations ago).
// U16LOG: the log buffer holds entry e of this lane at logb + e * 2 * MZ_LANES (maze_dfs_rows); otherwise two
// entries per lane dword, dword i at logb + i * 4 * MZ_LANES.
template <bool U16LOG>
APG_DEV void maze_memory_phase(MzWin &W, MzStack &K, bool done, bool more, const uint8_t *stream, int ng,
                               const Pcg64 &r0, double bp, char *ring, char *logb, uint8_t *spill, uint32_t *logg) {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (!done) mz_win_refill(W, stream, ng, r0.i_hi, r0.i_lo, bp);  // the staged groups into the window
  const int cnt = K.sp - K.lo;
  uint32_t *ringw = reinterpret_cast<uint32_t *>(ring);
  // (a) the chunk below the ring back into it, once there is room for it and a period of pushes
  if (K.pend && cnt <= MZ_RING - MZ_PERIOD - MZ_CHUNK) {
    const int w0 = ((K.lo - MZ_CHUNK) >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
    for (int i = 0; i < MZ_CHUNK / 4; i++) ringw[(w0 + i) * MZ_LANES] = K.pd[i];
    K.lo -= MZ_CHUNK;
    K.pend = false;
  } else if (cnt > MZ_RING - MZ_PERIOD) {
    // (b) spill the oldest chunk; it stays in registers as the chunk below the ring
    const int w0 = (K.lo >> 2) & (MZ_RING / 4 - 1);
#pragma unroll
    for (int i = 0; i < MZ_CHUNK / 4; i++) K.pd[i] = ringw[(w0 + i) * MZ_LANES];
    uint4 *dst = reinterpret_cast<uint4 *>(spill + K.lo);
#pragma unroll
    for (int i = 0; i < MZ_CHUNK / 16; i++)
      dst[i] = make_uint4(K.pd[4 * i], K.pd[4 * i + 1], K.pd[4 * i + 2], K.pd[4 * i + 3]);
    K.lo += MZ_CHUNK;
    K.pend = true;
  }
  // (c) the log buffer out in whole groups of 8 entries (16-byte stores); the rest moves to the front.
  // After the last period the tail is padded to a whole group.
  auto entry = [&](int e) -> uint16_t & {
    return *reinterpret_cast<uint16_t *>(U16LOG ? logb + e * (2 * MZ_LANES) : logb + (e >> 1) * (4 * MZ_LANES) + (e & 1) * 2);
  };
  if (!more && (K.lg & 7)) {
    for (int e = K.lg; e < ((K.lg + 7) & ~7); e++) entry(e) = (uint16_t)MZ_LOG_PAD;
    K.lg = (K.lg + 7) & ~7;
  }
  if (K.lg >= 8) {
    const int g = K.lg >> 3;  // groups: 1..3
    uint4 *dst = reinterpret_cast<uint4 *>(logg) + (K.logpos >> 3);
    if constexpr (U16LOG) {
      auto group = [&](int q) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = (uint32_t)entry(8 * q + 2 * i) | ((uint32_t)entry(8 * q + 2 * i + 1) << 16);
        dst[q] = make_uint4(w[0], w[1], w[2], w[3]);
      };
      group(0);
      if (g > 1) group(1);
      if (g > 2) group(2);
      // the leftover (< 8 entries) to the front
#pragma unroll
      for (int i = 0; i < 7; i++) {
        const int src = 8 * g + i;
        if (src < MZ_LOGBUF) entry(i) = entry(src);
      }
    } else {
      uint32_t *logw = reinterpret_cast<uint32_t *>(logb);  // log dword i at logw[i * MZ_LANES]
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
    }
    K.logpos += 8 * g;
    K.lg -= 8 * g;
  }
  // (d) prefetch the chunk below the ring (used at a later phase; the wait for it is the vmcnt(0) above)
  if (!K.pend && K.lo > 0) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(spill + K.lo - MZ_CHUNK);
#pragma unroll
    for (int i = 0; i < MZ_CHUNK / 8; i++) {
      const uint64_t v = mz_load_coherent(src + i);
      K.pd[2 * i] = (uint32_t)v;
      K.pd[2 * i + 1] = (uint32_t)(v >> 32);
    }
    K.pend = true;
  }
  if (!done) mz_win_stage(W, stream, ng, W.e >> 5);  // the groups after the window, for the next phase
}

// The first window (a synchronous load), the groups after it staged, and the start cell's permutation (drawn
// fresh: no buffered half).  Returns false when the draw does not fit a full window (never in practice).
APG_DEV bool maze_dfs_start(MzWin &W, const Pcg64 &r0, const uint8_t *stream, int ng, double bp, uint32_t &pidx) {
  mz_win_stage(W, stream, ng, 0);
  mz_win_refill(W, stream, ng, r0.i_hi, r0.i_lo, bp);
  mz_win_stage(W, stream, ng, W.e >> 5);
  const MzPerm pr = mz_perm_draw(W, W.h0, 0);
  if (!pr.ok) return false;
  pidx = pr.pidx;
  W.has32 = (uint32_t)(pr.q & 1);
  W.b2 = W.has32 ? (uint32_t)(W.h0 >> (4 * (pr.p - 1) + 2)) & 3u : 0u;
  mz_win_shift(W, pr.p);
  return true;
}

// maze_dfs for mazes of ncx <= 63 (one visited word per row; every maze up to 127 x 127).  The iteration is
// issue-bound (one wave per SIMD: one instruction per 4 cycles), so it is written for the fewest instructions:
//  * the cell is one index pos = cy * 64 + cx; a move adds {+1, -1, +64, -64}[direction] (a byte table);
//  * the rows the next iteration tests (row cy and column cx's words of rows cy +- 1; pad rows stand in for
//    rows -1 and ncy) are read right after this iteration's move and carve, so their LDS latency overlaps the
//    rest of the iteration; the parent frame is read at the top, the table entries of both possible next frames
//    (parent, drawn child) as soon as their indices are known;
//  * log entries are pos | direction << 13 (cy <= 126: 13 bits of pos), buffered as one u16 per lane and entry;
//  * the body is straight-line (selects; the long-permutation fallback, probability < 4^-14 per draw, is the only
//    lane-divergent branch): the wave executes every path any lane takes.  Loop-carried flags are integers.
template <bool BP1>
APG_DEV int maze_dfs_rows(const Pcg64 &r0, const uint8_t *stream, int ng, bool active, const MazeGeom &m, double bp,
                          char *lds, int lane, uint8_t *spill, uint32_t *logg, bool &bad) {
  constexpr int RB = 8 * MZ_LANES;                    // bytes per vis row (all lanes)
  constexpr uint32_t MZ_DELTA = 0xC040FF01u;          // direction (+x, -x, +y, -y) -> pos delta (int8 each)
  MzWin W{};
  char *vis = lds + maze_vis_off(m) + lane * 8;       // row 0 of this lane; rows -1 and ncy are the pads
  char *ring = lds + maze_ring_off(m) + lane * 4;
  char *logb = lds + maze_log_off(m) + lane * 2;      // entry e at logb + e * 2 * MZ_LANES
  const uint64_t pad = m.ncx >= 64 ? 0ULL : ~((1ULL << m.ncx) - 1ULL);
  for (int r = -1; r <= m.ncy; r++)
    *reinterpret_cast<uint64_t *>(vis + r * RB) = (r < 0 || r == m.ncy) ? ~0ULL : (r == 0 ? pad | 1ULL : pad);
  const uint4 *tab = reinterpret_cast<const uint4 *>(lds);

  MzStack K{};
  int pos = 0;
  // frame = code | from << 5 (the ring byte); rflag / rchild: the frame was just returned to from child
  // direction rchild (its resume positions come from its table entry, read at the end of the iteration)
  uint32_t done = active ? 0u : 1u, badf = 0u, first = 1u, frame = 0u, kmask = 0xFu, rflag = 0u, rchild = 0u;
  uint64_t Rc = pad | 1ULL;                              // row cy
  uint32_t Wu = m.ncy > 1 ? (uint32_t)pad : ~0u, Wd = ~0u;  // column cx's word of rows cy + 1, cy - 1
  if (active) {
    uint32_t pidx = 0;
    if (maze_dfs_start(W, r0, stream, ng, bp, pidx)) {
      frame = (pidx / 6u) | (((pidx % 6u) >> 1) << 2) | ((pidx & 1u) << 4);
    } else {
      bad = true;
      done = 1u;
    }
  }
  uint4 T = tab[frame];  // the current frame's table entry
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing in flight at the loop entry
  for (;;) {
    for (int it = 0; it < MZ_PERIOD; it++) {
      // ---- the parent frame (slot sp - 1), for a return
      const int ps = K.sp - 1;
      const uint32_t fb = (uint8_t)ring[((ps >> 2) & (MZ_RING / 4 - 1)) * (4 * MZ_LANES) + (ps & 3)];
      // ---- visited mask of the neighbours: columns cx - 1 .. cx + 1 of row cy (a 64-bit rotation by cx - 1;
      // column -1 is the pad bit 63), column cx of rows cy +- 1
      const int cx = pos & 63;
      const uint32_t n = (uint32_t)(cx - 1);  // cx = 0: 0xFFFFFFFF, the rotation by 63
      const bool nlo = n < 32u;
      const uint32_t rc = __builtin_amdgcn_alignbit(nlo ? (uint32_t)(Rc >> 32) : (uint32_t)Rc,
                                                    nlo ? (uint32_t)Rc : (uint32_t)(Rc >> 32), n);
      // 4 * the visited mask: the nibble of the table's map
      const uint32_t V4 = ((rc & 5u) << 2) | (__builtin_amdgcn_ubfe(Wu, (uint32_t)pos, 1u) << 3) |
                          (__builtin_amdgcn_ubfe(Wd, (uint32_t)pos, 1u) << 5);
      // ---- the unvisited permutation positions not tried yet, the first one, its direction
      kmask = rflag ? __builtin_amdgcn_ubfe(T.w, 4u * rchild, 4u) : kmask;
      const uint32_t pm = (uint32_t)((((uint64_t)T.y << 32) | T.x) >> V4) & kmask;
      const uint32_t j = (uint32_t)__builtin_ctz(pm | 0x10u);
      const uint32_t d = (T.z >> (2u * j)) & 3u;
      // ---- the draws (maze.py:42, 33): rng.random() when the branch is not the frame's first (always below
      // branching_prob >= 1: BP1), then the child's permutation from the outputs after it.  X = the halves
      // next_uint32 returns (the buffered one first).
      const uint32_t hasE = pm != 0u ? 1u : 0u;
      const uint32_t dneed = hasE & (first ^ 1u);
      const uint32_t want = BP1 ? hasE : hasE & (first | (W.d & 1u));
      const uint64_t hs = W.h0 >> (4u * dneed);
      const uint64_t X = (hs << (2u * W.has32)) | W.b2;
      const uint32_t xl = (uint32_t)X;
      const uint32_t kept = ~(xl & (xl >> 1)) & 0x55555554u;  // bit 2i (i >= 1): half i is not 3
      uint32_t i2x2, j21;
      if (__builtin_expect(kept != 0u, 1)) {
        i2x2 = (uint32_t)__builtin_ctz(kept);
        j21 = __builtin_amdgcn_alignbit((uint32_t)(X >> 32), xl, i2x2) & 7u;
      } else {  // 15 rejected halves: the rest of X
        const uint64_t k64 = ~(X & (X >> 1)) & 0x5555555555555554ULL;
        i2x2 = (uint32_t)__builtin_ctzll(k64 | (1ULL << 62));
        j21 = (uint32_t)(X >> i2x2) & 7u;
      }
      const uint32_t q = (i2x2 >> 1) + 2u - W.has32;  // halves taken from outputs
      const uint32_t p = (q + 1u) >> 1;               // outputs
      const uint32_t nhas = q & 1u;
      const uint32_t nb2 = nhas ? (uint32_t)(hs >> (4u * p - 2u)) & 3u : 0u;
      const int lim = W.avail < 15 ? W.avail : 15;  // a draw must fit the window (and its 64-bit X)
      const int need = (int)(dneed + (want ? p : 0u));
      const uint32_t go = (done == 0u && need <= lim) ? 1u : 0u;
      // a permutation of > 28 rejected halves (never in practice): the maze is abandoned and reported
      const uint32_t stuck = (go | done) == 0u && W.avail >= 15 ? 1u : 0u;
      badf |= stuck;
      done |= stuck;
      const uint32_t carve = want & go;
      const uint32_t ret = go & (hasE ^ 1u) & (K.sp > K.lo ? 1u : 0u);  // sp == lo > 0: parent chunk not back yet
      done |= go & (hasE ^ 1u) & (K.sp == 0 ? 1u : 0u);                  // carve(starting_pos) returned
      // ---- the window past this iteration's draws
      {
        const int used = go ? need : 0;
        const uint32_t s = 4u * (uint32_t)used;
        W.h0 = (W.h0 >> s) | ((W.h1 << 1) << (63u - s));
        W.h1 >>= s;
        if constexpr (!BP1) W.d >>= used;
        W.avail -= used;
      }
      W.has32 = carve ? nhas : W.has32;
      W.b2 = carve ? nb2 : W.b2;
      // ---- one move: into d (carve), or back against the entry direction (return); the carve's LDS writes,
      // issued unconditionally (without a carve: the frame byte lands in the free slot above the top, the visited
      // word is OR-ed with 0, the log entry lands in the free entry lg)
      const uint32_t from = frame >> 5;
      const uint32_t mv = carve ? d : (from ^ 1u);
      pos += (carve | ret) ? __builtin_amdgcn_sbfe((int)MZ_DELTA, 8u * mv, 8u) : 0;
      char *row = vis + (pos >> 6) * RB;
      char *wrow = row + ((pos >> 3) & 4);  // column cx's word
      ring[((K.sp >> 2) & (MZ_RING / 4 - 1)) * (4 * MZ_LANES) + (K.sp & 3)] = (char)frame;
      __hip_atomic_fetch_or(reinterpret_cast<uint32_t *>(wrow), carve << (pos & 31), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WAVEFRONT);
      *reinterpret_cast<uint16_t *>(logb + K.lg * (2 * MZ_LANES)) = (uint16_t)((uint32_t)pos | (d << 13));
      K.lg += (int)carve;
      K.sp += carve ? 1 : (ret ? -1 : 0);
      // ---- the next frame: the child (fresh), the parent (resumes after the child's position: rflag), or this
      // one (after a skipped branch, BP1 never: the positions after j)
      kmask = carve ? 0xFu : ((!BP1 && (go & hasE)) ? (0x1Eu << j) & 0xFu : kmask);
      rflag = ret;
      rchild = from;
      {  // (a bit blend: a select chain here compiles to lane-divergent branches)
        const uint32_t mc = 0u - carve, mr = 0u - ret;
        frame = (mc & ((j21 << 2) | (xl & 3u) | (d << 5))) | (mr & fb) | (~(mc | mr) & frame);
      }
      first = (carve | ret) ? carve : first;
      // ---- the next iteration's rows (after the carve's visited bit) and table entry
      Rc = *reinterpret_cast<const uint64_t *>(row);
      Wu = *reinterpret_cast<const uint32_t *>(wrow + RB);
      Wd = *reinterpret_cast<const uint32_t *>(wrow - RB);
      T = tab[frame & 31u];
    }
    const bool more = __ballot(done == 0u) != 0ULL;
    maze_memory_phase<true>(W, K, done != 0u, more, stream, ng, r0, bp, ring, logb, spill, logg);
    if (!more) break;
  }
  if (badf) bad = true;
  return K.logpos;
}

// maze_dfs for mazes of ncx > 63 (cw visited words per row): the current cell's rows are read from LDS each
// iteration, the row bounds are two compares.  Same iteration as maze_dfs_rows otherwise (pidx table entries).
APG_DEV int maze_dfs_words(const Pcg64 &r0, const uint8_t *stream, int ng, bool active, const MazeGeom &m, double bp,
                           char *lds, int lane, uint8_t *spill, uint32_t *logg, bool &bad) {
  MzWin W{};
  const int CW = m.cw;
  const int RB = CW * 8 * MZ_LANES;  // bytes per vis row (all lanes)
  char *vis = lds + maze_vis_off(m) + lane * 8;
  char *ring = lds + maze_ring_off(m) + lane * 4;
  char *logb = lds + maze_log_off(m) + lane * 4;
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

  MzStack K{};
  int cx = 0, cy = 0, k = 0;
  int arow = 0;  // byte offset of the current cell's vis row
  uint32_t from = 0, pidx = 0, pinfo = 0;
  uint64_t pmt = 0;
  bool first = true, done = !active;
  auto load_perm = [&](uint32_t p) {
    const uint4 t = tab[p];
    pmt = (uint64_t)t.x | ((uint64_t)t.y << 32);
    pinfo = t.z;
  };
  if (active) {
    if (maze_dfs_start(W, r0, stream, ng, bp, pidx)) {
      load_perm(pidx);
    } else {
      bad = true;
      done = true;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing in flight at the loop entry
  for (;;) {
    for (int it = 0; it < MZ_PERIOD; it++) {
      if (done) continue;
      // eligible directions of the current cell: in bounds (pad bits, row compares) and not visited
      const uint64_t *vr = reinterpret_cast<const uint64_t *>(vis + arow);
      const int wc = CW * MZ_LANES, kx = cx >> 6, kr = (cx + 1) >> 6, kl = (cx - 1) >> 6;
      const uint64_t ru = ~vr[(cy + 1 < m.ncy ? wc : 0) + kx * MZ_LANES], rd = ~vr[(cy > 0 ? -wc : 0) + kx * MZ_LANES];
      const uint64_t rr = ~vr[(kr < CW ? kr : kx) * MZ_LANES], rl = ~vr[(cx > 0 ? kl : kx) * MZ_LANES];
      const uint32_t E = ((uint32_t)(rr >> ((cx + 1) & 63)) & (uint32_t)(kr < CW) & 1u) |
                         (((uint32_t)(rl >> ((cx - 1) & 63)) & (uint32_t)(cx > 0) & 1u) << 1) |
                         (((uint32_t)(ru >> (cx & 63)) & (uint32_t)(cy + 1 < m.ncy) & 1u) << 2) |
                         (((uint32_t)(rd >> (cx & 63)) & (uint32_t)(cy > 0) & 1u) << 3);
      // the eligible permutation positions >= k
      const uint32_t pm = (uint32_t)(pmt >> (4 * E)) & (0xFu << k) & 0xFu;
      const int j = __builtin_ctz(pm | 0x10u);
      const uint32_t d = (pinfo >> (2 * j)) & 3u;
      // first eligible branch always; later ones only if rng.random() < branching_prob (maze.py:42): the
      // window's next output; a carve then draws the child's permutation from the outputs after it.  An
      // iteration whose draws are not all in the window waits for the next memory phase (go == false).
      const bool dneed = pm != 0u && !first;
      const bool want = pm != 0u && (first || (W.d & 1u) != 0u);
      const int u0 = dneed ? 1 : 0;
      const uint64_t hs = dneed ? ((W.h0 >> 4) | (W.h1 << 60)) : W.h0;
      const MzPerm pr = mz_perm_draw(W, hs, u0);
      const int need = u0 + (want ? pr.p : 0);
      const bool go = need <= W.avail && (!want || pr.ok);
      if (!go && W.avail == 32) {  // a permutation of > 30 rejected halves: abandoned, reported
        bad = true;
        done = true;
      }
      const bool carve = want && go;
      const bool back = go && pm == 0u && K.sp > K.lo;  // sp == lo > 0: the parent's chunk arrives at the next phase
      done = done || (go && pm == 0u && K.sp == 0);     // carve(starting_pos) returned
      W.has32 = carve ? (uint32_t)(pr.q & 1) : W.has32;
      W.b2 = carve ? (uint32_t)(hs >> (4 * (pr.p - 1) + 2)) & 3u : W.b2;
      mz_win_shift(W, go ? need : 0);
      k = go && pm != 0u ? j + 1 : k;
      // one move: into d, or back against the entry direction
      const bool move = carve || back;
      const uint32_t mv = carve ? d : (from ^ 1u);
      const int dx = move ? (mv == 0u) - (mv == 1u) : 0, dy = move ? (mv == 2u) - (mv == 3u) : 0;
      cx += dx;
      cy += dy;
      arow += dy * RB;
      const int slot = carve ? K.sp : K.sp - 1;
      char *rb = ring + ((slot >> 2) & (MZ_RING / 4 - 1)) * (4 * MZ_LANES) + (slot & 3);
      // the carve's three LDS writes, issued unconditionally (see maze_dfs_rows)
      char *wb = ring + ((K.sp >> 2) & (MZ_RING / 4 - 1)) * (4 * MZ_LANES) + (K.sp & 3);
      const uint32_t fb = (uint8_t)*rb;  // the parent frame (used on a return)
      *wb = (char)(pidx | (from << 5));
      __hip_atomic_fetch_or(reinterpret_cast<uint64_t *>(vis + arow + (cx >> 6) * 8 * MZ_LANES),
                            carve ? 1ULL << (cx & 63) : 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      *reinterpret_cast<uint16_t *>(logb + (K.lg >> 1) * (4 * MZ_LANES) + (K.lg & 1) * 2) =
          (uint16_t)((uint32_t)cx | ((uint32_t)cy << 7) | (d << 14));
      K.lg += carve ? 1 : 0;
      K.sp += carve ? 1 : (back ? -1 : 0);
      const uint32_t child = from;
      pidx = carve ? pr.pidx : (back ? fb & 31u : pidx);
      from = carve ? d : (back ? fb >> 5 : from);
      first = move ? carve : first;
      load_perm(pidx);  // (the same entry again when nothing moved)
      k = carve ? 0 : (back ? (int)((pinfo >> (8 + 2 * child)) & 3u) + 1 : k);
    }
    const bool more = __ballot(!done) != 0ULL;
    maze_memory_phase<false>(W, K, done, more, stream, ng, r0, bp, ring, logb, spill, logg);
    if (!more) break;
  }
  return K.logpos;
}

// The DFS of one maze per lane.  Every lane of the wave must call it (wave-uniform memory phases); lanes
// with active == false only take part in them.  `lds` is the workgroup's dynamic LDS (maze_table_init<ONEW>
// done), `spill` / `logg` / `stream` this maze's global scratch (16-byte aligned; the stream of ng groups written
// by k_maze_stream), r0 the maze's seeded generator (its increment steps the LCG past the stream).  ONEW: ncx
// <= 63.  Returns the log length in entries (a multiple of 8, the tail padded); `bad` is set when a draw does
// not fit in a full window (a permutation of ~30 rejected halves: never in practice) and that maze is abandoned.
template <bool ONEW>
APG_DEV int maze_dfs(const Pcg64 &r0, const uint8_t *stream, int ng, bool active, const MazeGeom &m, double bp,
                     char *lds, int lane, uint8_t *spill, uint32_t *logg, bool &bad) {
  if constexpr (ONEW) {
    if (bp >= 1.0) return maze_dfs_rows<true>(r0, stream, ng, active, m, bp, lds, lane, spill, logg, bad);
    return maze_dfs_rows<false>(r0, stream, ng, active, m, bp, lds, lane, spill, logg, bad);
  }
  else return maze_dfs_words(r0, stream, ng, active, m, bp, lds, lane, spill, logg, bad);
}

// Paint a maze's occupancy rows from its log into the LDS bitmap bm[h][wpr] (all walls, then the start cell
// (1, 1), every carved cell and the passage it was entered through) by NT cooperating threads t: one wave
// (NT = 64, wave fences) or a workgroup (__syncthreads).
template <int NT = 64>
APG_DEV void maze_paint(const MazeGeom &m, int wpr, const uint32_t *logg, int nlog, uint64_t *bm, int lane) {
  auto sync = [] {
    if constexpr (NT == 64) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      __syncthreads();
    }
  };
  for (int i = lane; i < m.h * wpr; i += NT) {
    const int y = i / wpr, kk = i - y * wpr, lo = 64 * kk;
    uint64_t v = 0;
    if (m.w > lo) v = (m.w - lo >= 64) ? ~0ULL : ((1ULL << (m.w - lo)) - 1ULL);
    if (y == 1 && kk == 0) v &= ~2ULL;  // maze[1, 1] = 0 (maze.py:51)
    bm[i] = v;
  }
  sync();
  const int nq = (nlog + 7) >> 3;  // 16-byte rows of 8 entries
  const uint4 *src = reinterpret_cast<const uint4 *>(logg);
  constexpr auto scope = NT == 64 ? __HIP_MEMORY_SCOPE_WAVEFRONT : __HIP_MEMORY_SCOPE_WORKGROUP;
#pragma unroll 4
  for (int q = lane; q < nq; q += NT) {  // unrolled: four rows' loads in flight before their atomics
    const uint4 v = src[q];
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint32_t e = (wv[t >> 1] >> (16 * (t & 1))) & 0xFFFFu;
      if (8 * q + t >= nlog || e == MZ_LOG_PAD) continue;
      // entries: cx | cy << 7 | d << 14 (maze_dfs_words), pos | d << 13 with pos = cy * 64 + cx (maze_dfs_rows)
      const bool onew = maze_onew(m);
      const int x = 2 * (int)(e & (onew ? 63u : 127u)) + 1, y = 2 * (int)((e >> (onew ? 6 : 7)) & 127u) + 1;
      const uint32_t d = (e >> (onew ? 13 : 14)) & 3u;
      const int px = x - ((d == 0u) - (d == 1u)), py = y - ((d == 2u) - (d == 3u));  // passage cell
      if (py == y) {  // same row: one or two words
        const int k0 = x >> 6, k1 = px >> 6;
        if (k0 == k1) {
          __hip_atomic_fetch_and(&bm[y * wpr + k0], ~((1ULL << (x & 63)) | (1ULL << (px & 63))), __ATOMIC_RELAXED, scope);
        } else {
          __hip_atomic_fetch_and(&bm[y * wpr + k0], ~(1ULL << (x & 63)), __ATOMIC_RELAXED, scope);
          __hip_atomic_fetch_and(&bm[y * wpr + k1], ~(1ULL << (px & 63)), __ATOMIC_RELAXED, scope);
        }
      } else {
        __hip_atomic_fetch_and(&bm[y * wpr + (x >> 6)], ~(1ULL << (x & 63)), __ATOMIC_RELAXED, scope);
        __hip_atomic_fetch_and(&bm[py * wpr + (px >> 6)], ~(1ULL << (px & 63)), __ATOMIC_RELAXED, scope);
      }
    }
  }
  sync();
}

// Words of the row-major linear bitmap bitmap_map_obs builds (bit c = cell c = y * w + x), + 1 zero word.
__host__ __device__ inline int bitmap_lin_words(int h, int w) { return (h * w + 63) / 64 + 1; }

// The f32 map observation of a painted bitmap (bool map / 255, lidar_localization2d.py:299) into dst[h * w],
// by NT cooperating threads (t = 0 .. NT - 1, NT >= 8; the caller synchronizes NT = 64 as a wave, NT > 64 with
// __syncthreads around the call).  The bitmap's rows are first re-laid as one row-major bit string in `lin`
// (bitmap_lin_words; cells c .. c + 3 are then four consecutive bits, read by 16 lanes at once), then the
// 16-byte-aligned body of the map's floats goes out in 16-byte non-temporal stores (4 cells each; a wave-store of
// dwords per row left the kernel store-issue bound), the unaligned head and tail in scalar stores.
template <int NT = 64>
APG_DEV void bitmap_map_obs(const uint64_t *bm, int h, int w, int wpr, float *dst, int lane, uint64_t *lin) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const float wall = 1.0f / 255.0f;
  const int cells = h * w, nlin = bitmap_lin_words(h, w);
  // bits [x, x + k) (k <= 64) of row y
  auto row_bits = [&](int y, int x, int k) -> uint64_t {
    const uint64_t *r = bm + y * wpr;
    const int q = x >> 6, o = x & 63;
    const uint64_t lo = r[q], hi = q + 1 < wpr ? r[q + 1] : 0ULL;
    const uint64_t v = (lo >> o) | ((hi << 1) << (63 - o));
    return k >= 64 ? v : v & ((1ULL << k) - 1ULL);
  };
  for (int i = lane; i < nlin; i += NT) {
    uint64_t v = 0;
    int c = 64 * i;
    if (c < cells) {
      int y = c / w, x = c - y * w, filled = 0;
      while (filled < 64 && y < h) {
        const int k = min(64 - filled, w - x);
        v |= row_bits(y, x, k) << filled;
        filled += k;
        x = 0;
        y++;
      }
    }
    lin[i] = v;
  }
  if constexpr (NT == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
  const int head = (int)(((16u - ((unsigned)(uintptr_t)dst & 15u)) & 15u) >> 2);  // floats before a 16-B boundary
  const int nbody = (cells - head) >> 2;
  for (int q = lane; q < nbody; q += NT) {
    const int c = head + 4 * q, wi = c >> 6;
    const uint32_t o = (uint32_t)c & 63u;
    const uint32_t nib = (uint32_t)((lin[wi] >> o) | ((lin[wi + 1] << 1) << (63u - o))) & 15u;
    f4 v;
    v.x = (nib & 1u) ? wall : 0.0f;
    v.y = (nib & 2u) ? wall : 0.0f;
    v.z = (nib & 4u) ? wall : 0.0f;
    v.w = (nib & 8u) ? wall : 0.0f;
    __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(dst + head) + q);
  }
  const int tail0 = head + 4 * nbody;
  if (lane < head || (lane >= 4 && lane - 4 < cells - tail0)) {
    const int c = lane < head ? lane : tail0 + lane - 4;
    dst[c] = ((lin[c >> 6] >> (c & 63)) & 1ULL) ? wall : 0.0f;
  }
}

}  // namespace apg
