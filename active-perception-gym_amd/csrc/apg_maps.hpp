// apg_maps.hpp — rooms floor maps on device, one GPU thread per map, bit-exact with
//   FloorMapDatasetRooms.get_data_point  ap_gym/envs/floor_map/floor_map_dataset_rooms.py:25-89
// (mazes: apg_maze.hpp)
// Occupancy is bit-packed: row y of a map is `wpr` uint64 words, bit x%64 of word x/64 set = wall.
// Bits at x >= width are always zero.
#pragma once
#include "apg_binom_table.hpp"
#include "apg_device.hpp"

namespace apg {

constexpr int ROOMS_MAX = 64;  // max_rooms of the generator (binomial draws of n = mrl - 2 < ROOMS_MAX)
struct BinomTable {  // random_binomial_inversion constants for n = 0..ROOMS_MAX-1 at p = 0.3 (host libm)
  double qn[ROOMS_MAX];
  int32_t bound[ROOMS_MAX];
  double p, q;
};
// In constant memory (tools/gen_binom_table.py): 784 bytes no kernel carries as an argument
static __constant__ BinomTable c_binom = {{APG_BINOM_QN}, {APG_BINOM_BOUND}, APG_BINOM_P, APG_BINOM_Q};

APG_DEV int64_t binomial_inv(Pcg64 &r, int64_t n, const BinomTable &bt) {
  if (n == 0) return 0;
  const double p = bt.p, q = bt.q, qn = bt.qn[n];
  const int64_t bound = bt.bound[n];
  int64_t X = 0;
  double px = qn;
  double U = next_double(r);
  while (U > px) {
    X++;
    if (X > bound) {
      X = 0;
      px = qn;
      U = next_double(r);
    } else {
      U = __dsub_rn(U, px);
      px = __ddiv_rn(__dmul_rn(__dmul_rn((double)(n - X + 1), p), px), __dmul_rn((double)X, q));
    }
  }
  return X;
}

APG_DEV int64_t pyfloordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
  return q;
}

// Working storage of the rooms generator, strided so that a workgroup can interleave its threads'
// copies in LDS ([index][thread], conflict-free) or a thread can point it at private arrays (stride 1):
// the task stack, the capacities and sizes of the current split, distribute_integers' cut points, and
// the output primitives prim[0] = nw | nd << 8, prim[1 + i] walls, prim[1 + maxw + i] doors (i < maxw =
// max_rooms - 1: every split adds k - 1 walls and doors to the k rooms it makes of one).
struct RoomsWork {
  uint64_t *stk;
  int16_t *cap, *size, *cut;
  uint32_t *prim;
  int st;       // element stride
  int stk_cap;  // stack capacity
  int maxw;     // walls (= doors) the primitives hold
  APG_DEV uint64_t &S(int i) const { return stk[i * st]; }
  APG_DEV int16_t &C(int i) const { return cap[i * st]; }
  APG_DEV int16_t &Z(int i) const { return size[i * st]; }
  APG_DEV int16_t &K(int i) const { return cut[i * st]; }
  APG_DEV uint32_t &P(int i) const { return prim[i * st]; }
};
constexpr int ROOMS_PRIM_WORDS = 33;  // 17 rooms (the fused step kernel's LDS layout)
__host__ __device__ constexpr int rooms_prim_words(int max_rooms) { return 1 + 2 * (max_rooms - 1); }

// distribute_integers(n, k) (rooms.py:36-40) with k <= ROOMS_MAX, n < 2^15: out(i) for i < k
template <class Out>
APG_DEV void distribute_integers(Pcg64 &r, int64_t n, int k, const RoomsWork &W, Out out) {
  const int64_t nz = k > n ? k - n : 0;
  const int64_t pop = nz + (n > 1 ? n - 1 : 0);
  const int kk = k - 1;
  // Generator.choice(pop, kk, replace=False): Floyd's algorithm, then _shuffle_int(kk, 1)
  for (int64_t j = pop - kk; j < pop; j++) {
    int64_t val = (int64_t)bounded_u64(r, (uint64_t)j);
    int idx = (int)(j - (pop - kk));
    bool found = false;
    for (int t = 0; t < idx; t++) found |= (W.K(t) == val);
    W.K(idx) = (int16_t)(found ? j : val);
  }
  for (int i = kk - 1; i >= 1; i--) {
    int jj = (int)bounded_u64(r, (uint64_t)i);
    const int16_t t = W.K(jj);
    W.K(jj) = W.K(i);
    W.K(i) = t;
  }
  for (int i = 0; i < kk; i++) {  // r[idx], then sorted (insertion sort)
    const int c = W.K(i);
    W.K(i) = (int16_t)(c < nz ? 0 : c - nz + 1);
  }
  for (int i = 1; i < kk; i++) {
    const int16_t v = W.K(i);
    int j = i - 1;
    while (j >= 0 && W.K(j) > v) {
      W.K(j + 1) = W.K(j);
      j--;
    }
    W.K(j + 1) = v;
  }
  int64_t prev = 0;
  for (int i = 0; i < kk; i++) {
    const int c = W.K(i);
    out(i) = (int16_t)(c - prev);
    prev = c;
  }
  out(kk) = (int16_t)(n - prev);
}

struct Bits {  // bit-packed rows in global memory
  uint64_t *w;
  int wpr;
  APG_DEV bool get(int y, int x) const { return (w[y * wpr + (x >> 6)] >> (x & 63)) & 1ULL; }
  APG_DEV void set(int y, int x) { w[y * wpr + (x >> 6)] |= 1ULL << (x & 63); }
  APG_DEV void clr(int y, int x) { w[y * wpr + (x >> 6)] &= ~(1ULL << (x & 63)); }
};

// Rooms: a view task is numpy's room[...] slice: element (i, j) is map cell
//   t == 0: (y0 + i, x0 + j)      t == 1: (y0 + j, x0 + i)
// Task and primitive encodings, narrow (the fused step kernel's generator: maps <= 128, <= 17 rooms; its code
// is register-sensitive) or wide (k_lidar_reset / k_map_generate_rooms: maps up to 511):
//   task  narrow y0 | x0 << 8 | t << 16 | n0 << 17 | n1 << 25 | max_rooms << 33
//         wide   y0 | x0 << 9 | t << 18 | n0 << 19 | n1 << 28 | max_rooms << 37
//   wall  narrow vertical << 31 | fixed << 16 | start << 8 | len;  wide vertical << 31 | fixed << 18 | start << 9 | len
//         the cells (fixed, start .. start + len) of a row (vertical = 0) or column
//   door  narrow r0 << 24 | c0 << 16 | hh << 8 | ww;  wide r0 << 23 | c0 << 14 | vertical << 13 | dw
//         the block of rows [r0, r0 + hh) and columns [c0, c0 + ww): (hh, ww) = (2 dw - 1, dw) across a row wall,
//         (dw, 2 dw - 1) across a column wall (dw = door_width; a door needs dw < m / 2)
// The final transpose flips a wall's `vertical` and swaps a door's rows and columns.
struct Wall {
  bool vertical;
  int fixed, start, len;
};
struct Door {
  int r0, c0, hh, ww;
};
template <bool WIDE>
struct RoomsFmt;
template <>
struct RoomsFmt<false> {
  static APG_DEV uint64_t task(int y0, int x0, int t, int n0, int n1, int mr) {
    return (uint64_t)y0 | ((uint64_t)x0 << 8) | ((uint64_t)t << 16) | ((uint64_t)n0 << 17) | ((uint64_t)n1 << 25) |
           ((uint64_t)mr << 33);
  }
  static APG_DEV void untask(uint64_t tk, int &y0, int &x0, int &t, int &n0, int &n1, int &mr) {
    y0 = (int)(tk & 255);
    x0 = (int)((tk >> 8) & 255);
    t = (int)((tk >> 16) & 1);
    n0 = (int)((tk >> 17) & 255);
    n1 = (int)((tk >> 25) & 255);
    mr = (int)((tk >> 33) & 255);
  }
  static APG_DEV uint32_t wall(uint32_t v, int fixed, int start, int len) {
    return (v << 31) | ((uint32_t)fixed << 16) | ((uint32_t)start << 8) | (uint32_t)len;
  }
  static APG_DEV Wall wall_of(uint32_t wl) {
    return {(wl >> 31) != 0u, (int)((wl >> 16) & 255u), (int)((wl >> 8) & 255u), (int)(wl & 255u)};
  }
  static APG_DEV uint32_t door(uint32_t v, int r0, int c0, int dw) {
    const uint32_t span = (uint32_t)(2 * dw - 1), w = (uint32_t)dw;
    return ((uint32_t)r0 << 24) | ((uint32_t)c0 << 16) | ((v ? w : span) << 8) | (v ? span : w);
  }
  static APG_DEV Door door_of(uint32_t d) {
    return {(int)(d >> 24), (int)((d >> 16) & 255u), (int)((d >> 8) & 255u), (int)(d & 255u)};
  }
  static APG_DEV uint32_t door_t(uint32_t d) {
    return (((d >> 16) & 255u) << 24) | (((d >> 24) & 255u) << 16) | ((d & 255u) << 8) | ((d >> 8) & 255u);
  }
};
template <>
struct RoomsFmt<true> {
  static APG_DEV uint64_t task(int y0, int x0, int t, int n0, int n1, int mr) {
    return (uint64_t)y0 | ((uint64_t)x0 << 9) | ((uint64_t)t << 18) | ((uint64_t)n0 << 19) | ((uint64_t)n1 << 28) |
           ((uint64_t)mr << 37);
  }
  static APG_DEV void untask(uint64_t tk, int &y0, int &x0, int &t, int &n0, int &n1, int &mr) {
    y0 = (int)(tk & 511);
    x0 = (int)((tk >> 9) & 511);
    t = (int)((tk >> 18) & 1);
    n0 = (int)((tk >> 19) & 511);
    n1 = (int)((tk >> 28) & 511);
    mr = (int)((tk >> 37) & 255);
  }
  static APG_DEV uint32_t wall(uint32_t v, int fixed, int start, int len) {
    return (v << 31) | ((uint32_t)fixed << 18) | ((uint32_t)start << 9) | (uint32_t)len;
  }
  static APG_DEV Wall wall_of(uint32_t wl) {
    return {(wl >> 31) != 0u, (int)((wl >> 18) & 511u), (int)((wl >> 9) & 511u), (int)(wl & 511u)};
  }
  static APG_DEV uint32_t door(uint32_t v, int r0, int c0, int dw) {
    return ((uint32_t)r0 << 23) | ((uint32_t)c0 << 14) | (v << 13) | (uint32_t)dw;
  }
  static APG_DEV Door door_of(uint32_t d) {
    const bool v = (d >> 13) & 1u;
    const int dw = (int)(d & 8191u);
    return {(int)(d >> 23), (int)((d >> 14) & 511u), v ? dw : 2 * dw - 1, v ? 2 * dw - 1 : dw};
  }
  static APG_DEV uint32_t door_t(uint32_t d) {
    return door(((d >> 13) & 1u) ^ 1u, (int)((d >> 14) & 511u), (int)(d >> 23), (int)(d & 8191u));
  }
};

// The reference paints walls (`room[wp] = where(room[wp] != -1, 1, -1)`) and doors (`= -1`) into an
// int8 map in task order, then maps -1 to free.  A cell ends up a wall iff it is on the border or
// covered by some wall segment, and covered by no door block: paint order never matters.  So the
// generator only records the segments and blocks (in map coordinates, W.P) and paints rows at the
// end, with the final 50% transpose applied to the primitives instead of the bitmap.
template <bool WIDE>
APG_DEV int rooms_primitives(Pcg64 &r, int m, int max_rooms, int door_width, const BinomTable &bt,
                             const RoomsWork &W) {
  const int min_size = door_width + 2;
  int nw = 0, nd = 0;
  int sp = 0;
  W.P(0) = 0u;
  using F = RoomsFmt<WIDE>;
  W.S(sp++) = F::task(1, 1, 0, m - 2, m - 2, max_rooms);
  while (sp > 0) {
    const uint64_t tk = W.S(--sp);
    int y0, x0, t, n0, n1, mr;
    F::untask(tk, y0, x0, t, n0, n1, mr);
    int64_t mrl = pyfloordiv(n0 - min_size, min_size + 1) + 1;
    if (mr < mrl) mrl = mr;
    if (mrl <= 1) continue;
    if (mrl > ROOMS_MAX) return -2;  // the binomial table: mrl - 2 < ROOMS_MAX
    const int k = (int)binomial_inv(r, mrl - 2, bt) + 2;
    distribute_integers(r, mrl, k, W, [&](int i) -> int16_t & { return W.C(i); });
    distribute_integers(r, n0 - (int64_t)k * (1 + min_size) + 1, k, W, [&](int i) -> int16_t & { return W.Z(i); });
    // sizes += min_size; room i spans view rows [starts[i], ends[i]] with ends[i] = acc_i - 1,
    // starts[i] = acc_{i-1} + 1 (starts[0] = 0), acc_i = sum_{j <= i} (sizes[j] + 1)
    for (int i = 0; i < k; i++) W.Z(i) = (int16_t)(W.Z(i) + min_size);
    if (nw + k - 1 > W.maxw) return -4;
    int acc = (int)W.Z(0) + 1;
    for (int i = 1; i < k; i++) {
      const int wp = acc;  // starts[i] - 1
      acc += (int)W.Z(i) + 1;
      const int dp = (int)integers(r, 0, n1 - door_width);
      if (wp - (door_width - 1) < 0 || wp + (door_width - 1) >= n0 || dp + door_width > n1) return -3;
      // wall: the whole view row wp; door: view rows wp-dw+1 .. wp+dw-1, columns dp .. dp+dw-1
      const int lo = wp - (door_width - 1);
      if (t == 0) {
        W.P(1 + nw++) = F::wall(0u, y0 + wp, x0, n1);
        W.P(1 + W.maxw + nd++) = F::door(0u, y0 + lo, x0 + dp, door_width);
      } else {
        W.P(1 + nw++) = F::wall(1u, x0 + wp, y0, n1);
        W.P(1 + W.maxw + nd++) = F::door(1u, y0 + dp, x0 + lo, door_width);
      }
    }
    // children room[s:e+1].T, depth-first in order => push in reverse (acc = acc_{k-1} here)
    if (sp + k > W.stk_cap) return -4;
    for (int i = k - 1; i >= 0; i--) {
      const int acc_prev = acc - ((int)W.Z(i) + 1);
      int64_t s = i == 0 ? 0 : acc_prev + 1, e = acc;  // starts[i], ends[i] + 1
      acc = acc_prev;
      if (e > n0) e = n0;
      if (s > n0) s = n0;
      const int cy0 = t ? y0 : y0 + (int)s, cx0 = t ? x0 + (int)s : x0;
      W.S(sp++) = F::task(cy0, cx0, 1 - t, n1, (int)(e - s), (int)W.C(i));
    }
  }
  if (integers(r, 0, 2) == 0) {  // map_int = map_int.T: transpose the primitives
    for (int i = 0; i < nw; i++) W.P(1 + i) ^= 1u << 31;
    for (int i = 0; i < nd; i++) W.P(1 + W.maxw + i) = F::door_t(W.P(1 + W.maxw + i));
  }
  W.P(0) = (uint32_t)nw | ((uint32_t)nd << 8);
  return 0;
}

// bits [s, s+l) of the 64-bit word covering columns [64k, 64k+64)
APG_DEV uint64_t span_mask(int s, int l, int k) {
  const int lo = s > 64 * k ? s : 64 * k, hi = (s + l) < 64 * k + 64 ? s + l : 64 * k + 64;
  if (hi <= lo) return 0ULL;
  const int n = hi - lo;
  return (n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL)) << (lo - 64 * k);
}

// Paint rows [m][wpr] = border | walls & ~doors, one primitive at a time (each primitive is read
// once; the row words are read-modify-written, so `rows` should be LDS: see k_lidar_reset).
template <bool WIDE>
APG_DEV void rooms_paint(const RoomsWork &W, int m, int wpr, uint64_t *rows) {
  using F = RoomsFmt<WIDE>;
  const int nw = (int)(W.P(0) & 255u), nd = (int)(W.P(0) >> 8);
  for (int y = 0; y < m; y++)
    for (int k = 0; k < wpr; k++)
      rows[y * wpr + k] = (y == 0 || y == m - 1) ? span_mask(0, m, k) : (span_mask(0, 1, k) | span_mask(m - 1, 1, k));
  for (int i = 0; i < nw; i++) {
    const Wall wl = F::wall_of(W.P(1 + i));
    if (wl.vertical) {  // column `fixed`, rows [start, start + len)
      const uint64_t bit = 1ULL << (wl.fixed & 63);
      for (int y = wl.start; y < wl.start + wl.len; y++) rows[y * wpr + (wl.fixed >> 6)] |= bit;
    } else {
      for (int k = 0; k < wpr; k++) rows[wl.fixed * wpr + k] |= span_mask(wl.start, wl.len, k);
    }
  }
  for (int i = 0; i < nd; i++) {
    const Door d = F::door_of(W.P(1 + W.maxw + i));
    for (int y = d.r0; y < d.r0 + d.hh; y++)
      for (int k = 0; k < wpr; k++) rows[y * wpr + k] &= ~span_mask(d.c0, d.ww, k);
  }
}

// generate + paint (wide encodings): occ rows [m][wpr]; working storage in this thread's private arrays, sized for
// MR rooms
template <int MR = 17>
APG_DEV int rooms_generate(Pcg64 &r, uint64_t *occ, int wpr, int m, int max_rooms, int door_width,
                           const BinomTable &bt) {
  uint64_t stk[MR + 7];
  int16_t cap[MR], size[MR], cut[MR - 1];
  uint32_t prim[rooms_prim_words(MR)];
  const RoomsWork W{stk, cap, size, cut, prim, 1, MR + 7, MR - 1};
  const int rc = rooms_primitives<true>(r, m, max_rooms, door_width, bt, W);
  rooms_paint<true>(W, m, wpr, occ);
  return rc;
}

}  // namespace apg
