// apg_maps.hpp — procedural floor maps on device, one GPU thread per map, bit-exact with
//   FloorMapDatasetRooms.get_data_point  ap_gym/envs/floor_map/floor_map_dataset_rooms.py:25-89
//   FloorMapDatasetMaze.get_data_point   ap_gym/envs/floor_map/floor_map_dataset_maze.py:24-55
// Occupancy is bit-packed: row y of a map is `wpr` uint64 words, bit x%64 of word x/64 set = wall.
// Bits at x >= width are always zero.
#pragma once
#include "apg_device.hpp"

namespace apg {

struct BinomTable {  // random_binomial_inversion constants for n = 0..15 at p = 0.3 (host libm)
  double qn[16];
  int32_t bound[16];
  double p, q;
};

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

// distribute_integers(n, k) (rooms.py:36-40) with k <= 16
APG_DEV void distribute_integers(Pcg64 &r, int64_t n, int k, int64_t *out) {
  int64_t cuts[16];
  const int64_t nz = k > n ? k - n : 0;
  const int64_t pop = nz + (n > 1 ? n - 1 : 0);
  const int kk = k - 1;
  // Generator.choice(pop, kk, replace=False): Floyd's algorithm, then _shuffle_int(kk, 1)
  for (int64_t j = pop - kk; j < pop; j++) {
    int64_t val = (int64_t)bounded_u64(r, (uint64_t)j);
    int idx = (int)(j - (pop - kk));
    bool found = false;
    for (int t = 0; t < idx; t++) found |= (cuts[t] == val);
    cuts[idx] = found ? j : val;
  }
  for (int i = kk - 1; i >= 1; i--) {
    int jj = (int)bounded_u64(r, (uint64_t)i);
    int64_t t = cuts[jj];
    cuts[jj] = cuts[i];
    cuts[i] = t;
  }
  for (int i = 0; i < kk; i++) cuts[i] = cuts[i] < nz ? 0 : cuts[i] - nz + 1;  // r[idx]
  for (int i = 1; i < kk; i++) {
    int64_t v = cuts[i];
    int j = i - 1;
    while (j >= 0 && cuts[j] > v) {
      cuts[j + 1] = cuts[j];
      j--;
    }
    cuts[j + 1] = v;
  }
  int64_t prev = 0;
  for (int i = 0; i < kk; i++) {
    out[i] = cuts[i] - prev;
    prev = cuts[i];
  }
  out[kk] = n - prev;
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
// packed as y0 | x0 << 8 | t << 16 | n0 << 17 | n1 << 25 | max_rooms << 33
APG_DEV uint64_t pack_task(int y0, int x0, int t, int n0, int n1, int mr) {
  return (uint64_t)y0 | ((uint64_t)x0 << 8) | ((uint64_t)t << 16) | ((uint64_t)n0 << 17) |
         ((uint64_t)n1 << 25) | ((uint64_t)mr << 33);
}

// Returns 0 on success. wall/door: [h][wpr] words, caller-zeroed not required.
APG_DEV int rooms_generate(Pcg64 &r, Bits wall, Bits door, int m, int max_rooms, int door_width,
                           const BinomTable &bt) {
  const int min_size = door_width + 2;
  for (int y = 0; y < m; y++)
    for (int k = 0; k < wall.wpr; k++) {
      wall.w[y * wall.wpr + k] = 0;
      door.w[y * door.wpr + k] = 0;
    }
  for (int x = 0; x < m; x++) {
    wall.set(0, x);
    wall.set(m - 1, x);
  }
  for (int y = 0; y < m; y++) {
    wall.set(y, 0);
    wall.set(y, m - 1);
  }
  uint64_t stack[64];
  int sp = 0;
  stack[sp++] = pack_task(1, 1, 0, m - 2, m - 2, max_rooms);
  while (sp > 0) {
    const uint64_t tk = stack[--sp];
    const int y0 = (int)(tk & 255), x0 = (int)((tk >> 8) & 255), t = (int)((tk >> 16) & 1);
    const int n0 = (int)((tk >> 17) & 255), n1 = (int)((tk >> 25) & 255), mr = (int)((tk >> 33) & 255);
    int64_t mrl = pyfloordiv(n0 - min_size, min_size + 1) + 1;
    if (mr < mrl) mrl = mr;
    if (mrl <= 1) continue;
    if (mrl > 16) return -2;
    const int k = (int)binomial_inv(r, mrl - 2, bt) + 2;
    int64_t cap[16], sizes[16], starts[16], ends[16], doors[16];
    distribute_integers(r, mrl, k, cap);
    distribute_integers(r, n0 - (int64_t)k * (1 + min_size) + 1, k, sizes);
    int64_t acc = 0;
    for (int i = 0; i < k; i++) {
      sizes[i] += min_size;
      acc += sizes[i] + 1;
      ends[i] = acc - 1;
    }
    starts[0] = 0;
    for (int i = 1; i < k; i++) starts[i] = ends[i - 1] + 2;
    for (int i = 0; i < k - 1; i++) doors[i] = integers(r, 0, n1 - door_width);
    // walls: room[wall_positions] = where(room != -1, 1, -1)
    for (int i = 1; i < k; i++) {
      const int wp = (int)(starts[i] - 1);
      if (wp < 0 || wp >= n0) return -3;
      for (int j = 0; j < n1; j++) {
        const int y = t ? y0 + j : y0 + wp, x = t ? x0 + wp : x0 + j;
        if (!door.get(y, x)) wall.set(y, x);
      }
    }
    // doors: cells (wp +- a, dp + b) become -1
    for (int i = 1; i < k; i++) {
      const int wp = (int)(starts[i] - 1), dp = (int)doors[i - 1];
      for (int a = 0; a < door_width; a++)
        for (int b = 0; b < door_width; b++)
          for (int s = 0; s < 2; s++) {
            const int vi = s ? wp - a : wp + a, vj = dp + b;
            if (vi < 0 || vi >= n0 || vj >= n1) return -3;
            const int y = t ? y0 + vj : y0 + vi, x = t ? x0 + vi : x0 + vj;
            door.set(y, x);
            wall.clr(y, x);
          }
    }
    // children room[s:e+1].T, depth-first in order => push in reverse
    if (sp + k > 64) return -4;
    for (int i = k - 1; i >= 0; i--) {
      int64_t s = starts[i], e = ends[i] + 1;
      if (e > n0) e = n0;
      if (s > n0) s = n0;
      const int cy0 = t ? y0 : y0 + (int)s, cx0 = t ? x0 + (int)s : x0;
      stack[sp++] = pack_task(cy0, cx0, 1 - t, n1, (int)(e - s), (int)cap[i]);
    }
  }
  if (integers(r, 0, 2) == 0) {  // map_int = map_int.T  (square maps only)
    for (int y = 0; y < m; y++)
      for (int x = 0; x < m; x++)
        if (wall.get(x, y)) door.set(y, x); else door.clr(y, x);
    for (int y = 0; y < m; y++)
      for (int kk = 0; kk < wall.wpr; kk++) wall.w[y * wall.wpr + kk] = door.w[y * door.wpr + kk];
  }
  return 0;
}

// Maze: recursive carve() as an explicit DFS. Frame (u16): perm 4x2 bits | k << 8 | first << 11 |
// from << 12. `stack` is frame-major: frame f of this map lives at stack[f * stride].
APG_DEV uint32_t draw_perm4(Pcg64 &r) {
  uint32_t p = 0 | (1u << 2) | (2u << 4) | (3u << 6);
#pragma unroll
  for (int i = 3; i >= 1; i--) {
    uint32_t j = random_interval_small(r, (uint32_t)i);
    uint32_t vi = (p >> (2 * i)) & 3u, vj = (p >> (2 * j)) & 3u;
    p &= ~((3u << (2 * i)) | (3u << (2 * j)));
    p |= (vj << (2 * i)) | (vi << (2 * j));
  }
  return p;
}

APG_DEV int maze_generate(Pcg64 &r, Bits occ, int h, int w, double branching_prob, uint16_t *stack,
                          size_t stride, int cap) {
  for (int y = 0; y < h; y++)
    for (int k = 0; k < occ.wpr; k++) {
      const int lo = k * 64;
      uint64_t v = 0;
      if (w > lo) v = (w - lo >= 64) ? ~0ULL : ((1ULL << (w - lo)) - 1ULL);
      occ.w[y * occ.wpr + k] = v;
    }
  occ.clr(1, 1);
  const int dxs[4] = {2, -2, 0, 0}, dys[4] = {0, 0, 2, -2};
  int x = 1, y = 1, sp = 1;
  uint32_t top = draw_perm4(r) | (1u << 11);  // k = 0, first = 1
  while (true) {
    const uint32_t k = (top >> 8) & 7u;
    if (k >= 4) {  // pop
      if (--sp == 0) break;
      const uint32_t from = (top >> 12) & 3u;
      x -= dxs[from];
      y -= dys[from];
      top = stack[(size_t)(sp - 1) * stride];
      continue;
    }
    const uint32_t d = (top >> (2 * k)) & 3u;
    top = (top & ~(7u << 8)) | ((k + 1) << 8);
    const int nx = x + dxs[d], ny = y + dys[d];
    if (0 < nx && 0 < ny && nx < w - 1 && ny < h - 1 && occ.get(ny, nx)) {
      const bool first = (top >> 11) & 1u;
      if (first || next_double(r) < branching_prob) {
        occ.clr(y + dys[d] / 2, x + dxs[d] / 2);
        occ.clr(ny, nx);
        top &= ~(1u << 11);
        if (sp >= cap) return -5;
        stack[(size_t)(sp - 1) * stride] = (uint16_t)top;
        sp++;
        x = nx;
        y = ny;
        top = draw_perm4(r) | (1u << 11) | (d << 12);
      }
    }
  }
  return 0;
}

}  // namespace apg
