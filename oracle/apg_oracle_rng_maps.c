/*
 * CPU restatement (TEST INFRASTRUCTURE ONLY) of
 *   - numpy 2.2 Generator(PCG64(SeedSequence)) draws used by ap_gym
 *     (numpy/random/bit_generator.pyx SeedSequence, numpy/random/src/pcg64/pcg64.h,
 *      numpy/random/src/distributions/distributions.c random_bounded_uint64 / random_interval /
 *      random_binomial_inversion, _generator.pyx choice(replace=False) Floyd branch + shuffle);
 *   - FloorMapDatasetRooms.get_data_point  (ap_gym/envs/floor_map/floor_map_dataset_rooms.py:25-89)
 *   - FloorMapDatasetMaze.get_data_point   (ap_gym/envs/floor_map/floor_map_dataset_maze.py:24-55)
 * Compiled with -ffp-contract=off so that float arithmetic is evaluated exactly as written.
 */
#include "apg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ---------------------------------------------------------------- SeedSequence */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t value, uint32_t *hc) {
  value ^= *hc;
  *hc *= SS_MULT_A;
  value *= *hc;
  value ^= value >> 16;
  return value;
}

static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> 16;
  return r;
}

/* SeedSequence(seed).generate_state(4, uint64) */
static void seed_sequence_state(uint64_t seed, uint64_t out[4]) {
  uint32_t ent[2];
  int n_ent = 0;
  if (seed == 0) {
    ent[n_ent++] = 0;
  } else {
    while (seed > 0) {
      ent[n_ent++] = (uint32_t)(seed & 0xffffffffu);
      seed >>= 32;
    }
  }
  uint32_t pool[4];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  /* n_ent <= 2 < pool size: no remaining entropy words */
  uint32_t words[8];
  uint32_t hb = SS_INIT_B;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i & 3];
    v ^= hb;
    hb *= SS_MULT_B;
    v *= hb;
    v ^= v >> 16;
    words[i] = v;
  }
  for (int i = 0; i < 4; i++) out[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
}

/* ---------------------------------------------------------------- PCG64 */
static const u128 PCG_MULT = (((u128)0x2360ED051FC65DA4ULL) << 64) | (u128)0x4385DF649FCCF645ULL;

static inline u128 st_get(const orc_pcg64 *s) { return ((u128)s->state_hi << 64) | s->state_lo; }
static inline u128 inc_get(const orc_pcg64 *s) { return ((u128)s->inc_hi << 64) | s->inc_lo; }
static inline void st_set(orc_pcg64 *s, u128 v) {
  s->state_hi = (uint64_t)(v >> 64);
  s->state_lo = (uint64_t)v;
}

void orc_seed(uint64_t seed, orc_pcg64 *s) {
  uint64_t v[4];
  seed_sequence_state(seed, v);
  u128 initstate = ((u128)v[0] << 64) | v[1];
  u128 initseq = ((u128)v[2] << 64) | v[3];
  u128 inc = (initseq << 1) | 1u;
  u128 st = 0;
  st = st * PCG_MULT + inc;
  st += initstate;
  st = st * PCG_MULT + inc;
  st_set(s, st);
  s->inc_hi = (uint64_t)(inc >> 64);
  s->inc_lo = (uint64_t)inc;
  s->has_uint32 = 0;
  s->uinteger = 0;
}

uint64_t orc_next64(orc_pcg64 *s) {
  u128 st = st_get(s) * PCG_MULT + inc_get(s);
  st_set(s, st);
  uint64_t hi = (uint64_t)(st >> 64), lo = (uint64_t)st;
  unsigned rot = (unsigned)(st >> 122);
  uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

uint32_t orc_next32(orc_pcg64 *s) {
  if (s->has_uint32) {
    s->has_uint32 = 0;
    return s->uinteger;
  }
  uint64_t n = orc_next64(s);
  s->has_uint32 = 1;
  s->uinteger = (uint32_t)(n >> 32);
  return (uint32_t)(n & 0xffffffffu);
}

double orc_next_double(orc_pcg64 *s) { return (double)(orc_next64(s) >> 11) * (1.0 / 9007199254740992.0); }

/* random_bounded_uint64(state, 0, rng, 0, use_masked=0) */
static uint64_t bounded_u64(orc_pcg64 *s, uint64_t rng) {
  if (rng == 0) return 0;
  if (rng <= 0xffffffffULL) {
    if (rng == 0xffffffffULL) return orc_next32(s);
    uint32_t r = (uint32_t)rng, rex = r + 1u;
    uint64_t m = (uint64_t)orc_next32(s) * rex;
    uint32_t left = (uint32_t)m;
    if (left < rex) {
      uint32_t thr = (0xffffffffu - r) % rex;
      while (left < thr) {
        m = (uint64_t)orc_next32(s) * rex;
        left = (uint32_t)m;
      }
    }
    return m >> 32;
  }
  if (rng == 0xffffffffffffffffULL) return orc_next64(s);
  uint64_t rex = rng + 1;
  u128 m = (u128)orc_next64(s) * rex;
  uint64_t left = (uint64_t)m;
  if (left < rex) {
    uint64_t thr = (0xffffffffffffffffULL - rng) % rex;
    while (left < thr) {
      m = (u128)orc_next64(s) * rex;
      left = (uint64_t)m;
    }
  }
  return (uint64_t)(m >> 64);
}

int64_t orc_integers(orc_pcg64 *s, int64_t lo, int64_t hi_excl) {
  return lo + (int64_t)bounded_u64(s, (uint64_t)(hi_excl - 1 - lo));
}

uint64_t orc_integers_u32_endpoint(orc_pcg64 *s) { return bounded_u64(s, 0x100000000ULL); }

uint64_t orc_random_interval(orc_pcg64 *s, uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = max, v;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  mask |= mask >> 32;
  if (max <= 0xffffffffULL) {
    while ((v = (orc_next32(s) & mask)) > max) {
    }
  } else {
    while ((v = (orc_next64(s) & mask)) > max) {
    }
  }
  return v;
}

/* random_binomial (p <= 0.5, n*p <= 30 => inversion). */
int64_t orc_binomial(orc_pcg64 *s, int64_t n, double p) {
  if (n == 0 || p == 0.0) return 0;
  if (!(p <= 0.5) || !(p * n <= 30.0)) abort(); /* BTPE branch not needed by ap_gym */
  double q = 1.0 - p;
  double qn = exp(n * log(q));
  double np = n * p;
  int64_t bound = (int64_t)fmin((double)n, np + 10.0 * sqrt(np * q + 1));
  int64_t X = 0;
  double px = qn;
  double U = orc_next_double(s);
  while (U > px) {
    X++;
    if (X > bound) {
      X = 0;
      px = qn;
      U = orc_next_double(s);
    } else {
      U -= px;
      px = ((n - X + 1) * p * px) / (X * q);
    }
  }
  return X;
}

double orc_uniform(orc_pcg64 *s, double lo, double hi) { return lo + (hi - lo) * orc_next_double(s); }

/* Generator.choice(arange(pop), k, replace=False) for pop <= 10000 (Floyd + _shuffle_int). */
static void choice_noreplace(orc_pcg64 *s, int64_t pop, int64_t k, int64_t *idx) {
  for (int64_t j = pop - k; j < pop; j++) {
    int64_t val = (int64_t)bounded_u64(s, (uint64_t)j);
    int found = 0;
    for (int64_t t = 0; t < j - (pop - k); t++)
      if (idx[t] == val) {
        found = 1;
        break;
      }
    idx[j - pop + k] = found ? j : val;
  }
  for (int64_t i = k - 1; i >= 1; i--) {
    int64_t jj = (int64_t)bounded_u64(s, (uint64_t)i);
    int64_t t = idx[jj];
    idx[jj] = idx[i];
    idx[i] = t;
  }
}

void orc_test_draws(uint64_t seed, int kind, int64_t a, int64_t b, double p, int n, double *out) {
  orc_pcg64 s;
  orc_seed(seed, &s);
  for (int i = 0; i < n; i++) {
    switch (kind) {
      case 0: out[i] = (double)orc_next64(&s); break;
      case 1: out[i] = (double)orc_next32(&s); break;
      case 2: out[i] = orc_next_double(&s); break;
      case 3: out[i] = (double)orc_integers(&s, a, b); break;
      case 4: out[i] = (double)orc_integers_u32_endpoint(&s); break;
      case 5: out[i] = (double)orc_binomial(&s, a, p); break;
      case 6: out[i] = orc_uniform(&s, (double)a, (double)b); break;
      case 7: out[i] = (double)orc_random_interval(&s, (uint64_t)a); break;
      default: out[i] = 0; break;
    }
  }
}

/* ---------------------------------------------------------------- Rooms
 * A "view" is numpy's (possibly transposed) 2-D slice of map_int: element (i, j) lives at map
 * row y0 + i*a0y + j*a1y, column x0 + i*a0x + j*a1x. Cell values: 0 free, 1 wall, -1 door. */
typedef struct {
  int y0, x0, a0y, a0x, a1y, a1x, n0, n1;
} rview;

typedef struct {
  int8_t *m;
  int w;
  orc_pcg64 *rng;
  int min_size, door_width;
} rooms_ctx;

static inline int8_t *rv_at(const rooms_ctx *c, const rview *v, int i, int j) {
  int y = v->y0 + i * v->a0y + j * v->a1y;
  int x = v->x0 + i * v->a0x + j * v->a1x;
  return &c->m[y * c->w + x];
}

/* distribute_integers(n, k) (floor_map_dataset_rooms.py:36-40):
 * r = concat(zeros(max(0, k-n)), arange(1, n)); cuts = sort(choice(r, k-1, replace=False));
 * returns diff([0, cuts..., n]). */
static void distribute_integers(orc_pcg64 *s, int64_t n, int64_t k, int64_t *out) {
  int64_t cuts[64];
  int64_t nz = k > n ? k - n : 0;
  int64_t pop = nz + (n > 1 ? n - 1 : 0);
  if (k - 1 > 63) abort();
  choice_noreplace(s, pop, k - 1, cuts);
  for (int64_t i = 0; i < k - 1; i++) cuts[i] = cuts[i] < nz ? 0 : cuts[i] - nz + 1; /* r[idx] */
  for (int64_t i = 1; i < k - 1; i++) { /* insertion sort */
    int64_t v = cuts[i], j = i - 1;
    while (j >= 0 && cuts[j] > v) {
      cuts[j + 1] = cuts[j];
      j--;
    }
    cuts[j + 1] = v;
  }
  int64_t prev = 0;
  for (int64_t i = 0; i < k - 1; i++) {
    out[i] = cuts[i] - prev;
    prev = cuts[i];
  }
  out[k - 1] = n - prev;
}

static int64_t pyfloordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
  return q;
}

static void split_room(rooms_ctx *c, rview v, int64_t max_rooms) {
  int64_t mrl = pyfloordiv(v.n0 - c->min_size, c->min_size + 1) + 1;
  if (max_rooms < mrl) mrl = max_rooms;
  if (mrl <= 1) return;
  int64_t k = orc_binomial(c->rng, mrl - 2, 0.3) + 2;
  int64_t cap[64], sizes[64], starts[64], ends[64], doors[64];
  distribute_integers(c->rng, mrl, k, cap);
  distribute_integers(c->rng, v.n0 - k * (1 + c->min_size) + 1, k, sizes);
  int64_t acc = 0;
  for (int64_t i = 0; i < k; i++) {
    sizes[i] += c->min_size;
    acc += sizes[i] + 1;
    ends[i] = acc - 1;
  }
  starts[0] = 0;
  for (int64_t i = 1; i < k; i++) starts[i] = ends[i - 1] + 2;
  for (int64_t i = 0; i < k - 1; i++) doors[i] = orc_integers(c->rng, 0, v.n1 - c->door_width);
  /* room[wall_positions] = where(room[wall_positions] != -1, 1, -1) */
  for (int64_t i = 1; i < k; i++) {
    int64_t wp = starts[i] - 1;
    if (wp < 0 || wp >= v.n0) abort();
    for (int j = 0; j < v.n1; j++) {
      int8_t *cell = rv_at(c, &v, (int)wp, j);
      if (*cell != -1) *cell = 1;
    }
  }
  /* door cells (both sides of each wall) become -1 */
  for (int64_t i = 1; i < k; i++) {
    int64_t wp = starts[i] - 1, dp = doors[i - 1];
    for (int a = 0; a < c->door_width; a++)
      for (int b = 0; b < c->door_width; b++) {
        if (wp + a >= v.n0 || wp - a < 0 || dp + b >= v.n1) abort();
        *rv_at(c, &v, (int)(wp + a), (int)(dp + b)) = -1;
      }
    for (int a = 0; a < c->door_width; a++)
      for (int b = 0; b < c->door_width; b++) *rv_at(c, &v, (int)(wp - a), (int)(dp + b)) = -1;
  }
  /* recurse into room[s:e+1].T (numpy slicing clips e+1 to n0) */
  for (int64_t i = 0; i < k; i++) {
    int64_t s = starts[i], e = ends[i] + 1;
    if (e > v.n0) e = v.n0;
    if (s > v.n0) s = v.n0;
    rview ch;
    ch.y0 = v.y0 + (int)s * v.a0y;
    ch.x0 = v.x0 + (int)s * v.a0x;
    ch.a0y = v.a1y;
    ch.a0x = v.a1x;
    ch.a1y = v.a0y;
    ch.a1x = v.a0x;
    ch.n0 = v.n1;
    ch.n1 = (int)(e - s);
    split_room(c, ch, cap[i]);
  }
}

int orc_rooms_map(uint64_t idx, int h, int w, int max_rooms, int door_width, uint8_t *out) {
  if (h != w || h < 3) return -1;
  orc_pcg64 rng;
  orc_seed(idx, &rng);
  int8_t *m = (int8_t *)calloc((size_t)h * w, 1);
  for (int x = 0; x < w; x++) m[x] = m[(h - 1) * w + x] = 1;
  for (int y = 0; y < h; y++) m[y * w] = m[y * w + w - 1] = 1;
  rooms_ctx c = {m, w, &rng, door_width + 2, door_width};
  rview top = {1, 1, 1, 0, 0, 1, h - 2, w - 2};
  split_room(&c, top, max_rooms);
  int transpose = orc_integers(&rng, 0, 2) == 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int8_t v = transpose ? m[x * w + y] : m[y * w + x];
      out[y * w + x] = (uint8_t)(v == 1);
    }
  free(m);
  return 0;
}

/* ---------------------------------------------------------------- Maze
 * Recursive carve() restated with an explicit stack (depth <= number of maze cells). */
int orc_maze_map(uint64_t idx, int h, int w, double branching_prob, uint8_t *out) {
  if ((h % 2) == 0 || (w % 2) == 0) return -1;
  static const int dirs[4][2] = {{2, 0}, {-2, 0}, {0, 2}, {0, -2}};
  orc_pcg64 rng;
  orc_seed(idx, &rng);
  memset(out, 1, (size_t)h * w);
  out[1 * w + 1] = 0;
  int cap = ((h + 1) / 2) * ((w + 1) / 2) + 4;
  typedef struct {
    int x, y, k, first;
    int perm[4];
  } frame;
  frame *st = (frame *)malloc(sizeof(frame) * (size_t)cap);
  int sp = 0;
#define PUSH_FRAME(PX, PY)                                          \
  do {                                                              \
    frame *f = &st[sp++];                                           \
    f->x = (PX);                                                    \
    f->y = (PY);                                                    \
    f->k = 0;                                                       \
    f->first = 1;                                                   \
    for (int t = 0; t < 4; t++) f->perm[t] = t;                     \
    for (int t = 3; t >= 1; t--) {                                  \
      int j = (int)orc_random_interval(&rng, (uint64_t)t);          \
      int tmp = f->perm[t];                                         \
      f->perm[t] = f->perm[j];                                      \
      f->perm[j] = tmp;                                             \
    }                                                               \
  } while (0)
  PUSH_FRAME(1, 1);
  while (sp > 0) {
    frame *f = &st[sp - 1];
    if (f->k >= 4) {
      sp--;
      continue;
    }
    const int *d = dirs[f->perm[f->k++]];
    int nx = f->x + d[0], ny = f->y + d[1];
    if (0 < nx && 0 < ny && nx < w - 1 && ny < h - 1 && out[ny * w + nx] == 1) {
      if (f->first || orc_next_double(&rng) < branching_prob) {
        out[(f->y + d[1] / 2) * w + (f->x + d[0] / 2)] = 0;
        out[ny * w + nx] = 0;
        f->first = 0; /* set before the child runs: the flag is only read after it returns */
        if (sp >= cap) abort();
        PUSH_FRAME(nx, ny);
      }
    }
  }
#undef PUSH_FRAME
  free(st);
  return 0;
}
