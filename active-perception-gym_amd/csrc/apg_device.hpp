// apg_device.hpp — device-side building blocks for the gfx950 LIDAR path.
//
//  * numpy Generator(PCG64(SeedSequence)) restated for one GPU thread per stream (bit-exact):
//    SeedSequence hashing, PCG64 XSL-RR, next_uint32 half-buffering, Lemire32/64 bounded draws,
//    masked random_interval, Floyd choice(replace=False) + shuffle, binomial inversion
//    (numpy/random/src/distributions/distributions.c, _generator.pyx).
//  * exact orientation predicate (Shewchuk filter + exact 6-product expansion fallback) and the
//    GEOS algorithm::Intersection::intersection formula, evaluated without FMA contraction.
//
// Everything here is compiled with -ffp-contract=off; FMAs appear only where written explicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define APG_DEV __device__ __forceinline__

namespace apg {

// ------------------------------------------------------------------ PCG64 stream state
struct Pcg64 {
  uint64_t s_hi, s_lo, i_hi, i_lo;
  uint32_t has32, u32;
};

static constexpr uint64_t PCG_MUL_HI = 0x2360ED051FC65DA4ULL;
static constexpr uint64_t PCG_MUL_LO = 0x4385DF649FCCF645ULL;

APG_DEV void pcg_step(uint64_t &hi, uint64_t &lo, uint64_t ihi, uint64_t ilo) {
  // (hi:lo) = (hi:lo) * MUL + inc  (mod 2^128)
  uint64_t nlo = lo * PCG_MUL_LO;
  uint64_t nhi = __umul64hi(lo, PCG_MUL_LO) + hi * PCG_MUL_LO + lo * PCG_MUL_HI;
  uint64_t rlo = nlo + ilo;
  nhi += ihi + (rlo < nlo ? 1ULL : 0ULL);
  hi = nhi;
  lo = rlo;
}

APG_DEV uint64_t next64(Pcg64 &r) {
  pcg_step(r.s_hi, r.s_lo, r.i_hi, r.i_lo);
  uint64_t x = r.s_hi ^ r.s_lo;
  unsigned rot = (unsigned)(r.s_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

APG_DEV uint32_t next32(Pcg64 &r) {
  if (r.has32) {
    r.has32 = 0;
    return r.u32;
  }
  uint64_t n = next64(r);
  r.has32 = 1;
  r.u32 = (uint32_t)(n >> 32);
  return (uint32_t)n;
}

APG_DEV double next_double(Pcg64 &r) {
  return (double)(next64(r) >> 11) * (1.0 / 9007199254740992.0);
}

// SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding (bit_generator.pyx, pcg64.pyx)
APG_DEV uint32_t ss_hashmix(uint32_t v, uint32_t &hc) {
  v ^= hc;
  hc *= 0x931e8875u;
  v *= hc;
  v ^= v >> 16;
  return v;
}
APG_DEV uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
  return r ^ (r >> 16);
}

APG_DEV Pcg64 seed_pcg64(uint64_t seed) {
  uint32_t ent0 = (uint32_t)seed, ent1 = (uint32_t)(seed >> 32);
  int n_ent = (seed >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;
#pragma unroll
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i == 0 ? ent0 : (i == 1 && n_ent == 2 ? ent1 : 0u), hc);
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  uint32_t hb = 0x8b51f9ddu, w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i & 3] ^ hb;
    hb *= 0x58f38dedu;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  Pcg64 r;
  // inc = initseq << 1 | 1 ; initseq = v2:v3 ; initstate = v0:v1
  r.i_hi = (v2 << 1) | (v3 >> 63);
  r.i_lo = (v3 << 1) | 1ULL;
  r.s_hi = 0;
  r.s_lo = 0;
  pcg_step(r.s_hi, r.s_lo, r.i_hi, r.i_lo);
  uint64_t lo = r.s_lo + v1;
  r.s_hi = r.s_hi + v0 + (lo < v1 ? 1ULL : 0ULL);
  r.s_lo = lo;
  pcg_step(r.s_hi, r.s_lo, r.i_hi, r.i_lo);
  r.has32 = 0;
  r.u32 = 0;
  return r;
}

// random_bounded_uint64(state, 0, rng, 0, use_masked=false)
APG_DEV uint64_t bounded_u64(Pcg64 &r, uint64_t rng) {
  if (rng == 0) return 0;
  if (rng <= 0xffffffffULL) {
    if (rng == 0xffffffffULL) return next32(r);
    uint32_t rr = (uint32_t)rng, rex = rr + 1u;
    uint64_t m = (uint64_t)next32(r) * rex;
    uint32_t left = (uint32_t)m;
    if (left < rex) {
      uint32_t thr = (0xffffffffu - rr) % rex;
      while (left < thr) {
        m = (uint64_t)next32(r) * rex;
        left = (uint32_t)m;
      }
    }
    return m >> 32;
  }
  if (rng == 0xffffffffffffffffULL) return next64(r);
  uint64_t rex = rng + 1;
  uint64_t x = next64(r);
  uint64_t left = x * rex, hi = __umul64hi(x, rex);
  if (left < rex) {
    uint64_t thr = (0xffffffffffffffffULL - rng) % rex;
    while (left < thr) {
      x = next64(r);
      left = x * rex;
      hi = __umul64hi(x, rex);
    }
  }
  return hi;
}

APG_DEV int64_t integers(Pcg64 &r, int64_t lo, int64_t hi_excl) {
  return lo + (int64_t)bounded_u64(r, (uint64_t)(hi_excl - 1 - lo));
}

APG_DEV uint32_t random_interval_small(Pcg64 &r, uint32_t max) {
  // random_interval(max) for max < 2^32: masked rejection on next_uint32
  if (max == 0) return 0;
  uint32_t mask = max;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = (next32(r) & mask)) > max) {
  }
  return v;
}

// ------------------------------------------------------------------ exact geometry
// sign of (qx-px)*(vy-py) - (qy-py)*(vx-px) for f32-valued p, q and integer-valued v.
// Fast path: Shewchuk's orient2d filter; fallback: the determinant expanded into six products of
// two f32-representable numbers (each exact in f64) summed exactly by grow-expansion.
APG_DEV void two_sum(double a, double b, double &s, double &e) {
  s = __dadd_rn(a, b);
  double bv = __dsub_rn(s, a);
  double av = __dsub_rn(s, bv);
  e = __dadd_rn(__dsub_rn(a, av), __dsub_rn(b, bv));
}

APG_DEV int orient_exact6(double px, double py, double qx, double qy, double vx, double vy) {
  double t[6] = {__dmul_rn(qx, vy), -__dmul_rn(qx, py), -__dmul_rn(px, vy),
                 -__dmul_rn(qy, vx), __dmul_rn(qy, px), __dmul_rn(py, vx)};
  // Grow-Expansion without zero elimination: fully unrolled, static register indexing.
  double h[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double q = t[i];
#pragma unroll
    for (int j = 0; j < i; j++) {
      double s, e;
      two_sum(q, h[j], s, e);
      q = s;
      h[j] = e;
    }
    h[i] = q;
  }
  int sgn = 0;
#pragma unroll
  for (int j = 5; j >= 0; j--)
    if (sgn == 0 && h[j] != 0.0) sgn = h[j] > 0.0 ? 1 : -1;
  return sgn;
}

APG_DEV int orient(double px, double py, double qx, double qy, double vx, double vy) {
  // orient2d(pa=p, pb=q, pc=v) with pc as origin
  double dl = __dmul_rn(__dsub_rn(px, vx), __dsub_rn(qy, vy));
  double dr = __dmul_rn(__dsub_rn(py, vy), __dsub_rn(qx, vx));
  double det = __dsub_rn(dl, dr);
  double bound = 3.3306690738754716e-16 * (fabs(dl) + fabs(dr));  // (3 + 16 eps) eps, eps = 2^-53
  if (det > bound) return 1;
  if (-det > bound) return -1;
  return orient_exact6(px, py, qx, qy, vx, vy);
}

// Same predicate for f32 p, q and integer lattice point (a, b): Shewchuk's filter evaluated in
// float32 first (error bound (3 + 16 eps) eps * (|dl| + |dr|), eps = 2^-24), then the f64 path.
APG_DEV int orient_lattice(float fpx, float fpy, float fqx, float fqy, int a, int b) {
  const float fa = (float)a, fb = (float)b;
  const float dl = __fmul_rn(__fsub_rn(fpx, fa), __fsub_rn(fqy, fb));
  const float dr = __fmul_rn(__fsub_rn(fpy, fb), __fsub_rn(fqx, fa));
  const float det = __fsub_rn(dl, dr);
  const float bound = 1.7881398e-7f * __fadd_rn(fabsf(dl), fabsf(dr));
  int r = det > bound ? 1 : (-det > bound ? -1 : 0);
  if (r == 0) r = orient(fpx, fpy, fqx, fqy, (double)a, (double)b);  // near-tie: f64 filter, then exact
  return r;
}

// GEOS algorithm::Intersection::intersection (midpoint-conditioned homogeneous formula).
APG_DEV void geos_intersection(double p1x_, double p1y_, double p2x_, double p2y_, double q1x_,
                               double q1y_, double q2x_, double q2y_, double &ox, double &oy) {
  double minX0 = p1x_ < p2x_ ? p1x_ : p2x_, minY0 = p1y_ < p2y_ ? p1y_ : p2y_;
  double maxX0 = p1x_ > p2x_ ? p1x_ : p2x_, maxY0 = p1y_ > p2y_ ? p1y_ : p2y_;
  double minX1 = q1x_ < q2x_ ? q1x_ : q2x_, minY1 = q1y_ < q2y_ ? q1y_ : q2y_;
  double maxX1 = q1x_ > q2x_ ? q1x_ : q2x_, maxY1 = q1y_ > q2y_ ? q1y_ : q2y_;
  double intMinX = minX0 > minX1 ? minX0 : minX1, intMaxX = maxX0 < maxX1 ? maxX0 : maxX1;
  double intMinY = minY0 > minY1 ? minY0 : minY1, intMaxY = maxY0 < maxY1 ? maxY0 : maxY1;
  double midx = __ddiv_rn(__dadd_rn(intMinX, intMaxX), 2.0);
  double midy = __ddiv_rn(__dadd_rn(intMinY, intMaxY), 2.0);
  double p1x = __dsub_rn(p1x_, midx), p1y = __dsub_rn(p1y_, midy);
  double p2x = __dsub_rn(p2x_, midx), p2y = __dsub_rn(p2y_, midy);
  double q1x = __dsub_rn(q1x_, midx), q1y = __dsub_rn(q1y_, midy);
  double q2x = __dsub_rn(q2x_, midx), q2y = __dsub_rn(q2y_, midy);
  double px = __dsub_rn(p1y, p2y), py = __dsub_rn(p2x, p1x);
  double pw = __dsub_rn(__dmul_rn(p1x, p2y), __dmul_rn(p2x, p1y));
  double qx = __dsub_rn(q1y, q2y), qy = __dsub_rn(q2x, q1x);
  double qw = __dsub_rn(__dmul_rn(q1x, q2y), __dmul_rn(q2x, q1y));
  double x = __dsub_rn(__dmul_rn(py, qw), __dmul_rn(qy, pw));
  double y = __dsub_rn(__dmul_rn(qx, pw), __dmul_rn(px, qw));
  double w = __dsub_rn(__dmul_rn(px, qy), __dmul_rn(qx, py));
  ox = __dadd_rn(__ddiv_rn(x, w), midx);
  oy = __dadd_rn(__ddiv_rn(y, w), midy);
}

// Correctly rounded float32 division and square root, evaluated in float64 and rounded once more:
// exact for IEEE binary32 because 53 >= 2*24 + 2 (innocuous double rounding).  The gfx950 native
// f32 sqrt/div sequences are not guaranteed to be correctly rounded.
APG_DEV float f32_div(float a, float b) { return (float)__ddiv_rn((double)a, (double)b); }
APG_DEV float f32_sqrt(float a) { return (float)__dsqrt_rn((double)a); }

// a / b for a divisor fixed per launch, from inv = 1.0 / (double)b (correctly rounded f64): the f64
// product is within 2^-52 (relative) of a / b, while a quotient of two f32 values is never an f32
// rounding midpoint (odd 25-bit x 24-bit significands need >= 25 bits) and, when not one, lies >= 2^-49
// (relative) from it -- so rounding the product to f32 gives the correctly rounded quotient, as
// f32_div does (normal f32 results; the callers' quotients are 0 or >= 2^-30).
APG_DEV float f32_div_inv(float a, double inv) { return (float)__dmul_rn((double)a, inv); }

// numpy norm of a float32 2-vector (OpenBLAS sdot: f32 products, f32 sum) then f32 sqrt.
APG_DEV float norm_f32(float dx, float dy) {
  float s = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
  return f32_sqrt(s);
}

}  // namespace apg
