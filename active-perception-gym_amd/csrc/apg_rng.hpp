// apg_rng.hpp — vector-level numpy streams drawn in parallel on the GPU.
//
// The image envs draw their per-reset batches from ONE numpy Generator each (DatasetBatchIterator:
// integers(0, len, N), dataset_iterator.py:52-57; ImagePerceptionModule: uniform(-1, 1, (N, 2)) and
// integers(0, 2, N), image_perception_module.py:130-161; ImageLocalizationVectorEnv:
// uniform(-1, 1, (k, 2)), image_localization.py:153-156).  A single stream is sequential, but PCG64
// is an LCG: the state after d steps is A^d s + C_d (pcg_advance_lcg_128), so a workgroup can give
// every thread its own stretch of the stream, and Lemire's rejections become a stream compaction
// (output i is the i-th accepted candidate).  Bit-exact with numpy, including the next_uint32
// half-buffer carried in the generator state.
#pragma once
#include "apg_device.hpp"

namespace apg {

struct U128 {
  uint64_t hi, lo;
};

APG_DEV U128 mul128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo * b.lo;
  r.hi = __umul64hi(a.lo, b.lo) + a.hi * b.lo + a.lo * b.hi;
  return r;
}

APG_DEV U128 add128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ULL : 0ULL);
  return r;
}

// Jumps of d = k * 256^i LCG steps (i < 4, k < 256): s -> A^d s + G(d) inc with G(d) = 1 + A + ... + A^(d-1)
// (mod 2^128), tabulated at compile time, so an advance by d < 2^32 is at most four such maps (eight 128-bit
// multiplies) instead of pcg_advance_lcg_128's square-and-multiply (four per bit of d: the per-thread jumps of
// the parallel stream draws were their kernels' longest chain).
struct PcgJump {
  uint64_t m_hi, m_lo, g_hi, g_lo;
};
struct PcgJumpTable {
  PcgJump e[4][256];
};
constexpr PcgJumpTable make_pcg_jump_table() {
  PcgJumpTable t{};
  using u128 = unsigned __int128;
  u128 base_m = ((u128)PCG_MUL_HI << 64) | PCG_MUL_LO, base_g = 1;  // A^step, G(step) for step = 256^i
  for (int i = 0; i < 4; i++) {
    u128 m = 1, g = 0;  // A^(k step), G(k step)
    for (int k = 0; k < 256; k++) {
      t.e[i][k] = PcgJump{(uint64_t)(m >> 64), (uint64_t)m, (uint64_t)(g >> 64), (uint64_t)g};
      g = g + m * base_g;  // G((k + 1) step) = G(k step) + A^(k step) G(step)
      m = m * base_m;
    }
    base_m = m;  // A^(256 step), G(256 step)
    base_g = g;
  }
  return t;
}
static __constant__ PcgJumpTable c_pcg_jump = make_pcg_jump_table();

// state <- state advanced by `delta` LCG steps (numpy pcg64 advance / pcg_advance_lcg_128)
APG_DEV void pcg_advance(Pcg64 &r, uint64_t delta) {
  if ((delta >> 32) == 0ULL) {
    U128 s{r.s_hi, r.s_lo};
    const U128 inc{r.i_hi, r.i_lo};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int k = (int)((delta >> (8 * i)) & 255ULL);
      if (k) {
        const PcgJump j = c_pcg_jump.e[i][k];
        s = add128(mul128(U128{j.m_hi, j.m_lo}, s), mul128(U128{j.g_hi, j.g_lo}, inc));
      }
    }
    r.s_hi = s.hi;
    r.s_lo = s.lo;
    return;
  }
  U128 acc_mult{0, 1}, acc_plus{0, 0}, cur_mult{PCG_MUL_HI, PCG_MUL_LO}, cur_plus{r.i_hi, r.i_lo};
  while (delta) {
    if (delta & 1ULL) {
      acc_mult = mul128(acc_mult, cur_mult);
      acc_plus = add128(mul128(acc_plus, cur_mult), cur_plus);
    }
    cur_plus = mul128(add128(cur_mult, U128{0, 1}), cur_plus);
    cur_mult = mul128(cur_mult, cur_mult);
    delta >>= 1;
  }
  const U128 s = add128(mul128(acc_mult, U128{r.s_hi, r.s_lo}), acc_plus);
  r.s_hi = s.hi;
  r.s_lo = s.lo;
}

// XSL-RR output of the state after one more step, without touching `r`
APG_DEV uint64_t pcg_output_next(Pcg64 r) {
  pcg_step(r.s_hi, r.s_lo, r.i_hi, r.i_lo);
  const uint64_t x = r.s_hi ^ r.s_lo;
  const unsigned rot = (unsigned)(r.s_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// i-th 32-bit word of the next_uint32 sequence that continues from `base` (numpy pcg64_next32:
// the buffered high half first when has32, then low, high halves of successive next64 outputs).
APG_DEV uint32_t next32_word(const Pcg64 &base, uint64_t i) {
  if (base.has32) {
    if (i == 0) return base.u32;
    i -= 1;
  }
  Pcg64 r = base;
  pcg_advance(r, i >> 1);
  const uint64_t v = pcg_output_next(r);
  return (i & 1ULL) ? (uint32_t)(v >> 32) : (uint32_t)v;
}

// Sequential reader of the next_uint32 words k0, k0+1, ... of the stream continuing from `base`
// (one jump to k0, then one LCG step per two words).
struct Next32Walker {
  Pcg64 r;
  uint64_t pair;
  uint32_t buffered;
  int state;  // 0: return `buffered` next, 1: high half of `pair` next, 2: draw a new pair next

  APG_DEV Next32Walker(const Pcg64 &base, uint64_t k0) : r(base), pair(0), buffered(base.u32), state(2) {
    uint64_t j = k0;
    if (base.has32) {
      if (k0 == 0) {
        state = 0;
        return;
      }
      j = k0 - 1;
    }
    pcg_advance(r, j >> 1);
    if (j & 1ULL) {
      pair = next64(r);
      state = 1;
    }
  }

  APG_DEV uint32_t next() {
    if (state == 0) {
      state = 2;
      return buffered;
    }
    if (state == 1) {
      state = 2;
      return (uint32_t)(pair >> 32);
    }
    pair = next64(r);
    state = 1;
    return (uint32_t)pair;
  }
};

// Generator state after `words` next_uint32 calls from `base`.
APG_DEV Pcg64 after_next32_words(const Pcg64 &base, uint64_t words) {
  Pcg64 r = base;
  if (words == 0) return r;
  if (r.has32) {
    r.has32 = 0;
    words -= 1;
  }
  pcg_advance(r, words >> 1);
  if (words & 1ULL) {  // a pair was drawn and its high half is buffered
    const uint64_t v = pcg_output_next(r);
    pcg_advance(r, 1);
    r.has32 = 1;
    r.u32 = (uint32_t)(v >> 32);
  }
  return r;
}

}  // namespace apg
