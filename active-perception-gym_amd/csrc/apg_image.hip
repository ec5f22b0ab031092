// apg_image.hip — gfx950 kernels + C ABI for the image glimpse envs (ImageClassificationVectorEnv,
// ImageLocalizationVectorEnv over ImagePerceptionModule; ap_gym/envs/image_*.py, image/*.py).
//
//   k_fill_*         a whole batch drawn from ONE numpy stream across the chip (apg_rng.hpp):
//                    PCG64 jump-ahead per thread, Lemire rejections as a stream compaction.
//   k_image_gather   labels of the newly drawn data points, optional label inversion (:130-139).
//   k_image_env      one thread per env: prediction/action NaN checks, normalized CE (f64) or MSE
//                    (f32) loss, project_sphere move + clip (f64), base reward, reward (:191-217,
//                    image_classification.py:113-127, image_localization.py:151-181).
//   k_glimpse        one thread per glimpse pixel: scipy RGI "linear" bilinear in f64 in
//                    _evaluate_linear's term order, clip(0, 1), float32 (:294-331).  Images stay in
//                    the resident uint8 pool; the u8 -> f32/255 conversion is a 256-entry table.
//   k_unique         one workgroup per env: glimpses of the P sampling-grid points are staged in LDS
//                    tile by tile, every unordered pair's mean squared difference is summed in
//                    numpy's pairwise order, min-reduced per point (LDS atomics), then one wave
//                    ranks the top k (:253-277).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "../../include/apgym_capi.h"
#include "apg_host.hpp"
#include "apg_pairwise.hpp"
#include "apg_rng.hpp"

using namespace apg;

namespace {

// ------------------------------------------------------------------ geometry of a glimpse
struct GlimpseGeo {
  int h, w, pc, c, s0, s1;
  double lim_x, lim_y;  // sensor_pos_lim_pixels (x first, like the reference)
  double scale, cy, cx;  // grid centres (h - 1) / 2, (w - 1) / 2
  int pool_f32;
  int tiled;             // APG_POOL_U8_TILED: RGBX pixels in 8 x 4-pixel 128-byte tiles
  int64_t trow;          // tiled: bytes per row of tiles, ceil(w / 8) * 128
  int64_t img_elems;     // h * w * pc (tiled: ceil(h / 4) * trow bytes)
  int64_t pitch;         // output floats per glimpse unit: s0 * s1 * c (dense), out_row_bytes / 4 (packed env rows)
};

GlimpseGeo make_geo(const apg_image_config *c) {
  GlimpseGeo g;
  g.h = c->height;
  g.w = c->width;
  g.pc = c->pool_channels;
  g.c = c->channels;
  g.s0 = c->sensor_h;
  g.s1 = c->sensor_w;
  g.scale = c->sensor_scale;
  // (flip(image_shape[1:3]) - 1) / 2 - (sensor_size * sensor_scale - 1) / 2   (:419-423)
  g.lim_x = ((double)c->width - 1.0) / 2.0 - ((double)c->sensor_h * c->sensor_scale - 1.0) / 2.0;
  g.lim_y = ((double)c->height - 1.0) / 2.0 - ((double)c->sensor_w * c->sensor_scale - 1.0) / 2.0;
  g.cy = ((double)c->height - 1.0) / 2.0;
  g.cx = ((double)c->width - 1.0) / 2.0;
  g.pool_f32 = c->pool_dtype == APG_POOL_F32;
  g.tiled = c->pool_dtype == APG_POOL_U8_TILED;
  g.trow = (int64_t)((c->width + 7) / 8) * 128;
  g.img_elems = g.tiled ? (int64_t)((c->height + 3) / 4) * g.trow : (int64_t)c->height * c->width * c->pool_channels;
  g.pitch = (int64_t)c->sensor_h * c->sensor_w * c->channels;
  return g;
}

// The geometry of the env's own glimpse outputs (one unit per env): packed rows step by out_row_bytes.
GlimpseGeo env_geo(const apg_image_config *c) {
  GlimpseGeo g = make_geo(c);
  if (c->out_row_bytes > 0) g.pitch = c->out_row_bytes / 4;
  return g;
}

// Output element j of env e: a dense [N][k] array, or (row > 0: apg_image_config.out_row_bytes) a field of env e's
// packed output row.
template <class T>
APG_DEV T &ro(T *p, int row, int e, int k, int j = 0) {
  return row ? *reinterpret_cast<T *>(reinterpret_cast<char *>(p) + (size_t)e * (size_t)row + (size_t)j * sizeof(T))
             : p[(size_t)e * k + j];
}
// statistic m of env e: dense [M][N], packed [N][M]
template <class T>
APG_DEV T &ro_t(T *p, int row, int n, int e, int m) {
  return row ? *reinterpret_cast<T *>(reinterpret_cast<char *>(p) + (size_t)e * (size_t)row + (size_t)m * sizeof(T))
             : p[(size_t)m * n + e];
}

// float32(v) / 255 for v = 0..255 (_process_imgs_np), staged in LDS by every glimpse workgroup:
// the f64 quotient rounded once more to f32 equals numpy's correctly rounded f32 division for all
// 256 values (checked bit for bit by the glimpse parity tests, which cover every u8 value)
APG_DEV float u8_value(unsigned v) { return (float)__dmul_rn((double)v, 1.0 / 255.0); }
// The same f32 value in registers: v * (1/255) as an unevaluated f32 pair c_hi + c_lo, fma(v, c_hi, v * c_lo).
// The pair carries 1/255 to ~2^-48 relative, and no v / 255 (v in 0..255; a repeating 8-bit pattern) lies that
// close to a rounding midpoint of f32, so the fma rounds to the correctly rounded v / 255 = u8_value(v) for every
// v (checked exhaustively with exact rationals, tests/test_host.py).  The glimpse's tap reads use it instead of
// the LDS table: random bytes of 64 lanes hit the table's 32 banks with ~2.5 extra cycles per read.
#ifndef APG_U8_ARITH
#define APG_U8_ARITH 1
#endif
constexpr float U8_C_HI = 0x1.010102p-8f, U8_C_LO = -0x1.fdfdfep-33f;
APG_DEV float u8_value_f32(uint32_t v) { return __fmaf_rn((float)v, U8_C_HI, __fmul_rn((float)v, U8_C_LO)); }
APG_DEV void load_u8_table(float *lut) {
  // v * (1/255) in f64 rounds to the same f32 as the correctly rounded v / 255 for every v in 0..255
  // (checked exhaustively against numpy on the host); cheaper than an f64 division per entry
  for (int v = threadIdx.x; v < 256; v += blockDim.x) lut[v] = u8_value((unsigned)v);
  __syncthreads();
}

// byte offsets of image row y / column x in a tiled pool (APG_POOL_U8_TILED): separable, pixel = row_off + col_off
APG_DEV int64_t tile_row_off(const GlimpseGeo &g, int y) { return (int64_t)(y >> 2) * g.trow + ((y & 3) << 5); }
APG_DEV int tile_col_off(int x) { return ((x >> 3) << 7) + ((x & 7) << 2); }

APG_DEV float pool_value(const GlimpseGeo &g, const void *pool, const float *lut, int64_t base, int y, int x, int ch) {
  const int64_t i = g.tiled ? base + tile_row_off(g, y) + tile_col_off(x) + ch
                            : base + (int64_t)((y * g.w + x) * g.pc + (g.pc == 1 ? 0 : ch));
  if (g.pool_f32) return static_cast<const float *>(pool)[i];
  const uint32_t v = static_cast<const uint8_t *>(pool)[i];
  return APG_U8_ARITH ? u8_value_f32(v) : lut[v];  // (random table reads conflict on the LDS banks)
}

// grid interval of v on the unit grid k - c (k = 0..n-1): g[i] <= v < g[i+1], clipped to [0, n-2]
// (scipy _rgi_cython.find_indices / find_interval_ascending); returns i and v - g[i]
APG_DEV int grid_interval(double v, double c, int n, double &frac) {
  double f = floor(__dadd_rn(v, c));
  int i = (int)f;
  if (i > n - 2) i = n - 2;
  if (i < 0) i = 0;
  if (__dsub_rn((double)i, c) > v && i > 0) i--;
  frac = __dsub_rn(v, __dsub_rn((double)i, c));
  return i;
}

// One glimpse pixel (i, j) of image `base` at normalized position (px, py): C channels into out.
// Returns APG_ERR_OOB_* bits for points outside the image grid (RGI bounds_error=True).
APG_DEV uint32_t glimpse_pixel(const GlimpseGeo &g, const void *pool, const float *lut, int64_t base, double px,
                               double py, int i, int j, float *out) {
  // flip(denormalize(pos)) + offsets: (y, x) = (pos_y * lim_y + o0[i], pos_x * lim_x + o1[j])
  const double o0 = __dmul_rn(__dsub_rn((double)i, ((double)g.s0 - 1.0) / 2.0), g.scale);
  const double o1 = __dmul_rn(__dsub_rn((double)j, ((double)g.s1 - 1.0) / 2.0), g.scale);
  const double y = __dadd_rn(__dmul_rn(py, g.lim_y), o0);
  const double x = __dadd_rn(__dmul_rn(px, g.lim_x), o1);
  uint32_t err = 0;
  if (!(y >= -g.cy && y <= g.cy)) err |= APG_ERR_OOB_Y;
  if (!(x >= -g.cx && x <= g.cx)) err |= APG_ERR_OOB_X;
  double wy, wx;
  const int iy = grid_interval(y, g.cy, g.h, wy);
  const int ix = grid_interval(x, g.cx, g.w, wx);
  const double ny = __dsub_rn(1.0, wy), nx = __dsub_rn(1.0, wx);
  // hypercube order of _evaluate_linear: (i0, j0), (i0, j0+1), (i0+1, j0), (i0+1, j0+1); w = (1*wy)*wx
  const double w00 = __dmul_rn(ny, nx), w01 = __dmul_rn(ny, wx), w10 = __dmul_rn(wy, nx), w11 = __dmul_rn(wy, wx);
  for (int ch = 0; ch < g.c; ch++) {
    double v = __dadd_rn(0.0, __dmul_rn((double)pool_value(g, pool, lut, base, iy, ix, ch), w00));
    v = __dadd_rn(v, __dmul_rn((double)pool_value(g, pool, lut, base, iy, ix + 1, ch), w01));
    v = __dadd_rn(v, __dmul_rn((double)pool_value(g, pool, lut, base, iy + 1, ix, ch), w10));
    v = __dadd_rn(v, __dmul_rn((double)pool_value(g, pool, lut, base, iy + 1, ix + 1, ch), w11));
    v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);  // np.clip(0, 1)
    out[ch] = (float)v;
  }
  return err;
}

// ------------------------------------------------------------------ stream draws (k_fill_*)
// A batch of n draws from ONE numpy stream, spread over the chip: every thread jumps to its own
// stretch of FILL_PER_THREAD words of the stream (pcg_advance) and walks it.  integers() rejects
// candidates (Lemire), so output i is the i-th accepted candidate: k_fill_count counts per thread,
// k_fill_write places each thread's accepted draws at its prefix, and its last workgroup to finish (a ticket
// counter in work[0], left at zero; last_block_done) advances the generator state past the consumed words (and,
// if the candidates ran out, which is astronomically rare for the sizes used, finishes sequentially) once every
// workgroup has read the state; uniform draws finish the same way when given a counter.  Few outputs per thread:
// the kernels' time is one thread's chain (the jump, then its outputs), not the chip's throughput.
constexpr int FILL_THREADS = 256;
#ifndef APG_FILL_PER_THREAD
#define APG_FILL_PER_THREAD 8
#endif
constexpr int FILL_PER_THREAD = APG_FILL_PER_THREAD;
constexpr int FILL_PER_BLOCK = FILL_THREADS * FILL_PER_THREAD;

struct FillArgs {
  int kind;
  int64_t n;
  int cols;
  double low[2], range[2];
  int64_t lo;
  uint64_t bound;   // exclusive range of integers(lo, lo + bound)
  int64_t cand;     // candidate words examined in parallel (>= n)
  int nblocks;
  // k_fill_count copies save_words words save_src -> save_dst first (apg_image_draw_ahead's snapshot of the streams,
  // taken by the first kernel of the draws instead of a separate copy launch)
  const uint64_t *save_src;
  uint64_t *save_dst;
  int save_words;
};

// work layout (int64): the finishing ticket counter, then (`wk` = work + 1) [nblocks] block totals,
// [nblocks * FILL_THREADS] thread counts, consumed
APG_DEV int64_t *fill_consumed(int64_t *wk, int nblocks) { return wk + (size_t)nblocks * (FILL_THREADS + 1); }

int64_t fill_work_elems(int64_t cand) {
  const int64_t nb = (cand + FILL_PER_BLOCK - 1) / FILL_PER_BLOCK;
  return 1 + nb * (FILL_THREADS + 1) + 1;
}

// true in exactly one thread of the grid: thread 0 of the last workgroup to get here (every workgroup calls it, all
// of its threads; the counter returns to zero).  No release / acquire fence (~3.5 us each on gfx950): what the last
// workgroup relies on is (1) every workgroup has read the generator state -- its loads returned before its barrier --
// and (2) the consumed-word count, written with an agent-scope (sc1) store and read with an agent-scope load, every
// wave having drained its stores (vmcnt(0)) before the barrier behind which lane 0 takes the ticket
// (MI355X_MICROARCH.md, inter-workgroup visibility: the sc1 store / load with a counter add form).
// last_block: the same test, true in every thread of that workgroup (block-uniform)
APG_DEV bool last_block(int64_t *counter) {
  __shared__ bool s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(counter), 1ULL,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == (unsigned long long)(gridDim.x - 1);
    if (s_last) __hip_atomic_store(reinterpret_cast<unsigned long long *>(counter), 0ULL, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last;
}

APG_DEV bool last_block_done(int64_t *counter) { return last_block(counter) && threadIdx.x == 0; }

// sum of v[0, n) over the workgroup's threads (strided loads issued together, not one dependent round trip per
// element), returned to every thread
APG_DEV int64_t block_sum(const int64_t *v, int n) {
  __shared__ int64_t s_red[FILL_THREADS / 64];
  int64_t t = 0;
  for (int k = threadIdx.x; k < n; k += FILL_THREADS) t += v[k];
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = t;
  __syncthreads();
  t = 0;
  for (int w = 0; w < FILL_THREADS / 64; w++) t += s_red[w];
  return t;
}

struct LemireSpec {
  bool full;
  uint32_t rex, thr;
};

APG_DEV LemireSpec lemire_spec(uint64_t bound) {
  LemireSpec l;
  const uint64_t rng = bound - 1;
  l.full = rng == 0xffffffffULL;
  l.rex = (uint32_t)(rng + 1);
  l.thr = l.full ? 0u : (uint32_t)((0xffffffffULL - rng) % l.rex);
  return l;
}

APG_DEV bool lemire_accept(const LemireSpec &l, uint32_t u) {
  return l.full || (uint32_t)((uint64_t)u * l.rex) >= l.thr;
}

APG_DEV int64_t lemire_value(const LemireSpec &l, uint32_t u) {
  return (int64_t)(l.full ? (uint64_t)u : (((uint64_t)u * l.rex) >> 32));
}

// counter != nullptr: the last workgroup advances the state (else k_fill_uniform_finish does, launched after)
__global__ __launch_bounds__(FILL_THREADS) void k_fill_uniform(apg_pcg64 *st, FillArgs a, double *out,
                                                               int64_t *counter) {
  // random_uniform: off + scale * next_double, one next64 per value, C order over (n, cols)
  const int64_t m = a.n * a.cols;
  const int64_t k0 = ((int64_t)blockIdx.x * FILL_THREADS + threadIdx.x) * FILL_PER_THREAD;
  if (k0 < m) {
    const int64_t k1 = k0 + FILL_PER_THREAD < m ? k0 + FILL_PER_THREAD : m;
    Pcg64 r = *reinterpret_cast<const Pcg64 *>(st);
    pcg_advance(r, (uint64_t)k0);
    for (int64_t k = k0; k < k1; k++) {
      const int c = a.cols == 1 ? 0 : (int)(k & 1);
      out[k] = __dadd_rn(a.low[c], __dmul_rn(a.range[c], next_double(r)));
    }
  }
  if (counter && last_block_done(counter)) {
    Pcg64 r = *reinterpret_cast<const Pcg64 *>(st);
    pcg_advance(r, (uint64_t)m);
    *reinterpret_cast<Pcg64 *>(st) = r;
  }
}

__global__ void k_fill_uniform_finish(apg_pcg64 *st, int64_t m) {
  Pcg64 r = *reinterpret_cast<const Pcg64 *>(st);
  pcg_advance(r, (uint64_t)m);
  *reinterpret_cast<Pcg64 *>(st) = r;
}

__global__ __launch_bounds__(FILL_THREADS) void k_fill_count(const apg_pcg64 *st, FillArgs a, int64_t *work_all) {
  int64_t *work = work_all + 1;
  __shared__ int s_sum[FILL_THREADS / 64];
  if (blockIdx.x == 0 && (int)threadIdx.x < a.save_words) a.save_dst[threadIdx.x] = a.save_src[threadIdx.x];
  const LemireSpec l = lemire_spec(a.bound);
  const int64_t k0 = ((int64_t)blockIdx.x * FILL_THREADS + threadIdx.x) * FILL_PER_THREAD;
  int cnt = 0;
  if (k0 < a.cand) {
    const int64_t k1 = k0 + FILL_PER_THREAD < a.cand ? k0 + FILL_PER_THREAD : a.cand;
    Next32Walker wk(*reinterpret_cast<const Pcg64 *>(st), (uint64_t)k0);
    for (int64_t k = k0; k < k1; k++) cnt += lemire_accept(l, wk.next()) ? 1 : 0;
  }
  work[a.nblocks + (size_t)blockIdx.x * FILL_THREADS + threadIdx.x] = cnt;
  int v = cnt;
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < FILL_THREADS / 64; w++) t += s_sum[w];
    work[blockIdx.x] = t;
  }
}

APG_DEV void fill_finish(apg_pcg64 *st, const FillArgs &a, int64_t *out, int64_t *work);

__global__ __launch_bounds__(FILL_THREADS) void k_fill_write(apg_pcg64 *st, FillArgs a, int64_t *out,
                                                             int64_t *work_all) {
  int64_t *work = work_all + 1;
  __shared__ int64_t s_wave[FILL_THREADS / 64];
  const LemireSpec l = lemire_spec(a.bound);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cnt = work[a.nblocks + (size_t)blockIdx.x * FILL_THREADS + threadIdx.x];
  int64_t inc = cnt;
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) s_wave[wave] = inc;
  // the accepted counts of the preceding workgroups (its barrier also publishes s_wave)
  int64_t q = block_sum(work, (int)blockIdx.x) + inc - cnt;
  for (int w = 0; w < wave; w++) q += s_wave[w];
  const int64_t k0 = ((int64_t)blockIdx.x * FILL_THREADS + threadIdx.x) * FILL_PER_THREAD;
  if (cnt != 0 && q < a.n) {
    const int64_t k1 = k0 + FILL_PER_THREAD < a.cand ? k0 + FILL_PER_THREAD : a.cand;
    Next32Walker wk(*reinterpret_cast<const Pcg64 *>(st), (uint64_t)k0);
    for (int64_t k = k0; k < k1 && q < a.n; k++) {
      const uint32_t u = wk.next();
      if (lemire_accept(l, u)) {
        out[q] = a.lo + lemire_value(l, u);
        if (q == a.n - 1)  // read by the last workgroup (last_block_done): an agent-scope store
          __hip_atomic_store(reinterpret_cast<unsigned long long *>(fill_consumed(work, a.nblocks)),
                             (unsigned long long)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        q++;
      }
    }
  }
  if (last_block(work_all)) fill_finish(st, a, out, work);  // block-uniform: the whole last workgroup
}

APG_DEV void fill_finish(apg_pcg64 *st, const FillArgs &a, int64_t *out, int64_t *work) {
  const int64_t total = block_sum(work, a.nblocks);
  if (threadIdx.x != 0) return;
  const LemireSpec l = lemire_spec(a.bound);
  const Pcg64 base = *reinterpret_cast<const Pcg64 *>(st);
  Pcg64 r;
  if (total >= a.n) {
    r = after_next32_words(base, (uint64_t)__hip_atomic_load(reinterpret_cast<unsigned long long *>(
                                        fill_consumed(work, a.nblocks)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  } else {  // not enough accepted candidates: continue sequentially after all of them
    r = after_next32_words(base, (uint64_t)a.cand);
    for (int64_t i = total; i < a.n; i++) {
      uint32_t u;
      do {
        u = next32(r);
      } while (!lemire_accept(l, u));
      out[i] = a.lo + lemire_value(l, u);
    }
  }
  *reinterpret_cast<Pcg64 *>(st) = r;
}

__global__ void k_fill_const(int64_t n, int64_t v, int64_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = v;
}

// ------------------------------------------------------------------ seeding chain
__global__ void k_image_seed(apg_pcg64 *rng, uint64_t seed) {
  // gymnasium VectorEnv.reset(seed): np_random = default_rng(seed); the _np_random setter seeds the
  // module with np_random.integers(0, 2**32 - 1, endpoint=True) (a full-range next_uint32);
  // module.seed: current_rng = default_rng(s); DatasetBatchIterator(seed=current_rng.integers(...))
  Pcg64 env = seed_pcg64(seed);
  const uint32_t s_module = next32(env);
  Pcg64 cur = seed_pcg64(s_module);
  const uint32_t s_iter = next32(cur);
  const Pcg64 it = seed_pcg64(s_iter);
  reinterpret_cast<Pcg64 *>(rng)[0] = env;
  reinterpret_cast<Pcg64 *>(rng)[1] = cur;
  reinterpret_cast<Pcg64 *>(rng)[2] = it;
}

// ------------------------------------------------------------------ k_image_gather
// This shard's slice of the batch draws: data point index, label (+ inversion), start position.
__global__ void k_image_gather(int n, int offset, const int32_t *pool_labels, const int64_t *idx_draw,
                               int invert, const int64_t *inv_draw, const double *pos_draw, int num_classes,
                               int64_t *index, int32_t *label, int32_t *inverted, double *pos) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int d = offset + e;
  const int64_t idx = idx_draw[d];
  index[e] = idx;
  int32_t l = pool_labels[idx];
  if (invert) {
    const int32_t inv = inv_draw[d] == 1 ? 1 : 0;  // integers(0, 2, N) == 1
    inverted[e] = inv;
    if (inv) l = num_classes - l - 1;
  }
  label[e] = l;
  pos[2 * e] = pos_draw[2 * d];
  pos[2 * e + 1] = pos_draw[2 * d + 1];
}

// ------------------------------------------------------------------ k_glimpse
template <class PosT>
__global__ __launch_bounds__(256) void k_glimpse(GlimpseGeo g, const void *pool, const int64_t *index,
                                                 const PosT *pos, int npos, int total, float *out, uint32_t *err) {
  __shared__ float s_lut[256];
  load_u8_table(s_lut);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // total < 2^31 (checked by the host)
  if (t >= total) return;
  const int per = g.s0 * g.s1;
  const int np_ = t / per, pix = t - np_ * per;  // np_ = env * npos + p
  const int i = pix / g.s1, j = pix - i * g.s1;
  const int e = np_ / npos;
  const double px = (double)pos[2 * np_], py = (double)pos[2 * np_ + 1];
  float v[3];
  const uint32_t bad = glimpse_pixel(g, pool, s_lut, index[e] * g.img_elems, px, py, i, j, v);
  float *dst = out + (size_t)np_ * g.pitch + (size_t)pix * g.c;
  for (int ch = 0; ch < g.c; ch++) dst[ch] = v[ch];
  if (bad) atomicOr(err, bad);
}

// k_glimpse_sep: the same pixels, UPB glimpse units (env x position) per workgroup, using that the
// bilinear coordinates are separable: the row interval / weight of pixel (i, j) depends on i only and
// the column ones on j only, so they are computed once per unit row and column (G0 + G1 values instead
// of G0 * G1) and shared through LDS; each pixel then forms its four weights and reads its taps.
// Divisions by the launch-invariant unit and row sizes use host-computed reciprocals (FastDiv).
constexpr int GS_THREADS = 256, GS_MAX_UNITS = 128, GS_MAX_SIDE = 256;
struct FastDiv {  // n / d for n < 2^32 / d: (n * ceil(2^32 / d)) >> 32
  uint32_t d, m;
  APG_DEV uint32_t div(uint32_t n) const { return d == 1 ? n : __umulhi(n, m); }
};
FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.m = d <= 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) + d - 1) / d);
  return f;
}

struct Axis {     // one sampling coordinate: pool offsets of its grid interval's two ends (rows: idx * w * pc and
  int off, off1;  // (idx + 1) * w * pc, columns: idx * pc and (idx + 1) * pc; tiled pools: tile_row_off /
  double w, nw;   // tile_col_off of idx and idx + 1), fractional weight, 1 - weight
};

// Separable glimpse of `nu` units (env x position) starting at unit u0, in two passes over a workgroup:
// gs_axes computes every unit's row and column grid intervals / weights once (into LDS s_ax, plus the
// pool offset of its image), gs_pixels then evaluates one pixel per thread from them.
template <int GT = GS_THREADS, class PosAt>
APG_DEV uint32_t gs_axes(const GlimpseGeo &g, const int64_t *index, PosAt pos_at, int u0, int nu, int npos,
                         FastDiv side_div, Axis *s_ax, int64_t *s_base) {
  const int side = g.s0 + g.s1;
  uint32_t bad = 0;
  for (int q = threadIdx.x; q < nu * side; q += GT) {
    const int u = (int)side_div.div((uint32_t)q), k = q - u * side;
    const bool row = k < g.s0;
    const int t = row ? k : k - g.s0;
    const double p = pos_at(u, row ? 1 : 0);
    // flip(denormalize(pos)) + offsets (glimpse_pixel): rows use pos[1], columns pos[0]
    const double off = __dmul_rn(__dsub_rn((double)t, ((double)(row ? g.s0 : g.s1) - 1.0) / 2.0), g.scale);
    const double c = __dadd_rn(__dmul_rn(p, row ? g.lim_y : g.lim_x), off);
    const double lim = row ? g.cy : g.cx;
    if (!(c >= -lim && c <= lim)) bad |= row ? APG_ERR_OOB_Y : APG_ERR_OOB_X;
    Axis ax;
    const int iv = grid_interval(c, lim, row ? g.h : g.w, ax.w);
    if (g.tiled) {
      ax.off = row ? (int)tile_row_off(g, iv) : tile_col_off(iv);
      ax.off1 = row ? (int)tile_row_off(g, iv + 1) : tile_col_off(iv + 1);
    } else {
      ax.off = iv * (row ? g.w * g.pc : g.pc);
      ax.off1 = ax.off + (row ? g.w * g.pc : g.pc);
    }
    ax.nw = __dsub_rn(1.0, ax.w);
    s_ax[q] = ax;
    if (k == 0 && index) s_base[u] = index[(u0 + u) / npos] * g.img_elems;  // index == nullptr: s_base is set
  }
  return bad;
}

// one instantiation per pool format (u8 / f32), pool channels PC and output channels C (validate() admits
// (1, 1), (1, 3), (3, 3)), so the channel loops unroll and the u8 table reads stay LDS reads
// u8 taps of one glimpse pixel: the dwords holding its two rows' 2 * PC tap bytes, and their byte offsets
struct U8Taps {
  uint32_t a00, a01, a02, a10, a11, a12;
  int o0, o1;
};
#ifndef APG_TAPS_WIDE
#define APG_TAPS_WIDE 1  // (0: the per-dword tap loads of round 4, A/B knob)
#endif

template <bool F32, int PC, int C, int GT = GS_THREADS, bool TILED = false>
APG_DEV void gs_pixels_t(const GlimpseGeo &g, const void *pool, int u0, int nu, FastDiv per_div, FastDiv s1_div,
                         const Axis *s_ax, const int64_t *s_base, const float *s_lut, float *out) {
  const int side = g.s0 + g.s1;
  const int per = g.s0 * g.s1;
  const int row_elems = g.w * PC;
  const int total = nu * per;
  auto coords = [&](int q, int &u, int &i, int &j) {
    u = (int)per_div.div((uint32_t)q);
    const int pix = q - u * per;
    i = (int)s1_div.div((uint32_t)pix);
    j = pix - i * g.s1;
  };
  // weights in the hypercube order of _evaluate_linear: (i0, j0), (i0, j0+1), (i0+1, j0), (i0+1, j0+1); (1*wy)*wx
  auto weights = [&](const Axis &ay, const Axis &axx, double &w00, double &w01, double &w10, double &w11) {
    w00 = __dmul_rn(ay.nw, axx.nw), w01 = __dmul_rn(ay.nw, axx.w), w10 = __dmul_rn(ay.w, axx.nw),
    w11 = __dmul_rn(ay.w, axx.w);
  };
  auto store = [&](int q, int u, const float *res) {
    float *dst = out + (size_t)(u0 + u) * g.pitch + (size_t)(q - u * per) * C;
    if constexpr (C == 3) {
      struct F3 {
        float x, y, z;
      };
      *reinterpret_cast<F3 *>(dst) = F3{res[0], res[1], res[2]};  // one 12-byte store per pixel
    } else {
      __builtin_nontemporal_store(res[0], dst);  // the glimpses are read by the consumer, not by this kernel
    }
  };
  if constexpr (TILED) {
    // RGBX tiles (APG_POOL_U8_TILED): each tap one aligned dword, its channels at fixed byte positions; the four
    // taps from the axes' two row and two column offsets (a tap pair may straddle a tile edge)
    static_assert(PC == 3 && C == 3, "tiled pools are RGB");
    const uint8_t *im = static_cast<const uint8_t *>(pool);
    for (int q = threadIdx.x; q < total; q += GT) {
      int u, i, j;
      coords(q, u, i, j);
      const Axis ay = s_ax[u * side + i], axx = s_ax[u * side + g.s0 + j];
      const uint8_t *b = im + s_base[u];
      const uint32_t t00 = *reinterpret_cast<const uint32_t *>(b + (ay.off + axx.off)),
                     t01 = *reinterpret_cast<const uint32_t *>(b + (ay.off + axx.off1)),
                     t10 = *reinterpret_cast<const uint32_t *>(b + (ay.off1 + axx.off)),
                     t11 = *reinterpret_cast<const uint32_t *>(b + (ay.off1 + axx.off1));
      double w00, w01, w10, w11;
      weights(ay, axx, w00, w01, w10, w11);
      auto tap = [&](uint32_t t, int ch) { return u8_value_f32((t >> (8 * ch)) & 0xffu); };
      float res[3];
#pragma unroll
      for (int ch = 0; ch < 3; ch++) {
        double v = __dmul_rn((double)tap(t00, ch), w00);
        v = __dadd_rn(v, __dmul_rn((double)tap(t01, ch), w01));
        v = __dadd_rn(v, __dmul_rn((double)tap(t10, ch), w10));
        v = __dadd_rn(v, __dmul_rn((double)tap(t11, ch), w11));
        res[ch] = (float)fmin(v, 1.0);
      }
      store(q, u, res);
    }
  } else if constexpr (F32) {
    const float *im = static_cast<const float *>(pool);
    for (int q = threadIdx.x; q < total; q += GT) {
      int u, i, j;
      coords(q, u, i, j);
      const Axis ay = s_ax[u * side + i], axx = s_ax[u * side + g.s0 + j];
      double w00, w01, w10, w11;
      weights(ay, axx, w00, w01, w10, w11);
      const int64_t r0 = s_base[u] + (ay.off + axx.off), r1 = r0 + row_elems;
      float res[C];
#pragma unroll
      for (int ch = 0; ch < C; ch++) {
        const int cc = PC == 1 ? 0 : ch;
        double v = __dadd_rn(0.0, __dmul_rn((double)im[r0 + cc], w00));
        v = __dadd_rn(v, __dmul_rn((double)im[r0 + PC + cc], w01));
        v = __dadd_rn(v, __dmul_rn((double)im[r1 + cc], w10));
        v = __dadd_rn(v, __dmul_rn((double)im[r1 + PC + cc], w11));
        res[ch] = (float)(v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));  // np.clip(0, 1)
      }
      store(q, u, res);
    }
  } else {
    // the 2 * PC tap bytes of each row are contiguous: aligned dword loads, only the ones they occupy (issuing
    // the next pixel's loads ahead of this pixel's arithmetic measured slower: register pressure)
    const uint8_t *im = static_cast<const uint8_t *>(pool);
    constexpr int span = 2 * PC;
    auto fetch = [&](int q) {
      int u, i, j;
      coords(q, u, i, j);
      const int64_t r0 = s_base[u] + (s_ax[u * side + i].off + s_ax[u * side + g.s0 + j].off), r1 = r0 + row_elems;
      U8Taps t;
      t.o0 = (int)(reinterpret_cast<uintptr_t>(im + r0) & 3u);
      t.o1 = (int)(reinterpret_cast<uintptr_t>(im + r1) & 3u);
      // pointer arithmetic (not integer round trips) keeps the loads global rather than flat
      const uint32_t *d0 = reinterpret_cast<const uint32_t *>(im + (r0 - t.o0)),
                     *d1 = reinterpret_cast<const uint32_t *>(im + (r1 - t.o1));
      if constexpr (APG_TAPS_WIDE && span > 4) {
        // RGB: one dwordx3 load per row instead of up to three dword loads (a third of the address work:
        // TinyImageNetLoc 31.1-31.5 -> 30.6 us); it reads up to 6 bytes past the row's taps (u8 pools carry
        // APG_U8_POOL_PAD bytes of slack after the last image, apgym_capi.h).  Grey pools keep the per-dword
        // loads (an unconditional dwordx2 measured 11.4 -> 11.6 us at MNIST)
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        u32x3 v0, v1;
        __builtin_memcpy(&v0, d0, 12);
        __builtin_memcpy(&v1, d1, 12);
        t.a00 = v0.x, t.a01 = v0.y, t.a02 = v0.z;
        t.a10 = v1.x, t.a11 = v1.y, t.a12 = v1.z;
      } else {
        t.a00 = d0[0];
        t.a10 = d1[0];
        t.a01 = t.o0 + span > 4 ? d0[1] : 0u;
        t.a11 = t.o1 + span > 4 ? d1[1] : 0u;
        t.a02 = t.a12 = 0u;
        if constexpr (span > 4) {
          t.a02 = t.o0 + span > 8 ? d0[2] : 0u;
          t.a12 = t.o1 + span > 8 ? d1[2] : 0u;
        }
      }
      return t;
    };
    for (int q = threadIdx.x; q < total; q += GT) {
      const U8Taps cur = fetch(q);
      int u, i, j;
      coords(q, u, i, j);
      const Axis ay = s_ax[u * side + i], axx = s_ax[u * side + g.s0 + j];
      double w00, w01, w10, w11;
      weights(ay, axx, w00, w01, w10, w11);
      // the span bytes realigned to byte 0 (funnel shifts by the runtime offset), so every tap sits at a
      // compile-time byte position
      const uint32_t b0[2] = {__builtin_amdgcn_alignbit(cur.a01, cur.a00, 8u * cur.o0),
                              __builtin_amdgcn_alignbit(cur.a02, cur.a01, 8u * cur.o0)};
      const uint32_t b1[2] = {__builtin_amdgcn_alignbit(cur.a11, cur.a10, 8u * cur.o1),
                              __builtin_amdgcn_alignbit(cur.a12, cur.a11, 8u * cur.o1)};
      auto tap = [&](const uint32_t *b, int t) {
        const uint32_t v = (b[t >> 2] >> (8 * (t & 3))) & 0xffu;  // a compile-time byte: v_cvt_f32_ubyteN
        return APG_U8_ARITH ? u8_value_f32(v) : s_lut[v];
      };
      float res[C];
#pragma unroll
      for (int ch = 0; ch < C; ch++) {
        const int cc = PC == 1 ? 0 : ch;
        // u8 taps and the weights are >= +0: 0.0 + t00 * w00 is t00 * w00 and only the upper clip applies
        double v = __dmul_rn((double)tap(b0, cc), w00);
        v = __dadd_rn(v, __dmul_rn((double)tap(b0, PC + cc), w01));
        v = __dadd_rn(v, __dmul_rn((double)tap(b1, cc), w10));
        v = __dadd_rn(v, __dmul_rn((double)tap(b1, PC + cc), w11));
        res[ch] = (float)fmin(v, 1.0);
      }
      store(q, u, res);
    }
  }
}

APG_DEV void gs_pixels(const GlimpseGeo &g, const void *pool, int u0, int nu, FastDiv per_div, FastDiv s1_div,
                       const Axis *s_ax, const int64_t *s_base, const float *s_lut, float *out) {
#define APG_GS_PIXELS(F, P, C) gs_pixels_t<F, P, C>(g, pool, u0, nu, per_div, s1_div, s_ax, s_base, s_lut, out)
  if (g.tiled) {
    gs_pixels_t<false, 3, 3, GS_THREADS, true>(g, pool, u0, nu, per_div, s1_div, s_ax, s_base, s_lut, out);
  } else if (g.pool_f32) {
    if (g.pc == 3) APG_GS_PIXELS(true, 3, 3);
    else if (g.c == 3) APG_GS_PIXELS(true, 1, 3);
    else APG_GS_PIXELS(true, 1, 1);
  } else {
    if (g.pc == 3) APG_GS_PIXELS(false, 3, 3);
    else if (g.c == 3) APG_GS_PIXELS(false, 1, 3);
    else APG_GS_PIXELS(false, 1, 1);
  }
#undef APG_GS_PIXELS
}

template <class PosT>
__global__ __launch_bounds__(GS_THREADS) void k_glimpse_sep(GlimpseGeo g, const void *pool, const int64_t *index,
                                                            const PosT *pos, int npos, int units, int upb,
                                                            FastDiv per_div, FastDiv s1_div, FastDiv side_div,
                                                            float *out, uint32_t *err) {
  __shared__ float s_lut[256];
  extern __shared__ Axis s_ax[];  // [unit][rows s0 | columns s1]
  __shared__ int64_t s_base[GS_MAX_UNITS];
  if (!APG_U8_ARITH) for (int v = threadIdx.x; v < 256; v += GS_THREADS) s_lut[v] = u8_value((unsigned)v);
  const int u0 = blockIdx.x * upb, nu = units - u0 < upb ? units - u0 : upb;
  const uint32_t bad = gs_axes(g, index, [&](int u, int c) { return (double)pos[2 * (u0 + u) + c]; }, u0, nu, npos,
                               side_div, s_ax, s_base);
  __syncthreads();
  gs_pixels(g, pool, u0, nu, per_div, s1_div, s_ax, s_base, s_lut, out);
  if (bad) atomicOr(err, bad);
}

// ------------------------------------------------------------------ k_image_env
struct EnvArgs {
  int n, kind, k, resetting, log_stats, limit, t_new;
  int row;  // apg_image_config.out_row_bytes (0: dense outputs)
  double msl[2];
  double ce_scale, ce_offset;
  float mse_scale, mse_offset;
  float time_value;
  float loss_weight;  // 1, or for the -sparse ids terminated.astype(float32) (one value: episodes end together)
  int copy_target;  // localize, steps without a target refresh: prediction_target = target.copy() here
  float *target_st;  // the state's targets (localize)
  // the batch autoreset with its draws made ahead (apg_image_draw_ahead), k_image_gather and k_loc_target folded
  // into the step kernel: draws of env e at d = offset + e, the index / inversion draws at ahead_i64[d] /
  // [nt + d], the start / target draws at ahead_f64[2 d] / [2 nt + 2 d]; NULL: the draws (if any) are installed
  // already.  (Few fields: the kernel's SGPR budget holds the arguments without spilling.)
  const int64_t *ahead_i64;
  const double *ahead_f64;
  const int32_t *pool_labels;
  int32_t *inverted_st;
  int invert, offset, nt;
};


// numpy's float32 exp and log (the AVX-512F loops np.exp / np.log run on contiguous float32 arrays, numpy 2.2:
// simd_exp_f32 / simd_log_f32), restated operation by operation so that the CE loss (scipy.special.log_softmax:
// np.exp of x - max, np.log of the pairwise sum) is bit-exact.  The constants are numpy's float32 coefficients (read
// from the loops' constant pool of the installed numpy); checked bit for bit against np.exp on every float32 in
// [-103.97, 0] and np.log on every float32 in [1, 65536] (the ranges a log-softmax feeds them), tests/test_host.py.
// exp: x = q ln2 + r with q = rint(x log2e) (the 1.5 * 2^23 magic), r by two Cody-Waite fmas; exp(r) as a [5/2]
// rational in fmas and one correctly rounded division; scaled by 2^q with one rounding (vscalefps); x >= 88.72 -> inf,
// x <= -103.97 -> 0.
APG_DEV float np_expf(float x) {
  if (x != x) return x;
  if (x >= 88.72283935546875f) return __int_as_float(0x7f800000);
  if (x <= -103.97208404541015625f) return 0.0f;
  const float q = __fsub_rn(__fadd_rn(__fmul_rn(x, 1.4426950216293335f), 12582912.0f), 12582912.0f);
  float r = __fmaf_rn(q, -0.693145751953125f, x);
  r = __fmaf_rn(q, -1.428606765330187e-06f, r);
  r = __fmaf_rn(q, 0.0f, r);
  float num = __fmaf_rn(5.082762800157070e-04f, r, 6.757896859198809e-03f);
  num = __fmaf_rn(num, r, 5.1145121455192566e-02f);
  num = __fmaf_rn(num, r, 2.4736154079437256e-01f);
  num = __fmaf_rn(num, r, 7.2576647996902466e-01f);
  num = __fmaf_rn(num, r, 1.0f);
  float den = __fmaf_rn(2.1595094352960587e-02f, r, -2.7423354983329773e-01f);
  den = __fmaf_rn(den, r, 1.0f);
  const float poly = f32_div(num, den);
  // poly * 2^q (q integral in [-150, 128]): exact in f64, one rounding to f32 (subnormal results included)
  return __double2float_rn(__dmul_rn((double)poly, __longlong_as_double((long long)(1023 + (int)q) << 52)));
}
// log: x = m 2^e with m in [0.5, 1) (vgetmantps / vgetexpps); m <= sqrt(1/2) is doubled (e - 1); log(m) as a [5/5]
// rational of m - 1 in fmas and one correctly rounded division, + e ln2 by one fma.  0 -> -inf, < 0 / NaN -> NaN,
// inf -> inf.
APG_DEV float np_logf(float x) {
  if (!(x > 0.0f)) return x == 0.0f ? __int_as_float(0xff800000) : __int_as_float(0x7fc00000);
  if (x == __int_as_float(0x7f800000)) return x;
  int e;
  float m = frexpf(x, &e);
  float ex = (float)e;
  if (m <= 0.70710676908493042f) {
    m = __fadd_rn(m, m);
    ex = __fsub_rn(ex, 1.0f);
  }
  const float r = __fsub_rn(m, 1.0f);
  float num = __fmaf_rn(2.5899792090058327e-02f, r, 3.8088378310203552e-01f);
  num = __fmaf_rn(num, r, 1.4800006151199341f);
  num = __fmaf_rn(num, r, 2.1126775741577148f);
  num = __fmaf_rn(num, r, 1.0f);
  num = __fmaf_rn(num, r, 0.0f);
  float den = __fmaf_rn(5.8750952593982220e-03f, r, 1.5464763343334198e-01f);
  den = __fmaf_rn(den, r, 9.8649430274963379e-01f);
  den = __fmaf_rn(den, r, 2.4530060291290283f);
  den = __fmaf_rn(den, r, 2.6126775741577148f);
  den = __fmaf_rn(den, r, 1.0f);
  return __fmaf_rn(ex, 0.69314718246459961f, f32_div(num, den));
}

// scipy.special.log_softmax(row)[target] in float32 (x_max zeroed when not finite); -> -value
APG_DEV float ce_f32(const float *row, int k, int target) {
  float m = row[0];
  bool nan = false;
  for (int i = 0; i < k; i++) {
    const float v = row[i];
    if (v != v) nan = true;
    m = v > m ? v : m;
  }
  if (nan || isinf(m)) m = 0.0f;  // np.amax propagates NaN; x_max[~isfinite] = 0
  auto ex = [&](int i) { return np_expf(__fsub_rn(row[i], m)); };
  const float s = pw_sum<MAX_PW_DEPTH>(ex, 0, k);
  const float out = __fsub_rn(__fsub_rn(row[target], m), np_logf(s));
  return -out;
}

// Vector log wrappers of the registered ids (active_classification_env.py:116-197,
// active_regression_env.py:160-227, util.py:40-80): the per-step metric of the episode is recorded
// at index t - 1 (the autoreset step clears the wrapper's deque and records nothing); on the
// episode's last step final = value at t - 1 and avg = np.mean(list) (numpy's pairwise f32 mean).
APG_DEV float episode_mean(const float *h, int len) {
  return f32_div(__fadd_rn(0.0f, pw_sum_ptr(h, len)), (float)len);
}

APG_DEV void log_regression(const EnvArgs &a, int e, const apg_image_outputs &out, float *hist, float ed, float mse) {
  if (!a.log_stats || a.resetting) return;
  float *h0 = hist + (size_t)e * 2 * a.limit, *h1 = h0 + a.limit;
  h0[a.t_new - 1] = ed;
  h1[a.t_new - 1] = mse;
  if (a.t_new < a.limit) return;
  ro_t(out.stats, a.row, a.n, e, 0) = ed;
  ro_t(out.stats, a.row, a.n, e, 1) = mse;
  ro_t(out.stats, a.row, a.n, e, 2) = episode_mean(h0, a.limit);
  ro_t(out.stats, a.row, a.n, e, 3) = episode_mean(h1, a.limit);
}

APG_DEV void log_classification(const EnvArgs &a, int e, const apg_image_outputs &out, float *hist, float prob) {
  if (!a.log_stats || a.resetting) return;
  float *h = hist + (size_t)e * 2 * a.limit;
  h[a.t_new - 1] = prob;
  if (a.t_new < a.limit) return;
  // accuracy = correct_label_prob > 1 / num_classes (the Python float compared as float32, NEP 50)
  const float thr = (float)(1.0 / (double)a.k);
  float *acc = h + a.limit;
  int first_correct = -1, last_incorrect = -1;
  for (int i = 0; i < a.limit; i++) {
    const bool c = h[i] > thr;
    acc[i] = c ? 1.0f : 0.0f;
    if (c && first_correct < 0) first_correct = i;
    if (!c) last_incorrect = i;
  }
  ro_t(out.stats, a.row, a.n, e, 0) = prob;
  ro_t(out.stats, a.row, a.n, e, 1) = acc[a.limit - 1];
  ro_t(out.stats, a.row, a.n, e, 2) = episode_mean(h, a.limit);
  ro_t(out.stats, a.row, a.n, e, 3) = episode_mean(acc, a.limit);
  ro_t(out.stats_idx, a.row, a.n, e, 0) = first_correct;
  ro_t(out.stats_idx, a.row, a.n, e, 1) = last_incorrect;
}

// ImagePerceptionModule.step's move (:197-213): project_sphere (util.py:94-97) in f32, then
// max_step_length (f64) * step, clip(-1, 1); returns |action| (f32) for the base reward.
APG_DEV float move_pos(const EnvArgs &a, float a0, float a1, double &px, double &py) {
  const float mag = norm_f32(a0, a1);
  float s0 = a0, s1 = a1;
  if (mag > 1.0f) {
    s0 = __fmul_rn(f32_div(a0, mag), 1.0f);
    s1 = __fmul_rn(f32_div(a1, mag), 1.0f);
  }
  px = __dadd_rn(px, __dmul_rn(a.msl[0], (double)s0));
  py = __dadd_rn(py, __dmul_rn(a.msl[1], (double)s1));
  px = px < -1.0 ? -1.0 : (px > 1.0 ? 1.0 : px);
  py = py < -1.0 ? -1.0 : (py > 1.0 ? 1.0 : py);
  return mag;
}

// Per-env inputs of the env step, loaded up front (the fused kernel loads them before its glimpse
// passes, so their latency hides behind the glimpse).
struct EnvIn {
  float a0, a1;          // action (not read on the autoreset step)
  double px, py;         // position before this step's move
  float p0, p1, t0, t1;  // localization: prediction, target before the autoreset update
  int32_t label;         // classification
};
// The batch autoreset of env e from the draws made ahead (k_image_gather + k_loc_target): the new data point,
// its label (inverted when drawn so), start position, and (localize) the pre-update target as this step's
// prediction target, the refreshed target into the state.  Returns the new image's pool index.
APG_DEV int64_t install_ahead(const EnvArgs &a, int e, const apg_image_outputs &out, double *pos, EnvIn &in,
                              int64_t *index_st, int32_t *label_st) {
  const int d = a.offset + e;
  const int64_t idx = a.ahead_i64[d];
  index_st[e] = idx;
  int32_t l = a.pool_labels[idx];
  if (a.invert) {
    const int32_t inv = a.ahead_i64[(size_t)a.nt + d] == 1 ? 1 : 0;  // integers(0, 2, N) == 1
    a.inverted_st[e] = inv;
    if (inv) l = a.k - l - 1;
  }
  label_st[e] = l;
  in.label = l;
  in.px = a.ahead_f64[2 * d];
  in.py = a.ahead_f64[2 * d + 1];
  pos[2 * e] = in.px;
  pos[2 * e + 1] = in.py;
  if (a.kind == APG_IMAGE_LOCALIZE) {  // prediction_target = target.copy(); target[prev_done] = uniform draws
    in.t0 = a.target_st[2 * e];
    in.t1 = a.target_st[2 * e + 1];
    ro(out.target, a.row, e, 2, 0) = in.t0;
    ro(out.target, a.row, e, 2, 1) = in.t1;
    a.target_st[2 * e] = (float)a.ahead_f64[2 * ((size_t)a.nt + d)];
    a.target_st[2 * e + 1] = (float)a.ahead_f64[2 * ((size_t)a.nt + d) + 1];
  }
  return idx;
}

template <int KIND>
APG_DEV EnvIn load_env_in(const EnvArgs &a, int e, const float *__restrict__ act, const float *__restrict__ pred,
                          const int32_t *label, const double *pos, const apg_image_outputs &out) {
  EnvIn in{};
  if (!a.resetting) {
    in.a0 = act[2 * e];
    in.a1 = act[2 * e + 1];
  }
  in.px = pos[2 * e];
  in.py = pos[2 * e + 1];
  if constexpr (KIND == APG_IMAGE_LOCALIZE) {
    in.p0 = pred[2 * e];
    in.p1 = pred[2 * e + 1];
    in.t0 = a.copy_target ? a.target_st[2 * e] : ro(out.target, a.row, e, 2, 0);
    in.t1 = a.copy_target ? a.target_st[2 * e + 1] : ro(out.target, a.row, e, 2, 1);
  } else {
    in.label = label[e];
  }
  return in;
}

// The per-env tail of ImagePerceptionModule.step (:197-213) + ActivePerceptionVectorEnv.step
// (reward = base_reward - loss): move (or not, on the autoreset step), rewards, glimpse_pos, time.
APG_DEV uint32_t env_tail(const EnvArgs &a, int e, const EnvIn &in, double *pos, const apg_image_outputs &out,
                          double loss_d, float loss_f) {
  uint32_t err = 0;
  double px = in.px, py = in.py;
  // WeightedLossFn (loss_fn.py:307-316): loss * weight; f64 * f32 -> f64 (classify), f32 * f32 (localize).
  // weight 1 leaves the loss bit-identical (including inf / NaN), so the dense ids share this path.
  loss_d = __dmul_rn(loss_d, (double)a.loss_weight);
  loss_f = __fmul_rn(loss_f, a.loss_weight);
  if (a.kind != APG_IMAGE_CLASSIFY) loss_d = (double)loss_f;
  if (a.resetting) {
    // module.reset() replaced the batch; base_reward = np.zeros(N) (float64)
    ro(out.base_reward, a.row, e, 1) = 0.0f;
    ro(out.reward, a.row, e, 1) = __dsub_rn(0.0, loss_d);
  } else {
    const float a0 = in.a0, a1 = in.a1;
    if (a0 != a0 || a1 != a1) err |= APG_ERR_NAN_ACTION;
    const float mag = move_pos(a, a0, a1, px, py);
    pos[2 * e] = px;
    pos[2 * e + 1] = py;
    const float base = __fmul_rn(-mag, 1e-3f);  // -norm(action) * 1e-3 (f32, weak Python scalar)
    ro(out.base_reward, a.row, e, 1) = base;
    ro(out.reward, a.row, e, 1) = a.kind == APG_IMAGE_CLASSIFY ? __dsub_rn((double)base, loss_d)
                                                               : (double)__fsub_rn(base, loss_f);
  }
  ro(out.glimpse_pos, a.row, e, 2, 0) = (float)px;
  ro(out.glimpse_pos, a.row, e, 2, 1) = (float)py;
  ro(out.time_step, a.row, e, 1) = a.time_value;
  return err;
}

// Localization step of env e: MSE against the target before the autoreset update.
APG_DEV void loc_env(const EnvArgs &a, int e, const EnvIn &in, double *pos, const apg_image_outputs &out,
                     float *hist) {
  uint32_t err = 0;
  const float p0 = in.p0, p1 = in.p1;
  if (p0 != p0 || p1 != p1) err |= APG_ERR_NAN_PREDICTION;  // 1 - |pred - target| / 2 is NaN
  const float t0 = in.t0, t1 = in.t1;
  if (a.copy_target) {  // k_loc_target folded in (no refresh this step)
    ro(out.target, a.row, e, 2, 0) = t0;
    ro(out.target, a.row, e, 2, 1) = t1;
  }
  const float d0 = __fsub_rn(p0, t0), d1 = __fsub_rn(p1, t1);
  // np.mean(f32 [2]): (0 + d0^2 + d1^2) / 2, then * scale + offset in f32
  const float mse = f32_div(__fadd_rn(__fadd_rn(0.0f, __fmul_rn(d0, d0)), __fmul_rn(d1, d1)), 2.0f);
  const float loss_f = __fadd_rn(__fmul_rn(mse, a.mse_scale), a.mse_offset);
  ro(out.loss_f32, a.row, e, 1) = loss_f;
  log_regression(a, e, out, hist, norm_f32(d0, d1), mse);  // |target - prediction|: signs do not matter
  err |= env_tail(a, e, in, pos, out, (double)loss_f, loss_f);
  if (err) atomicOr(out.err, err);
}

// Localization: one thread per env.
__global__ __launch_bounds__(256) void k_image_env_loc(EnvArgs a, const float *__restrict__ act,
                                                       const float *__restrict__ pred, double *pos,
                                                       apg_image_outputs out, float *hist) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < a.n) loc_env(a, e, load_env_in<APG_IMAGE_LOCALIZE>(a, e, act, pred, nullptr, pos, out), pos, out, hist);
}

// numpy pairwise sum of x[off .. off+n) by the 8 lanes of a group (lane j owns accumulator j of
// every <= 128 block; the combine and the < 8 tail are evaluated identically by all 8 lanes)
APG_DEV float pw_leaf8(const float *x, int off, int n, int j) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; i++) r = __fadd_rn(r, x[off + i]);
    return r;
  }
  float r = x[off + j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) r = __fadd_rn(r, x[off + i + j]);
  const int g0 = (int)(threadIdx.x & 63u) & ~7;
  float q[8];
#pragma unroll
  for (int k = 0; k < 8; k++) q[k] = __shfl(r, g0 + k, 64);
  float res = __fadd_rn(__fadd_rn(__fadd_rn(q[0], q[1]), __fadd_rn(q[2], q[3])),
                        __fadd_rn(__fadd_rn(q[4], q[5]), __fadd_rn(q[6], q[7])));
  for (; i < n; i++) res = __fadd_rn(res, x[off + i]);
  return res;
}

template <int DEPTH>
APG_DEV float pw_sum8(const float *x, int off, int n, int j) {
  if constexpr (DEPTH == 0) {
    return pw_leaf8(x, off, n, j);
  } else {
    if (n <= 128) return pw_leaf8(x, off, n, j);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __fadd_rn(pw_sum8<DEPTH - 1>(x, off, n2, j), pw_sum8<DEPTH - 1>(x, off + n2, n - n2, j));
  }
}

// Classification: 8 lanes per env, the block's logits staged in LDS with coalesced loads.
// Cross entropy = -(x[t] - m - log(sum(exp(x - m)))) in f32 (scipy.special.log_softmax), the exp
// sum in numpy's pairwise order; normalized with the f64 affine (loss_fn.py:100-110).
constexpr int CLS_LANES = 8;
__global__ __launch_bounds__(256) void k_image_env_cls(EnvArgs a, int envs_per_block, const float *__restrict__ act,
                                                       const float *__restrict__ pred, const int32_t *label,
                                                       double *pos, apg_image_outputs out, float *hist) {
  extern __shared__ float s_logit[];  // [envs_per_block][k + 1]
  const int k = a.k, stride = k + 1;
  const int e0 = blockIdx.x * envs_per_block;
  const int ne = a.n - e0 < envs_per_block ? a.n - e0 : envs_per_block;
  for (int q = threadIdx.x; q < ne * k; q += blockDim.x) {
    const int r = q / k;
    s_logit[r * stride + (q - r * k)] = pred[(size_t)e0 * k + q];
  }
  __syncthreads();
  const int grp = threadIdx.x / CLS_LANES, j = threadIdx.x % CLS_LANES;
  const bool live = grp < ne;
  float *row = s_logit + (live ? grp : 0) * stride;
  // max (NaN-propagating like np.amax) and the softmax NaN condition, over the 8 lanes
  float m = -INFINITY;
  bool nan = false, pos_inf = false, all_neg_inf = true;
  for (int i = j; i < k; i += CLS_LANES) {
    const float v = row[i];
    nan |= v != v;
    pos_inf |= v == INFINITY;
    all_neg_inf &= v == -INFINITY;
    m = v > m ? v : m;
  }
  for (int d = 1; d < CLS_LANES; d <<= 1) {
    const float om = __shfl_xor(m, d, 64);
    m = om > m ? om : m;
    nan |= __shfl_xor((int)nan, d, 64) != 0;
    pos_inf |= __shfl_xor((int)pos_inf, d, 64) != 0;
    all_neg_inf &= __shfl_xor((int)all_neg_inf, d, 64) != 0;
  }
  if (nan || isinf(m)) m = 0.0f;  // x_max[~isfinite(x_max)] = 0
  const int32_t l = live ? label[e0 + grp] : 0;
  const int lc = l < 0 ? 0 : (l >= k ? k - 1 : l);
  const float xt = row[lc];
  __syncthreads();
  if (live)  // lanes of the tail groups (grp >= ne) alias row 0 and must not write it
    for (int i = j; i < k; i += CLS_LANES) row[i] = np_expf(__fsub_rn(row[i], m));
  __syncthreads();
  const float sum = pw_sum8<MAX_PW_DEPTH>(row, 0, k, j);
  if (!live || j != 0) return;
  const int e = e0 + grp;
  uint32_t err = (nan || pos_inf || all_neg_inf) ? APG_ERR_NAN_PREDICTION : 0u;
  const float ce = -__fsub_rn(__fsub_rn(xt, m), np_logf(sum));
  const double loss_d = __dadd_rn(__dmul_rn((double)ce, a.ce_scale), a.ce_offset);
  ro(out.loss_f64, a.row, e, 1) = loss_d;
  ro(out.label_target, a.row, e, 1) = l;
  // scipy.special.softmax(prediction)[label] = exp(x_l - max) / sum(exp(x - max)) (finite logits)
  log_classification(a, e, out, hist, f32_div(row[lc], sum));
  err |= env_tail(a, e, load_env_in<APG_IMAGE_CLASSIFY>(a, e, act, pred, label, pos, out), pos, out, loss_d, 0.0f);
  if (err) atomicOr(out.err, err);
}

// Classification for few classes (K <= CLS1_MAX_K, e.g. MNIST / CIFAR-10): thread = env.  With 8 lanes
// per env most lanes idle for K = 10 and the tail (loss, stats, move) runs on one lane of eight; here a
// 128-thread block stages its 128 rows of logits in LDS with coalesced loads and every thread evaluates
// its own row: max, exp, numpy's pairwise sum (n <= 128: 8 strided accumulators, ((0+1)+(2+3))+((4+5)+(6+7)),
// then the tail — the order pw_leaf8 distributes over 8 lanes), log, with the same device libm calls.
constexpr int CLS1_ENVS = 128;
constexpr int CLS1_MAX_K = 16;
APG_DEV void cls1_env(const EnvArgs &a, int e, float *row, const EnvIn &in, double *pos, const apg_image_outputs &out,
                      float *hist);
// LDS row stride of a K-logit row: odd, so lanes = envs hit distinct banks (k + 1 is even for odd K)
APG_DEV int cls1_stride(int k) { return k + 1 + (k & 1); }

__global__ __launch_bounds__(CLS1_ENVS) void k_image_env_cls1(EnvArgs a, const float *__restrict__ act,
                                                             const float *__restrict__ pred, const int32_t *label,
                                                             double *pos, apg_image_outputs out, float *hist) {
  extern __shared__ float s_logit[];  // [CLS1_ENVS][cls1_stride(k)]
  const int k = a.k, stride = cls1_stride(k);
  const int e0 = blockIdx.x * CLS1_ENVS;
  const int ne = a.n - e0 < CLS1_ENVS ? a.n - e0 : CLS1_ENVS;
  for (int q = threadIdx.x; q < ne * k; q += CLS1_ENVS) {
    const int r = q / k;
    s_logit[r * stride + (q - r * k)] = pred[(size_t)e0 * k + q];
  }
  __syncthreads();
  if ((int)threadIdx.x >= ne) return;
  const int e = e0 + threadIdx.x;
  cls1_env(a, e, s_logit + threadIdx.x * stride, load_env_in<APG_IMAGE_CLASSIFY>(a, e, act, pred, label, pos, out), pos,
           out, hist);
}

// Classification step of env e for K <= CLS1_MAX_K from its logit row (in LDS; overwritten with the exps).
APG_DEV void cls1_env(const EnvArgs &a, int e, float *row, const EnvIn &in, double *pos, const apg_image_outputs &out,
                      float *hist) {
  const int k = a.k;
  float m = -INFINITY;
  bool nan = false, pos_inf = false, all_neg_inf = true;
  for (int i = 0; i < k; i++) {
    const float v = row[i];
    nan |= v != v;
    pos_inf |= v == INFINITY;
    all_neg_inf &= v == -INFINITY;
    m = v > m ? v : m;
  }
  if (nan || isinf(m)) m = 0.0f;  // x_max[~isfinite(x_max)] = 0
  const int32_t l = in.label;
  const int lc = l < 0 ? 0 : (l >= k ? k - 1 : l);
  const float xt = row[lc];
  for (int i = 0; i < k; i++) row[i] = np_expf(__fsub_rn(row[i], m));
  float sum = 0.0f;
  if (k < 8) {
    for (int i = 0; i < k; i++) sum = __fadd_rn(sum, row[i]);
  } else {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = row[j];
    int i = 8;
    for (; i < k - (k % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; j++) r[j] = __fadd_rn(r[j], row[i + j]);
    }
    sum = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                    __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < k; i++) sum = __fadd_rn(sum, row[i]);
  }
  uint32_t err = (nan || pos_inf || all_neg_inf) ? APG_ERR_NAN_PREDICTION : 0u;
  const float ce = -__fsub_rn(__fsub_rn(xt, m), np_logf(sum));
  const double loss_d = __dadd_rn(__dmul_rn((double)ce, a.ce_scale), a.ce_offset);
  ro(out.loss_f64, a.row, e, 1) = loss_d;
  ro(out.label_target, a.row, e, 1) = l;
  log_classification(a, e, out, hist, f32_div(row[lc], sum));
  err |= env_tail(a, e, in, pos, out, loss_d, 0.0f);
  if (err) atomicOr(out.err, err);
}

// One launch per step: a workgroup computes the glimpses of its `nu` envs at their new positions (gs_axes /
// gs_pixels) and runs their env steps (loc_env / cls1_env: loss, stats, move).  On the batch autoreset step
// (a.resetting, after module_reset's draws and gather) nothing moves: the glimpses are taken at the new batch's
// start positions, as observe() does.  KIND:
// APG_IMAGE_LOCALIZE, or APG_IMAGE_CLASSIFY with K <= CLS1_MAX_K (logits staged in LDS with coalesced loads,
// one thread per env as k_image_env_cls1).
// ENVW: the workgroup is GT glimpse threads plus one env wave.  The env wave loads the env inputs,
// moves the units (positions into LDS for the axes), and after the second barrier runs the env steps while
// the glimpse waves compute the pixels: the serial per-env tail (exp / log / stats / move) overlaps the
// glimpse instead of following it.  Without ENVW the first GT threads do both in turn.  GT: 256, or 448 for the
// env-wave instances (eight waves per workgroup: four workgroups fill a CU's 32 wave slots, so a grid of up to
// 1024 workgroups is resident at once with each glimpse thread on fewer pixels).
#ifndef APG_FUSED_MIN_WAVES
#define APG_FUSED_MIN_WAVES 8  // <= 64 VGPRs: every workgroup of the grid resident at once
#endif
constexpr int ENV_WAVE = 64;
template <int KIND, bool F32, int PC, int C, bool ENVW, int GT = GS_THREADS, bool TILED = false>
__global__ __launch_bounds__(ENVW ? GT + ENV_WAVE : GT)
__attribute__((amdgpu_waves_per_eu(APG_FUSED_MIN_WAVES))) void k_image_step_fused(EnvArgs a, GlimpseGeo g, const void *pool, const int64_t *index, const float *__restrict__ act,
                   const float *__restrict__ pred, const int32_t *label, double *pos, apg_image_outputs out,
                   float *hist, int upb, FastDiv per_div, FastDiv s1_div, FastDiv side_div, FastDiv k_div) {
  __shared__ float s_lut[256];
  __shared__ int64_t s_base[GS_MAX_UNITS];
  __shared__ double s_npos[GS_MAX_UNITS][2];  // the units' positions after this step's move
  extern __shared__ Axis s_ax[];  // [unit][rows s0 | columns s1], then (classify) the logits [unit][stride]
  const int tid = threadIdx.x;
  const int u0 = blockIdx.x * upb, nu = a.n - u0 < upb ? a.n - u0 : upb;
  float *s_logit = reinterpret_cast<float *>(s_ax + (size_t)upb * (g.s0 + g.s1));
  // env inputs of unit u by thread r of `nr` (the env wave, or the first GS_THREADS threads): logits staged,
  // inputs loaded, image offset and the move (the env step repeats it for its outputs) into LDS for the axes
  // (classify) the units' logits staged in LDS for the env step: off the move's path, so the env wave stages them
  // between the two barriers while the glimpse waves compute the axes
  auto stage_logits = [&](int r, int nr) {
    if constexpr (KIND == APG_IMAGE_CLASSIFY) {
      const int k = a.k, stride = cls1_stride(k);
      for (int q = r; q < nu * k; q += nr) {
        const int row = (int)k_div.div((uint32_t)q);
        s_logit[row * stride + (q - row * k)] = pred[(size_t)u0 * k + q];
      }
    }
  };
  auto env_inputs = [&](int r, int nr, EnvIn &in) {
    in = EnvIn{};
    if (r < nu) {
      const int e = u0 + r;
      if (a.ahead_i64) {  // the batch autoreset, its draws made ahead: installed here (k_image_gather folded in)
        if constexpr (KIND == APG_IMAGE_LOCALIZE) {
          in.p0 = pred[2 * e];
          in.p1 = pred[2 * e + 1];
        }
        s_base[r] = install_ahead(a, e, out, pos, in, const_cast<int64_t *>(index), const_cast<int32_t *>(label)) *
                    g.img_elems;
      } else {
        in = load_env_in<KIND>(a, e, act, pred, label, pos, out);
        s_base[r] = index[e] * g.img_elems;
      }
      double px = in.px, py = in.py;
      if (!a.resetting) move_pos(a, in.a0, in.a1, px, py);  // the autoreset step observes the new batch in place
      s_npos[r][0] = px;
      s_npos[r][1] = py;
    }
  };
  auto env_step = [&](int r, const EnvIn &in) {
    if (r >= nu) return;
    if constexpr (KIND == APG_IMAGE_CLASSIFY)
      cls1_env(a, u0 + r, s_logit + r * cls1_stride(a.k), in, pos, out, hist);
    else
      loc_env(a, u0 + r, in, pos, out, hist);
  };
  if constexpr (ENVW) {
    if (tid >= GT) {  // the env wave (wave-uniform branch; it takes part in both barriers)
      EnvIn in;
      env_inputs(tid - GT, ENV_WAVE, in);
      __syncthreads();
      stage_logits(tid - GT, ENV_WAVE);
      __syncthreads();
      env_step(tid - GT, in);
      return;
    }
    if (!APG_U8_ARITH) for (int v = tid; v < 256; v += GT) s_lut[v] = u8_value((unsigned)v);
    __syncthreads();
    const uint32_t bad =
        gs_axes<GT>(g, nullptr, [&](int u, int c) { return s_npos[u][c]; }, u0, nu, 1, side_div, s_ax, s_base);
    __syncthreads();
    gs_pixels_t<F32, PC, C, GT, TILED>(g, pool, u0, nu, per_div, s1_div, s_ax, s_base, s_lut, out.glimpse);
    if (bad) atomicOr(out.err, bad);
  } else {
    if (!APG_U8_ARITH) for (int v = tid; v < 256; v += GT) s_lut[v] = u8_value((unsigned)v);
    EnvIn in;
    env_inputs(tid, GT, in);
    stage_logits(tid, GT);
    __syncthreads();
    const uint32_t bad =
        gs_axes<GT>(g, nullptr, [&](int u, int c) { return s_npos[u][c]; }, u0, nu, 1, side_div, s_ax, s_base);
    __syncthreads();
    gs_pixels_t<F32, PC, C, GT, TILED>(g, pool, u0, nu, per_div, s1_div, s_ax, s_base, s_lut, out.glimpse);
    env_step(tid, in);
    if (bad) atomicOr(out.err, bad);
  }
}

// ------------------------------------------------------------------ k_unique
constexpr int UNIQ_THREADS = 256;
constexpr int UNIQ_LDS_FLOATS = 24 * 1024;  // 96 KiB of glimpse tiles (two tiles)
constexpr int UNIQ_MAX_POINTS = 4096;

// tile of T glimpses (rows p0 .. p0+T-1 of the sampling grid) into LDS rows of stride L + 1
APG_DEV void unique_tile(const GlimpseGeo &g, const void *pool, const float *lut, int64_t base, const double *grid,
                         int p0, int T, int P, int L, float *tile) {
  const int per = g.s0 * g.s1;
  for (int q = threadIdx.x; q < T * per; q += UNIQ_THREADS) {
    const int r = q / per, pix = q % per, p = p0 + r;
    if (p >= P) continue;
    float v[3];
    glimpse_pixel(g, pool, lut, base, grid[2 * p], grid[2 * p + 1], pix / g.s1, pix % g.s1, v);
    for (int ch = 0; ch < g.c; ch++) tile[r * (L + 1) + pix * g.c + ch] = v[ch];
  }
}

__global__ __launch_bounds__(UNIQ_THREADS) void k_unique(GlimpseGeo g, const void *pool, const int64_t *index,
                                                         const double *grid, int P, int T, int k, int32_t *top_k,
                                                         float *uniq) {
  extern __shared__ float s_dyn[];
  __shared__ uint32_t s_min[UNIQ_MAX_POINTS];
  __shared__ float s_lut[256];
  load_u8_table(s_lut);
  const int e = blockIdx.x;
  const int L = g.s0 * g.s1 * g.c;
  float *tA = s_dyn, *tB = s_dyn + T * (L + 1);
  const int64_t base = index[e] * g.img_elems;
  for (int p = threadIdx.x; p < P; p += UNIQ_THREADS) s_min[p] = 0x7f800000u;  // +inf
  const int tiles = (P + T - 1) / T;
  const float inv_l_den = (float)L;
  for (int A = 0; A < tiles; A++) {
    __syncthreads();
    unique_tile(g, pool, s_lut, base, grid, A * T, T, P, L, tA);
    for (int B = A; B < tiles; B++) {
      __syncthreads();
      if (B != A) unique_tile(g, pool, s_lut, base, grid, B * T, T, P, L, tB);
      __syncthreads();
      const float *sb = B == A ? tA : tB;
      const int na = A * T + T <= P ? T : P - A * T, nb = B * T + T <= P ? T : P - B * T;
      for (int q = threadIdx.x; q < na * nb; q += UNIQ_THREADS) {
        const int ra = q / nb, rb = q % nb;
        if (B == A && rb <= ra) continue;  // unordered pairs a < b (the mean is symmetric)
        const float *xa = tA + ra * (L + 1), *xb = sb + rb * (L + 1);
        auto sq = [&](int l) {
          const float d = __fsub_rn(xb[l], xa[l]);
          return __fmul_rn(d, d);
        };
        // np.mean over the (G, G, C) block: (0 + pairwise_sum) / L in f32
        const float m = f32_div(__fadd_rn(0.0f, pw_sum<MAX_PW_DEPTH>(sq, 0, L)), inv_l_den);
        const uint32_t bits = __float_as_uint(m);  // m >= 0: unsigned order == float order
        atomicMin(&s_min[A * T + ra], bits);
        atomicMin(&s_min[B * T + rb], bits);
      }
    }
  }
  __syncthreads();
  if (uniq)
    for (int p = threadIdx.x; p < P; p += UNIQ_THREADS) uniq[(size_t)e * P + p] = __uint_as_float(s_min[p]);
  // top k by descending uniqueness, exact ties by ascending index: one wave, k selection rounds
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    for (int r = 0; r < k; r++) {
      uint32_t best = 0;
      int bi = 0x7fffffff;
      for (int p = lane; p < P; p += 64) {
        const uint32_t v = s_min[p];
        if (v != 0xffffffffu && (bi == 0x7fffffff || v > best)) {
          best = v;
          bi = p;
        }
      }
      for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t ob = __shfl_xor(best, d, 64);
        const int oi = __shfl_xor(bi, d, 64);
        if (oi != 0x7fffffff && (bi == 0x7fffffff || ob > best || (ob == best && oi < bi))) {
          best = ob;
          bi = oi;
        }
      }
      if (lane == 0) {
        top_k[(size_t)e * k + r] = bi;
        s_min[bi] = 0xffffffffu;  // taken
      }
      __builtin_amdgcn_wave_barrier();
      __threadfence_block();
    }
  }
}

// ---- k_unique_blk: the same ranking, register-blocked (the path for L = G*G*C <= 2048).
// The P glimpses of an env are computed once into a per-workgroup global slot; pairs are then
// processed as (32-row A tile) x (64-row B tile), leaf by leaf of numpy's pairwise sum over L: each
// thread owns a 2 x 4 block of pairs (A rows ia, ia+16; B rows ib + 16j) with the leaf's eight
// strided accumulators per pair in packed f32 registers, so one LDS read feeds 2 or 4 pairs.  Leaf
// results are combined in the recursion's post order through a small shifting stack (the combine
// counts come from the host, UniqPlan).  Per-point minima are kept on the pair TOTALS and divided
// by L at the end: rounding x / L is monotone, so min(x) / L == min(x / L) bit for bit.
#ifndef APG_UQ_STAGED
#define APG_UQ_STAGED 1  // k_unique_blk's pair loop in stage order (0: per pair; A/B 189.5 -> 187.6 ms, ab/unique_staged.txt)
#endif
#ifndef APG_UQ_WAVES
#define APG_UQ_WAVES 3  // k_unique_blk's occupancy bound (waves per SIMD; A/B knob)
#endif
constexpr int UQ_TA = 32, UQ_TB = 64, UQ_THREADS = 256, UQ_MAX_LEAVES = 16, UQ_MAX_L = 2048;
struct UniqPlan {
  int nleaves, ls;  // leaves of the pairwise sum over L; LDS row stride (>= longest leaf, ls % 8 == 4)
  int16_t off[UQ_MAX_LEAVES], len[UQ_MAX_LEAVES];
  int8_t comb[UQ_MAX_LEAVES];  // combines of the two top partial sums right after leaf j
};
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int SD>
__global__ __launch_bounds__(UQ_THREADS, APG_UQ_WAVES) void k_unique_blk(GlimpseGeo g, const void *pool, const int64_t *index,
                                                           const double *grid, int n, int P, int k, int32_t *top_k,
                                                           float *uniq, float *scratch, UniqPlan plan) {
  extern __shared__ float s_dyn[];  // [UQ_TA + UQ_TB][ls] leaf tiles, then s_min[P]
  __shared__ float s_lut[256];
  load_u8_table(s_lut);
  const int L = g.s0 * g.s1 * g.c, ls = plan.ls;
  float *s_a = s_dyn, *s_b = s_dyn + UQ_TA * ls;
  uint32_t *s_min = reinterpret_cast<uint32_t *>(s_dyn + (UQ_TA + UQ_TB) * ls);
  float *glim = scratch + (size_t)blockIdx.x * P * L;
  const int tid = threadIdx.x, ia = tid >> 4, ib = tid & 15;
  const int per = g.s0 * g.s1;
  const bool vec4 = L % 4 == 0;  // glimpse rows 16-byte aligned (leaf offsets are multiples of 8)
  for (int e = blockIdx.x; e < n; e += gridDim.x) {
    const int64_t base = index[e] * g.img_elems;
    __syncthreads();  // the previous env's ranking is done with s_min
    for (int q = tid; q < P * per; q += UQ_THREADS) {
      const int p = q / per, pix = q - p * per;
      float v[3];
      glimpse_pixel(g, pool, s_lut, base, grid[2 * p], grid[2 * p + 1], pix / g.s1, pix % g.s1, v);
      for (int ch = 0; ch < g.c; ch++) glim[(size_t)p * L + pix * g.c + ch] = v[ch];
    }
    for (int p = tid; p < P; p += UQ_THREADS) s_min[p] = 0x7f800000u;  // +inf
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // read the slot's fresh glimpses, not stale L1 lines
    for (int A0 = 0; A0 < P; A0 += UQ_TA) {
      for (int B0 = A0; B0 < P; B0 += UQ_TB) {
        float st[SD][8];  // partial sums of the pairwise tree, st[0] on top; pair index i * 4 + j
#pragma unroll
        for (int d = 0; d < SD; d++)
#pragma unroll
          for (int q = 0; q < 8; q++) st[d][q] = 0.0f;
        for (int lf = 0; lf < plan.nleaves; lf++) {
          const int lo = plan.off[lf], ln = plan.len[lf];
          // stage the leaf's columns of the 96 tile rows: 32 lanes per row (4 columns each), 8 rows at a
          // time; the loads of each half of the rows are all issued before its first LDS store
          __syncthreads();  // tiles free
#pragma unroll 1
          for (int half = 0; half < 2; half++) {
            constexpr int RPASS = UQ_THREADS / 32, NPASS = (UQ_TA + UQ_TB) / RPASS / 2;
            const int c4 = tid & 31, c = 4 * c4, r0 = (tid >> 5) + half * RPASS * NPASS;
            f4 v[NPASS];
            if (vec4) {
#pragma unroll
              for (int rr = 0; rr < NPASS; rr++) {
                const int r = r0 + RPASS * rr, p = r < UQ_TA ? A0 + r : B0 + (r - UQ_TA);
                v[rr] = f4{0.0f, 0.0f, 0.0f, 0.0f};
                if (c < ln && p < P) v[rr] = *reinterpret_cast<const f4 *>(glim + (size_t)p * L + lo + c);
              }
            } else {
#pragma unroll
              for (int rr = 0; rr < NPASS; rr++) {
                const int r = r0 + RPASS * rr, p = r < UQ_TA ? A0 + r : B0 + (r - UQ_TA);
                const float *src = glim + (size_t)p * L + lo + c;
                const bool ok = p < P;
                v[rr].x = ok && c < ln ? src[0] : 0.0f;
                v[rr].y = ok && c + 1 < ln ? src[1] : 0.0f;
                v[rr].z = ok && c + 2 < ln ? src[2] : 0.0f;
                v[rr].w = ok && c + 3 < ln ? src[3] : 0.0f;
              }
            }
#pragma unroll
            for (int rr = 0; rr < NPASS; rr++) {
              const int r = r0 + RPASS * rr;
              // 16-byte aligned (ls and c are multiples of 4): one ds_write_b128 per row piece, 8 lanes per 128 B;
              // without the assumption the store splits into ds_write2_b32 pairs whose lanes (4 dwords apart)
              // meet on every fourth bank
              f4 *dst = static_cast<f4 *>(__builtin_assume_aligned(s_dyn + r * ls + c, 16));
              if (c < ln) *dst = v[rr];
            }
          }
          __syncthreads();
          const float *pa0 = s_a + ia * ls, *pa1 = s_a + (ia + 16) * ls;
          const float *pb0 = s_b + ib * ls, *pb1 = s_b + (ib + 16) * ls, *pb2 = s_b + (ib + 32) * ls,
                      *pb3 = s_b + (ib + 48) * ls;
          // acc[i][j][h]: a row i, b row j, strided accumulators (2h, 2h+1) packed: the 16-byte row reads
          // land in register pairs the packed f32 ops take as they are
          f2 acc[2][4][4];
#pragma unroll
          for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
              for (int h = 0; h < 4; h++) acc[i][j][h] = f2{0.0f, 0.0f};
          const int groups = ln >> 3;
          for (int gi = 0; gi < groups; gi++) {
            const int c = gi * 8;
            f2 av[2][4], bv[4][4];
#pragma unroll
            for (int i = 0; i < 2; i++) {
              const float *pa = i ? pa1 : pa0;
              const f4 lo4 = *reinterpret_cast<const f4 *>(pa + c), hi4 = *reinterpret_cast<const f4 *>(pa + c + 4);
              av[i][0] = lo4.xy;
              av[i][1] = lo4.zw;
              av[i][2] = hi4.xy;
              av[i][3] = hi4.zw;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const float *pb = j == 0 ? pb0 : (j == 1 ? pb1 : (j == 2 ? pb2 : pb3));
              const f4 lo4 = *reinterpret_cast<const f4 *>(pb + c), hi4 = *reinterpret_cast<const f4 *>(pb + c + 4);
              bv[j][0] = lo4.xy;
              bv[j][1] = lo4.zw;
              bv[j][2] = hi4.xy;
              bv[j][3] = hi4.zw;
            }
#if APG_UQ_STAGED
            // per column pair h: the 8 pairs' differences, then their squares, then the adds (independent
            // chains side by side instead of sub -> mul -> add back to back on one temporary)
#pragma unroll
            for (int h = 0; h < 4; h++) {
              f2 d[8];
#pragma unroll
              for (int q = 0; q < 8; q++) d[q] = bv[q & 3][h] - av[q >> 2][h];
#pragma unroll
              for (int q = 0; q < 8; q++) d[q] = d[q] * d[q];
#pragma unroll
              for (int q = 0; q < 8; q++) acc[q >> 2][q & 3][h] = acc[q >> 2][q & 3][h] + d[q];
            }
#else
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
              for (int j = 0; j < 4; j++)
#pragma unroll
                for (int h = 0; h < 4; h++) {
                  const f2 d = bv[j][h] - av[i][h];
                  acc[i][j][h] = acc[i][j][h] + d * d;
                }
#endif
          }
          // leaf sums: ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) (0 for a leaf shorter than 8), in-order tail
          float res[8];
#pragma unroll
          for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const f2 *r = acc[i][j];
              const float t = __fadd_rn(__fadd_rn(__fadd_rn(r[0].x, r[0].y), __fadd_rn(r[1].x, r[1].y)),
                                        __fadd_rn(__fadd_rn(r[2].x, r[2].y), __fadd_rn(r[3].x, r[3].y)));
              res[i * 4 + j] = groups ? t : 0.0f;
            }
          for (int c = groups * 8; c < ln; c++) {
            const float a[2] = {pa0[c], pa1[c]};
            const float b[4] = {pb0[c], pb1[c], pb2[c], pb3[c]};
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const float d = __fsub_rn(b[j], a[i]);
                res[i * 4 + j] = __fadd_rn(res[i * 4 + j], __fmul_rn(d, d));
              }
          }
          // push, then the post-order combines (left = st[1], right = st[0])
#pragma unroll
          for (int d = SD - 1; d > 0; d--)
#pragma unroll
            for (int q = 0; q < 8; q++) st[d][q] = st[d - 1][q];
#pragma unroll
          for (int q = 0; q < 8; q++) st[0][q] = res[q];
          for (int cb = 0; cb < plan.comb[lf]; cb++) {
#pragma unroll
            for (int q = 0; q < 8; q++) st[0][q] = __fadd_rn(st[1][q], st[0][q]);
#pragma unroll
            for (int d = 1; d < SD - 1; d++)
#pragma unroll
              for (int q = 0; q < 8; q++) st[d][q] = st[d + 1][q];
          }
        }
        // per-point minima over the valid pairs a < b < P (totals are >= 0: unsigned order == float order)
        const int a[2] = {A0 + ia, A0 + ia + 16};
        const int b[4] = {B0 + ib, B0 + ib + 16, B0 + ib + 32, B0 + ib + 48};
        uint32_t colmin[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
#pragma unroll
        for (int i = 0; i < 2; i++) {
          uint32_t rowmin = 0xffffffffu;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (a[i] < b[j] && b[j] < P) {
              const uint32_t bits = __float_as_uint(st[0][i * 4 + j]);
              rowmin = bits < rowmin ? bits : rowmin;
              colmin[j] = bits < colmin[j] ? bits : colmin[j];
            }
          }
          if (rowmin != 0xffffffffu) atomicMin(&s_min[a[i]], rowmin);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (colmin[j] != 0xffffffffu) atomicMin(&s_min[b[j]], colmin[j]);
      }
    }
    __syncthreads();
    // np.mean = (0 + total) / L on the minimum total of each point
    const float lden = (float)L;
    for (int p = tid; p < P; p += UQ_THREADS) {
      const float m = f32_div(__fadd_rn(0.0f, __uint_as_float(s_min[p])), lden);
      s_min[p] = __float_as_uint(m);
      if (uniq) uniq[(size_t)e * P + p] = m;
    }
    __syncthreads();
    if (tid < 64) {  // top k by descending uniqueness, exact ties by ascending index
      const int lane = tid;
      for (int r = 0; r < k; r++) {
        uint32_t best = 0;
        int bi = 0x7fffffff;
        for (int p = lane; p < P; p += 64) {
          const uint32_t v = s_min[p];
          if (v != 0xffffffffu && (bi == 0x7fffffff || v > best)) {
            best = v;
            bi = p;
          }
        }
        for (int d = 32; d >= 1; d >>= 1) {
          const uint32_t ob = __shfl_xor(best, d, 64);
          const int oi = __shfl_xor(bi, d, 64);
          if (oi != 0x7fffffff && (bi == 0x7fffffff || ob > best || (ob == best && oi < bi))) {
            best = ob;
            bi = oi;
          }
        }
        if (lane == 0) {
          top_k[(size_t)e * k + r] = bi;
          s_min[bi] = 0xffffffffu;  // taken
        }
        __builtin_amdgcn_wave_barrier();
        __threadfence_block();
      }
    }
  }
}

// target = clip(grid[top_k[sel]] + jitter, -1, 1).astype(float32)  (:281-292, image_localization.py:139-143)
__global__ void k_unique_finish(int n, int offset, int k, const int32_t *top_k, const int64_t *sel,
                                const double *grid, const double *jitter, float *target) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int d = offset + e;
  const int p = top_k[(size_t)e * k + sel[d]];
  for (int c = 0; c < 2; c++) {
    double v = __dadd_rn(grid[2 * p + c], jitter[2 * d + c]);
    v = v < -1.0 ? -1.0 : (v > 1.0 ? 1.0 : v);
    target[2 * e + c] = (float)v;
  }
}

// target[prev_done] = np_random.uniform(-1, 1, (k, 2)).astype(float32); out_prev = pre-update copy
__global__ void k_loc_target(int n, int offset, int refresh, const double *draw, float *target, float *out_prev,
                             int row) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  for (int c = 0; c < 2; c++) {
    ro(out_prev, row, e, 2, c) = target[2 * e + c];
    if (refresh) target[2 * e + c] = (float)draw[2 * (offset + e) + c];
  }
}

// glimpse_pos = pos.astype(float32); time_step = full(N, value)
__global__ void k_obs_pos(int n, const double *pos, float *glimpse_pos, float *time_step, float value, int row) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  ro(glimpse_pos, row, e, 2, 0) = (float)pos[2 * e];
  ro(glimpse_pos, row, e, 2, 1) = (float)pos[2 * e + 1];
  ro(time_step, row, e, 1) = value;
}

// ------------------------------------------------------------------ standalone losses
__global__ void k_loss_ce(const float *logits, const int32_t *target, int n, int k, double scale, double offset,
                          double *out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  out[e] = __dadd_rn(__dmul_rn((double)ce_f32(logits + (size_t)e * k, k, target[e]), scale), offset);
}

__global__ void k_loss_mse(const float *pred, const float *target, int n, int d, float scale, float offset,
                           float *out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float *p = pred + (size_t)e * d, *t = target + (size_t)e * d;
  auto sq = [&](int i) {
    const float x = __fsub_rn(p[i], t[i]);
    return __fmul_rn(x, x);
  };
  const float m = f32_div(__fadd_rn(0.0f, pw_sum<MAX_PW_DEPTH>(sq, 0, d)), (float)d);
  out[e] = __fadd_rn(__fmul_rn(m, scale), offset);
}

// ------------------------------------------------------------------ host side
int grid_for(int64_t n, int threads) { return (int)((n + threads - 1) / threads); }

// Bytes of a packed output row (apg_image_config.out_row_bytes): reward (f64), the glimpse, glimpse_pos, time_step,
// base_reward; classification: loss_f64, label_target; localization: target, loss_f32; stats (4 f32)
// with log_stats, stats_idx (2 i32) for classification
int image_min_row_bytes(const apg_image_config *c) {
  const int64_t glimpse = 4LL * c->sensor_h * c->sensor_w * c->channels;
  int64_t b = 8 + glimpse + 8 + 4 + 4;
  if (c->kind == APG_IMAGE_CLASSIFY) b += 8 + 4 + (c->log_stats ? 8 : 0);
  else b += 8 + 4;  // (the target glimpse stays dense)
  if (c->log_stats) b += 16;
  b = (b + 7) & ~7LL;
  return b > 0x7fffffff ? 0x7fffffff : (int)b;
}

int validate(const apg_image_config *c) {
  if (c->num_envs <= 0) return fail(APG_E_INVALID, "num_envs must be positive");
  if (c->height < 2 || c->width < 2) return fail(APG_E_INVALID, "images must be at least 2 x 2");
  if (c->pool_channels != 1 && c->pool_channels != 3) return fail(APG_E_INVALID, "pool channels must be 1 or 3");
  if (c->channels != 1 && c->channels != 3) return fail(APG_E_INVALID, "Target channels must be either 1 or 3");
  if (c->pool_channels == 3 && c->channels == 1)
    return fail(APG_E_INVALID, "Invalid image format. Expected 1 channels but got 3");
  if (c->pool_dtype != APG_POOL_U8 && c->pool_dtype != APG_POOL_F32 && c->pool_dtype != APG_POOL_U8_TILED)
    return fail(APG_E_INVALID, "unknown pool_dtype");
  if (c->pool_dtype == APG_POOL_U8_TILED && c->pool_channels != 3)
    return fail(APG_E_INVALID, "tiled pools (APG_POOL_U8_TILED) hold RGB images (pool_channels 3)");
  if (c->sensor_h <= 0 || c->sensor_w <= 0) return fail(APG_E_INVALID, "sensor size must be positive");
  if ((int64_t)c->sensor_h * c->sensor_w * c->channels > MAX_PW_N)
    return fail(APG_E_INVALID, "glimpse too large");
  if (c->pool_len <= 0 || c->pool_len > 0xffffffffLL) return fail(APG_E_INVALID, "pool_len must be in [1, 2**32]");
  if (c->step_limit <= 0) return fail(APG_E_INVALID, "step_limit must be positive");
  if (c->kind == APG_IMAGE_CLASSIFY && (c->num_classes <= 0 || c->num_classes > MAX_PW_N))
    return fail(APG_E_INVALID, "num_classes out of range");
  if (c->kind != APG_IMAGE_CLASSIFY && c->kind != APG_IMAGE_LOCALIZE) return fail(APG_E_INVALID, "unknown image env kind");
  if (c->log_stats && c->step_limit > PW_PTR_MAX_N) return fail(APG_E_INVALID, "log_stats needs step_limit <= 968");
  if (c->env_offset < 0 || (int64_t)c->env_offset + c->num_envs > c->num_envs_total)
    return fail(APG_E_INVALID, "shard [env_offset, env_offset + num_envs) must lie inside num_envs_total");
  if (c->out_row_bytes < 0 || (c->out_row_bytes & 7)) return fail(APG_E_INVALID, "out_row_bytes must be a multiple of 8");
  if (c->out_row_bytes > 0 && c->out_row_bytes < image_min_row_bytes(c))
    return fail(APG_E_INVALID, "out_row_bytes is smaller than the packed output row of the enabled fields");
  return APG_OK;
}

// candidates examined for n integers draws: n / P(accept) plus eight standard deviations
int64_t fill_candidates(int64_t n, uint64_t bound) {
  const uint64_t rng = bound - 1;
  double p_rej = 0.0;
  if (rng != 0xffffffffULL && rng != 0) p_rej = (double)((0xffffffffULL - rng) % (rng + 1)) / 4294967296.0;
  const double expect = (double)n / (1.0 - p_rej);
  int64_t cand = (int64_t)(expect + 8.0 * std::sqrt(expect * p_rej + 1.0) + 64.0);
  return cand < n ? n : cand;
}

// save_src / save_dst (optional): save_words words copied by the first kernel before any draw (or by a copy when no
// kernel of this call reads the stream)
int launch_integers(apg_pcg64 *state, int64_t n, int64_t lo, uint64_t bound, int64_t *out, int64_t *work,
                    hipStream_t s, const apg_pcg64 *save_src = nullptr, apg_pcg64 *save_dst = nullptr,
                    int save_count = 0) {
  if (save_dst && (n <= 0 || bound == 1) &&
      hipMemcpyAsync(save_dst, save_src, save_count * sizeof(apg_pcg64), hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipMemcpyAsync (stream snapshot)");
  if (n <= 0) return APG_OK;
  if (bound == 1) {  // integers(lo, lo + 1): no draw at all
    hipLaunchKernelGGL(k_fill_const, dim3(grid_for(n, 256)), dim3(256), 0, s, n, lo, out);
    return check_launch("k_fill_const");
  }
  FillArgs a{};
  if (save_dst) {
    static_assert(sizeof(apg_pcg64) % 8 == 0, "apg_pcg64: whole 8-byte words");
    a.save_src = reinterpret_cast<const uint64_t *>(save_src);
    a.save_dst = reinterpret_cast<uint64_t *>(save_dst);
    a.save_words = save_count * (int)(sizeof(apg_pcg64) / 8);
  }
  a.kind = APG_DRAW_INTEGERS;
  a.n = n;
  a.cols = 1;
  a.lo = lo;
  a.bound = bound;
  a.cand = fill_candidates(n, bound);
  a.nblocks = grid_for(a.cand, FILL_PER_BLOCK);
  hipLaunchKernelGGL(k_fill_count, dim3(a.nblocks), dim3(FILL_THREADS), 0, s, state, a, work);
  hipLaunchKernelGGL(k_fill_write, dim3(a.nblocks), dim3(FILL_THREADS), 0, s, state, a, out, work);
  return check_launch("k_fill_*");
}

// counter: a zeroed int64 the last workgroup uses to finish in the same launch (left at zero), or nullptr
int launch_uniform(apg_pcg64 *state, int64_t n, int cols, const double *low, const double *range, double *out,
                   hipStream_t s, int64_t *counter = nullptr) {
  if (n <= 0) return APG_OK;
  FillArgs a{};
  a.kind = APG_DRAW_UNIFORM;
  a.n = n;
  a.cols = cols;
  for (int c = 0; c < cols; c++) {
    a.low[c] = low[c];
    a.range[c] = range[c];
  }
  const int64_t m = n * cols;
  hipLaunchKernelGGL(k_fill_uniform, dim3(grid_for(m, FILL_PER_BLOCK)), dim3(FILL_THREADS), 0, s, state, a, out,
                     counter);
  if (!counter) hipLaunchKernelGGL(k_fill_uniform_finish, dim3(1), dim3(1), 0, s, state, m);
  return check_launch("k_fill_uniform");
}

// Glimpse units (env x position) per k_glimpse_sep / k_image_step_fused workgroup: about APG_GLIMPSE_PPT
// (default 4, clamped to [1, 16]: the Axis LDS stays far below 64 KiB) pixels per thread.  The output
// does not depend on it.
int glimpse_units_per_block(int per, int ppt_default = 4) {
  static const int forced = getenv("APG_GLIMPSE_PPT") ? std::max(1, std::min(16, atoi(getenv("APG_GLIMPSE_PPT")))) : 0;
  const int ppt = forced ? forced : ppt_default;
  return std::max(1, std::min(GS_MAX_UNITS, (ppt * GS_THREADS + per - 1) / per));
}

template <class PosT>
int launch_glimpse(const GlimpseGeo &g, const void *pool, const int64_t *index, const PosT *pos, int n, int npos,
                   float *out, uint32_t *err, hipStream_t s) {
  const int64_t total = (int64_t)n * npos * g.s0 * g.s1;
  if (total >= (int64_t)1 << 31) return fail(APG_E_INVALID, "glimpse batch too large (>= 2**31 pixels)");
  static const bool generic = getenv("APG_GLIMPSE_GENERIC") != nullptr;
  if (g.s0 <= GS_MAX_SIDE && g.s1 <= GS_MAX_SIDE && !generic) {
    const int per = g.s0 * g.s1, units = n * npos;
    const int upb = glimpse_units_per_block(per);
    const size_t dyn = (size_t)upb * (g.s0 + g.s1) * sizeof(Axis);
    hipLaunchKernelGGL(k_glimpse_sep<PosT>, dim3(grid_for(units, upb)), dim3(GS_THREADS), dyn, s, g, pool, index, pos,
                       npos, units, upb, make_fastdiv((uint32_t)per), make_fastdiv((uint32_t)g.s1),
                       make_fastdiv((uint32_t)(g.s0 + g.s1)), out, err);
    return check_launch("k_glimpse_sep");
  }
  hipLaunchKernelGGL(k_glimpse<PosT>, dim3(grid_for(total, 256)), dim3(256), 0, s, g, pool, index, pos, npos,
                     (int)total, out, err);
  return check_launch("k_glimpse");
}

int unique_tile_rows(int L) {
  int T = UNIQ_LDS_FLOATS / (2 * (L + 1));
  if (T > 32) T = 32;
  return T;
}

// numpy's pairwise recursion over L as a leaf list with post-order combine counts; returns the
// partial-sum stack depth it needs, or 0 when it does not fit the blocked kernel
int unique_plan(int L, UniqPlan &pl) {
  memset(&pl, 0, sizeof(pl));
  int depth = 0, maxdepth = 0, longest = 0;
  bool ok = true;
  auto rec = [&](auto &&self, int off, int len) -> void {
    if (len <= 128) {
      if (pl.nleaves >= UQ_MAX_LEAVES) {
        ok = false;
        return;
      }
      pl.off[pl.nleaves] = (int16_t)off;
      pl.len[pl.nleaves] = (int16_t)len;
      pl.nleaves++;
      longest = len > longest ? len : longest;
      depth++;
      maxdepth = depth > maxdepth ? depth : maxdepth;
      return;
    }
    int n2 = len / 2;
    n2 -= n2 % 8;
    self(self, off, n2);
    self(self, off + n2, len - n2);
    if (!ok) return;
    pl.comb[pl.nleaves - 1]++;
    depth--;
  };
  rec(rec, 0, L);
  if (!ok || L > UQ_MAX_L) return 0;
  pl.ls = ((longest + 3) / 4) * 4;
  if (pl.ls % 8 == 0) pl.ls += 4;  // ls / 4 odd: the 16-byte row reads of 16 lanes hit distinct banks
  return maxdepth;
}

float *unique_scratch(size_t bytes) {  // per-device slot buffer of k_unique_blk, grown on demand (resets only)
  static float *buf[64] = {};
  static size_t cap[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (cap[dev] < bytes) {
    if (buf[dev]) (void)hipFree(buf[dev]);
    buf[dev] = nullptr;
    cap[dev] = 0;
    if (hipMalloc(reinterpret_cast<void **>(&buf[dev]), bytes) != hipSuccess) return nullptr;
    cap[dev] = bytes;
  }
  return buf[dev];
}

template <int SD>
int launch_unique_blk(const GlimpseGeo &g, const void *pool, const int64_t *index, const double *grid, int n, int P,
                      int k, int32_t *top_k, float *uniq, const UniqPlan &pl, hipStream_t s) {
  const int L = g.s0 * g.s1 * g.c;
  const size_t dyn = ((size_t)(UQ_TA + UQ_TB) * pl.ls + P) * sizeof(float);
  if (dyn > 64 * 1024 &&
      hipFuncSetAttribute((const void *)k_unique_blk<SD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn) !=
          hipSuccess)
    return fail(APG_E_LAUNCH, "hipFuncSetAttribute(k_unique_blk) failed");
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_unique_blk<SD>, UQ_THREADS, dyn) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return fail(APG_E_LAUNCH, "k_unique_blk occupancy query failed");
  int blocks = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
  if (const char *cap = getenv("APG_UNIQUE_GRID")) blocks = atoi(cap) > 0 ? atoi(cap) : blocks;  // tests: striding
  if (blocks > n) blocks = n;
  float *scratch = unique_scratch((size_t)blocks * P * L * sizeof(float));
  if (!scratch) return fail(APG_E_LAUNCH, "hipMalloc of the uniqueness glimpse slots failed");
  hipLaunchKernelGGL(k_unique_blk<SD>, dim3(blocks), dim3(UQ_THREADS), dyn, s, g, pool, index, grid, n, P, k, top_k,
                     uniq, scratch, pl);
  return check_launch("k_unique_blk");
}

int launch_unique(const GlimpseGeo &g, const void *pool, const int64_t *index, const double *grid, int n, int P,
                  int k, int32_t *top_k, float *uniq, hipStream_t s) {
  const int L = g.s0 * g.s1 * g.c;
  if (P > UNIQ_MAX_POINTS) return fail(APG_E_INVALID, "too many unique-sampling grid points");
  if (k < 1 || k > P) return fail(APG_E_INVALID, "top_k must be in [1, P]");
  UniqPlan pl;
  const int sd = getenv("APG_UNIQUE_GENERIC") ? 0 : unique_plan(L, pl);
  if (sd >= 1 && sd <= 2) return launch_unique_blk<2>(g, pool, index, grid, n, P, k, top_k, uniq, pl, s);
  if (sd == 3) return launch_unique_blk<3>(g, pool, index, grid, n, P, k, top_k, uniq, pl, s);
  if (sd >= 4 && sd <= 5) return launch_unique_blk<5>(g, pool, index, grid, n, P, k, top_k, uniq, pl, s);
  const int T = unique_tile_rows(L);
  if (T < 1) return fail(APG_E_INVALID, "glimpse too large for the uniqueness tiles");
  if (P > UNIQ_MAX_POINTS) return fail(APG_E_INVALID, "too many unique-sampling grid points");
  if (k < 1 || k > P) return fail(APG_E_INVALID, "top_k must be in [1, P]");
  const size_t dyn = (size_t)2 * T * (L + 1) * sizeof(float);
  static bool big = false;
  if (!big) {
    if (hipFuncSetAttribute((const void *)k_unique, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) !=
        hipSuccess)
      return fail(APG_E_LAUNCH, "hipFuncSetAttribute(k_unique) failed");
    big = true;
  }
  hipLaunchKernelGGL(k_unique, dim3(n), dim3(UNIQ_THREADS), dyn, s, g, pool, index, grid, P, T, k, top_k, uniq);
  return check_launch("k_unique");
}

}  // namespace

extern "C" {

int64_t apg_rng_fill_work_elems(int64_t n, uint64_t bound) {
  if (n <= 0 || bound < 1 || bound > 0x100000000ULL) return 0;
  return fill_work_elems(fill_candidates(n, bound));
}

int apg_rng_fill(apg_pcg64 *state, int kind, int64_t n, int cols, const double *low, const double *range, int64_t lo,
                 uint64_t bound, void *out, int64_t *work, apg_stream_t stream) {
  if (!state || !out || n < 0) return fail(APG_E_INVALID, "bad apg_rng_fill arguments");
  if (n == 0) return APG_OK;
  hipStream_t s = (hipStream_t)stream;
  if (kind == APG_DRAW_UNIFORM) {
    if (cols < 1 || cols > 2 || !low || !range) return fail(APG_E_INVALID, "uniform draws need 1 or 2 columns");
    return launch_uniform(state, n, cols, low, range, static_cast<double *>(out), s, work);
  }
  if (kind == APG_DRAW_INTEGERS) {
    if (bound < 1 || bound > 0x100000000ULL) return fail(APG_E_INVALID, "integers range must be in [1, 2**32]");
    if (!work && bound > 1) return fail(APG_E_INVALID, "integers draws need apg_rng_fill_work_elems() of work");
    return launch_integers(state, n, lo, bound, static_cast<int64_t *>(out), work, s);
  }
  return fail(APG_E_INVALID, "unknown draw kind");
}

int apg_image_seed(const apg_image_config *cfg, const apg_image_state *st, uint64_t seed, apg_stream_t stream) {
  if (int rc = validate(cfg)) return rc;
  hipLaunchKernelGGL(k_image_seed, dim3(1), dim3(1), 0, (hipStream_t)stream, st->rng, seed);
  return check_launch("k_image_seed");
}

static int module_reset(const apg_image_config *c, const apg_image_state *st, const apg_image_outputs *out,
                        hipStream_t s) {
  const int n = c->num_envs, nt = c->num_envs_total;
  int64_t *idx_draw = st->scratch_i64, *inv_draw = st->scratch_i64 + nt;
  int rc;
  // next(DatasetBatchIterator): integers(0, len(dataset), N)
  if ((rc = launch_integers(st->rng + 2, nt, 0, (uint64_t)c->pool_len, idx_draw, st->rng_work, s))) return rc;
  // randomly_invert_labels: current_rng.integers(0, 2, size=N) == 1
  if (c->invert_labels && (rc = launch_integers(st->rng + 1, nt, 0, 2, inv_draw, st->rng_work, s))) return rc;
  // current_rng.uniform(-1, 1, size=(N, 2))
  const double low[2] = {-1.0, -1.0}, range[2] = {2.0, 2.0};
  if ((rc = launch_uniform(st->rng + 1, nt, 2, low, range, st->scratch_f64, s, st->rng_work))) return rc;
  hipLaunchKernelGGL(k_image_gather, dim3(grid_for(n, 256)), dim3(256), 0, s, n, c->env_offset, st->pool_labels,
                     idx_draw, c->invert_labels, inv_draw, st->scratch_f64, c->num_classes, st->index, st->label,
                     st->inverted, st->pos);
  return check_launch("k_image_gather");
}

static int observe(const apg_image_config *c, const apg_image_state *st, const apg_image_outputs *out, hipStream_t s,
                   bool target_changed) {
  const GlimpseGeo g = env_geo(c);
  int rc = launch_glimpse<double>(g, st->pool, st->index, st->pos, c->num_envs, 1, out->glimpse, out->err, s);
  if (rc || c->kind != APG_IMAGE_LOCALIZE || !target_changed) return rc;
  // the target glimpse is never part of a packed row (dense pitch)
  return launch_glimpse<float>(make_geo(c), st->pool, st->index, st->target, c->num_envs, 1, out->target_glimpse,
                               out->err, s);
}

int apg_image_reset(const apg_image_config *c, const apg_image_state *st, const apg_image_outputs *out,
                    apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int n = c->num_envs;
  int rc;
  if ((rc = module_reset(c, st, out, s))) return rc;
  if (c->kind == APG_IMAGE_LOCALIZE) {
    // sample_unique_glimpse_positions: rank, then current_rng.integers(0, k, N) and
    // current_rng.uniform(-cell, cell, (N, 2)); ImageLocalizationVectorEnv keeps it as float32
    const GlimpseGeo g = make_geo(c);
    if ((rc = launch_unique(g, st->pool, st->index, st->unique_grid, n, c->unique_points, c->top_k, st->top_k,
                            nullptr, s)))
      return rc;
    const int nt = c->num_envs_total;
    if ((rc = launch_integers(st->rng + 1, nt, 0, (uint64_t)c->top_k, st->scratch_i64, st->rng_work, s))) return rc;
    const double low[2] = {-c->cell[0], -c->cell[1]};
    const double range[2] = {c->cell[0] - -c->cell[0], c->cell[1] - -c->cell[1]};
    if ((rc = launch_uniform(st->rng + 1, nt, 2, low, range, st->scratch_f64, s, st->rng_work))) return rc;
    hipLaunchKernelGGL(k_unique_finish, dim3(grid_for(n, 256)), dim3(256), 0, s, n, c->env_offset, c->top_k,
                       st->top_k, st->scratch_i64, st->unique_grid, st->scratch_f64, st->target);
    if ((rc = check_launch("k_unique_finish"))) return rc;
  }
  // obs: glimpse, glimpse_pos, time_step (= (0 / limit) * 2 - 1 = -1)
  hipLaunchKernelGGL(k_obs_pos, dim3(grid_for(n, 256)), dim3(256), 0, s, n, st->pos, out->glimpse_pos,
                     out->time_step, -1.0f, c->out_row_bytes);
  if ((rc = check_launch("k_obs_pos"))) return rc;
  return observe(c, st, out, s, true);
}

int apg_image_step(const apg_image_config *c, const apg_image_state *st, const float *action,
                   const float *prediction, int32_t t, int32_t prev_done, const apg_image_outputs *out,
                   apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  if (!action || !prediction) return fail(APG_E_INVALID, "null action/prediction");
  if (c->log_stats && (!st->stats_hist || !out->stats || (c->kind == APG_IMAGE_CLASSIFY && !out->stats_idx)))
    return fail(APG_E_INVALID, "log_stats needs stats_hist, stats (and stats_idx) buffers");
  hipStream_t s = (hipStream_t)stream;
  const int n = c->num_envs, nt = c->num_envs_total;
  const bool ahead = (prev_done & 2) != 0;
  prev_done &= 1;
  if (ahead && (!prev_done || !st->ahead_i64 || !st->ahead_f64))
    return fail(APG_E_INVALID, "draws made ahead are installed by a batch autoreset step with the ahead buffers");
  int rc;
  // tuning knobs, read once: APG_IMAGE_UNFUSED (two launches per step), APG_GLIMPSE_GENERIC, APG_CLS_LANES8
  static const bool unfused = getenv("APG_IMAGE_UNFUSED") != nullptr, generic = getenv("APG_GLIMPSE_GENERIC") != nullptr,
                    lanes8 = getenv("APG_CLS_LANES8") != nullptr;
  const GlimpseGeo g = env_geo(c);
  const bool fusable = !unfused && !generic && !lanes8 && g.s0 <= GS_MAX_SIDE && g.s1 <= GS_MAX_SIDE &&
                       (c->kind == APG_IMAGE_LOCALIZE || c->num_classes <= CLS1_MAX_K);
  const bool fold = ahead && fusable;  // the fused step kernel installs the draws made ahead itself
  if (c->kind == APG_IMAGE_LOCALIZE && prev_done && !fold) {
    // prediction_target = target.copy(); target[prev_done] = np_random.uniform(-1, 1, (k, 2)) as f32
    const double *draw = ahead ? st->ahead_f64 + 2 * (size_t)nt : st->scratch_f64;
    if (!ahead) {
      const double low[2] = {-1.0, -1.0}, range[2] = {2.0, 2.0};
      if ((rc = launch_uniform(st->rng + 0, nt, 2, low, range, st->scratch_f64, s, st->rng_work))) return rc;
    }
    // (steps without a refresh fold the copy into the env kernels)
    hipLaunchKernelGGL(k_loc_target, dim3(grid_for(n, 256)), dim3(256), 0, s, n, c->env_offset, prev_done, draw,
                       st->target, out->target, c->out_row_bytes);
    if ((rc = check_launch("k_loc_target"))) return rc;
  }
  if (prev_done && !ahead && (rc = module_reset(c, st, out, s))) return rc;
  if (prev_done && ahead && !fold) {  // the draws made ahead, installed as module_reset's gather would
    hipLaunchKernelGGL(k_image_gather, dim3(grid_for(n, 256)), dim3(256), 0, s, n, c->env_offset, st->pool_labels,
                       st->ahead_i64, c->invert_labels, st->ahead_i64 + nt, st->ahead_f64, c->num_classes,
                       st->index, st->label, st->inverted, st->pos);
    if ((rc = check_launch("k_image_gather"))) return rc;
  }
  EnvArgs a{};
  a.n = n;
  a.kind = c->kind;
  a.k = c->num_classes;
  a.resetting = prev_done ? 1 : 0;
  a.msl[0] = c->max_step[0];
  a.msl[1] = c->max_step[1];
  a.ce_scale = c->ce_scale;
  a.ce_offset = c->ce_offset;
  a.mse_scale = c->mse_scale;
  a.mse_offset = c->mse_offset;
  a.log_stats = c->log_stats ? 1 : 0;
  a.limit = c->step_limit;
  const int32_t t_new = prev_done ? 0 : t + 1;
  a.t_new = t_new;
  a.time_value = (float)(((double)t_new / (double)c->step_limit) * 2.0 - 1.0);
  a.loss_weight = !c->sparse ? 1.0f : (!prev_done && t_new >= c->step_limit ? 1.0f : 0.0f);
  a.copy_target = c->kind == APG_IMAGE_LOCALIZE && !prev_done ? 1 : 0;
  a.target_st = st->target;
  a.row = c->out_row_bytes;
  if (fold) {
    a.ahead_i64 = st->ahead_i64;
    a.ahead_f64 = st->ahead_f64;
    a.nt = (int)nt;
    a.pool_labels = st->pool_labels;
    a.invert = c->invert_labels;
    a.offset = c->env_offset;
    a.inverted_st = st->inverted;
  }
  if (fusable) {
    const int per = g.s0 * g.s1;
    // The env wave (the workgroup's units at its 64 lanes) runs the serial per-env tail beside the glimpse waves:
    // with 448 glimpse threads it pays off for both kinds (MI355X, fused step rocprof medians: MNIST 13.08 ->
    // 12.46 us, TinyImageNetLoc 31.15 -> 30.3 us; with 256 glimpse threads localization's short tail did not
    // repay the extra wave, 29.7 vs 28.0 us in round 3).  APG_IMAGE_ENV_WAVE=0|1 overrides (A/B knob; results
    // do not depend on it).
    static const int envw_knob = getenv("APG_IMAGE_ENV_WAVE") ? atoi(getenv("APG_IMAGE_ENV_WAVE")) : -1;
    const bool envw = envw_knob >= 0 ? envw_knob != 0 : true;
    static const int gt_knob = getenv("APG_IMAGE_GT") ? atoi(getenv("APG_IMAGE_GT")) : 448;
    const bool gt448 = gt_knob == 448;
    int upb = envw ? std::min(ENV_WAVE, glimpse_units_per_block(per, 8)) : glimpse_units_per_block(per, 4);
    // Whole generations: four eight-wave workgroups are resident per CU, and a grid of 2.13 such generations
    // leaves the chip mostly idle in its last one.  From one full generation up, the units per workgroup are
    // re-chosen so the grid is the nearest whole number of generations (TinyImageNetLoc: 15 units, 2185
    // workgroups, 31.3 / 30.8 us -> 16 units, 2048 workgroups, 30.2 / 29.8 us, rocprof medians of two rounds).
    // Not when APG_GLIMPSE_PPT forces the size (A/B knob); results do not depend on it.
    static const bool ppt_forced = getenv("APG_GLIMPSE_PPT") != nullptr;
    if (envw && gt448 && !ppt_forced) {
      static int resident = 0;
      if (!resident) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
          cus = 256;
        resident = 4 * cus;
      }
      const double gens = (double)n / ((double)upb * resident);
      if (gens >= 1.0) {
        const int whole = (int)std::lround(gens);
        upb = std::min(ENV_WAVE, (int)(((int64_t)n + (int64_t)whole * resident - 1) / ((int64_t)whole * resident)));
      }
    }
    size_t dyn = (size_t)upb * (g.s0 + g.s1) * sizeof(Axis);
    if (c->kind == APG_IMAGE_CLASSIFY) dyn += (size_t)upb * (c->num_classes + 2) * sizeof(float);
    const dim3 grid(grid_for(n, upb)), block(GS_THREADS);
    const FastDiv pd = make_fastdiv((uint32_t)per), sd = make_fastdiv((uint32_t)g.s1),
                  sid = make_fastdiv((uint32_t)(g.s0 + g.s1)), kd = make_fastdiv((uint32_t)std::max(1, c->num_classes));
    // one instance per env kind and pool format (u8 / f32, pool channels, glimpse channels)
    // glimpse threads of the env-wave instances: 448 (eight-wave workgroups) unless APG_IMAGE_GT=256 (A/B knob;
    // results do not depend on it)
    const dim3 block_e((gt448 ? 448 : GS_THREADS) + ENV_WAVE);
    // one instance per env kind and pool format (u8 / f32, pool channels, glimpse channels)
#define APG_FUSED(K, F, P, C, TL)                                                                                \
  do {                                                                                                           \
    if (envw && gt448)                                                                                           \
      hipLaunchKernelGGL((k_image_step_fused<K, F, P, C, true, 448, TL>), grid, block_e, dyn, s, a, g, st->pool, \
                         st->index, action, prediction, st->label, st->pos, *out, st->stats_hist, upb, pd, sd, sid, \
                         kd);                                                                                    \
    else if (envw)                                                                                               \
      hipLaunchKernelGGL((k_image_step_fused<K, F, P, C, true, GS_THREADS, TL>), grid, block_e, dyn, s, a, g,    \
                         st->pool, st->index, action, prediction, st->label, st->pos, *out, st->stats_hist, upb, pd, \
                         sd, sid, kd);                                                                           \
    else                                                                                                         \
      hipLaunchKernelGGL((k_image_step_fused<K, F, P, C, false, GS_THREADS, TL>), grid, block, dyn, s, a, g,     \
                         st->pool, st->index, action, prediction, st->label, st->pos, *out, st->stats_hist, upb, pd, \
                         sd, sid, kd);                                                                           \
  } while (0)
#define APG_FUSED_KIND(K)                                   \
  do {                                                      \
    if (g.tiled) {                                          \
      APG_FUSED(K, false, 3, 3, true);                      \
    } else if (g.pool_f32) {                                \
      if (g.pc == 3) APG_FUSED(K, true, 3, 3, false);       \
      else if (g.c == 3) APG_FUSED(K, true, 1, 3, false);   \
      else APG_FUSED(K, true, 1, 1, false);                 \
    } else {                                                \
      if (g.pc == 3) APG_FUSED(K, false, 3, 3, false);      \
      else if (g.c == 3) APG_FUSED(K, false, 1, 3, false);  \
      else APG_FUSED(K, false, 1, 1, false);                \
    }                                                       \
  } while (0)
    if (c->kind == APG_IMAGE_LOCALIZE) APG_FUSED_KIND(APG_IMAGE_LOCALIZE);
    else APG_FUSED_KIND(APG_IMAGE_CLASSIFY);
#undef APG_FUSED_KIND
#undef APG_FUSED
    if ((rc = check_launch("k_image_step_fused"))) return rc;
    // the target glimpse only changes with the target and the images, i.e. on the autoreset step
    if (!prev_done || c->kind != APG_IMAGE_LOCALIZE) return APG_OK;
    return launch_glimpse<float>(make_geo(c), st->pool, st->index, st->target, n, 1, out->target_glimpse, out->err, s);
  }
  if (c->kind == APG_IMAGE_CLASSIFY && c->num_classes <= CLS1_MAX_K && !lanes8) {
    const size_t lds = (size_t)CLS1_ENVS * (c->num_classes + 2) * sizeof(float);
    hipLaunchKernelGGL(k_image_env_cls1, dim3(grid_for(n, CLS1_ENVS)), dim3(CLS1_ENVS), lds, s, a, action, prediction,
                       st->label, st->pos, *out, st->stats_hist);
  } else if (c->kind == APG_IMAGE_CLASSIFY) {
    int epb = 256 / CLS_LANES;
    while (epb > 1 && (size_t)epb * (c->num_classes + 1) * sizeof(float) > 64 * 1024) epb /= 2;
    const size_t lds = (size_t)epb * (c->num_classes + 1) * sizeof(float);
    hipLaunchKernelGGL(k_image_env_cls, dim3(grid_for(n, epb)), dim3(epb * CLS_LANES), lds, s, a, epb, action,
                       prediction, st->label, st->pos, *out, st->stats_hist);
  } else {
    hipLaunchKernelGGL(k_image_env_loc, dim3(grid_for(n, 256)), dim3(256), 0, s, a, action, prediction, st->pos,
                       *out, st->stats_hist);
  }
  if ((rc = check_launch("k_image_env"))) return rc;
  // the target glimpse only changes with the target or the images, i.e. on the autoreset step
  return observe(c, st, out, s, prev_done != 0);
}

int apg_image_draw_ahead(const apg_image_config *c, const apg_image_state *st, apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  if (!st->ahead_i64 || !st->ahead_f64 || !st->rng_saved) return fail(APG_E_INVALID, "null ahead buffers");
  hipStream_t s = (hipStream_t)stream;
  const int nt = c->num_envs_total;
  int rc;
  // module_reset's draws in its order: next(DatasetBatchIterator), label inversions, start positions; the first
  // kernel also keeps the three streams as they were before (rng_saved, for apg_image_discard_ahead)
  if ((rc = launch_integers(st->rng + 2, nt, 0, (uint64_t)c->pool_len, st->ahead_i64, st->rng_work, s, st->rng,
                            st->rng_saved, 3)))
    return rc;
  if (c->invert_labels && (rc = launch_integers(st->rng + 1, nt, 0, 2, st->ahead_i64 + nt, st->rng_work, s))) return rc;
  const double low[2] = {-1.0, -1.0}, range[2] = {2.0, 2.0};
  if ((rc = launch_uniform(st->rng + 1, nt, 2, low, range, st->ahead_f64, s, st->rng_work))) return rc;
  // ImageLocalizationVectorEnv's target refresh on the autoreset step: np_random.uniform(-1, 1, (N, 2))
  if (c->kind == APG_IMAGE_LOCALIZE &&
      (rc = launch_uniform(st->rng + 0, nt, 2, low, range, st->ahead_f64 + 2 * (size_t)nt, s, st->rng_work)))
    return rc;
  return APG_OK;
}

int apg_image_discard_ahead(const apg_image_config *c, const apg_image_state *st, apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  if (!st->rng_saved) return fail(APG_E_INVALID, "null rng_saved");
  if (hipMemcpyAsync(st->rng, st->rng_saved, 3 * sizeof(apg_pcg64), hipMemcpyDeviceToDevice, (hipStream_t)stream) !=
      hipSuccess)
    return fail(APG_E_LAUNCH, "hipMemcpyAsync (restore the streams)");
  return APG_OK;
}

int apg_image_glimpse(const apg_image_config *c, const void *pool, const int64_t *index, const void *pos,
                      int pos_is_f32, int32_t npos, float *out, uint32_t *err, apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  if (npos <= 0) return fail(APG_E_INVALID, "npos must be positive");
  const GlimpseGeo g = make_geo(c);
  hipStream_t s = (hipStream_t)stream;
  if (pos_is_f32)
    return launch_glimpse<float>(g, pool, index, static_cast<const float *>(pos), c->num_envs, npos, out, err, s);
  return launch_glimpse<double>(g, pool, index, static_cast<const double *>(pos), c->num_envs, npos, out, err, s);
}

int apg_image_unique_top_k(const apg_image_config *c, const void *pool, const int64_t *index, const double *grid,
                           int32_t npoints, int32_t k, int32_t *top_k, float *uniq, apg_stream_t stream) {
  if (int rc = validate(c)) return rc;
  return launch_unique(make_geo(c), pool, index, grid, c->num_envs, npoints, k, top_k, uniq, (hipStream_t)stream);
}

int apg_loss_ce(const float *logits, const int32_t *target, int32_t n, int32_t k, double scale, double offset,
                double *out, apg_stream_t stream) {
  if (n <= 0 || k <= 0 || k > MAX_PW_N) return fail(APG_E_INVALID, "bad apg_loss_ce shape");
  hipLaunchKernelGGL(k_loss_ce, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, logits, target, n, k,
                     scale, offset, out);
  return check_launch("k_loss_ce");
}

int apg_loss_mse(const float *pred, const float *target, int32_t n, int32_t d, float scale, float offset, float *out,
                 apg_stream_t stream) {
  if (n <= 0 || d <= 0 || d > MAX_PW_N) return fail(APG_E_INVALID, "bad apg_loss_mse shape");
  hipLaunchKernelGGL(k_loss_mse, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, pred, target, n, d,
                     scale, offset, out);
  return check_launch("k_loss_mse");
}

}  // extern "C"
