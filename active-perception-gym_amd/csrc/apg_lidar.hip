// apg_lidar.hip — gfx950 kernels + C ABI for the LIDAR localization hot path.
//
//   k_lidar_reset   one thread per env: reseed (reset(seed)), next map index from the
//                   DatasetIterator stream, rooms/maze generation, start-cell draw
//                   (lidar_localization2d.py:293-315, :547-557; dataset_iterator.py:26-32)
//                   The same wave then rewrites the float32 map obs of each env that reset (:299).
//   k_lidar_step    64 envs per 256-thread workgroup.  Phase 1 (lane = env): autoreset bookkeeping,
//                   NaN check, reward, move + collide + slide, termination, target, normalized MSE,
//                   TimeLimit (lidar_localization2d.py:317-389, time_limit.py:118-139,
//                   active_perception_env.py:101-121).  Phase 2 (lane = beam): each env's 32-column
//                   occupancy window is staged in LDS, then every beam runs the exact scan
//                   (:238-277, :496-536).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

#include "../../include/apgym_capi.h"
#include "apg_host.hpp"
#include "apg_maps.hpp"
#include "apg_pairwise.hpp"
#include "apg_scan.hpp"

using namespace apg;

namespace apg {
namespace {
thread_local char g_err[512] = "";
}

int fail(int code, const char *msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return APG_E_LAUNCH;
  }
  return APG_OK;
}
}  // namespace apg

namespace {

constexpr uint8_t F_AUTORESET = 1, F_JUST_RESET = 2, F_FIRST = 4;
#ifndef APG_STEP_EPB
#define APG_STEP_EPB 64
#endif
constexpr int EPB = APG_STEP_EPB;        // envs per step workgroup (lane = env in phases 1 and 2a)
constexpr int STEP_THREADS = 4 * EPB;    // phase 2a: 4 beams at a time per env
static_assert(EPB == 16 || EPB == 32 || EPB == 64, "EPB: power of two, at most one wave");
constexpr int MAX_WIN_ROWS = 32;
constexpr int WIN_STRIDE = MAX_WIN_ROWS + 1;  // LDS words per env window (+1: lanes = envs hit distinct banks)
constexpr int MAX_STAGED_BEAMS = 64;          // lidar rows staged in LDS for coalesced stores

BinomTable make_binom_table() {
  BinomTable t;
  t.p = 0.3;
  t.q = 1.0 - t.p;
  for (int n = 0; n < 16; n++) {
    // random_binomial_inversion's cached constants, evaluated with the host libm like numpy
    double np_ = n * t.p;
    t.qn[n] = std::exp(n * std::log(t.q));
    double b = np_ + 10.0 * std::sqrt(np_ * t.q + 1);
    t.bound[n] = (int32_t)(n < b ? n : b);
  }
  return t;
}

struct Geo {
  int n, h, w, wpr, is_static, kind, max_rooms, door_width, frames;
  double bp;
};

Geo make_geo(const apg_lidar_config *c) {
  Geo g;
  g.n = c->num_envs;
  g.h = c->height;
  g.w = c->width;
  g.wpr = (c->width + 63) / 64;
  g.is_static = c->is_static;
  g.kind = c->map_kind;
  g.max_rooms = c->max_rooms;
  g.door_width = c->door_width;
  g.frames = ((c->height + 1) / 2) * ((c->width + 1) / 2) + 4;
  g.bp = c->branching_prob;
  return g;
}

int validate(const apg_lidar_config *c) {
  if (!c) return fail(APG_E_INVALID, "null config");
  if (c->num_envs <= 0) return fail(APG_E_INVALID, "num_envs must be positive");
  if (c->height < 3 || c->width < 3 || c->height > 128 || c->width > 128)
    return fail(APG_E_INVALID, "map size must be within [3, 128]");
  if (c->map_kind == APG_MAP_ROOMS) {
    if (c->height != c->width) return fail(APG_E_INVALID, "rooms maps must be square");
    if (c->max_rooms < 1 || c->max_rooms > 17) return fail(APG_E_INVALID, "max_rooms must be in [1, 17]");
    if (c->door_width < 1) return fail(APG_E_INVALID, "door_width must be positive");
  } else if (c->map_kind == APG_MAP_MAZE) {
    if ((c->height % 2) == 0 || (c->width % 2) == 0)
      return fail(APG_E_INVALID, "Width and height must be odd.");
  } else {
    return fail(APG_E_INVALID, "unknown map kind");
  }
  if (c->beams <= 0 || c->beams > 4096) return fail(APG_E_INVALID, "beams must be in [1, 4096]");
  if (!(c->lidar_range > 0.0f) || c->lidar_range > 10.0f)
    return fail(APG_E_INVALID, "lidar_range must be in (0, 10] (occupancy window of the fused step kernel)");
  if (c->step_limit <= 0) return fail(APG_E_INVALID, "step_limit must be positive");
  if (c->log_stats && c->step_limit > PW_PTR_MAX_N) return fail(APG_E_INVALID, "log_stats needs step_limit <= 968");
  return APG_OK;
}

// ------------------------------------------------------------------ map helpers
APG_DEV int place_start(Pcg64 &rng, const uint64_t *rows, int h, int w, int wpr, float &px, float &py) {
  int nocc = 0;
  for (int i = 0; i < h * wpr; i++) nocc += __popcll(rows[i]);
  const int64_t nfree = (int64_t)h * w - nocc;
  if (nfree <= 0) return -1;
  int64_t pick = integers(rng, 0, nfree);
  for (int y = 0; y < h; y++) {
    int occ_row = 0;
    for (int k = 0; k < wpr; k++) occ_row += __popcll(rows[y * wpr + k]);
    const int free_row = w - occ_row;
    if (pick >= free_row) {
      pick -= free_row;
      continue;
    }
    for (int x = 0; x < w; x++) {
      if (!((rows[y * wpr + (x >> 6)] >> (x & 63)) & 1ULL)) {
        if (pick == 0) {
          px = __fadd_rn((float)x, 0.5f);
          py = __fadd_rn((float)y, 0.5f);
          return 0;
        }
        pick--;
      }
    }
  }
  return -1;
}

// ------------------------------------------------------------------ kernels
// Map generator of a kernel instance (template parameter GEN): static maps are generated once by
// apg_lidar_init, so the reset kernel for them only draws start cells.
enum : int { GEN_NONE = 0, GEN_ROOMS = 1, GEN_MAZE = 2 };

template <int GEN>
APG_DEV int generate_one(const Geo &g, Pcg64 &r, uint64_t *occ, uint16_t *stack, const BinomTable &bt) {
  if constexpr (GEN == GEN_MAZE) return maze_generate(r, Bits{occ, g.wpr}, g.h, g.w, g.bp, stack, 1, g.frames);
  else return rooms_generate(r, occ, g.wpr, g.h, g.max_rooms, g.door_width, bt);
}

// Rooms maps are painted into the lane's LDS bitmap (row words are read-modify-written once per
// primitive), then the wave copies its bitmaps out with coalesced stores.
APG_DEV void copy_out_maps(const uint64_t *s_maps, unsigned long long done, size_t words, uint64_t *dst, int lane) {
  while (done) {
    const int j = __ffsll((long long)done) - 1;
    done &= done - 1ULL;
    for (size_t k = lane; k < words; k += 64) dst[(size_t)j * words + k] = s_maps[(size_t)j * words + k];
  }
}

template <int GEN>
__global__ __launch_bounds__(64) void k_map_generate(Geo g, const uint64_t *idx, int n, uint64_t *occ,
                                                     uint16_t *stack, uint32_t *err, BinomTable bt, int lanes) {
  extern __shared__ uint64_t s_rows[];  // rooms: [lanes][h * wpr]
  const int lane = threadIdx.x;
  const int i = blockIdx.x * lanes + lane;
  const bool active = lane < lanes && i < n;
  const size_t words = (size_t)g.h * g.wpr;
  int rc = 0;
  if (active) {
    Pcg64 r = seed_pcg64(idx[i]);
    if constexpr (GEN == GEN_ROOMS)
      rc = rooms_generate(r, s_rows + lane * words, g.wpr, g.h, g.max_rooms, g.door_width, bt);
    else
      rc = generate_one<GEN>(g, r, occ + (size_t)i * words, stack ? stack + (size_t)i * g.frames : nullptr, bt);
  }
  if constexpr (GEN == GEN_ROOMS) copy_out_maps(s_rows, __ballot(active), words, occ + (size_t)blockIdx.x * lanes * words, lane);
  if (rc != 0 && err) atomicOr(err, APG_ERR_MAPGEN);
}

// reset of env e (lidar_localization2d.py:293-315 with the _np_random setter :547-557 on reset(seed)):
// reseed (use_seed) or continue the env's streams, next map index from the DatasetIterator stream,
// map generation into `own` (rooms: the caller's LDS bitmap; maze: the env's occupancy rows), start
// cell draw.  Returns the env's new flags.
template <int GEN>
APG_DEV uint8_t reset_one(const Geo &g, const apg_lidar_state &S, int e, uint8_t f, bool use_seed, uint64_t seed,
                          uint64_t *own, uint64_t *out_map_idx, uint32_t *err, const BinomTable &bt) {
  Pcg64 rng;
  Pcg64 it;
  if (use_seed) {
    rng = seed_pcg64(seed + (uint64_t)e);
    if constexpr (GEN != GEN_NONE) it = seed_pcg64(bounded_u64(rng, 0x100000000ULL));  // integers(0, 2**32, endpoint=True)
  } else {
    rng = *reinterpret_cast<const Pcg64 *>(&S.rng[e]);
    if constexpr (GEN != GEN_NONE) it = *reinterpret_cast<const Pcg64 *>(&S.it_rng[e]);
  }
  uint64_t midx;
  float px = 0.5f, py = 0.5f;
  if constexpr (GEN != GEN_NONE) {
    midx = next32(it);  // DatasetIterator: integers(0, len(dataset) = 2**32)
    Pcg64 map_rng = seed_pcg64(midx);  // FloorMapDataset*.get_data_point: default_rng(idx)
    int rc;
    if constexpr (GEN == GEN_ROOMS)
      rc = rooms_generate(map_rng, own, g.wpr, g.h, g.max_rooms, g.door_width, bt);
    else
      rc = generate_one<GEN>(g, map_rng, own, S.stack + (size_t)e * g.frames, bt);
    if (place_start(rng, own, g.h, g.w, g.wpr, px, py) != 0) rc = -6;
    if (rc != 0) atomicOr(err, APG_ERR_MAPGEN);
    *reinterpret_cast<Pcg64 *>(&S.it_rng[e]) = it;
    S.map_idx[e] = midx;
  } else {
    midx = S.map_idx[e];
    if (place_start(rng, S.occ, g.h, g.w, g.wpr, px, py) != 0) atomicOr(err, APG_ERR_MAPGEN);
  }
  S.pos[2 * e] = px;
  S.pos[2 * e + 1] = py;
  S.init_pos[2 * e] = px;
  S.init_pos[2 * e + 1] = py;
  S.elapsed[e] = 0;
  const uint8_t nf = (uint8_t)((f & F_AUTORESET) | F_JUST_RESET | F_FIRST);
  S.flags[e] = nf;
  *reinterpret_cast<Pcg64 *>(&S.rng[e]) = rng;
  if (out_map_idx) out_map_idx[e] = midx;
  return nf;
}

// reset(seed) of all envs (and, for maps too large for the fused step kernel's LDS, the autoresets):
// one wave per `lanes` (<= 64) envs.  Map generation is a long serial, divergent chain per env whose
// speed is set by instruction latency, not by lanes, so the host spreads the envs over as many waves
// as fit on the chip at once (gen_lanes).  Waves with nothing to reset exit after one flag load.
template <int GEN>
__global__ __launch_bounds__(64) void k_lidar_reset(Geo g, apg_lidar_state S, uint64_t seed, int use_seed,
                                                    int all, uint64_t *out_map_idx, uint32_t *err, BinomTable bt,
                                                    int lanes) {
  extern __shared__ uint64_t s_rows[];  // rooms: [lanes][h * wpr]
  const int lane = threadIdx.x;
  const int e = blockIdx.x * lanes + lane;
  const bool mine = lane < lanes && e < g.n;
  const uint8_t f = mine ? S.flags[e] : 0;
  const bool active = mine && (all || (f & F_AUTORESET));
  const unsigned long long todo = __ballot(active);
  if (todo == 0ULL) return;
  const size_t words = (size_t)g.h * g.wpr;
  if (active) {
    uint64_t *own = GEN == GEN_ROOMS ? s_rows + lane * words : S.occ + (size_t)e * words;
    reset_one<GEN>(g, S, e, f, use_seed != 0, seed, own, out_map_idx, err, bt);
  }
  if constexpr (GEN == GEN_ROOMS) copy_out_maps(s_rows, todo, words, S.occ + (size_t)blockIdx.x * lanes * words, lane);
}

struct StepParams {
  int n, h, w, wpr, beams, step_limit, is_static, R, wrows, log_stats, sparse;
  float range, loss_scale, loss_offset;
};

// ActiveRegressionLogWrapper (active_regression_env.py:131-159): per step |target - prediction| and
// mean((target - prediction)^2) in float32; at the episode end avg = float(np.mean(list)) (numpy's
// pairwise float32 mean) and final = the last value.  Stats for the steps of this episode live in
// hist[0 .. len) (euclidean distance) and hist[step_limit ..) (mse).
APG_DEV void log_episode_stats(const StepParams &P, const apg_lidar_outputs &O, int e, const float *hist, int len) {
  for (int m = 0; m < 2; m++) {
    const float *h = hist + m * P.step_limit;
    const float avg = f32_div(__fadd_rn(0.0f, pw_sum_ptr(h, len)), (float)len);
    O.stats[(size_t)m * P.n + e] = avg;
    O.stats[(size_t)(2 + m) * P.n + e] = h[len - 1];
  }
  O.stats_len[e] = len;
}

// Occupancy window per env, staged in LDS from the PRE-move position p0: the 32 x 32 cells
// [floor(p0) - 15, floor(p0) + 17)^2 (zero outside the map).  A step moves the agent by at most
// ~2 cells (clamped move <= 1, slide <= 1), and every cell a scan of length <= R from the new
// position p can touch lies within [floor(p) - R - 2, floor(p) + R + 1] (+1 column for the 2-bit
// quad reads), i.e. within [floor(p0) - R - 5, floor(p0) + R + 5]: inside the window for R <= 10.
#ifdef APG_STEP_PROFILE  // tuning builds only (tools/step_phase_profile.py): per-workgroup phase timestamps
__device__ unsigned long long g_step_prof[16384][8];
#define STEP_MARK(k) \
  if (threadIdx.x == 0 && blockIdx.x < 16384) g_step_prof[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
#else
#define STEP_MARK(k)
#endif
#ifndef APG_STEP_MIN_WAVES
#define APG_STEP_MIN_WAVES 4  // keep k_lidar_step at <= 128 VGPRs: 4 waves per SIMD
#endif
// GEN / FUSED: FUSED instances start with phase R, the NEXT_STEP autoresets of the envs whose episode
// ended at the previous step (map generation of kind GEN, start cell), so a step is one launch; the
// unfused instance (reset(seed)'s observation pass, and autoresets of rooms maps too large for the LDS
// budget, which k_lidar_reset does first) skips it.
template <int GEN, bool FUSED>
__global__ __launch_bounds__(STEP_THREADS, APG_STEP_MIN_WAVES) void k_lidar_step(StepParams P, Geo g, apg_lidar_state S,
                                                             const float *__restrict__ act,
                                                             const float *__restrict__ pred,
                                                             apg_lidar_outputs O, BinomTable bt) {
  __shared__ float s_pos[EPB][2];
  __shared__ int s_x0[EPB], s_y0[EPB];
  // dynamic LDS (step_lds_bytes): occupancy windows, then (beams <= MAX_STAGED_BEAMS) the lidar rows
  // staged for coalesced stores and the phase-2b work list of (beam << 6) | env entries
  extern __shared__ uint32_t s_dyn[];
  uint32_t *s_win = s_dyn;
  const int LS = P.beams + 1;  // odd row stride: lanes = envs hit distinct banks
  float *s_lid = reinterpret_cast<float *>(s_dyn + EPB * WIN_STRIDE);
  uint16_t *s_queue = reinterpret_cast<uint16_t *>(s_lid + EPB * LS);
  __shared__ int s_qn;
  __shared__ float s_dirs[MAX_STAGED_BEAMS][2];  // beam_dirs, read inside the beam loops (LDS, not HBM latency)
  const int tid = threadIdx.x;
  const int base = blockIdx.x * EPB;
  const size_t words = (size_t)P.h * P.wpr;
  STEP_MARK(0)
#ifdef APG_STEP_PROFILE
  const unsigned long long prof_clk0 = __builtin_amdgcn_s_memtime();
#endif

  // ---------------- phase R: NEXT_STEP autoresets (fused instances).  Envs are spread 16 per wave over
  // the four waves (map generation is a serial divergent chain per env, latency-bound: more waves in
  // flight, fewer lanes each).  Rooms maps are painted in LDS (aliasing the windows, which are staged
  // later) and copied out with the map observation; maze maps go straight to the occupancy rows.
  __shared__ unsigned long long s_reset;
  if constexpr (FUSED) {
    __shared__ unsigned long long s_pend;
    if (tid < EPB) {
      const int e = base + tid;
      const bool pend = e < P.n && (S.flags[e] & F_AUTORESET);
      const unsigned long long m = __ballot(pend);
      if (tid == 0) s_pend = m;
    }
    __syncthreads();
    const unsigned long long pend = s_pend;
    if (pend != 0ULL) {
      uint64_t *s_maps = reinterpret_cast<uint64_t *>(s_dyn);  // rooms: [EPB][h * wpr]
      const int lane = tid & 63, el = (tid >> 6) * (EPB / 4) + lane;
      if (lane < EPB / 4 && ((pend >> el) & 1ULL)) {
        const int e = base + el;
        uint64_t *own = GEN == GEN_ROOMS ? s_maps + (size_t)el * words : S.occ + (size_t)e * words;
        reset_one<GEN>(g, S, e, S.flags[e], false, 0, own, O.map_idx, O.err, bt);
      }
      __syncthreads();
      if constexpr (GEN == GEN_ROOMS) {  // occupancy rows out, coalesced over the workgroup
        for (int k = tid; k < EPB * (int)words; k += STEP_THREADS) {
          const int el2 = k / (int)words;
          if (((pend >> el2) & 1ULL) && base + el2 < P.n) S.occ[(size_t)base * words + k] = s_maps[k];
        }
        __syncthreads();
      }
    }
  }

  // ---------------- phase 0: window origins from the pre-move positions; which envs reset
  if (P.beams <= MAX_STAGED_BEAMS && tid < 2 * P.beams) s_dirs[tid >> 1][tid & 1] = S.beam_dirs[tid];
  if (tid < EPB) {
    const int e = base + tid;
    bool rs = false;
    if (e < P.n) {
      s_x0[tid] = (int)floorf(S.pos[2 * e]) - 15;
      s_y0[tid] = (int)floorf(S.pos[2 * e + 1]) - 15;
      rs = (S.flags[e] & F_JUST_RESET) != 0;
    }
    const unsigned long long m = __ballot(rs);
    if (tid == 0) {
      s_reset = m;
      s_qn = 0;
    }
  }
  __syncthreads();
  // map obs of the envs that reset this step: bool map / 255 (lidar_localization2d.py:299), written by
  // the whole workgroup with float4 stores (only in reset steps; the maps came from k_lidar_reset)
  if (s_reset != 0ULL && O.map_obs && !P.is_static) {
    const float wall = 1.0f / 255.0f;
    const int cells = P.h * P.w;
    unsigned long long m = s_reset;
    while (m) {
      const int j = __ffsll((long long)m) - 1;
      m &= m - 1ULL;
      const uint64_t *rows = S.occ + (size_t)(base + j) * words;
      float *dst = O.map_obs + (size_t)(base + j) * cells;
      if ((P.w & 3) == 0) {  // 4 cells of one row per float4: one row-word load, non-temporal stores
        const int q = P.w >> 2;
        for (int k4 = tid; k4 < cells / 4; k4 += STEP_THREADS) {
          const int y = k4 / q, x = (k4 - y * q) * 4;
          const uint32_t b = (uint32_t)(rows[y * P.wpr + (x >> 6)] >> (x & 63));
          typedef float f4 __attribute__((ext_vector_type(4)));
          f4 v;
          v.x = (b & 1u) ? wall : 0.0f;
          v.y = (b & 2u) ? wall : 0.0f;
          v.z = (b & 4u) ? wall : 0.0f;
          v.w = (b & 8u) ? wall : 0.0f;
          __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(dst) + k4);
        }
      } else {
        for (int k = tid; k < cells; k += STEP_THREADS) {
          const int y = k / P.w, x = k - y * P.w;
          dst[k] = ((rows[y * P.wpr + (x >> 6)] >> (x & 63)) & 1ULL) ? wall : 0.0f;
        }
      }
    }
  }
  for (int r = tid; r < EPB * P.wrows; r += STEP_THREADS) {
    const int el = r / P.wrows, row = r - el * P.wrows;
    const int e = base + el;
    uint32_t v = 0;
    if (e < P.n) {
      const int y = s_y0[el] + row;
      if ((unsigned)y < (unsigned)P.h)
        v = extract_window_row(S.occ + (P.is_static ? 0 : e * words) + (size_t)y * P.wpr, P.wpr, s_x0[el]);
    }
    s_win[el * WIN_STRIDE + row] = v;
  }
  __syncthreads();
  STEP_MARK(1)

  // ---------------- phase 1: one lane per env
  if (tid < EPB) {
    const int e = base + tid;
    uint32_t errbits = 0;
    if (e < P.n) {
      const RowsWindow rw{&s_win[tid * WIN_STRIDE], s_x0[tid], s_y0[tid], P.wrows};
      uint8_t f = S.flags[e];
      const bool was_reset = f & F_JUST_RESET;
      float pos0 = S.pos[2 * e], pos1 = S.pos[2 * e + 1];
      const float mapw = (float)P.w, maph = (float)P.h;
      if (was_reset) {  // NEXT_STEP autoreset: this env returned reset obs, reward 0
        O.reward[e] = 0.0;
        O.terminated[e] = 0;
        O.truncated[e] = 0;
        O.base_reward[e] = 0.0f;
        O.target[2 * e] = 0.0f;
        O.target[2 * e + 1] = 0.0f;
        O.loss[e] = 0.0f;
        O.info_mask[e] = 0;
        if (P.log_stats) O.stats_len[e] = 0;
        if (P.sparse) O.weight[e] = 0.0;
        f &= (uint8_t)~(F_JUST_RESET | F_AUTORESET);
      } else {
        float ax = act[2 * e], ay = act[2 * e + 1];
        const float prx = pred[2 * e], pry = pred[2 * e + 1];
        if (isnan(ax) || isnan(ay)) errbits |= APG_ERR_NAN_ACTION;
        if (isnan(prx) || isnan(pry)) errbits |= APG_ERR_NAN_PREDICTION;
        if (errbits) {  // the reference raises ValueError before touching this env's state
          O.reward[e] = 0.0;
          O.terminated[e] = 0;
          O.truncated[e] = 0;
          O.base_reward[e] = 0.0f;
          O.target[2 * e] = 0.0f;
          O.target[2 * e + 1] = 0.0f;
          O.loss[e] = 0.0f;
          O.info_mask[e] = 0;
          if (P.log_stats) O.stats_len[e] = 0;
          if (P.sparse) O.weight[e] = 0.0;
        } else {
          const float lpx = pos0, lpy = pos1;
          const float br = __fsub_rn(0.1f, __fmul_rn(0.001f, __fadd_rn(__fmul_rn(ax, ax), __fmul_rn(ay, ay))));
          const float mag = norm_f32(ax, ay);
          if (mag > 1.0f) {
            ax = f32_div(ax, mag);
            ay = f32_div(ay, mag);
          }
          const float tx = __fadd_rn(pos0, ax), ty = __fadd_rn(pos1, ay);
          float dirx = __fsub_rn(tx, pos0), diry = __fsub_rn(ty, pos1);
          const float total = norm_f32(dirx, diry);
          if (total > 0.0f) {
            dirx = f32_div(dirx, total);
            diry = f32_div(diry, total);
            const float d = lidar_scan(rw, pos0, pos1, tx, ty).dist;
            pos0 = __fadd_rn(pos0, __fmul_rn(dirx, d));
            pos1 = __fadd_rn(pos1, __fmul_rn(diry, d));
            const float rem = __fsub_rn(total, d);
            if (rem > 1e-5f) {  // slide along the wall (:345-364)
              const float rvx = __fmul_rn(dirx, rem), rvy = __fmul_rn(diry, rem);
              const bool kx = rvx > 1e-5f, ky = rvy > 1e-5f;
              if (kx || ky) {
                const float c0x = kx ? rvx : rvy, c1y = ky ? rvy : rvx;  // eye(2) * kept
                const float d0 = lidar_scan(rw, pos0, pos1, __fadd_rn(pos0, c0x), __fadd_rn(pos1, 0.0f)).dist;
                const float d1 = lidar_scan(rw, pos0, pos1, __fadd_rn(pos0, 0.0f), __fadd_rn(pos1, c1y)).dist;
                float cx, cy, dd;
                if (d0 > 0.0f) {
                  cx = c0x;
                  cy = 0.0f;
                  dd = d0;
                } else {
                  cx = 0.0f;
                  cy = c1y;
                  dd = d1;
                }
                const float nrm = norm_f32(cx, cy);
                pos0 = __fadd_rn(pos0, __fmul_rn(f32_div(cx, nrm), dd));
                pos1 = __fadd_rn(pos1, __fmul_rn(f32_div(cy, nrm), dd));
              }
            }
          }
          if (f & F_FIRST) {  // initial_pos aliases pos until np.clip rebinds it (:305, :371)
            S.init_pos[2 * e] = pos0;
            S.init_pos[2 * e + 1] = pos1;
            f &= (uint8_t)~F_FIRST;
          }
          bool term = pos0 < 0.0f || pos1 < 0.0f || pos0 >= mapw || pos1 >= maph;
          pos0 = fminf(fmaxf(pos0, 0.0f), mapw);
          pos1 = fminf(fmaxf(pos1, 0.0f), maph);
          const float tgx = __fsub_rn(__fmul_rn(f32_div(lpx, mapw), 2.0f), 1.0f);
          const float tgy = __fsub_rn(__fmul_rn(f32_div(lpy, maph), 2.0f), 1.0f);
          const int el = S.elapsed[e] + 1;
          S.elapsed[e] = el;
          if (el >= P.step_limit) term = true;  // TimeLimit(issue_termination=True)
          const float ex = __fsub_rn(prx, tgx), ey = __fsub_rn(pry, tgy);
          const float mse = f32_div(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), 2.0f);
          const float loss = __fadd_rn(__fmul_rn(mse, P.loss_scale), P.loss_offset);
          if (P.log_stats) {
            float *hist = S.stats_hist + (size_t)e * 2 * P.step_limit;
            hist[el - 1] = norm_f32(ex, ey);  // |target - prediction|: the signs do not matter
            hist[P.step_limit + el - 1] = mse;
            if (term) log_episode_stats(P, O, e, hist, el);
            else O.stats_len[e] = 0;
          }
          O.base_reward[e] = br;
          O.target[2 * e] = tgx;
          O.target[2 * e + 1] = tgy;
          O.loss[e] = loss;
          if (P.sparse) {  // SparsifyWrapper: base_reward - loss * (1.0 if terminated else 0.0), in f32
            O.weight[e] = term ? 1.0 : 0.0;
            O.reward[e] = (double)__fsub_rn(br, __fmul_rn(loss, term ? 1.0f : 0.0f));
          } else {
            O.reward[e] = (double)__fsub_rn(br, loss);
          }
          O.terminated[e] = term;
          O.truncated[e] = 0;
          O.info_mask[e] = 1;
          if (term) f |= F_AUTORESET;
          S.pos[2 * e] = pos0;
          S.pos[2 * e + 1] = pos1;
        }
      }
      S.flags[e] = f;
      if (O.reset_mask) O.reset_mask[e] = was_reset;
      // odometry (:263-270) and TimeLimit time_step (time_limit.py:113-116)
      const float ox = __fsub_rn(pos0, S.init_pos[2 * e]), oy = __fsub_rn(pos1, S.init_pos[2 * e + 1]);
      O.odometry[2 * e] = __fsub_rn(__fmul_rn(f32_div(__fadd_rn(ox, mapw), __fadd_rn(mapw, mapw)), 2.0f), 1.0f);
      O.odometry[2 * e + 1] = __fsub_rn(__fmul_rn(f32_div(__fadd_rn(oy, maph), __fadd_rn(maph, maph)), 2.0f), 1.0f);
      O.time_step[e] = (float)(2.0 * (double)S.elapsed[e] / (double)P.step_limit - 1.0);
      s_pos[tid][0] = pos0;
      s_pos[tid][1] = pos1;
    }
    if (errbits) atomicOr(O.err, errbits);  // rare: NaN inputs only
  }
  __syncthreads();
  STEP_MARK(2)

  // ---------------- phase 2a: lane = env, wave = beam index (all 64 lanes of a wave cast the same
  // beam direction).  Beams whose bounding box holds no occupied cell are SCAN_EMPTY and finish
  // here; the others are queued (env, beam) in LDS, grouped by beam, for 2b.
  const int el = tid & (EPB - 1), e = base + el;
  const bool staged = P.beams <= MAX_STAGED_BEAMS;
  const float px = s_pos[el][0], py = s_pos[el][1];
  const RowsWindow rw{&s_win[el * WIN_STRIDE], s_x0[el], s_y0[el], P.wrows};
  for (int beam = tid / EPB; beam < P.beams; beam += STEP_THREADS / EPB) {
    bool walk = false;
    if (e < P.n) {
      const float dx = staged ? s_dirs[beam][0] : S.beam_dirs[2 * beam];
      const float dy = staged ? s_dirs[beam][1] : S.beam_dirs[2 * beam + 1];
      const float qx = __fadd_rn(px, dx), qy = __fadd_rn(py, dy);
      walk = scan_may_hit(rw, px, py, qx, qy);
      if (!walk || !staged) {
        const float d = walk ? lidar_scan_walk(rw, px, py, qx, qy).dist : scan_empty(px, py, qx, qy).dist;
        const float v = fminf(fmaxf(f32_div(d, P.range), -1.0f), 1.0f);
        if (staged)
          s_lid[el * LS + beam] = v;
        else
          O.lidar[(size_t)e * P.beams + beam] = v;
      }
    }
    if (staged) {
      const int lane = tid & 63;
      const unsigned long long m = __ballot(walk);
      int qbase = 0;
      if (lane == 0 && m) qbase = atomicAdd(&s_qn, __popcll(m));
      qbase = __shfl(qbase, 0);
      if (walk) s_queue[qbase + __popcll(m & ((1ULL << lane) - 1ULL))] = (uint16_t)((beam << 6) | el);
    }
  }
  if (staged) {
    __syncthreads();
    STEP_MARK(3)
    // ---------------- phase 2b: the queued scans, densely over all lanes of the workgroup
    const int nq = s_qn;
    for (int i = tid; i < nq; i += STEP_THREADS) {
      const int ent = s_queue[i], qe = ent & (EPB - 1), beam = ent >> 6;
      const float qpx = s_pos[qe][0], qpy = s_pos[qe][1];
      const RowsWindow qrw{&s_win[qe * WIN_STRIDE], s_x0[qe], s_y0[qe], P.wrows};
      const float qx = __fadd_rn(qpx, s_dirs[beam][0]), qy = __fadd_rn(qpy, s_dirs[beam][1]);
      const float d = lidar_scan_walk(qrw, qpx, qpy, qx, qy).dist;
      s_lid[qe * LS + beam] = fminf(fmaxf(f32_div(d, P.range), -1.0f), 1.0f);
    }
    __syncthreads();
    STEP_MARK(4)
    const int nenv = P.n - base < EPB ? P.n - base : EPB;
    for (int i = tid; i < nenv * P.beams; i += STEP_THREADS) {
      const int l = i / P.beams, beam = i - l * P.beams;
      O.lidar[(size_t)base * P.beams + i] = s_lid[l * LS + beam];
    }
  }
#ifdef APG_STEP_PROFILE
  __syncthreads();
  STEP_MARK(5)
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    g_step_prof[blockIdx.x][6] = s_qn;
    g_step_prof[blockIdx.x][7] = __builtin_amdgcn_s_memtime() - prof_clk0;
  }
#endif
}

__global__ void k_scan_batch(const uint64_t *occ, const int32_t *map_index, int h, int w, int wpr,
                             const float *seg, int n, float *dist, int32_t *kind) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float px = seg[4 * i], py = seg[4 * i + 1], qx = seg[4 * i + 2], qy = seg[4 * i + 3];
  const RowsGlobal rg{occ + (size_t)map_index[i] * h * wpr, h, wpr, (int)floorf(fminf(px, qx)) - 1};
  ScanOut o = lidar_scan(rg, px, py, qx, qy);
  dist[i] = o.dist;
  if (kind) kind[i] = o.kind;
}

// ------------------------------------------------------------------ render tracking (render path only)
// LIDARLocalization2DEnv keeps render-only state the hot kernels do not: the observation_map of every
// cell its beams saw (__get_obs, lidar_localization2d.py:239-261), the trajectory deque (:327, :377-380),
// the last lidar readings (:242) and last pos / prediction (:326-327).  One workgroup per tracked env
// rebuilds it after every reset / step from the new position: each beam re-scanned with the reference's
// contact point, the contact cell and the non-occluded scan points OR-ed into an observation bitmap.
constexpr int RT_THREADS = 256;
constexpr int RT_MAX_BEAMS = 1024;

__global__ __launch_bounds__(RT_THREADS) void k_lidar_render_track(StepParams P, apg_lidar_state S, const float *pred,
                                                                 apg_lidar_outputs O, apg_lidar_render_state R) {
  __shared__ float s_dist[RT_MAX_BEAMS];
  const int t = blockIdx.x, e = R.env[t];
  const int wpr32 = (P.w + 31) / 32;
  uint32_t *om = R.obs_map + (size_t)t * P.h * wpr32;
  float *pose = R.pose + 6 * (size_t)t;
  const bool was_reset = O.reset_mask[e] != 0;
  const float px = S.pos[2 * e], py = S.pos[2 * e + 1];
  if (was_reset)
    for (int k = threadIdx.x; k < P.h * wpr32; k += RT_THREADS) om[k] = 0u;  // np.zeros_like(map) (:301)
  if (threadIdx.x == 0) {
    if (was_reset) {  // trajectory.clear(); last_pred = last_pos = None (:312-313)
      R.traj_len[t] = 0;
      R.has_last[t] = 0;
    } else if (pred) {
      const float lx = pose[4], ly = pose[5];  // last_pos = pos.copy() before the move (:327)
      const float ax = pred[2 * e], ay = pred[2 * e + 1];
      pose[0] = lx;
      pose[1] = ly;
      // last_pred = (prediction + 1) / 2 * map_size (:323-326); / 2 == * 0.5 exactly
      pose[2] = __fmul_rn(__fmul_rn(__fadd_rn(ax, 1.0f), 0.5f), (float)P.w);
      pose[3] = __fmul_rn(__fmul_rn(__fadd_rn(ay, 1.0f), 0.5f), (float)P.h);
      // prediction_quality = 1 - |prediction - normalized_last_pos| / 0.25 (:377-380); the step's target is
      // normalized_last_pos, and / 0.25 == * 4 exactly
      const float d = norm_f32(__fsub_rn(ax, O.target[2 * e]), __fsub_rn(ay, O.target[2 * e + 1]));
      const float q = __fsub_rn(1.0f, __fmul_rn(d, 4.0f));
      const int k = R.traj_len[t];
      if (k < P.step_limit) {
        float *tr = R.traj + ((size_t)t * P.step_limit + k) * 3;
        tr[0] = lx;
        tr[1] = ly;
        tr[2] = q > 1.0f ? 1.0f : q;  // np.minimum(quality, 1)
        R.traj_len[t] = k + 1;
      }
      R.has_last[t] = 1;
    }
  }
  __syncthreads();
  const uint64_t *occ = S.occ + (P.is_static ? 0 : (size_t)e * P.h * P.wpr);
  for (int b = threadIdx.x; b < P.beams; b += RT_THREADS) {
    const float qx = __fadd_rn(px, S.beam_dirs[2 * b]), qy = __fadd_rn(py, S.beam_dirs[2 * b + 1]);
    const RowsGlobal rg{occ, P.h, P.wpr, (int)floorf(fminf(px, qx)) - 1};
    ScanContact c{(double)qx, (double)qy, true};
    const float dist = lidar_scan_walk<RowsGlobal, true>(rg, px, py, qx, qy, &c).dist;
    s_dist[b] = dist;
    R.lidar_dist[(size_t)t * P.beams + b] = dist;
    if (dist < norm_f32(__fsub_rn(qx, px), __fsub_rn(qy, py))) {
      // coords = floor(contact); coords[exact & (target < pos)] -= 1 (:529-533), in the contact's dtype
      int ix, iy;
      if (c.is_f32) {
        const float cx = (float)c.x, cy = (float)c.y, fx = floorf(cx), fy = floorf(cy);
        ix = (int)fx - ((fabsf(__fsub_rn(fx, cx)) < 1e-5f && qx < px) ? 1 : 0);
        iy = (int)fy - ((fabsf(__fsub_rn(fy, cy)) < 1e-5f && qy < py) ? 1 : 0);
      } else {
        const double fx = floor(c.x), fy = floor(c.y);
        ix = (int)fx - ((fabs(__dsub_rn(fx, c.x)) < 1e-5 && qx < px) ? 1 : 0);
        iy = (int)fy - ((fabs(__dsub_rn(fy, c.y)) < 1e-5 && qy < py) ? 1 : 0);
      }
      if (ix >= 0 && iy >= 0 && ix < P.w && iy < P.h) atomicOr(&om[iy * wpr32 + (ix >> 5)], 1u << (ix & 31));
    }
  }
  __syncthreads();
  // scan points within the measured distance and in bounds (:250-261); the reference tests (x, y) against
  // map.shape = (H, W), i.e. x < H and y < W, and indexes [y, x]
  const int npts = P.beams * R.scan_points;
  for (int k = threadIdx.x; k < npts; k += RT_THREADS) {
    if (!(R.scan_norm[k] <= (double)s_dist[k / R.scan_points])) continue;
    const double fx = floor(__dadd_rn((double)px, R.scan_xy[2 * k]));
    const double fy = floor(__dadd_rn((double)py, R.scan_xy[2 * k + 1]));
    if (fx < 0.0 || fy < 0.0 || fx >= (double)P.h || fy >= (double)P.w || fx >= (double)P.w || fy >= (double)P.h)
      continue;
    const int ix = (int)fx, iy = (int)fy;
    atomicOr(&om[iy * wpr32 + (ix >> 5)], 1u << (ix & 31));
  }
  if (threadIdx.x == 0) {
    pose[4] = px;
    pose[5] = py;
  }
}

__global__ void k_rng_draws(const uint64_t *seeds, int m, int kind, int64_t a, int64_t b, int n,
                            double *out, BinomTable bt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  Pcg64 r = seed_pcg64(seeds[i]);
  for (int k = 0; k < n; k++) {
    double v = 0;
    switch (kind) {
      case 0: v = (double)next64(r); break;
      case 1: v = (double)next32(r); break;
      case 2: v = next_double(r); break;
      case 3: v = (double)integers(r, a, b); break;
      case 4: v = (double)bounded_u64(r, 0x100000000ULL); break;
      case 5: v = (double)binomial_inv(r, a, bt); break;
      default: break;
    }
    out[(size_t)i * n + k] = v;
  }
}

int grid_for(int n, int threads) { return (n + threads - 1) / threads; }

// Envs per 64-lane workgroup (one wave) for the serial map-generation kernels.  Each env's map is a
// long divergent chain: with one wave per SIMD its instruction latency is exposed, with many waves of
// few lanes the SIMD issues the same divergent instruction stream for little work.  Measured best
// (maze 127 x 127 and rooms 64 x 64 on MI355X): about APG_GEN_WAVES_PER_SIMD waves per SIMD.
#ifndef APG_GEN_WAVES_PER_SIMD
#define APG_GEN_WAVES_PER_SIMD 2
#endif
int gen_lanes(int n) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t waves = (int64_t)cus * 4 * APG_GEN_WAVES_PER_SIMD;
  int lanes = 1;
  while (lanes < 64 && (int64_t)grid_for(n, lanes) > waves) lanes *= 2;
  return lanes;
}

// Dynamic LDS of a map-generation launch: rooms bitmaps [lanes][h * wpr] (opted in above 64 KiB).
template <class K>
int gen_lds(K kernel, int gen, const Geo &g, int lanes, size_t &dyn) {
  dyn = gen == GEN_ROOMS ? (size_t)lanes * g.h * g.wpr * sizeof(uint64_t) : 0;
  if (dyn > 64 * 1024 &&
      hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return APG_OK;
}

template <int GEN>
int launch_reset_gen(const Geo &g, const apg_lidar_state *st, uint64_t seed, int use_seed, int all,
                     const apg_lidar_outputs *out, hipStream_t s) {
  const int lanes = GEN == GEN_NONE ? 64 : gen_lanes(g.n);
  size_t dyn;
  if (int rc = gen_lds(k_lidar_reset<GEN>, GEN, g, lanes, dyn)) return rc;
  hipLaunchKernelGGL(k_lidar_reset<GEN>, dim3(grid_for(g.n, lanes)), dim3(64), dyn, s, g, *st, seed, use_seed, all,
                     out->map_idx, out->err, make_binom_table(), lanes);
  return check_launch("k_lidar_reset");
}

int launch_reset(const Geo &g, const apg_lidar_state *st, uint64_t seed, int use_seed, int all,
                 const apg_lidar_outputs *out, hipStream_t s) {
  if (g.is_static) return launch_reset_gen<GEN_NONE>(g, st, seed, use_seed, all, out, s);
  if (g.kind == APG_MAP_MAZE) return launch_reset_gen<GEN_MAZE>(g, st, seed, use_seed, all, out, s);
  return launch_reset_gen<GEN_ROOMS>(g, st, seed, use_seed, all, out, s);
}

template <int GEN>
int launch_map_generate(const Geo &g, const uint64_t *idx, int n, uint64_t *occ, uint16_t *stack, uint32_t *err,
                        hipStream_t s) {
  const int lanes = gen_lanes(n);
  size_t dyn;
  if (int rc = gen_lds(k_map_generate<GEN>, GEN, g, lanes, dyn)) return rc;
  hipLaunchKernelGGL(k_map_generate<GEN>, dim3(grid_for(n, lanes)), dim3(64), dyn, s, g, idx, n, occ, stack, err,
                     make_binom_table(), lanes);
  return check_launch("k_map_generate");
}

int launch_map_generate_any(const Geo &g, const uint64_t *idx, int n, uint64_t *occ, uint16_t *stack,
                            uint32_t *err, hipStream_t s) {
  if (g.kind == APG_MAP_MAZE) return launch_map_generate<GEN_MAZE>(g, idx, n, occ, stack, err, s);
  return launch_map_generate<GEN_ROOMS>(g, idx, n, occ, stack, err, s);
}

size_t step_lds_bytes(int beams) {
  size_t b = (size_t)EPB * WIN_STRIDE * sizeof(uint32_t);
  if (beams <= MAX_STAGED_BEAMS) b += (size_t)EPB * (beams + 1) * sizeof(float) + (size_t)EPB * beams * sizeof(uint16_t);
  return b;
}

// Rooms maps of a fused step workgroup live in its dynamic LDS during phase R: keep that within the
// budget of four resident workgroups per CU (the step kernel's occupancy); larger rooms maps take
// the two-launch path (k_lidar_reset, then the unfused step kernel).
constexpr size_t FUSED_ROOMS_LDS_MAX = 36 * 1024;
size_t fused_rooms_lds(const Geo &g) { return (size_t)EPB * g.h * g.wpr * sizeof(uint64_t); }
int step_gen(const Geo &g) {
  if (g.is_static) return GEN_NONE;
  if (g.kind == APG_MAP_MAZE) return GEN_MAZE;
  return fused_rooms_lds(g) <= FUSED_ROOMS_LDS_MAX ? GEN_ROOMS : -1;  // -1: not fusable
}

int launch_step_kernel(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *act,
                       const float *pred, const apg_lidar_outputs *out, hipStream_t s, bool fused) {
  StepParams P;
  P.n = cfg->num_envs;
  P.h = cfg->height;
  P.w = cfg->width;
  P.wpr = (cfg->width + 63) / 64;
  P.beams = cfg->beams;
  P.step_limit = cfg->step_limit;
  P.log_stats = cfg->log_stats ? 1 : 0;
  P.sparse = cfg->sparse ? 1 : 0;
  P.is_static = cfg->is_static;
  P.R = (int)ceilf(cfg->lidar_range);
  P.wrows = MAX_WIN_ROWS;
  P.range = cfg->lidar_range;
  P.loss_scale = cfg->loss_scale;
  P.loss_offset = cfg->loss_offset;
  const Geo g = make_geo(cfg);
  const dim3 grid(grid_for(P.n, EPB)), block(STEP_THREADS);
  const BinomTable bt = make_binom_table();
  size_t lds = step_lds_bytes(P.beams);
  const int gen = fused ? step_gen(g) : -1;
  if (gen == GEN_ROOMS && fused_rooms_lds(g) > lds) lds = fused_rooms_lds(g);
  switch (gen) {
    case GEN_NONE:
      hipLaunchKernelGGL((k_lidar_step<GEN_NONE, true>), grid, block, lds, s, P, g, *st, act, pred, *out, bt);
      break;
    case GEN_ROOMS:
      hipLaunchKernelGGL((k_lidar_step<GEN_ROOMS, true>), grid, block, lds, s, P, g, *st, act, pred, *out, bt);
      break;
    case GEN_MAZE:
      hipLaunchKernelGGL((k_lidar_step<GEN_MAZE, true>), grid, block, lds, s, P, g, *st, act, pred, *out, bt);
      break;
    default:
      hipLaunchKernelGGL((k_lidar_step<GEN_NONE, false>), grid, block, lds, s, P, g, *st, act, pred, *out, bt);
  }
  return check_launch("k_lidar_step");
}

}  // namespace

extern "C" {

const char *apg_version(void) { return "apgym-mi355x 0.1.0 (gfx950)"; }
const char *apg_last_error(void) { return g_err; }

int apg_lidar_query_sizes(const apg_lidar_config *cfg, apg_lidar_state_sizes *o) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!o) return fail(APG_E_INVALID, "null output");
  Geo g = make_geo(cfg);
  const size_t words = (size_t)g.h * g.wpr;
  o->wpr = g.wpr;
  o->maze_frames = g.frames;
  o->occ_bytes = (g.is_static ? 1 : (size_t)g.n) * words * sizeof(uint64_t);
  o->scratch_bytes = 0;  // reserved (rooms maps are painted from primitives, no scratch plane)
  o->stack_bytes = g.kind == APG_MAP_MAZE ? (size_t)g.frames * (g.is_static ? 1 : (size_t)g.n) * sizeof(uint16_t) : 0;
  return APG_OK;
}

int apg_lidar_init(const apg_lidar_config *cfg, const apg_lidar_state *st, apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!cfg->is_static) return APG_OK;
  // One map for every env: generate dataset[static_map_index] once.
  Geo g = make_geo(cfg);
  hipStream_t s = (hipStream_t)stream;
  // map_idx[0] already holds static_map_index (the host fills the state before init)
  return launch_map_generate_any(g, (const uint64_t *)st->map_idx, 1, st->occ, st->stack, nullptr, s);
}

int apg_lidar_reset(const apg_lidar_config *cfg, const apg_lidar_state *st, uint64_t seed, int use_seed,
                    const apg_lidar_outputs *out, apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  Geo g = make_geo(cfg);
  if ((rc = launch_reset(g, st, seed, use_seed, 1, out, s))) return rc;
  return launch_step_kernel(cfg, st, nullptr, nullptr, out, s, false);
}

int apg_lidar_step_profiled(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *action,
                            const float *prediction, const apg_lidar_outputs *out, apg_stream_t stream,
                            void *ev_begin, void *ev_end) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!action || !prediction) return fail(APG_E_INVALID, "null action/prediction");
  if (cfg->log_stats && (!st->stats_hist || !out->stats || !out->stats_len))
    return fail(APG_E_INVALID, "log_stats needs stats_hist, stats and stats_len buffers");
  if (cfg->sparse && !out->weight) return fail(APG_E_INVALID, "sparse needs the weight buffer");
  hipStream_t s = (hipStream_t)stream;
  Geo g = make_geo(cfg);
  // one launch per step: the fused step kernel performs the NEXT_STEP autoresets itself; only rooms
  // maps beyond its LDS budget are generated by k_lidar_reset first
  const bool fused = step_gen(g) >= 0;
  if (!fused && (rc = launch_reset(g, st, 0, 0, 0, out, s))) return rc;
  if (ev_begin && hipEventRecord((hipEvent_t)ev_begin, s) != hipSuccess) return fail(APG_E_LAUNCH, "hipEventRecord");
  rc = launch_step_kernel(cfg, st, action, prediction, out, s, fused);
  if (rc == APG_OK && ev_end && hipEventRecord((hipEvent_t)ev_end, s) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipEventRecord");
  return rc;
}

int apg_lidar_step(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *action,
                   const float *prediction, const apg_lidar_outputs *out, apg_stream_t stream) {
  return apg_lidar_step_profiled(cfg, st, action, prediction, out, stream, nullptr, nullptr);
}

int apg_map_generate(int map_kind, const uint64_t *idx, int n, int h, int w, int max_rooms, int door_width,
                     double branching_prob, uint64_t *occ, uint64_t *scratch, uint16_t *stack, uint32_t *err,
                     apg_stream_t stream) {
  apg_lidar_config c;
  memset(&c, 0, sizeof(c));
  c.num_envs = n;
  c.height = h;
  c.width = w;
  c.map_kind = map_kind;
  c.beams = 1;
  c.step_limit = 1;
  c.lidar_range = 1.0f;
  c.max_rooms = max_rooms;
  c.door_width = door_width;
  c.branching_prob = branching_prob;
  int rc = validate(&c);
  if (rc) return rc;
  if (map_kind == APG_MAP_MAZE && !stack) return fail(APG_E_INVALID, "maze maps need stack");
  Geo g = make_geo(&c);
  (void)scratch;  // unused since rooms maps are painted from primitives; kept for ABI stability
  return launch_map_generate_any(g, idx, n, occ, stack, err, (hipStream_t)stream);
}

int apg_lidar_scan_batch(const uint64_t *occ, const int32_t *map_index, int h, int w, const float *seg, int n,
                         float *dist, int32_t *kind, apg_stream_t stream) {
  if (n <= 0 || h <= 0 || w <= 0 || w > 128) return fail(APG_E_INVALID, "bad scan batch arguments");
  // segments must span <= 28 columns (32-column row window); callers check this on the host
  hipLaunchKernelGGL(k_scan_batch, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, occ, map_index, h,
                     w, (w + 63) / 64, seg, n, dist, kind);
  return check_launch("k_scan_batch");
}

int apg_lidar_render_track(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *prediction,
                           const apg_lidar_outputs *out, const apg_lidar_render_state *rs, apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!st || !out || !rs || !out->reset_mask || !out->target)
    return fail(APG_E_INVALID, "render tracking needs the state, reset_mask and target buffers");
  if (rs->num_tracked <= 0) return APG_OK;
  if (cfg->beams > RT_MAX_BEAMS) return fail(APG_E_INVALID, "render tracking supports at most 1024 beams");
  if (rs->scan_points < 0 || !rs->env || !rs->obs_map || !rs->traj || !rs->traj_len || !rs->pose ||
      !rs->has_last || !rs->lidar_dist || (rs->scan_points > 0 && (!rs->scan_xy || !rs->scan_norm)))
    return fail(APG_E_INVALID, "null render state buffer");
  StepParams P;
  memset(&P, 0, sizeof(P));
  P.n = cfg->num_envs;
  P.h = cfg->height;
  P.w = cfg->width;
  P.wpr = (cfg->width + 63) / 64;
  P.beams = cfg->beams;
  P.step_limit = cfg->step_limit;
  P.is_static = cfg->is_static;
  hipLaunchKernelGGL(k_lidar_render_track, dim3(rs->num_tracked), dim3(RT_THREADS), 0, (hipStream_t)stream, P, *st,
                     prediction, *out, *rs);
  return check_launch("k_lidar_render_track");
}

int apg_rng_draws(const uint64_t *seeds, int m, int kind, int64_t a, int64_t b, int n, double *out,
                  apg_stream_t stream) {
  if (m <= 0 || n <= 0 || kind < 0 || kind > 5) return fail(APG_E_INVALID, "bad rng draw arguments");
  if (kind == 5 && (a < 0 || a > 15)) return fail(APG_E_INVALID, "binomial n must be in [0, 15]");
  hipLaunchKernelGGL(k_rng_draws, dim3(grid_for(m, 64)), dim3(64), 0, (hipStream_t)stream, seeds, m, kind, a, b,
                     n, out, make_binom_table());
  return check_launch("k_rng_draws");
}

#ifdef APG_STEP_PROFILE
int apg_debug_step_profile(void *dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_step_prof), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
}  // extern "C"
