// apg_lidar.hip — gfx950 kernels + C ABI for the LIDAR localization hot path.
//
//   k_lidar_reset   one thread per env: reseed (reset(seed)), next map index from the
//                   DatasetIterator stream, rooms/maze generation, start-cell draw
//                   (lidar_localization2d.py:293-315, :547-557; dataset_iterator.py:26-32)
//                   The same wave then rewrites the float32 map obs of each env that reset (:299).
//   k_lidar_step    256 envs per 1024-thread workgroup (one per CU; 64 / 256 threads for small
//                   batches).  Phase R: the NEXT_STEP autoresets (map generation, start cell).
//                   Phase 1 (env-major, 16 envs per wave): autoreset bookkeeping, NaN check, reward,
//                   move + collide + slide, termination, target, normalized MSE, TimeLimit
//                   (lidar_localization2d.py:317-389, time_limit.py:118-139,
//                   active_perception_env.py:101-121).  Phase 2: each env's 32 x 32 occupancy window
//                   is staged in LDS, every beam runs the exact scan (:238-277, :496-536): a bounding-
//                   box pre-test, then the queued walks spread over the workgroup's waves.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <deque>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/apgym_capi.h"
#include "apg_host.hpp"
#include "apg_maps.hpp"
#include "apg_maze.hpp"
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
constexpr int MAX_WIN_ROWS = 32;
constexpr int MAX_WIN_RANGE = 10;  // scan lengths the staged window covers (k_lidar_step); longer: RowsGlobal
constexpr int WIN_STRIDE = MAX_WIN_ROWS + 1;  // LDS words per env window (+1: lanes = envs hit distinct banks)
constexpr int MAX_STAGED_BEAMS = 64;          // lidar rows staged in LDS for coalesced stores
// SCAN_EMPTY beam values by the bit pattern of |q - p|^2 (f32) around range^2: a beam of length range
// from p lands within ~1e-4 of it (f32 rounding of p + dir), i.e. within a few hundred f32 steps
constexpr int EMPTY_TAB = 1024;

struct Geo {
  int n, h, w, wpr, is_static, kind, max_rooms, door_width, frames, row, pool_len;
  double bp;
  int64_t stream_len;  // APG_MAP_POOL streamed maps: len(dataset) of the draw; the map is slot e of the pool (0: pool)
};

// Output element j of env e: a dense [N][k] array, or (row > 0: apg_lidar_config.out_row_bytes) a field of env
// e's packed output row, the layout ShardedVectorEnv all-gathers without a packing copy.
template <class T>
APG_DEV T &oat(T *p, int row, int e, int k, int j = 0) {
  return row ? *reinterpret_cast<T *>(reinterpret_cast<char *>(p) + (size_t)e * (size_t)row + (size_t)j * sizeof(T))
             : p[(size_t)e * k + j];
}

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
  g.frames = (int)(maze_scratch_bytes(c->height, c->width) / 2);  // maze scratch, in u16 units
  g.bp = c->branching_prob;
  g.row = c->out_row_bytes;
  g.pool_len = c->map_kind == APG_MAP_POOL ? c->pool_len : 0;
  g.stream_len = c->map_kind == APG_MAP_POOL && !c->is_static ? c->stream_len : 0;
  return g;
}

// Bytes of a packed output row (apg_lidar_config.out_row_bytes): reward, map_idx (8 B each), weight (sparse),
// lidar, odometry, target, time_step, base_reward, loss, stats + stats_len (log_stats), four flag bytes
int min_row_bytes(const apg_lidar_config *c) {
  const int b = 16 + (c->sparse ? 8 : 0) + 4 * c->beams + 8 + 8 + 12 + (c->log_stats ? 20 : 0) + 4;
  return (b + 7) & ~7;
}

int validate(const apg_lidar_config *c) {
  if (!c) return fail(APG_E_INVALID, "null config");
  if (c->num_envs <= 0) return fail(APG_E_INVALID, "num_envs must be positive");
  if (c->map_kind == APG_MAP_POOL) {  // any FloorMapDataset: any H x W
    if (c->height < 1 || c->width < 1 || c->height > 511 || c->width > 511)
      return fail(APG_E_INVALID, "pool maps must be 1 .. 511 cells on each side");
    if (c->pool_len < 1) return fail(APG_E_INVALID, "the map pool must hold at least one map");
    if (c->is_static && (c->static_map_index < 0 || c->static_map_index >= c->pool_len))
      return fail(APG_E_INVALID, "static_map_index is outside the map pool");
    if (c->stream_len < 0) return fail(APG_E_INVALID, "stream_len must be >= 0");
    if (c->stream_len > 0 && !c->is_static && c->pool_len != c->num_envs)
      return fail(APG_E_INVALID, "streamed maps need one pool slot per env (pool_len == num_envs)");
  } else if (c->height < 3 || c->width < 3) {
    return fail(APG_E_INVALID, "map size must be at least 3");
  }
  if (c->map_kind == APG_MAP_POOL) {
  } else if (c->map_kind == APG_MAP_ROOMS) {
    if (c->height > 511 || c->width > 511) return fail(APG_E_INVALID, "rooms maps must be at most 511 x 511");
    if (c->height != c->width) return fail(APG_E_INVALID, "rooms maps must be square");
    if (c->max_rooms < 1 || c->max_rooms > ROOMS_MAX) return fail(APG_E_INVALID, "max_rooms must be in [1, 64]");
    if (c->door_width < 1) return fail(APG_E_INVALID, "door_width must be positive");
  } else if (c->map_kind == APG_MAP_MAZE) {
    if ((c->height % 2) == 0 || (c->width % 2) == 0)
      return fail(APG_E_INVALID, "Width and height must be odd.");
    if (c->height > 511 || c->width > 511) return fail(APG_E_INVALID, "maze maps must be at most 511 x 511");
  } else {
    return fail(APG_E_INVALID, "unknown map kind");
  }
  if (c->beams <= 0 || c->beams > 4096) return fail(APG_E_INVALID, "beams must be in [1, 4096]");
  if (!(c->lidar_range > 0.0f) || c->lidar_range > 60.0f)
    return fail(APG_E_INVALID, "lidar_range must be in (0, 60] (64-column scan windows)");
  if (c->step_limit <= 0) return fail(APG_E_INVALID, "step_limit must be positive");
  if (c->log_stats && c->step_limit > PW_DEEP_MAX_N) return fail(APG_E_INVALID, "log_stats needs step_limit <= 15368");
  if (c->out_row_bytes < 0 || (c->out_row_bytes & 7)) return fail(APG_E_INVALID, "out_row_bytes must be a multiple of 8");
  if (c->out_row_bytes > 0 && c->out_row_bytes < min_row_bytes(c))
    return fail(APG_E_INVALID, "out_row_bytes is smaller than the packed output row of the enabled fields");
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
// GEN_POOL: maps of the resident pool (APG_MAP_POOL, any FloorMapDataset)
enum : int { GEN_NONE = 0, GEN_ROOMS = 1, GEN_PF = 2, GEN_POOL = 3 };  // mazes: k_maze (synchronous) or prefetched (GEN_PF)

// Rooms maps are painted into the lane's LDS bitmap (row words are read-modify-written once per
// primitive), then the wave copies its bitmaps out with coalesced stores.
APG_DEV void copy_out_maps(const uint64_t *s_maps, unsigned long long done, size_t words, uint64_t *dst, int lane) {
  while (done) {
    const int j = __ffsll((long long)done) - 1;
    done &= done - 1ULL;
    for (size_t k = lane; k < words; k += 64) dst[(size_t)j * words + k] = s_maps[(size_t)j * words + k];
  }
}

template <int MR>
__global__ __launch_bounds__(64) void k_map_generate_rooms(Geo g, const uint64_t *idx, int n, uint64_t *occ,
                                                           uint32_t *err, int lanes) {
  const BinomTable &bt = c_binom;
  extern __shared__ uint64_t s_rows[];  // [lanes][h * wpr]
  const int lane = threadIdx.x;
  const int i = blockIdx.x * lanes + lane;
  const bool active = lane < lanes && i < n;
  const size_t words = (size_t)g.h * g.wpr;
  int rc = 0;
  if (active) {
    Pcg64 r = seed_pcg64(idx[i]);
    rc = rooms_generate<MR>(r, s_rows + lane * words, g.wpr, g.h, g.max_rooms, g.door_width, bt);
  }
  copy_out_maps(s_rows, __ballot(active), words, occ + (size_t)blockIdx.x * lanes * words, lane);
  if (rc != 0 && err) atomicOr(err, APG_ERR_MAPGEN);
}

APG_DEV int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

APG_DEV int wave_inclusive_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// position of the k-th set bit (k < popcount(m)) of m: binary search on popcounts
APG_DEV int select_bit(uint64_t m, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(m & ((1ULL << w) - 1ULL));
    if (k >= c) {
      k -= c;
      m >>= w;
      pos += w;
    }
  }
  return pos;
}

// reset of env e (lidar_localization2d.py:293-315 with the _np_random setter :547-557 on reset(seed)):
// reseed (use_seed) or continue the env's streams, next map index from the DatasetIterator stream,
// rooms map generation into `own` (the caller's LDS bitmap), start cell draw.  Mazes: k_maze.
// Returns the env's new flags.
template <int GEN, int MR = 17>
APG_DEV uint8_t reset_one(const Geo &g, const apg_lidar_state &S, int e, uint8_t f, bool use_seed, uint64_t seed,
                          uint64_t *own, uint64_t *out_map_idx, uint32_t *err, const BinomTable &bt) {
  static_assert(GEN == GEN_NONE || GEN == GEN_ROOMS || GEN == GEN_POOL, "mazes reset in k_maze");
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
  if constexpr (GEN == GEN_POOL) {
    // DatasetIterator: integers(0, len(dataset)) (dataset_iterator.py:26-32), then get_data_point(idx) is pool map idx
    // (streamed maps: the host fetched get_data_point(idx) of this very draw into slot e ahead of the reset)
    midx = (uint64_t)integers(it, 0, g.stream_len ? g.stream_len : (int64_t)g.pool_len);
    const size_t words = (size_t)g.h * g.wpr;
    uint64_t *rows = S.occ + (size_t)e * words;
    const uint64_t *src = S.pool_occ + (g.stream_len ? (uint64_t)e : midx) * words;
    for (size_t q = 0; q < words; q++) rows[q] = src[q];
    if (place_start(rng, rows, g.h, g.w, g.wpr, px, py) != 0) atomicOr(err, APG_ERR_NO_FREE_CELL);
    *reinterpret_cast<Pcg64 *>(&S.it_rng[e]) = it;
    S.map_idx[e] = midx;
  } else if constexpr (GEN != GEN_NONE) {
    midx = next32(it);  // DatasetIterator: integers(0, len(dataset) = 2**32)
    Pcg64 map_rng = seed_pcg64(midx);  // FloorMapDataset*.get_data_point: default_rng(idx)
    int rc = rooms_generate<MR>(map_rng, own, g.wpr, g.h, g.max_rooms, g.door_width, bt);
    if (place_start(rng, own, g.h, g.w, g.wpr, px, py) != 0) rc = -6;
    if (rc != 0) atomicOr(err, APG_ERR_MAPGEN);
    *reinterpret_cast<Pcg64 *>(&S.it_rng[e]) = it;
    S.map_idx[e] = midx;
  } else {
    midx = S.map_idx[e];
    if (place_start(rng, S.occ, g.h, g.w, g.wpr, px, py) != 0)
      atomicOr(err, g.kind == APG_MAP_POOL ? APG_ERR_NO_FREE_CELL : APG_ERR_MAPGEN);
  }
  S.pos[2 * e] = px;
  S.pos[2 * e + 1] = py;
  S.init_pos[2 * e] = px;
  S.init_pos[2 * e + 1] = py;
  S.elapsed[e] = 0;
  const uint8_t nf = (uint8_t)((f & F_AUTORESET) | F_JUST_RESET | F_FIRST);
  S.flags[e] = nf;
  *reinterpret_cast<Pcg64 *>(&S.rng[e]) = rng;
  if (out_map_idx) oat(out_map_idx, g.row, e, 1) = midx;
  return nf;
}

// reset(seed) of all envs (static maps and rooms; mazes: k_maze): one wave per `lanes` (<= 64) envs.
// Map generation is a long serial, divergent chain per env whose speed is set by instruction latency,
// not by lanes, so the host spreads the envs over as many waves as fit on the chip at once (gen_lanes).
// Waves with nothing to reset exit after one flag load.
template <int GEN, int MR = 17>
__global__ __launch_bounds__(64) void k_lidar_reset(Geo g, apg_lidar_state S, uint64_t seed, int use_seed,
                                                    int all, uint64_t *out_map_idx, uint32_t *err,
                                                    int lanes) {
  const BinomTable &bt = c_binom;
  extern __shared__ uint64_t s_rows[];  // rooms: [lanes][h * wpr]
  const int lane = threadIdx.x;
  const int e = blockIdx.x * lanes + lane;
  const bool mine = lane < lanes && e < g.n;
  const uint8_t f = mine ? S.flags[e] : 0;
  const bool active = mine && (all || (f & F_AUTORESET));
  const unsigned long long todo = __ballot(active);
  if (todo == 0ULL) return;
  const size_t words = (size_t)g.h * g.wpr;
  if (active) reset_one<GEN, MR>(g, S, e, f, use_seed != 0, seed, s_rows + lane * words, out_map_idx, err, bt);
  if constexpr (GEN == GEN_ROOMS) copy_out_maps(s_rows, todo, words, S.occ + (size_t)blockIdx.x * lanes * words, lane);
}

// Mazes (FloorMapDatasetMaze.get_data_point, floor_map_dataset_maze.py:24-55, see apg_maze.hpp) in three
// launches: k_maze_stream (the random streams), k_maze (the DFS, one lane per maze, `lanes` <= 64 mazes per
// one-wave workgroup, carve logs into the scratch), k_maze_paint (rows, map obs, start cell, state), for
//   MZ_MAPS   maps of dataset indices idx[0, n) into occ (static map, dataset access);
//   MZ_RESET  reset_one for mazes: the envs that reset (all, or those with an autoreset pending), their
//             streams, map index, maze into S.occ, its f32 map obs (bool map / 255, lidar_localization2d.py:299:
//             the step kernel launched after it is given no map obs), start cell (place_start), state.
enum : int { MZ_MAPS = 0, MZ_RESET = 1 };

// ------------------------------------------------------------------ map prefetch (apgym_capi.h, "map prefetch")
// apg_lidar_state.prefetch holds, per env, the result of its NEXT reset computed ahead (the reference's
// DataLoader prefetch thread, lidar_localization2d.py:130-131, buffered_iterator.py:11-61): map index, occupancy
// rows, start cell, and the env / iterator streams after those draws.  Ownership: gen[] (resets done) is written
// only by the step / reset kernels on the env's stream; every other field by the prefetch batch on the side
// stream (and by the synchronous reset kernels, which run ordered against the batches by events).  A record is
// valid for the env's current episode when pf_gen[e] == gen[e].  Its streams are the env's current streams from
// the moment its reset installs them (S.rng = rng), so a batch draws the next reset from the record alone and reads
// nothing the concurrently running step kernel writes except gen, which that kernel stores after its reads of the
// record (a coherent relaxed atomic: the batch overwrites a record only once it sees the reset that consumed it).
// The step kernel consumes a record only after its stream waited for the batch that wrote it.
struct PfLayout {
  size_t gen, pf_gen, sel_gen, start, list, ctl, idx, rng, it, occ, bytes;
};
__host__ __device__ inline PfLayout pf_layout(int n, int h, int wpr) {
  PfLayout L;
  size_t o = 0;
  auto take = [&](size_t &f, size_t bytes) {
    f = o;
    o = (o + bytes + 255) & ~(size_t)255;
  };
  const size_t N = (size_t)n;
  take(L.gen, 4 * N);
  take(L.pf_gen, 4 * N);
  take(L.sel_gen, 4 * N);
  take(L.start, 4 * N);
  take(L.list, 4 * N);
  take(L.ctl, 64);  // [0] envs selected by the batch, [1] resets of the current step, [2] step workgroup ticket
  take(L.idx, 8 * N);
  take(L.rng, sizeof(Pcg64) * N);
  take(L.it, sizeof(Pcg64) * N);
  take(L.occ, 8 * N * (size_t)h * (size_t)wpr);
  L.bytes = o;
  return L;
}
struct PfView {
  uint32_t *gen, *pf_gen, *sel_gen, *start, *list;
  unsigned long long *ctl;
  uint64_t *idx;
  Pcg64 *rng, *it;
  uint64_t *occ;
  uint32_t *host_slot;  // step kernels: pinned host word that receives the step's reset count (NULL: none)
};
PfView pf_view(uint8_t *base, int n, int h, int wpr) {
  const PfLayout L = pf_layout(n, h, wpr);
  PfView v;
  v.gen = reinterpret_cast<uint32_t *>(base + L.gen);
  v.pf_gen = reinterpret_cast<uint32_t *>(base + L.pf_gen);
  v.sel_gen = reinterpret_cast<uint32_t *>(base + L.sel_gen);
  v.start = reinterpret_cast<uint32_t *>(base + L.start);
  v.list = reinterpret_cast<uint32_t *>(base + L.list);
  v.ctl = reinterpret_cast<unsigned long long *>(base + L.ctl);
  v.idx = reinterpret_cast<uint64_t *>(base + L.idx);
  v.rng = reinterpret_cast<Pcg64 *>(base + L.rng);
  v.it = reinterpret_cast<Pcg64 *>(base + L.it);
  v.occ = reinterpret_cast<uint64_t *>(base + L.occ);
  v.host_slot = nullptr;
  return v;
}
static_assert(sizeof(Pcg64) == sizeof(apg_pcg64), "prefetch records hold apg_pcg64 streams");
// relaxed, agent scope: coherent across the XCDs' L2s without the L2 write-back of a release fence
APG_DEV uint32_t pf_load_gen(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
APG_DEV void pf_store_gen(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Batch kernel 1: the envs whose record is stale (pf_gen != gen), appended to the list.  ctl[0] was zeroed before
// the launch.
__global__ __launch_bounds__(256) void k_pf_select(int n, PfView V) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  bool sel = false;
  uint32_t g = 0;
  if (e < n) {
    g = pf_load_gen(&V.gen[e]);
    sel = g != V.pf_gen[e];
  }
  const unsigned long long m = __ballot(sel);
  if (m == 0ULL) return;
  const int lane = threadIdx.x & 63;
  unsigned long long base = 0;
  if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&V.ctl[0], (unsigned long long)__popcll(m));
  base = __shfl(base, __ffsll((long long)m) - 1);
  if (sel) {
    V.sel_gen[e] = g;
    V.list[base + __popcll(m & ((1ULL << lane) - 1ULL))] = (uint32_t)e;
  }
}

// The dataset index of maze i (MZ_MAPS: idx[i]; MZ_RESET: the env's DatasetIterator draw, from its streams
// or, on reset(seed), from default_rng(seed + i)), with the env's streams after it.
APG_DEV uint64_t maze_index(const apg_lidar_state &S, const uint64_t *idx, int i, int mode, uint64_t seed,
                            int use_seed, Pcg64 &rng, Pcg64 &it) {
  if (mode != MZ_RESET) return idx[i];
  if (use_seed) {
    rng = seed_pcg64(seed + (uint64_t)i);
    it = seed_pcg64(bounded_u64(rng, 0x100000000ULL));  // integers(0, 2**32, endpoint=True)
  } else {
    rng = *reinterpret_cast<const Pcg64 *>(&S.rng[i]);
    it = *reinterpret_cast<const Pcg64 *>(&S.it_rng[i]);
  }
  return next32(it);  // DatasetIterator: integers(0, len(dataset) = 2**32)
}

// The random streams of the mazes k_maze is about to generate (apg_maze.hpp): a workgroup per MZS_MAZES
// mazes seeds them (default_rng(idx)) and tabulates the jumps to every item's first output, then its threads
// generate the items (MZ_ITEM_GROUPS groups of 32 outputs each) and the state after the last one.  Full
// occupancy, so the LCG work that held the DFS at one wave per SIMD runs at chip rate here.
constexpr int MZS_THREADS = 256, MZS_MAZES = 64;
static_assert(MZ_MAX_ITEMS + 1 <= MZS_THREADS - MZS_MAZES, "a jump-table entry per thread after the seeding ones");
__global__ __launch_bounds__(MZS_THREADS) void k_maze_stream(Geo g, apg_lidar_state S, const uint64_t *idx, int n,
                                                             uint8_t *scratch, int mode, uint64_t seed, int use_seed,
                                                             int all, int ng) {
  __shared__ uint64_t s_seed[MZS_MAZES][4];  // s_hi, s_lo, i_hi, i_lo
  __shared__ MzJump s_jump[MZ_MAX_ITEMS + 1];
  const int tid = threadIdx.x, nitems = ng / MZ_ITEM_GROUPS;
  const int i = blockIdx.x * MZS_MAZES + tid;
  bool act = false;
  if (tid < MZS_MAZES && i < n) act = mode != MZ_RESET || all || (S.flags[i] & F_AUTORESET);
  if (__syncthreads_or(act) == 0) return;  // (most steps: no autoreset pending)
  if (tid < MZS_MAZES) {
    if (act) {
      Pcg64 rng, it;
      const Pcg64 mr = seed_pcg64(maze_index(S, idx, i, mode, seed, use_seed, rng, it));
      s_seed[tid][0] = mr.s_hi;
      s_seed[tid][1] = mr.s_lo;
      s_seed[tid][2] = mr.i_hi;
      s_seed[tid][3] = mr.i_lo;
    } else {
      s_seed[tid][2] = s_seed[tid][3] = 0ULL;  // inactive: increments are odd, 0 never is one
    }
  } else if (tid - MZS_MAZES <= nitems) {  // nitems <= MZ_MAX_ITEMS = MZS_THREADS - MZS_MAZES - 1
    s_jump[tid - MZS_MAZES] = mz_jump((uint64_t)(tid - MZS_MAZES) * MZ_ITEM_GROUPS * MZ_GROUP);
  }
  __syncthreads();
  const size_t sb = maze_scratch_bytes(g.h, g.w), so = maze_stream_off(g.h, g.w);
  for (int q = tid; q < MZS_MAZES * (nitems + 1); q += MZS_THREADS) {
    const int j = q / (nitems + 1), c = q - j * (nitems + 1);
    if (s_seed[j][3] == 0ULL) continue;
    uint8_t *stream = scratch + (size_t)(blockIdx.x * MZS_MAZES + j) * sb + so;
    if (c < nitems) {
      maze_stream_item(s_seed[j][0], s_seed[j][1], s_seed[j][2], s_seed[j][3], s_jump[c], g.bp, c, stream, ng);
    } else {  // the state after the stream, for a maze that draws past it
      uint64_t hi = s_seed[j][0], lo = s_seed[j][1];
      mz_jump_state(s_jump[c], hi, lo, s_seed[j][2], s_seed[j][3]);
      uint64_t *st = reinterpret_cast<uint64_t *>(stream + maze_stream_state_off(ng));
      st[0] = hi;
      st[1] = lo;
    }
  }
}

template <bool ONEW>
__global__ __launch_bounds__(64) void k_maze(Geo g, apg_lidar_state S, const uint64_t *idx, int n, uint8_t *scratch,
                                             int mode, uint64_t seed, int use_seed, int all, uint32_t *err, int lanes,
                                             int ng) {
  extern __shared__ uint64_t s_mz[];  // apg_maze.hpp's workgroup layout
  const int lane = threadIdx.x;
  const int i = blockIdx.x * lanes + lane;
  const bool mine = lane < lanes && i < n;
  const MazeGeom m = maze_geom(g.h, g.w);
  const size_t sb = maze_scratch_bytes(g.h, g.w), lb = maze_log_bytes(g.h, g.w);
  const bool active = mine && (mode != MZ_RESET || all || (S.flags[i] & F_AUTORESET));
  if (__ballot(active) == 0ULL) return;
  char *lds = reinterpret_cast<char *>(s_mz);
  maze_table_init<ONEW>(lds, lane);
  __syncthreads();
  Pcg64 mr{};
  if (active) {  // get_data_point: default_rng(idx) (its increment; the stream: k_maze_stream)
    Pcg64 rng, it;
    mr = seed_pcg64(maze_index(S, idx, i, mode, seed, use_seed, rng, it));
  }
  uint8_t *mine_scr = scratch + (size_t)(active ? i : 0) * sb;
  bool bad = false;
  const int nlog = maze_dfs<ONEW>(mr, mine_scr + maze_stream_off(g.h, g.w), ng, active, m, g.bp, lds, lane,
                                  mine_scr + lb, reinterpret_cast<uint32_t *>(mine_scr), bad);
  if (bad) atomicOr(err, APG_ERR_MAPGEN);
  if (active) *reinterpret_cast<int *>(mine_scr + maze_stream_off(g.h, g.w) + maze_stream_state_off(ng) + 16) = nlog;
}

// Mazes past the LDS layout of k_maze (maze_big: maps wider or taller than 255, up to 511): the reference's carve()
// recursion (floor_map_dataset_maze.py:24-55) one thread per maze, as an explicit frame stack in the maze scratch
// (frame: cell x | y << 9 | permutation index << 18 | next position << 23 | first << 26), the visited bits beside
// it, the draws straight from default_rng(idx): rng.permutation(directions) as numpy's shuffle (random_interval 3,
// 2, 1 on next_uint32) on entering a cell, rng.random() for a non-first eligible branch.  The occupancy rows are
// carved in place (all walls first); k_maze_paint (prepainted) then writes the map obs and the start cell.  Slow
// (global memory, one lane per maze) but exact: these sizes are off the benched configurations.
__global__ __launch_bounds__(64) void k_maze_big(Geo g, apg_lidar_state S, const uint64_t *idx, int n, uint64_t *occ,
                                                 uint8_t *scratch, int mode, uint64_t seed, int use_seed, int all) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  if (mode == MZ_RESET && !all && !(S.flags[i] & F_AUTORESET)) return;
  Pcg64 rng, it;
  Pcg64 r = seed_pcg64(maze_index(S, idx, i, mode, seed, use_seed, rng, it));
  const MazeGeom m = maze_geom(g.h, g.w);
  const int words = g.h * g.wpr;
  uint64_t *rows = (mode == MZ_RESET ? S.occ : occ) + (size_t)i * words;
  uint8_t *scr = scratch + (size_t)i * maze_scratch_bytes(g.h, g.w);
  uint64_t *vis = reinterpret_cast<uint64_t *>(scr);
  uint32_t *stk = reinterpret_cast<uint32_t *>(scr + maze_big_vis_bytes(g.h, g.w));
  for (int q = 0; q < words; q++) {  // all walls
    const int lo = 64 * (q % g.wpr);
    rows[q] = g.w - lo >= 64 ? ~0ULL : ((1ULL << (g.w - lo)) - 1ULL);
  }
  for (int q = 0; q < m.ncy * m.cw; q++) vis[q] = 0ULL;
  auto open_cell = [&](int x, int y) { rows[y * g.wpr + (x >> 6)] &= ~(1ULL << (x & 63)); };
  auto visited = [&](int cx, int cy) { return (vis[cy * m.cw + (cx >> 6)] >> (cx & 63)) & 1ULL; };
  auto visit = [&](int cx, int cy) { vis[cy * m.cw + (cx >> 6)] |= 1ULL << (cx & 63); };
  auto draw_perm = [&]() {  // numpy shuffle of the 4 directions: swap(3, j3), swap(2, j2), swap(1, j1)
    const uint32_t j3 = random_interval_small(r, 3u), j2 = random_interval_small(r, 2u), j1 = random_interval_small(r, 1u);
    return j3 * 6u + j2 * 2u + j1;
  };
  auto pack = [](uint32_t cx, uint32_t cy, uint32_t p, uint32_t k, uint32_t first) {
    return cx | (cy << 9) | (p << 18) | (k << 23) | (first << 26);
  };
  open_cell(1, 1);  // maze[1, 1] = 0 (maze.py:51)
  visit(0, 0);
  stk[0] = pack(0u, 0u, draw_perm(), 0u, 1u);
  int sp = 1;
  while (sp > 0) {
    const uint32_t f = stk[sp - 1];
    const int cx = (int)(f & 511u), cy = (int)((f >> 9) & 511u);
    const uint32_t p = (f >> 18) & 31u, k = (f >> 23) & 7u;
    uint32_t first = (f >> 26) & 1u;
    if (k >= 4u) {  // every direction tried: return to the parent
      sp--;
      continue;
    }
    const uint32_t d = (mz_perm_of(p) >> (2u * k)) & 3u;
    const int dx = (d == 0u) - (d == 1u), dy = (d == 2u) - (d == 3u);
    const int nx = cx + dx, ny = cy + dy;
    bool carve = false;
    if (nx >= 0 && nx < m.ncx && ny >= 0 && ny < m.ncy && !visited(nx, ny))  // 0 < next < dims - 1, maze[next] == 1
      carve = first || next_double(r) < g.bp;  // maze.py:42
    if (carve) first = 0u;
    stk[sp - 1] = pack((uint32_t)cx, (uint32_t)cy, p, k + 1u, first);
    if (carve) {
      open_cell(2 * cx + 1 + dx, 2 * cy + 1 + dy);  // the passage, then the cell
      open_cell(2 * nx + 1, 2 * ny + 1);
      visit(nx, ny);
      stk[sp++] = pack((uint32_t)nx, (uint32_t)ny, draw_perm(), 0u, 1u);  // carve(next_pos)
    }
  }
}

// After k_maze's DFS, at full occupancy: a workgroup per MP_ENVS consecutive envs lists the mazes k_maze
// generated and, one maze at a time with all its threads, paints the occupancy rows from the carve log
// (maze_paint), writes them out (occ, or S.occ), and for MZ_RESET writes the map obs (bool map / 255,
// lidar_localization2d.py:299), draws the start cell like place_start (reset :304: the pick-th free cell in
// row-major order, pick = integers(0, nfree) on the env's stream) and resets the env's state.
#ifndef APG_MP_ENVS
#define APG_MP_ENVS 4  // mazes per k_maze_paint / k_pf_paint workgroup (64: 4.80 ms, 16: 4.51, 8: 4.49, 4: 4.44 at cfg 3)
#endif
constexpr int MP_THREADS = 256, MP_ENVS = APG_MP_ENVS;
__global__ __launch_bounds__(MP_THREADS) void k_maze_paint(Geo g, apg_lidar_state S, const uint64_t *idx, int n,
                                                           uint64_t *occ, const uint8_t *scratch, int mode,
                                                           uint64_t seed, int use_seed, int all, int ng,
                                                           uint64_t *out_map_idx, float *map_obs, uint32_t *err,
                                                           PfView pv, int prepainted) {
  __shared__ uint16_t s_list[MP_ENVS];
  __shared__ int s_cnt, s_wsum[MP_THREADS / 64], s_hit[2];
  extern __shared__ uint64_t s_bm[];  // one maze's rows, then bitmap_map_obs's linear bitmap
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, e0 = blockIdx.x * MP_ENVS;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  if (tid < MP_ENVS && e0 + tid < n && (mode != MZ_RESET || all || (S.flags[e0 + tid] & F_AUTORESET)))
    s_list[atomicAdd(&s_cnt, 1)] = (uint16_t)tid;
  __syncthreads();
  const int cnt = s_cnt;
  const MazeGeom m = maze_geom(g.h, g.w);
  const size_t words = (size_t)g.h * g.wpr, sb = maze_scratch_bytes(g.h, g.w);
  for (int k = 0; k < cnt; k++) {
    const int e = e0 + s_list[k];
    const uint8_t *scr = scratch + (size_t)e * sb;
    uint64_t *dst = (mode == MZ_RESET ? S.occ : occ) + (size_t)e * words;
    if (prepainted) {  // k_maze_big wrote the rows: into the LDS bitmap
      for (int q = tid; q < (int)words; q += MP_THREADS) s_bm[q] = dst[q];
      __syncthreads();
    } else {
      const int nlog = *reinterpret_cast<const int *>(scr + maze_stream_off(g.h, g.w) + maze_stream_state_off(ng) + 16);
      maze_paint<MP_THREADS>(m, g.wpr, reinterpret_cast<const uint32_t *>(scr), nlog, s_bm, tid);
      for (int q = tid; q < (int)words; q += MP_THREADS) dst[q] = s_bm[q];
    }
    if (mode != MZ_RESET) {
      __syncthreads();  // the bitmap is read before the next maze paints it
      continue;
    }
    if (map_obs) bitmap_map_obs<MP_THREADS>(s_bm, g.h, g.w, g.wpr, map_obs + (size_t)e * g.h * g.w, tid, s_bm + words);
    // free cells per row, their inclusive scan (rpt consecutive rows per thread: maps up to 2 * MP_THREADS rows),
    // the row holding the pick
    const int rpt = (g.h + MP_THREADS - 1) / MP_THREADS;
    auto row_free = [&](int y) {
      int oc = 0;
      for (int kk = 0; kk < g.wpr; kk++) oc += __popcll(s_bm[y * g.wpr + kk]);
      return g.w - oc;
    };
    int fr = 0;
    for (int rr = 0; rr < rpt; rr++)
      if (tid * rpt + rr < g.h) fr += row_free(tid * rpt + rr);
    const int incl_w = wave_inclusive_scan(fr, lane);
    if (lane == 63) s_wsum[wave] = incl_w;
    if (tid == 0) s_hit[0] = -1;
    __syncthreads();
    int before = 0, nfree = 0;
#pragma unroll
    for (int w2 = 0; w2 < MP_THREADS / 64; w2++) {
      before += w2 < wave ? s_wsum[w2] : 0;
      nfree += s_wsum[w2];
    }
    const int incl = incl_w + before, excl = incl - fr;
    Pcg64 rng, it;
    const uint64_t midx = maze_index(S, idx, e, mode, seed, use_seed, rng, it);
    const long long pick = nfree > 0 ? (long long)integers(rng, 0, nfree) : -1;  // every thread: same draw
    if (tid * rpt < g.h && pick >= excl && pick < incl) {
      int k2 = (int)(pick - excl), hx = -1, hy = tid * rpt;
      for (int rr = 0; rr < rpt; rr++) {  // the row of this thread's rows that holds the pick
        const int y = tid * rpt + rr, c = y < g.h ? row_free(y) : 0;
        if (k2 < c) {
          hy = y;
          break;
        }
        k2 -= c;
      }
      for (int kk = 0; kk < g.wpr && hx < 0; kk++) {
        const int lo = 64 * kk;
        const uint64_t valid = g.w - lo >= 64 ? ~0ULL : ((1ULL << (g.w - lo)) - 1ULL);
        const uint64_t fm = ~s_bm[hy * g.wpr + kk] & valid;
        const int c = __popcll(fm);
        if (k2 < c) hx = lo + select_bit(fm, k2);
        else k2 -= c;
      }
      s_hit[0] = hx;
      s_hit[1] = hy;
    }
    __syncthreads();
    if (tid == 0) {
      const uint8_t f = S.flags[e];
      float px = 0.5f, py = 0.5f;
      if (s_hit[0] < 0) {
        atomicOr(err, APG_ERR_MAPGEN);
      } else {
        px = __fadd_rn((float)s_hit[0], 0.5f);
        py = __fadd_rn((float)s_hit[1], 0.5f);
      }
      S.pos[2 * e] = px;
      S.pos[2 * e + 1] = py;
      S.init_pos[2 * e] = px;
      S.init_pos[2 * e + 1] = py;
      S.elapsed[e] = 0;
      S.flags[e] = (uint8_t)((f & F_AUTORESET) | F_JUST_RESET | F_FIRST);
      *reinterpret_cast<Pcg64 *>(&S.rng[e]) = rng;
      *reinterpret_cast<Pcg64 *>(&S.it_rng[e]) = it;
      S.map_idx[e] = midx;
      if (out_map_idx) oat(out_map_idx, g.row, e, 1) = midx;
      if (pv.gen) {  // the record's streams follow the env's; a prefetched next map is stale now
        pv.rng[e] = rng;
        pv.it[e] = it;
        pf_store_gen(&pv.gen[e], pv.gen[e] + 1u);
      }
    }
    __syncthreads();  // s_hit / the bitmap are reused by the next maze
  }
}

// Batch kernel 2: the random streams of the listed envs' next mazes (k_maze_stream's work): the DatasetIterator
// draw of each env's next map index (lidar_localization2d.py:296-298, dataset_iterator.py:26-32) from the record's
// iterator stream, then default_rng(idx)'s outputs into the env's maze scratch.
__global__ __launch_bounds__(MZS_THREADS) void k_pf_stream(Geo g, PfView V, uint8_t *scratch, int ng) {
  __shared__ uint64_t s_seed[MZS_MAZES][4];
  __shared__ uint32_t s_env[MZS_MAZES];
  __shared__ MzJump s_jump[MZ_MAX_ITEMS + 1];
  const int tid = threadIdx.x, nitems = ng / MZ_ITEM_GROUPS;
  const int cnt = (int)V.ctl[0];
  const int i0 = blockIdx.x * MZS_MAZES;
  if (i0 >= cnt) return;  // workgroup-uniform: most of the grid when few envs reset
  if (tid < MZS_MAZES) {
    if (i0 + tid < cnt) {
      const uint32_t e = V.list[i0 + tid];
      Pcg64 it = V.it[e];
      const uint64_t midx = next32(it);  // DatasetIterator: integers(0, len(dataset) = 2**32)
      V.it[e] = it;
      V.idx[e] = midx;
      const Pcg64 mr = seed_pcg64(midx);  // FloorMapDatasetMaze.get_data_point: default_rng(idx)
      s_seed[tid][0] = mr.s_hi;
      s_seed[tid][1] = mr.s_lo;
      s_seed[tid][2] = mr.i_hi;
      s_seed[tid][3] = mr.i_lo;
      s_env[tid] = e;
    } else {
      s_seed[tid][2] = s_seed[tid][3] = 0ULL;
    }
  } else if (tid - MZS_MAZES <= nitems) {
    s_jump[tid - MZS_MAZES] = mz_jump((uint64_t)(tid - MZS_MAZES) * MZ_ITEM_GROUPS * MZ_GROUP);
  }
  __syncthreads();
  const size_t sb = maze_scratch_bytes(g.h, g.w), so = maze_stream_off(g.h, g.w);
  for (int q = tid; q < MZS_MAZES * (nitems + 1); q += MZS_THREADS) {
    const int j = q / (nitems + 1), c = q - j * (nitems + 1);
    if (s_seed[j][3] == 0ULL) continue;
    uint8_t *stream = scratch + (size_t)s_env[j] * sb + so;
    if (c < nitems) {
      maze_stream_item(s_seed[j][0], s_seed[j][1], s_seed[j][2], s_seed[j][3], s_jump[c], g.bp, c, stream, ng);
    } else {
      uint64_t hi = s_seed[j][0], lo = s_seed[j][1];
      mz_jump_state(s_jump[c], hi, lo, s_seed[j][2], s_seed[j][3]);
      uint64_t *st = reinterpret_cast<uint64_t *>(stream + maze_stream_state_off(ng));
      st[0] = hi;
      st[1] = lo;
    }
  }
}

// Batch kernel 3: the DFS of the listed envs' next mazes (k_maze's work), carve logs into their scratch.
template <bool ONEW>
__global__ __launch_bounds__(64) void k_pf_dfs(Geo g, PfView V, uint8_t *scratch, uint32_t *err, int lanes, int ng) {
  extern __shared__ uint64_t s_mz[];
  const int lane = threadIdx.x;
  const int cnt = (int)V.ctl[0];
  if (blockIdx.x * lanes >= cnt) return;
  const int i = blockIdx.x * lanes + lane;
  const bool active = lane < lanes && i < cnt;
  const uint32_t e = active ? V.list[i] : 0u;
  const MazeGeom m = maze_geom(g.h, g.w);
  const size_t sb = maze_scratch_bytes(g.h, g.w), lb = maze_log_bytes(g.h, g.w);
  char *lds = reinterpret_cast<char *>(s_mz);
  maze_table_init<ONEW>(lds, lane);
  __syncthreads();
  Pcg64 mr{};
  if (active) mr = seed_pcg64(V.idx[e]);
  uint8_t *mine_scr = scratch + (size_t)e * sb;
  bool bad = false;
  const int nlog = maze_dfs<ONEW>(mr, mine_scr + maze_stream_off(g.h, g.w), ng, active, m, g.bp, lds, lane,
                                  mine_scr + lb, reinterpret_cast<uint32_t *>(mine_scr), bad);
  if (bad) atomicOr(err, APG_ERR_MAPGEN);
  if (active) *reinterpret_cast<int *>(mine_scr + maze_stream_off(g.h, g.w) + maze_stream_state_off(ng) + 16) = nlog;
}

// Batch kernel 4: the listed envs' next occupancy rows painted from their carve logs (k_maze_paint's work) into the
// records, the start cell drawn like place_start (lidar_localization2d.py:304: the pick-th free cell in row-major
// order, pick = integers(0, nfree) on the env's stream), the record's env stream advanced past that draw, and the
// record published for the generation k_pf_select saw.  Maps of <= MP_THREADS rows.
__global__ __launch_bounds__(MP_THREADS) void k_pf_paint(Geo g, PfView V, const uint8_t *scratch, int ng,
                                                         uint32_t *err) {
  __shared__ int s_wsum[MP_THREADS / 64], s_hit[2];
  extern __shared__ uint64_t s_bm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cnt = (int)V.ctl[0];
  const int i0 = blockIdx.x * MP_ENVS;
  if (i0 >= cnt) return;
  const int kn = cnt - i0 < MP_ENVS ? cnt - i0 : MP_ENVS;
  const MazeGeom m = maze_geom(g.h, g.w);
  const size_t words = (size_t)g.h * g.wpr, sb = maze_scratch_bytes(g.h, g.w);
  for (int k = 0; k < kn; k++) {
    const uint32_t e = V.list[i0 + k];
    const uint8_t *scr = scratch + (size_t)e * sb;
    const int nlog = *reinterpret_cast<const int *>(scr + maze_stream_off(g.h, g.w) + maze_stream_state_off(ng) + 16);
    maze_paint<MP_THREADS>(m, g.wpr, reinterpret_cast<const uint32_t *>(scr), nlog, s_bm, tid);
    uint64_t *dst = V.occ + (size_t)e * words;
    for (int q = tid; q < (int)words; q += MP_THREADS) dst[q] = s_bm[q];
    int fr = 0;
    if (tid < g.h) {
      int oc = 0;
      for (int kk = 0; kk < g.wpr; kk++) oc += __popcll(s_bm[tid * g.wpr + kk]);
      fr = g.w - oc;
    }
    const int incl_w = wave_inclusive_scan(fr, lane);
    if (lane == 63) s_wsum[wave] = incl_w;
    if (tid == 0) s_hit[0] = -1;
    __syncthreads();
    int before = 0, nfree = 0;
#pragma unroll
    for (int w2 = 0; w2 < MP_THREADS / 64; w2++) {
      before += w2 < wave ? s_wsum[w2] : 0;
      nfree += s_wsum[w2];
    }
    const int incl = incl_w + before, excl = incl - fr;
    Pcg64 rng = V.rng[e];
    const long long pick = nfree > 0 ? (long long)integers(rng, 0, nfree) : -1;  // every thread: the same draw
    if (tid < g.h && pick >= excl && pick < incl) {
      int k2 = (int)(pick - excl), hx = -1;
      for (int kk = 0; kk < g.wpr && hx < 0; kk++) {
        const int lo = 64 * kk;
        const uint64_t valid = g.w - lo >= 64 ? ~0ULL : ((1ULL << (g.w - lo)) - 1ULL);
        const uint64_t fm = ~s_bm[tid * g.wpr + kk] & valid;
        const int c = __popcll(fm);
        if (k2 < c) hx = lo + select_bit(fm, k2);
        else k2 -= c;
      }
      s_hit[0] = hx;
      s_hit[1] = tid;
    }
    __syncthreads();
    if (tid == 0) {
      if (s_hit[0] < 0) atomicOr(err, APG_ERR_MAPGEN);
      V.start[e] = s_hit[0] < 0 ? ~0u : ((uint32_t)s_hit[1] << 8) | (uint32_t)s_hit[0];
      V.rng[e] = rng;
      V.pf_gen[e] = V.sel_gen[e];
    }
    __syncthreads();  // s_hit / the bitmap are reused by the next maze
  }
}

struct StepParams {
  int n, h, w, wpr, beams, step_limit, is_static, R, wrows, log_stats, sparse, row, wlo, whi;
  int lidar16;  // dense lidar rows 16-byte aligned (base pointer and row pitch): vector stores
  int pretest;  // phase 2a's bounding-box pre-test (rooms: ~1/3 of the beams walk); 0: every beam walks (mazes:
                // ~98 % of the beams touch a wall, the pre-test only delays them)
  int p4;       // the pre-test reads a 4-row OR table of the windows (built by phase 1's idle waves; step_lds_bytes)
  float range, loss_scale, loss_offset;
};

// ActiveRegressionLogWrapper (active_regression_env.py:131-159): per step |target - prediction| and
// mean((target - prediction)^2) in float32; at the episode end avg = float(np.mean(list)) (numpy's
// pairwise float32 mean) and final = the last value.  The history is step-major,
// stats_hist[metric][step][env] (metric 0 euclidean distance, 1 mse), so the per-step stores of a
// wave are coalesced; the episode-end sums read an env's column with stride N.
// DEEP: episodes longer than PW_PTR_MAX_N steps (k_episode_stats, after the step kernel, which left their
// stats_len set and the sums to it).
template <bool DEEP = false>
APG_DEV void log_episode_stats(const StepParams &P, const apg_lidar_outputs &O, int e, const float *hist, int len) {
  for (int m = 0; m < 2; m++) {
    const float *h = hist + (size_t)m * P.step_limit * P.n + e;
    const float sum = DEEP ? pw_sum_ptr_deep(h, len, (size_t)P.n) : pw_sum_ptr(h, len, (size_t)P.n);
    const float avg = f32_div(__fadd_rn(0.0f, sum), (float)len);
    const float fin = h[(size_t)(len - 1) * P.n];
    if (P.row) {
      oat(O.stats, P.row, e, 4, m) = avg;
      oat(O.stats, P.row, e, 4, 2 + m) = fin;
    } else {
      O.stats[(size_t)m * P.n + e] = avg;
      O.stats[(size_t)(2 + m) * P.n + e] = fin;
    }
  }
  oat(O.stats_len, P.row, e, 1) = len;
}

// Occupancy window per env, staged in LDS from the PRE-move position p0: the 32 x 32 cells
// [floor(p0) - 15, floor(p0) + 17)^2 (zero outside the map).  A step moves the agent by at most
// ~2 cells (clamped move <= 1, slide <= 1), and every cell a scan of length <= R from the new
// position p can touch lies within [floor(p) - R - 2, floor(p) + R + 1] (+1 column for the 2-bit
// quad reads), i.e. within [floor(p0) - R - 5, floor(p0) + R + 5]: inside the window for R <= 10.
// APG_STEP_STOP=k (tuning builds only, tools/phase_pmc.py): the kernel returns after phase mark k, so
// PMC counts of the variants split the instruction mix by phase.  Outputs are then meaningless.
#ifdef APG_STEP_STOP
#define STEP_STOP(k) \
  if (APG_STEP_STOP == (k)) return;
#else
#define STEP_STOP(k)
#endif
#ifdef APG_STEP_PROFILE  // tuning builds only (tools/step_phase_profile.py): per-workgroup phase timestamps
__device__ unsigned long long g_step_prof[16384][16];
#define STEP_MARK(k) \
  if (threadIdx.x == 0 && blockIdx.x < 16384) g_step_prof[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
// per wave (lane 0): [0] phase R1 (generation) done, [1] phase R2 (paint) done
__device__ unsigned long long g_step_prof_w[16384][16][2];
#define STEP_MARK_W(k)                                    \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 16384) \
    g_step_prof_w[blockIdx.x][threadIdx.x >> 6][k] = __builtin_amdgcn_s_memrealtime();
#else
#define STEP_MARK(k)
#define STEP_MARK_W(k)
#endif
#ifndef APG_SLIDE_SPLIT
#define APG_SLIDE_SPLIT 1  // phase 1: second slide scan on the idle waves (0: both on the env's lane; A/B 36.4 -> 35.8 us)
#endif
#ifndef APG_MAPOBS_NT
#define APG_MAPOBS_NT 1  // the fused rooms autoreset's f32 map obs as non-temporal 16-byte stores (0: plain; A/B knob)
#endif
#ifndef APG_R2_LANES
#define APG_R2_LANES 1  // rooms autoreset paint: primitives via v_readlane (scalar decode); 0: per-lane LDS reads (A/B)
#endif
#ifndef APG_STEP_MIN_WAVES
#define APG_STEP_MIN_WAVES 4  // keep k_lidar_step at <= 128 VGPRs: 4 waves per SIMD
#endif

// Workgroup shape of a k_lidar_step instance: EPB envs, 4 threads per env (phase 2a: 4 beams at a
// time per env), W waves.  Phases R and 1 are "env-major": env slot el runs on wave el % W, lane
// el / W, i.e. every wave carries EPB / W = 16 envs, so the serial per-env chains (map generation,
// the move scans) run on all W waves at once instead of on the first EPB / 64.
template <int EPB>
struct StepShape {
  static constexpr int T = 4 * EPB, W = T / 64, LPW = EPB / W;
  static_assert(EPB == 64 || EPB == 128 || EPB == 256, "EPB: 64, 128 or 256 (256 / 512 / 1024 threads)");
  static_assert(LPW == 16, "16 envs per wave in the env-major phases");
};
constexpr int MAX_MAP_ROWS = 128;
// GEN_PF phase R, per wave: an env's occupancy rows (<= 128 x 2 words), then bitmap_map_obs's linear bitmap
constexpr int PF_WAVE_WORDS = MAX_MAP_ROWS * 2 + (MAX_MAP_ROWS * 128 + 63) / 64 + 1;

// Row y of a rooms map painted from its (narrow) primitives (rooms_paint's result, one row at a time): border
// | walls & ~doors.  Word k covers columns [64k, 64k + 64); the primitives are pr[i * st].
APG_DEV uint64_t rooms_row_word(const uint32_t *pr, int st, int m, int y, int k) {
  const int nw = (int)(pr[0] & 255u), nd = (int)(pr[0] >> 8);
  uint64_t v = (y == 0 || y == m - 1) ? span_mask(0, m, k) : (span_mask(0, 1, k) | span_mask(m - 1, 1, k));
  for (int i = 0; i < nw; i++) {
    const Wall wl = RoomsFmt<false>::wall_of(pr[(1 + i) * st]);
    if (wl.vertical) {
      if (y >= wl.start && y < wl.start + wl.len && (wl.fixed >> 6) == k) v |= 1ULL << (wl.fixed & 63);
    } else if (wl.fixed == y) {
      v |= span_mask(wl.start, wl.len, k);
    }
  }
  for (int i = 0; i < nd; i++) {
    const Door d = RoomsFmt<false>::door_of(pr[(17 + i) * st]);
    if (y >= d.r0 && y < d.r0 + d.hh) v &= ~span_mask(d.c0, d.ww, k);
  }
  return v;
}

// rooms_row_word with the env's primitives held one per lane (prv = pr[lane * st] on lanes 0 .. ROOMS_PRIM_WORDS - 1)
// and taken into scalar registers with v_readlane: the primitives' decode and span masks run on the scalar unit,
// and each lane keeps a range compare and a masked OR / AND per primitive (the reset step's paint is VALU-bound
// with four waves per SIMD)
APG_DEV uint64_t rooms_row_word_lanes(uint32_t prv, int m, int y, int k) {
  const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)prv, 0);
  const int nw = (int)(p0 & 255u), nd = (int)(p0 >> 8);
  const uint64_t full = span_mask(0, m, k), side = span_mask(0, 1, k) | span_mask(m - 1, 1, k);
  uint64_t v = (y == 0 || y == m - 1) ? full : side;
  for (int i = 0; i < nw; i++) {
    const Wall wl = RoomsFmt<false>::wall_of((uint32_t)__builtin_amdgcn_readlane((int)prv, 1 + i));
    if (wl.vertical) {
      const uint64_t bit = (wl.fixed >> 6) == k ? 1ULL << (wl.fixed & 63) : 0ULL;
      if (y >= wl.start && y < wl.start + wl.len) v |= bit;
    } else {
      const uint64_t sm = span_mask(wl.start, wl.len, k);
      if (y == wl.fixed) v |= sm;
    }
  }
  for (int i = 0; i < nd; i++) {
    const Door d = RoomsFmt<false>::door_of((uint32_t)__builtin_amdgcn_readlane((int)prv, 17 + i));
    const uint64_t keep = ~span_mask(d.c0, d.ww, k);
    if (y >= d.r0 && y < d.r0 + d.hh) v &= keep;
  }
  return v;
}

// Phase-R LDS of the fused rooms autoresets (dynamic region, before the windows are staged), all
// [index][EPB] so each thread's generator state is interleaved: primitives, task stack, split
// capacities and sizes, cut points, then each wave's copy of the map being painted.
constexpr int ROOMS_STACK = 20;  // pending tasks carry >= 1 room each: at most max_rooms <= 17
template <int EPB>
struct RoomsLds {
  static constexpr size_t prim = 0;
  static constexpr size_t stk = prim + (size_t)ROOMS_PRIM_WORDS * EPB * 4;
  static constexpr size_t cap = stk + (size_t)ROOMS_STACK * EPB * 8;
  static constexpr size_t size = cap + (size_t)17 * EPB * 2;
  static constexpr size_t cut = size + (size_t)17 * EPB * 2;
  static constexpr size_t mrow = (cut + (size_t)16 * EPB * 2 + 7) & ~(size_t)7;
  static constexpr size_t bytes = mrow + (size_t)(4 * EPB / 64) * MAX_MAP_ROWS * 2 * 8;
};

// GEN / FUSED: FUSED instances start with phase R, the NEXT_STEP autoresets of the envs whose episode
// ended at the previous step (map generation of kind GEN, start cell), so a step is one launch; the
// unfused instance (reset(seed)'s observation pass after k_lidar_reset) skips it.
// GR: every scan reads the occupancy rows from global memory through its own 32-column window (RowsGlobal at
// floor(min(p.x, q.x)) - 1: scans up to 28 cells long) instead of the staged 32 x 32 window around the env,
// for lidar_range > 10 (the staged window covers R <= 10).
// ROWP: packed output rows (apg_lidar_config.out_row_bytes > 0); the dense instance has P.row = 0 folded in.
template <int GEN, bool FUSED, int EPB, bool GR = false, bool ROWP = false>
__global__ __launch_bounds__(4 * EPB, APG_STEP_MIN_WAVES) void k_lidar_step(StepParams P_in, Geo g, apg_lidar_state S,
                                                                 const float *__restrict__ act,
                                                                 const float *__restrict__ pred,
                                                                 apg_lidar_outputs O, PfView V) {
  const BinomTable &bt = c_binom;
  using SS = StepShape<EPB>;
  constexpr int T = SS::T, W = SS::W, LPW = SS::LPW;
  StepParams P = P_in;
  if constexpr (!ROWP) P.row = 0;
  __shared__ float s_pos[EPB][2];
  __shared__ int s_x0[EPB], s_y0[EPB];
  __shared__ uint16_t s_rlist[EPB];  // envs that reset this step (map obs pass)
  __shared__ uint32_t s_start[EPB];  // rooms autoreset: start cell y << 8 | x, or ~0u (no free cell)
  __shared__ int s_cnt[4];           // 0: reset-list length, 1: queued walks, 2: walk / chunk cursor
  __shared__ float s_dirs[MAX_STAGED_BEAMS][2];  // beam_dirs, read inside the beam loops (LDS, not HBM latency)
#if APG_SLIDE_SPLIT
  __shared__ float s_slide[EPB];  // phase 1: the second slide candidate's length, then its scan distance
#endif
  // dynamic LDS (step_lds_bytes): occupancy windows, then (beams <= MAX_STAGED_BEAMS) the lidar rows
  // staged for coalesced stores and the phase-2b work list of (beam << 8) | env entries.  Phase R
  // (rooms) uses the same bytes first for the primitives and each wave's map rows.
  extern __shared__ uint32_t s_dyn[];
  uint32_t *s_win = s_dyn;
  const int LS = P.beams + 1;  // odd row stride: lanes = envs hit distinct banks
  float *s_lid = reinterpret_cast<float *>(s_dyn + EPB * WIN_STRIDE);
  uint16_t *s_queue = reinterpret_cast<uint16_t *>(s_lid + EPB * LS);
  float *s_tab = reinterpret_cast<float *>(s_queue + EPB * P.beams);  // EMPTY_TAB entries (staged instances)
  // (P.p4) s_win4[el * WIN_STRIDE + r] = OR of window rows r .. r + 3 of env slot el, for r in [wlo, whi - 3)
  uint32_t *s_win4 = reinterpret_cast<uint32_t *>(s_tab + EMPTY_TAB);
  // first table entry's bit pattern (recomputed where used: nothing stays live across the phases)
  auto tab_base = [&]() { return __float_as_uint(__fmul_rn(P.range, P.range)) - (uint32_t)(EMPTY_TAB / 2); };
  // the occupancy rows a scan of env slot el from x = ax to x = bx reads
  auto rows_of = [&](int el, float ax, float bx) {
    if constexpr (GR)
      return RowsGlobal{S.occ + (P.is_static ? 0 : (size_t)(blockIdx.x * EPB + el) * (size_t)P.h * P.wpr), P.h, P.wpr,
                        (int)floorf(fminf(ax, bx)) - 1};
    else
      return RowsWindow{&s_win[el * WIN_STRIDE], s_x0[el], s_y0[el], P.wrows};
  };
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int base = blockIdx.x * EPB;
  const size_t words = (size_t)P.h * P.wpr;
  // env-major slot of this thread (phases R, 0, 1)
  const bool env_thread = lane < LPW;
  const int my_el = lane * W + wave, my_e = base + my_el;
  const bool my_valid = env_thread && my_e < P.n;
  STEP_MARK(0)
#ifdef APG_STEP_PROFILE
  const unsigned long long prof_clk0 = __builtin_amdgcn_s_memtime();
#endif

  if (tid == 0) {
    s_cnt[0] = 0;
    s_cnt[1] = 0;
    s_cnt[2] = 0;
    s_cnt[3] = 0;
  }
  // Phases 0 and 1 run lane = env on the first EPB / 64 waves (thread tid owns env base + tid).  Its
  // inputs are loaded here, before any barrier, so their latency overlaps phase R and the window loads
  // (reloaded after phase R where resets happened).
  const int oe = base + tid;
  const bool own = tid < EPB && oe < P.n;
  uint8_t pf_f = 0;
  float pf_px = 0.0f, pf_py = 0.0f, pf_ax = 0.0f, pf_ay = 0.0f, pf_prx = 0.0f, pf_pry = 0.0f, pf_ix = 0.0f,
        pf_iy = 0.0f;
  int pf_el = 0;
  if (own) {
    pf_f = S.flags[oe];
    pf_px = S.pos[2 * oe];
    pf_py = S.pos[2 * oe + 1];
    pf_ix = S.init_pos[2 * oe];
    pf_iy = S.init_pos[2 * oe + 1];
    pf_el = S.elapsed[oe];
    if (act) {
      pf_ax = act[2 * oe];
      pf_ay = act[2 * oe + 1];
      pf_prx = pred[2 * oe];
      pf_pry = pred[2 * oe + 1];
    }
  }
  // The occupancy windows (32 x 32 cells from the pre-move position, see above): each thread's rows of
  // up to WIN_ITERS envs, loaded first thing from the envs' positions in HBM, so their latency overlaps
  // the input loads (a workgroup with autoresets reloads them after phase R).  Beam directions likewise.
  constexpr int WIN_ITERS = EPB * MAX_WIN_ROWS / T;
  uint32_t wv[WIN_ITERS];
  auto load_windows = [&]() {
#pragma unroll
    for (int k = 0; k < WIN_ITERS; k++) {
      const int r = tid + k * T;
      const int el = r / MAX_WIN_ROWS, row = r - el * MAX_WIN_ROWS;
      wv[k] = 0;
      if (base + el < P.n && row >= P.wlo && row < P.whi) {  // rows outside [wlo, whi) are never read
#ifdef APG_TIMING_NO_POSDEP  // timing experiment only (wrong results): window rows at a fixed origin, no pos load
        const float wpx = 20.5f, wpy = 20.5f;
#else
        const float wpx = S.pos[2 * (base + el)], wpy = S.pos[2 * (base + el) + 1];
#endif
        const int y = (int)floorf(wpy) - 15 + row;
        if ((unsigned)y < (unsigned)P.h)
          wv[k] = extract_window_row(S.occ + (P.is_static ? 0 : (size_t)(base + el) * words) + (size_t)y * P.wpr,
                                     P.wpr, (int)floorf(wpx) - 15);
      }
    }
  };
  if constexpr (!GR) load_windows();
  const bool dir_thread = P.beams <= MAX_STAGED_BEAMS && tid < 2 * P.beams;
  const float dir_v = dir_thread ? S.beam_dirs[tid] : 0.0f;
  if constexpr (!FUSED) __syncthreads();

  // ---------------- phase R: NEXT_STEP autoresets (fused instances), env-major.  The barrier of
  // __syncthreads_or also publishes the counters above.
  if constexpr (FUSED) {
    const uint8_t f0 = my_valid ? S.flags[my_e] : 0;
    const bool pend = my_valid && (f0 & F_AUTORESET);
    int npend;
    if constexpr (GEN == GEN_PF) {
      // the step's reset count to the prefetcher (pinned host word): every workgroup adds its count, the last one
      // to finish this point (ticket) publishes the total and rearms the counters for the next step
      npend = __syncthreads_count(pend);
      if (tid == 0) {  // (coherent relaxed atomics, ordered by a vmcnt wait instead of a release fence's L2 flush)
        if (npend) __hip_atomic_fetch_add(&V.ctl[1], (unsigned long long)npend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the count is added before the ticket is taken
        const unsigned long long t = __hip_atomic_fetch_add(&V.ctl[2], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
          const unsigned long long tot = __hip_atomic_load(&V.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (V.host_slot) __hip_atomic_store(V.host_slot, (uint32_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&V.ctl[1], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&V.ctl[2], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else {
      npend = __syncthreads_or(pend);
    }
    STEP_MARK(8)
    if (npend) {
      if constexpr (GEN == GEN_PF) {
        // Prefetched mazes (the record written by the side stream's batch, k_pf_*): each wave copies the next
        // occupancy rows of its pending envs (coalesced, into S.occ and the wave's LDS copy) and writes their f32
        // map obs (bool map / 255, lidar_localization2d.py:299) from that copy; the env's lane then installs the
        // reset state (start cell, streams after the reset's draws, map index: :293-315) and publishes the new
        // generation (release: the side stream's select reads the streams after acquiring it)
        uint64_t *mrow = reinterpret_cast<uint64_t *>(s_dyn) + (size_t)wave * PF_WAVE_WORDS;  // rows, linear bitmap
        const int m = P.h, wpr = P.wpr;
        const int words = m * wpr;
        uint32_t g0 = 0;
        bool ready = false;
        if (pend) {
          g0 = V.gen[my_e];
          ready = V.pf_gen[my_e] == g0;
        }
        for (int j = 0; j < LPW; j++) {
          if (!__shfl((int)(pend && ready), j)) continue;  // wave-uniform
          const int e = base + j * W + wave;
          const uint64_t *src = V.occ + (size_t)e * words;
          uint64_t *dst = S.occ + (size_t)e * words;
          for (int q = lane; q < words; q += 64) {
            const uint64_t v = src[q];
            dst[q] = v;
            mrow[q] = v;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (O.map_obs) bitmap_map_obs<64>(mrow, m, P.w, wpr, O.map_obs + (size_t)e * m * P.w, lane, mrow + words);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();  // mrow is rewritten by the next env
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (pend) {
          float px = 0.5f, py = 0.5f;
          if (ready) {
            const uint32_t sc = V.start[my_e];
            if (sc == ~0u) {
              atomicOr(O.err, APG_ERR_MAPGEN);
            } else {
              px = __fadd_rn((float)(sc & 255u), 0.5f);
              py = __fadd_rn((float)(sc >> 8), 0.5f);
            }
            *reinterpret_cast<Pcg64 *>(&S.rng[my_e]) = V.rng[my_e];
            *reinterpret_cast<Pcg64 *>(&S.it_rng[my_e]) = V.it[my_e];
            const uint64_t midx = V.idx[my_e];
            S.map_idx[my_e] = midx;
            if (O.map_idx) oat(O.map_idx, P.row, my_e, 1) = midx;
          } else {
            atomicOr(O.err, APG_ERR_PREFETCH);  // the host protocol guarantees a record: never in practice
          }
          S.pos[2 * my_e] = px;
          S.pos[2 * my_e + 1] = py;
          S.init_pos[2 * my_e] = px;
          S.init_pos[2 * my_e + 1] = py;
          S.elapsed[my_e] = 0;
          S.flags[my_e] = (uint8_t)((f0 & F_AUTORESET) | F_JUST_RESET | F_FIRST);
          // a consumed record moves the env to its next generation; a missing one (APG_ERR_PREFETCH, raised to the
          // caller) leaves the generation alone, so the next batch still selects this env and later records stay
          // in step with its resets
          if (ready) pf_store_gen(&V.gen[my_e], g0 + 1u);
        }
      } else if constexpr (GEN == GEN_POOL) {
        // Maps of the resident pool (any FloorMapDataset, APG_MAP_POOL).  The env's lane draws the DatasetIterator
        // index, integers(0, len(dataset)) (dataset_iterator.py:26-32), and the start-cell pick from the pool map's
        // free-cell count (lidar_localization2d.py:302-304); then each wave copies the pool rows of its pending envs
        // into their occupancy (lane = row, coalesced) and finds the pick-th free cell in row-major order on the way.
        // The f32 map obs (:299) is written from the copied rows by phase 0 like every unfused reset.
        Pcg64 rng, it;
        uint64_t midx = 0;
        long long pick = -1;
        if (pend) {
          rng = *reinterpret_cast<const Pcg64 *>(&S.rng[my_e]);
          it = *reinterpret_cast<const Pcg64 *>(&S.it_rng[my_e]);
          midx = (uint64_t)integers(it, 0, g.stream_len ? g.stream_len : (int64_t)g.pool_len);
          const int nfree = S.pool_free[g.stream_len ? (uint64_t)my_e : midx];  // (streamed: slot = env)
          if (nfree > 0) pick = (long long)integers(rng, 0, nfree);
        }
        const int wpr = P.wpr;
        for (int j = 0; j < LPW; j++) {
          if (!__shfl((int)pend, j)) continue;  // wave-uniform
          const int el = j * W + wave, e = base + el;
          const uint64_t mj = ((uint64_t)(uint32_t)__shfl((int)(midx >> 32), j) << 32) | (uint32_t)__shfl((int)midx, j);
          const long long pj = ((long long)__shfl((int)((unsigned long long)pick >> 32), j) << 32) |
                               (uint32_t)__shfl((int)pick, j);
          const uint64_t *src = S.pool_occ + (g.stream_len ? (uint64_t)e : mj) * words;
          uint64_t *dst = S.occ + (size_t)e * words;
          if (lane == 0) s_start[el] = ~0u;
          int off = 0;
          for (int y0 = 0; y0 < P.h; y0 += 64) {
            const int y = y0 + lane;
            int fr = 0;
            if (y < P.h) {
              int occ = 0;
              for (int k = 0; k < wpr; k++) {
                const uint64_t v = src[(size_t)y * wpr + k];
                dst[(size_t)y * wpr + k] = v;
                occ += __popcll(v);
              }
              fr = P.w - occ;
            }
            const int incl = wave_inclusive_scan(fr, lane) + off;
            const int excl = incl - fr;
            if (y < P.h && pj >= excl && pj < incl) {  // the pick-th free cell is in this lane's row
              int k2 = (int)(pj - excl), x = -1;
              for (int k = 0; k < wpr && x < 0; k++) {
                const int lo = 64 * k;
                const uint64_t valid = P.w - lo >= 64 ? ~0ULL : ((1ULL << (P.w - lo)) - 1ULL);
                const uint64_t fm = ~src[(size_t)y * wpr + k] & valid;
                const int c = __popcll(fm);
                if (k2 < c) x = lo + select_bit(fm, k2);
                else k2 -= c;
              }
              s_start[el] = ((uint32_t)y << 16) | (uint32_t)x;
            }
            off = __shfl(incl, 63);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // s_start of the wave's envs
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (pend) {
          const uint32_t sc = s_start[my_el];
          float px = 0.5f, py = 0.5f;
          if (sc == ~0u) {
            atomicOr(O.err, APG_ERR_NO_FREE_CELL);  // integers(0, 0): numpy's ValueError
          } else {
            px = __fadd_rn((float)(sc & 0xFFFFu), 0.5f);
            py = __fadd_rn((float)(sc >> 16), 0.5f);
          }
          S.pos[2 * my_e] = px;
          S.pos[2 * my_e + 1] = py;
          S.init_pos[2 * my_e] = px;
          S.init_pos[2 * my_e + 1] = py;
          S.elapsed[my_e] = 0;
          S.flags[my_e] = (uint8_t)((f0 & F_AUTORESET) | F_JUST_RESET | F_FIRST);
          *reinterpret_cast<Pcg64 *>(&S.rng[my_e]) = rng;
          *reinterpret_cast<Pcg64 *>(&S.it_rng[my_e]) = it;
          S.map_idx[my_e] = midx;
          if (O.map_idx) oat(O.map_idx, P.row, my_e, 1) = midx;
        }
      } else if constexpr (GEN == GEN_ROOMS) {
        // R1: the env's streams, its next map index and the map's primitives, generated with the
        // working storage interleaved in LDS (a private-array generator would live in scratch memory)
        using L = RoomsLds<EPB>;
        char *s_raw = reinterpret_cast<char *>(s_dyn);
        uint32_t *s_prims = reinterpret_cast<uint32_t *>(s_raw + L::prim);
        uint64_t *s_mrow = reinterpret_cast<uint64_t *>(s_raw + L::mrow);
        Pcg64 rng, it;
        uint64_t midx = 0;
        if (pend) {
          rng = *reinterpret_cast<const Pcg64 *>(&S.rng[my_e]);
          it = *reinterpret_cast<const Pcg64 *>(&S.it_rng[my_e]);
          midx = next32(it);  // DatasetIterator: integers(0, len(dataset) = 2**32)
          Pcg64 map_rng = seed_pcg64(midx);  // FloorMapDatasetRooms.get_data_point: default_rng(idx)
          const RoomsWork wk{reinterpret_cast<uint64_t *>(s_raw + L::stk) + my_el,
                             reinterpret_cast<int16_t *>(s_raw + L::cap) + my_el,
                             reinterpret_cast<int16_t *>(s_raw + L::size) + my_el,
                             reinterpret_cast<int16_t *>(s_raw + L::cut) + my_el, s_prims + my_el, EPB, ROOMS_STACK,
                             16};  // ROOMS_PRIM_WORDS: 17 rooms (larger max_rooms: k_lidar_reset + unfused step)
          const int rc = rooms_primitives<false>(map_rng, g.h, g.max_rooms, g.door_width, bt, wk);
          if (rc != 0) atomicOr(O.err, APG_ERR_MAPGEN);
        }
        // R2 reads only the primitives its own wave wrote in R1 (wave w owns the envs j * W + w): a wave
        // barrier suffices, so waves that finish generating start their map stores while others still
        // generate (the 4 * H * W-byte f32 map obs of every reset env is this step's dominant traffic)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        STEP_MARK(10)  // (wave 0's view)
        STEP_MARK_W(0)
        // R2: each wave paints the maps of its own envs one after the other, lane = row: occupancy rows
        // out (coalesced), the f32 map obs from the wave's row copy in LDS, the free-cell count and the
        // start cell (place_start: the pick-th free cell in row-major order, drawn by the env's lane)
        uint64_t *mrow = s_mrow + (size_t)wave * MAX_MAP_ROWS * 2;
        const int m = P.h, wpr = P.wpr;
        for (int j = 0; j < LPW; j++) {
          if (!__shfl((int)pend, j)) continue;  // wave-uniform
          const int el = j * W + wave, e = base + el;
          const uint32_t *pr = s_prims + el;
          const uint32_t prv = lane < ROOMS_PRIM_WORDS ? pr[lane * EPB] : 0u;
          uint64_t *dst = S.occ + (size_t)e * words;
          int fr[2] = {0, 0};
          uint64_t rw[2][2] = {{0ULL, 0ULL}, {0ULL, 0ULL}};
#pragma unroll
          for (int rr = 0; rr < 2; rr++) {
            const int y = lane + 64 * rr;
            if (y < m) {
              int occ = 0;
              for (int k = 0; k < wpr; k++) {
#if APG_R2_LANES
                const uint64_t v = rooms_row_word_lanes(prv, m, y, k);
#else
                const uint64_t v = rooms_row_word(pr, EPB, m, y, k);
#endif
                rw[rr][k] = v;
                dst[y * wpr + k] = v;
                mrow[y * 2 + k] = v;
                occ += __popcll(v);
              }
              fr[rr] = P.w - occ;
            }
          }
          const int nfree = wave_sum(fr[0] + fr[1]);
          long long pick = -1;
          if (lane == j && nfree > 0) pick = (long long)integers(rng, 0, nfree);
          pick = __shfl(pick, j);
          int off = 0;
          if (lane == 0) s_start[el] = ~0u;
#pragma unroll
          for (int rr = 0; rr < 2; rr++) {
            const int incl = wave_inclusive_scan(fr[rr], lane) + off;
            const int excl = incl - fr[rr];
            if (pick >= excl && pick < incl) {  // the pick-th free cell is in this lane's row
              int k2 = (int)(pick - excl), x = -1;
              for (int k = 0; k < wpr && x < 0; k++) {
                const int lo = 64 * k;
                const uint64_t valid = P.w - lo >= 64 ? ~0ULL : ((1ULL << (P.w - lo)) - 1ULL);
                const uint64_t fm = ~rw[rr][k] & valid;
                const int c = __popcll(fm);
                if (k2 < c) x = lo + select_bit(fm, k2);
                else k2 -= c;
              }
              s_start[el] = ((uint32_t)(lane + 64 * rr) << 8) | (uint32_t)x;
            }
            off = __shfl(incl, 63);
          }
          if (O.map_obs && (P.w & 3) == 0) {  // bool map / 255 (lidar_localization2d.py:299), float4 stores
            const float wall = 1.0f / 255.0f;
            typedef float f4 __attribute__((ext_vector_type(4)));
            float *mo = O.map_obs + (size_t)e * m * P.w;
            const int q4 = P.w >> 2;
            for (int k4 = lane; k4 < m * q4; k4 += 64) {
              const int y = k4 / q4, x = (k4 - y * q4) * 4;
              const uint32_t bits = (uint32_t)(mrow[y * 2 + (x >> 6)] >> (x & 63));
              f4 v;
              v.x = (bits & 1u) ? wall : 0.0f;
              v.y = (bits & 2u) ? wall : 0.0f;
              v.z = (bits & 4u) ? wall : 0.0f;
              v.w = (bits & 8u) ? wall : 0.0f;
#if APG_MAPOBS_NT
              __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(mo) + k4);
#else
              reinterpret_cast<f4 *>(mo)[k4] = v;
#endif
            }
          } else if (O.map_obs) {
            float *mo = O.map_obs + (size_t)e * m * P.w;
            for (int k = lane; k < m * P.w; k += 64) {
              const int y = k / P.w, x = k - y * P.w;
              mo[k] = ((mrow[y * 2 + (x >> 6)] >> (x & 63)) & 1ULL) ? 1.0f / 255.0f : 0.0f;
            }
          }
        }
        STEP_MARK(11)
        STEP_MARK_W(1)
        // R3: the env's lane finishes its reset (lidar_localization2d.py:293-315 tail)
        if (pend) {
          const uint32_t sc = s_start[my_el];
          float px = 0.5f, py = 0.5f;
          if (sc == ~0u) {
            atomicOr(O.err, APG_ERR_MAPGEN);
          } else {
            px = __fadd_rn((float)(sc & 255u), 0.5f);
            py = __fadd_rn((float)(sc >> 8), 0.5f);
          }
          S.pos[2 * my_e] = px;
          S.pos[2 * my_e + 1] = py;
          S.init_pos[2 * my_e] = px;
          S.init_pos[2 * my_e + 1] = py;
          S.elapsed[my_e] = 0;
          S.flags[my_e] = (uint8_t)((f0 & F_AUTORESET) | F_JUST_RESET | F_FIRST);
          *reinterpret_cast<Pcg64 *>(&S.rng[my_e]) = rng;
          *reinterpret_cast<Pcg64 *>(&S.it_rng[my_e]) = it;
          S.map_idx[my_e] = midx;
          if (O.map_idx) oat(O.map_idx, P.row, my_e, 1) = midx;
        }
      } else {
        // static maps only draw a start cell
        if (pend) reset_one<GEN>(g, S, my_e, f0, false, 0, nullptr, O.map_idx, O.err, bt);
      }
      __syncthreads();
      STEP_MARK(12)
      if (own && (pf_f & F_AUTORESET)) {  // this env was reset above
        pf_f = S.flags[oe];
        pf_px = S.pos[2 * oe];
        pf_py = S.pos[2 * oe + 1];
        pf_ix = S.init_pos[2 * oe];
        pf_iy = S.init_pos[2 * oe + 1];
        pf_el = S.elapsed[oe];
      }
      if constexpr (!GR) load_windows();  // the reset envs' new maps and positions
    }
  }

  // ---------------- phase 0: window origins from the pre-move positions; which envs reset
  if (dir_thread) s_dirs[tid >> 1][tid & 1] = dir_v;
  constexpr bool kMapObsHere = !(FUSED && (GEN == GEN_ROOMS || GEN == GEN_PF));  // fused resets wrote it in phase R
  if (own) {
    s_x0[tid] = (int)floorf(pf_px) - 15;
    s_y0[tid] = (int)floorf(pf_py) - 15;
    if (kMapObsHere && (pf_f & F_JUST_RESET)) s_rlist[atomicAdd(&s_cnt[0], 1)] = (uint16_t)tid;
  }
  if constexpr (kMapObsHere) __syncthreads();
  // map obs of the envs that reset this step: bool map / 255 (lidar_localization2d.py:299), written by
  // the whole workgroup with float4 stores
  if (kMapObsHere && s_cnt[0] != 0 && O.map_obs && !P.is_static) {
    const float wall = 1.0f / 255.0f;
    const int cells = P.h * P.w, nr = s_cnt[0];
    for (int r = 0; r < nr; r++) {
      const int j = s_rlist[r];
      const uint64_t *rows = S.occ + (size_t)(base + j) * words;
      float *dst = O.map_obs + (size_t)(base + j) * cells;
      if ((P.w & 3) == 0) {  // 4 cells of one row per float4: one row-word load, non-temporal stores
        const int q = P.w >> 2;
        for (int k4 = tid; k4 < cells / 4; k4 += T) {
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
        for (int k = tid; k < cells; k += T) {
          const int y = k / P.w, x = k - y * P.w;
          dst[k] = ((rows[y * P.wpr + (x >> 6)] >> (x & 63)) & 1ULL) ? wall : 0.0f;
        }
      }
    }
  }
  {
    // while the rows are in flight: the SCAN_EMPTY value table, v(s) = clip(f32 sqrt(s) / range, -1, 1)
    if (P.beams <= MAX_STAGED_BEAMS) {
      const double inv_range = 1.0 / (double)P.range;
      for (int k = tid; k < EMPTY_TAB; k += T) {
        const float d = f32_sqrt(__uint_as_float(tab_base() + (uint32_t)k));
        s_tab[k] = fminf(fmaxf(f32_div_inv(d, inv_range), -1.0f), 1.0f);
      }
    }
#pragma unroll
    for (int k = 0; k < WIN_ITERS; k++) {
      const int r = tid + k * T;
      const int el = r / MAX_WIN_ROWS, row = r - el * MAX_WIN_ROWS;
      s_win[el * WIN_STRIDE + row] = wv[k];
    }
  }
  STEP_MARK(9)
  __syncthreads();
  STEP_MARK(1)
  STEP_STOP(1)

  // ---------------- phase 1: lane = env (the prefetched inputs).  1a: NaN checks, base reward, the move up
  // to the first wall (:318-344); slides (:345-364) need two more scans from the stopped position, which
  // are independent of each other: with APG_SLIDE_SPLIT the second runs on the next EPB threads (waves
  // that are idle in this phase) between two barriers.  1b: slide, clip, loss, TimeLimit, stats, obs.
  {
  const int e = oe, el = tid;
  uint32_t errbits = 0;
  bool was_reset = false, moved = false, slide = false;
  uint8_t f = pf_f;
  float pos0 = pf_px, pos1 = pf_py, ipx = pf_ix, ipy = pf_iy;
  const float prx = pf_prx, pry = pf_pry;
  float br = 0.0f, c0x = 0.0f, c1y = 0.0f;
  const float lpx = pf_px, lpy = pf_py;
  if (tid < EPB && own) {
    was_reset = f & F_JUST_RESET;
    if (!was_reset) {
      float ax = pf_ax, ay = pf_ay;
      if (isnan(ax) || isnan(ay)) errbits |= APG_ERR_NAN_ACTION;
      if (isnan(prx) || isnan(pry)) errbits |= APG_ERR_NAN_PREDICTION;
      if (!errbits) {  // else the reference raises ValueError before touching this env's state
        moved = true;
        br = __fsub_rn(0.1f, __fmul_rn(0.001f, __fadd_rn(__fmul_rn(ax, ax), __fmul_rn(ay, ay))));
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
          const float d = lidar_scan(rows_of(el, pos0, tx), pos0, pos1, tx, ty).dist;
          pos0 = __fadd_rn(pos0, __fmul_rn(dirx, d));
          pos1 = __fadd_rn(pos1, __fmul_rn(diry, d));
          const float rem = __fsub_rn(total, d);
          if (rem > 1e-5f) {  // slide along the wall (:345-364)
            const float rvx = __fmul_rn(dirx, rem), rvy = __fmul_rn(diry, rem);
            const bool kx = rvx > 1e-5f, ky = rvy > 1e-5f;
            if (kx || ky) {
              slide = true;
              c0x = kx ? rvx : rvy;  // eye(2) * kept
              c1y = ky ? rvy : rvx;  // > 1e-5: 0 marks "no slide" below
            }
          }
        }
      }
    }
  }
  float d0 = 0.0f, d1 = 0.0f;
  if (!GR && P.p4 && tid >= 2 * EPB) {
    // waves idle in phase 1 (beyond the env lanes and the second slide scans): phase 2a's 4-row OR table, each
    // thread sliding down half of an env's staged rows (one LDS read and one write per entry; lanes = envs, so
    // the row reads of a wave hit distinct banks)
    const int hi = min(P.whi, MAX_WIN_ROWS) - 3, mid = (P.wlo + hi + 1) / 2;
    for (int q = tid - 2 * EPB; q < 2 * EPB; q += T - 2 * EPB) {
      const int sl = q & (EPB - 1), r0 = q < EPB ? P.wlo : mid, r1 = q < EPB ? mid : hi;
      const uint32_t *w = s_win + sl * WIN_STRIDE;
      uint32_t *w4 = s_win4 + sl * WIN_STRIDE;
      if (r0 >= r1) continue;
      uint32_t a = w[r0], b = w[r0 + 1], c = w[r0 + 2];
      for (int r = r0; r < r1; r++) {
        const uint32_t d = w[r + 3];
        w4[r] = a | b | c | d;
        a = b;
        b = c;
        c = d;
      }
    }
  }
#if APG_SLIDE_SPLIT
  if (tid < EPB) {
    s_pos[tid][0] = pos0;
    s_pos[tid][1] = pos1;
    s_slide[tid] = slide ? c1y : 0.0f;
  }
  __syncthreads();
  if (tid >= EPB && tid < 2 * EPB) {  // the second slide candidate of env tid - EPB
    const int j = tid - EPB;
    const float cy = s_slide[j];
    if (cy > 0.0f) {
      const float q0 = s_pos[j][0], q1 = s_pos[j][1];
      s_slide[j] = lidar_scan(rows_of(j, q0, q0), q0, q1, __fadd_rn(q0, 0.0f), __fadd_rn(q1, cy)).dist;
    }
  }
  if (slide) {
    const float bx = __fadd_rn(pos0, c0x);
    d0 = lidar_scan(rows_of(el, pos0, bx), pos0, pos1, bx, __fadd_rn(pos1, 0.0f)).dist;
  }
  __syncthreads();
  if (slide) d1 = s_slide[tid];
#else
  if (slide) {
    const float bx = __fadd_rn(pos0, c0x);
    d0 = lidar_scan(rows_of(el, pos0, bx), pos0, pos1, bx, __fadd_rn(pos1, 0.0f)).dist;
    d1 = lidar_scan(rows_of(el, pos0, pos0), pos0, pos1, __fadd_rn(pos0, 0.0f), __fadd_rn(pos1, c1y)).dist;
  }
#endif
  if (tid < EPB) {
    if (own) {
      const float mapw = (float)P.w, maph = (float)P.h;
      if (was_reset || errbits) {  // NEXT_STEP autoreset (this env returned reset obs, reward 0) or NaN inputs
        oat(O.reward, P.row, e, 1) = 0.0;
        oat(O.terminated, P.row, e, 1) = 0;
        oat(O.truncated, P.row, e, 1) = 0;
        oat(O.base_reward, P.row, e, 1) = 0.0f;
        oat(O.target, P.row, e, 2, 0) = 0.0f;
        oat(O.target, P.row, e, 2, 1) = 0.0f;
        oat(O.loss, P.row, e, 1) = 0.0f;
        oat(O.info_mask, P.row, e, 1) = 0;
        if (P.log_stats) oat(O.stats_len, P.row, e, 1) = 0;
        if (P.sparse) oat(O.weight, P.row, e, 1) = 0.0;
        if (was_reset) f &= (uint8_t)~(F_JUST_RESET | F_AUTORESET);
      }
      if (moved) {
        if (slide) {
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
        if (f & F_FIRST) {  // initial_pos aliases pos until np.clip rebinds it (:305, :371)
          S.init_pos[2 * e] = pos0;
          S.init_pos[2 * e + 1] = pos1;
          ipx = pos0;
          ipy = pos1;
          f &= (uint8_t)~F_FIRST;
        }
        bool term = pos0 < 0.0f || pos1 < 0.0f || pos0 >= mapw || pos1 >= maph;
        pos0 = fminf(fmaxf(pos0, 0.0f), mapw);
        pos1 = fminf(fmaxf(pos1, 0.0f), maph);
        const float tgx = __fsub_rn(__fmul_rn(f32_div_inv(lpx, 1.0 / (double)mapw), 2.0f), 1.0f);
        const float tgy = __fsub_rn(__fmul_rn(f32_div_inv(lpy, 1.0 / (double)maph), 2.0f), 1.0f);
        const int el2 = pf_el + 1;
        pf_el = el2;
        S.elapsed[e] = el2;
        if (el2 >= P.step_limit) term = true;  // TimeLimit(issue_termination=True)
        const float ex = __fsub_rn(prx, tgx), ey = __fsub_rn(pry, tgy);
        const float mse = __fmul_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), 0.5f);  // exact / 2
        const float loss = __fadd_rn(__fmul_rn(mse, P.loss_scale), P.loss_offset);
        if (P.log_stats) {
          float *hist = S.stats_hist;
          hist[(size_t)(el2 - 1) * P.n + e] = norm_f32(ex, ey);  // |target - prediction|: the signs do not matter
          hist[(size_t)(P.step_limit + el2 - 1) * P.n + e] = mse;
          if (term && el2 <= PW_PTR_MAX_N) log_episode_stats(P, O, e, hist, el2);
          else oat(O.stats_len, P.row, e, 1) = term ? el2 : 0;  // > PW_PTR_MAX_N steps: k_episode_stats
        }
        oat(O.base_reward, P.row, e, 1) = br;
        oat(O.target, P.row, e, 2, 0) = tgx;
        oat(O.target, P.row, e, 2, 1) = tgy;
        oat(O.loss, P.row, e, 1) = loss;
        if (P.sparse) {  // SparsifyWrapper: base_reward - loss * (1.0 if terminated else 0.0), in f32
          oat(O.weight, P.row, e, 1) = term ? 1.0 : 0.0;
          oat(O.reward, P.row, e, 1) = (double)__fsub_rn(br, __fmul_rn(loss, term ? 1.0f : 0.0f));
        } else {
          oat(O.reward, P.row, e, 1) = (double)__fsub_rn(br, loss);
        }
        oat(O.terminated, P.row, e, 1) = term;
        oat(O.truncated, P.row, e, 1) = 0;
        oat(O.info_mask, P.row, e, 1) = 1;
        if (term) f |= F_AUTORESET;
        S.pos[2 * e] = pos0;
        S.pos[2 * e + 1] = pos1;
      }
      S.flags[e] = f;
      if (O.reset_mask) oat(O.reset_mask, P.row, e, 1) = was_reset;
      // odometry (:263-270) and TimeLimit time_step (time_limit.py:113-116)
      const float ox = __fsub_rn(pos0, ipx), oy = __fsub_rn(pos1, ipy);
      oat(O.odometry, P.row, e, 2, 0) =
          __fsub_rn(__fmul_rn(f32_div_inv(__fadd_rn(ox, mapw), 1.0 / (double)__fadd_rn(mapw, mapw)), 2.0f), 1.0f);
      oat(O.odometry, P.row, e, 2, 1) =
          __fsub_rn(__fmul_rn(f32_div_inv(__fadd_rn(oy, maph), 1.0 / (double)__fadd_rn(maph, maph)), 2.0f), 1.0f);
      oat(O.time_step, P.row, e, 1) = (float)(2.0 * (double)pf_el / (double)P.step_limit - 1.0);
      s_pos[el][0] = pos0;
      s_pos[el][1] = pos1;
    }
    if (errbits) atomicOr(O.err, errbits);  // rare: NaN inputs only
  }
  }
  __syncthreads();
  STEP_MARK(2)
  STEP_STOP(2)

  // ---------------- phase 2a: lane = env, wave = beam index (all 64 lanes of a wave cast the same
  // beam direction).  Beams whose bounding box holds no occupied cell are SCAN_EMPTY and finish
  // here; the others are queued (env, beam) in LDS, grouped by beam, for 2b.  Up to MAX_STAGED_BEAMS
  // beams (every configuration of the reference) the lidar rows are staged in LDS; the instance for more
  // beams walks in place and stores straight to HBM.
  const int el = tid & (EPB - 1), e = base + el;
  const float px = s_pos[el][0], py = s_pos[el][1];
  const double inv_range = 1.0 / (double)P.range;
  auto beam_value = [&](float d) { return fminf(fmaxf(f32_div_inv(d, inv_range), -1.0f), 1.0f); };
  if (P.beams > MAX_STAGED_BEAMS) {
    for (int beam = tid / EPB; beam < P.beams; beam += T / EPB) {
      if (e < P.n) {
        const float qx = __fadd_rn(px, S.beam_dirs[2 * beam]), qy = __fadd_rn(py, S.beam_dirs[2 * beam + 1]);
        oat(O.lidar, P.row, e, P.beams, beam) = beam_value(lidar_scan(rows_of(el, px, qx), px, py, qx, qy).dist);
      }
    }
    return;
  }
  // the wave's walk flags first (bit it of wbits: iteration it's beam), then ONE queue reservation per wave
  // (an LDS atomic per beam iteration serialized the waves' pre-tests), then the entries, grouped by beam
  uint32_t wbits = 0;
  int wtot = 0;  // wave-uniform
  if (!P.pretest) {  // every (env, beam) walks: queue entry i is (beam i / EPB, env slot i % EPB), implicitly
    if (tid == 0) s_cnt[1] = EPB * P.beams;
  } else
  for (int beam = tid / EPB, it = 0; beam < P.beams; beam += T / EPB, it++) {
    bool walk = false;
    if (e < P.n) {
      const float dy = s_dirs[beam][1];
      const float qx = __fadd_rn(px, s_dirs[beam][0]), qy = __fadd_rn(py, dy);
      // the box spans <= floor(|qy - py|) + 2 <= floor(|dy| + 1e-4) + 2 rows (positions < 1024): a bound
      // uniform per wave
      const int hmax = __builtin_amdgcn_readfirstlane((int)floorf(fabsf(dy) + 1e-4f) + 2);
      if (!GR && P.p4) {
        // the box's rows [j0, j1] (h = j1 - j0 + 1 <= hmax) from the 4-row table: two reads when h >= 4 (rows
        // j0..j0+3 and j1-3..j1), the rows themselves below; a lane with h < 4 in a wave with hmax >= 4 reads
        // directly too (branch-free selects)
        const int i0 = (int)ceilf(fminf(px, qx)) - 1, i1 = (int)floorf(fmaxf(px, qx));
        const int j0 = (int)ceilf(fminf(py, qy)) - 1, j1 = (int)floorf(fmaxf(py, qy));
        const int h = j1 - j0 + 1, o = el * WIN_STRIDE + (j0 - s_y0[el]);
        uint32_t acc;
        if (hmax >= 4) {  // (wave-uniform)
          const bool t4 = h >= 4;
          acc = (t4 ? s_win4[o] : s_win[o]) | (t4 ? s_win4[o + h - 4] : (h > 1 ? s_win[o + 1] : 0u)) |
                (!t4 && h > 2 ? s_win[o + 2] : 0u);
          // the middle rows of boxes taller than 8 (lidar_range > 6): rows 4.. in 4-row steps, the last group
          // overlapping the tail read above
          for (int t = 4; t < h - 4; t += 4) acc |= s_win4[o + t];
        } else {
          acc = s_win[o] | (h > 1 ? s_win[o + 1] : 0u) | (h > 2 ? s_win[o + 2] : 0u);
        }
        const uint32_t mask = ((1u << (i1 - i0 + 1)) - 1u) << (i0 - s_x0[el]);
        walk = (acc & mask) != 0u;
      } else {
        walk = scan_may_hit(rows_of(el, px, qx), px, py, qx, qy, hmax);
      }
      if (!walk) {  // SCAN_EMPTY: |q - p| (f32 norm), its value from the table
        const float ex = __fsub_rn(qx, px), ey = __fsub_rn(qy, py);
        const float s2 = __fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
        const uint32_t k = __float_as_uint(s2) - tab_base();
        s_lid[el * LS + beam] = k < (uint32_t)EMPTY_TAB ? s_tab[k] : beam_value(f32_sqrt(s2));
      }
    }
    wbits |= walk ? 1u << it : 0u;
    wtot += __popcll(__ballot(walk));
  }
  {
    int qbase = 0;
    if (lane == 0 && wtot) qbase = atomicAdd(&s_cnt[1], wtot);
    qbase = __shfl(qbase, 0);
    for (int beam = tid / EPB, it = 0; beam < P.beams && wtot; beam += T / EPB, it++) {
      const bool walk = (wbits >> it) & 1u;
      const unsigned long long m = __ballot(walk);
      if (walk) s_queue[qbase + __popcll(m & ((1ULL << lane) - 1ULL))] = (uint16_t)((beam << 8) | el);
      qbase += __popcll(m);
    }
  }
  __syncthreads();
  STEP_MARK(3)
  STEP_STOP(3)
  // ---------------- phase 2b: the queued scans, densely over the workgroup's waves; each wave takes
  // the next 64 entries from a shared cursor, so waves with short walks take more of them
  const int nq = s_cnt[1];
  for (;;) {
    int start = 0;
    if (lane == 0) start = atomicAdd(&s_cnt[2], 64);
    start = __shfl(start, 0);
    if (start >= nq) break;
    const int i = start + lane;
    const int ent = P.pretest ? (i < nq ? (int)s_queue[i] : 0) : (i / EPB) << 8 | (i & (EPB - 1));
    const int qe = ent & 255, beam = ent >> 8;
    if (i < nq && (P.pretest || base + qe < P.n)) {
      const float qpx = s_pos[qe][0], qpy = s_pos[qe][1];
      const float qx = __fadd_rn(qpx, s_dirs[beam][0]), qy = __fadd_rn(qpy, s_dirs[beam][1]);
      s_lid[qe * LS + beam] = beam_value(lidar_scan_walk(rows_of(qe, qpx, qx), qpx, qpy, qx, qy).dist);
    }
  }
  __syncthreads();
  STEP_MARK(4)
  STEP_STOP(4)
  const int nenv = P.n - base < EPB ? P.n - base : EPB;
  if (!ROWP && P.lidar16) {  // dense rows 16-byte aligned: four beams per 16-byte store
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int B4 = P.beams >> 2, dl = T / B4, db = T - dl * B4;
    int l = tid / B4, b4 = tid - l * B4;
    for (int i = tid; i < nenv * B4; i += T) {
      const float *src = s_lid + l * LS + 4 * b4;
      __builtin_nontemporal_store(f4{src[0], src[1], src[2], src[3]},
                                  reinterpret_cast<f4 *>(O.lidar + (size_t)(base + l) * P.beams + 4 * b4));
      l += dl;
      b4 += db;
      if (b4 >= B4) {
        b4 -= B4;
        l++;
      }
    }
  } else {
    const int B = P.beams, dl = T / B, db = T - dl * B;  // (env, beam) of element i advanced without divisions
    int l = tid / B, beam = tid - l * B;
    for (int i = tid; i < nenv * B; i += T) {
      oat(O.lidar, P.row, base + l, B, beam) = s_lid[l * LS + beam];
      l += dl;
      beam += db;
      if (beam >= B) {
        beam -= B;
        l++;
      }
    }
  }
#ifdef APG_STEP_PROFILE
  __syncthreads();
  STEP_MARK(5)
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    g_step_prof[blockIdx.x][6] = s_cnt[1];
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
  const bool was_reset = oat(O.reset_mask, P.row, e, 1) != 0;
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
      const float d = norm_f32(__fsub_rn(ax, oat(O.target, P.row, e, 2, 0)), __fsub_rn(ay, oat(O.target, P.row, e, 2, 1)));
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
                            double *out) {
  const BinomTable &bt = c_binom;
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

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: the bytes opted in are remembered per
// (kernel, device), so an env on a second GPU of the process opts its kernels in too (the call costs host
// time, so it is not repeated on every launch).
int opt_in_lds(const void *kern, size_t bytes) {
  if (bytes <= 64 * 1024) return APG_OK;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(APG_E_LAUNCH, "hipGetDevice failed");
  static std::mutex mu;
  static std::map<std::pair<const void *, int>, size_t> opted;
  std::lock_guard<std::mutex> lock(mu);
  size_t &have = opted[std::make_pair(kern, dev)];
  if (have >= bytes) return APG_OK;
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  have = bytes;
  return APG_OK;
}

// Dynamic LDS of a map-generation launch: rooms bitmaps [lanes][h * wpr] (opted in above 64 KiB).
template <class K>
int gen_lds(K kernel, int gen, const Geo &g, int lanes, size_t &dyn) {
  dyn = gen == GEN_ROOMS ? (size_t)lanes * g.h * g.wpr * sizeof(uint64_t) : 0;
  return opt_in_lds((const void *)kernel, dyn);
}

// lanes of a rooms-generation wave: gen_lanes(n), fewer when their LDS bitmaps would pass 160 KiB (large maps)
int rooms_lanes(const Geo &g, int n) {
  int lanes = gen_lanes(n);
  const size_t per = (size_t)g.h * g.wpr * sizeof(uint64_t);
  while (lanes > 1 && lanes * per > 160 * 1024) lanes /= 2;
  return lanes;
}

template <int GEN, int MR>
int launch_reset_mr(const Geo &g, const apg_lidar_state *st, uint64_t seed, int use_seed, int all,
                    const apg_lidar_outputs *out, hipStream_t s) {
  const int lanes = GEN == GEN_ROOMS ? rooms_lanes(g, g.n) : 64;
  size_t dyn;
  if (int rc = gen_lds(k_lidar_reset<GEN, MR>, GEN, g, lanes, dyn)) return rc;
  hipLaunchKernelGGL((k_lidar_reset<GEN, MR>), dim3(grid_for(g.n, lanes)), dim3(64), dyn, s, g, *st, seed, use_seed,
                     all, out->map_idx, out->err, lanes);
  return check_launch("k_lidar_reset");
}

// the generator's private arrays hold 17 rooms (every registered env), ROOMS_MAX for larger max_rooms
template <int GEN>
int launch_reset_gen(const Geo &g, const apg_lidar_state *st, uint64_t seed, int use_seed, int all,
                     const apg_lidar_outputs *out, hipStream_t s) {
  if (GEN == GEN_ROOMS && g.max_rooms > 17) return launch_reset_mr<GEN, ROOMS_MAX>(g, st, seed, use_seed, all, out, s);
  return launch_reset_mr<GEN, 17>(g, st, seed, use_seed, all, out, s);
}

// k_maze over n mazes (MZ_MAPS: occ / idx; MZ_RESET: the state's envs, all or the pending autoresets).
// Dynamic LDS: the lanes' DFS state, at least one paint bitmap.
// Lanes (mazes) per one-wave k_maze / k_pf_dfs workgroup for n mazes; APG_MAZE_LANES overrides (tuning A/B only:
// the mazes do not depend on it)
int maze_lanes(int n) {
  int lanes = gen_lanes(n);
  static int forced = -1;
  if (forced < 0) {
    const char *e = getenv("APG_MAZE_LANES");
    forced = e ? atoi(e) : 0;
  }
  if (forced > 0 && forced <= 64) lanes = forced;
  return lanes;
}

// Stream groups per maze: APG_MAZE_STREAM_GROUPS (tests: fewer, so the DFS steps the LCG past them; the mazes do not
// depend on it) is clamped to [MZ_ITEM_GROUPS, maze_stream_groups], a multiple of MZ_ITEM_GROUPS
int maze_ng(const Geo &g) {
  static int forced_ng = -1;
  if (forced_ng < 0) {
    const char *e = getenv("APG_MAZE_STREAM_GROUPS");
    forced_ng = e ? atoi(e) : 0;
  }
  int ng = maze_stream_groups(g.h, g.w);
  if (forced_ng > 0) ng = std::max(MZ_ITEM_GROUPS, std::min(ng, forced_ng / MZ_ITEM_GROUPS * MZ_ITEM_GROUPS));
  return ng;
}

int launch_maze(const Geo &g, const apg_lidar_state &st, const uint64_t *idx, int n, uint64_t *occ, uint8_t *scratch,
                int mode, uint64_t seed, int use_seed, int all, uint64_t *out_map_idx, float *map_obs, uint32_t *err,
                hipStream_t s, const PfView *pv = nullptr) {
  if (!scratch) return fail(APG_E_INVALID, "maze maps need the maze scratch buffer (stack)");
  const MazeGeom m = maze_geom(g.h, g.w);
  const size_t paint_lds = ((size_t)g.h * g.wpr + bitmap_lin_words(g.h, g.w)) * sizeof(uint64_t);
  if (maze_big(g.h, g.w)) {  // maps past 255: one thread per maze, then the prepainted finish
    hipLaunchKernelGGL(k_maze_big, dim3(grid_for(n, 64)), dim3(64), 0, s, g, st, idx, n, occ, scratch, mode, seed,
                       use_seed, all);
    if (int rc = check_launch("k_maze_big")) return rc;
    if (mode != MZ_RESET) return APG_OK;
    hipLaunchKernelGGL(k_maze_paint, dim3(grid_for(n, MP_ENVS)), dim3(MP_THREADS), paint_lds, s, g, st, idx, n, occ,
                       scratch, mode, seed, use_seed, all, 0, out_map_idx, map_obs, err, pv ? *pv : PfView{}, 1);
    return check_launch("k_maze_paint");
  }
  const int lanes = maze_lanes(n);
  const size_t dyn = maze_wg_lds_bytes(g.h, g.w);  // laid out for 64 lanes whatever `lanes` is
  const bool onew = m.ncx <= 63;
  const void *kern = onew ? (const void *)k_maze<true> : (const void *)k_maze<false>;
  if (int rc = opt_in_lds(kern, dyn)) return rc;
  const int ng = maze_ng(g);
  if (ng / MZ_ITEM_GROUPS > MZ_MAX_ITEMS) return fail(APG_E_INVALID, "maze stream too long");
  hipLaunchKernelGGL(k_maze_stream, dim3(grid_for(n, MZS_MAZES)), dim3(MZS_THREADS), 0, s, g, st, idx, n, scratch, mode,
                     seed, use_seed, all, ng);
  if (int rc = check_launch("k_maze_stream")) return rc;
  if (onew)
    hipLaunchKernelGGL(k_maze<true>, dim3(grid_for(n, lanes)), dim3(64), dyn, s, g, st, idx, n, scratch, mode, seed,
                       use_seed, all, err, lanes, ng);
  else
    hipLaunchKernelGGL(k_maze<false>, dim3(grid_for(n, lanes)), dim3(64), dyn, s, g, st, idx, n, scratch, mode, seed,
                       use_seed, all, err, lanes, ng);
  if (int rc = check_launch("k_maze")) return rc;
  hipLaunchKernelGGL(k_maze_paint, dim3(grid_for(n, MP_ENVS)), dim3(MP_THREADS), paint_lds, s, g, st, idx, n, occ,
                     scratch, mode, seed, use_seed, all, ng, out_map_idx, map_obs, err, pv ? *pv : PfView{}, 0);
  return check_launch("k_maze_paint");
}

int launch_reset(const Geo &g, const apg_lidar_state *st, uint64_t seed, int use_seed, int all,
                 const apg_lidar_outputs *out, hipStream_t s) {
  if (g.is_static) return launch_reset_gen<GEN_NONE>(g, st, seed, use_seed, all, out, s);
  if (g.kind == APG_MAP_POOL) return launch_reset_gen<GEN_POOL>(g, st, seed, use_seed, all, out, s);
  if (g.kind == APG_MAP_MAZE)
    return launch_maze(g, *st, nullptr, g.n, nullptr, reinterpret_cast<uint8_t *>(st->stack), MZ_RESET, seed, use_seed,
                       all, out->map_idx, out->map_obs, out->err, s);
  return launch_reset_gen<GEN_ROOMS>(g, st, seed, use_seed, all, out, s);
}

int launch_map_generate_any(const Geo &g, const uint64_t *idx, int n, uint64_t *occ, uint16_t *stack,
                            uint32_t *err, hipStream_t s) {
  if (g.kind == APG_MAP_MAZE) {
    apg_lidar_state none;
    memset(&none, 0, sizeof(none));
    return launch_maze(g, none, idx, n, occ, reinterpret_cast<uint8_t *>(stack), MZ_MAPS, 0, 0, 1, nullptr, nullptr, err,
                       s);
  }
  const int lanes = rooms_lanes(g, n);
  size_t dyn;
  const bool big = g.max_rooms > 17;
  const void *kern = big ? (const void *)k_map_generate_rooms<ROOMS_MAX> : (const void *)k_map_generate_rooms<17>;
  if (int rc = gen_lds(kern, GEN_ROOMS, g, lanes, dyn)) return rc;
  if (big)
    hipLaunchKernelGGL(k_map_generate_rooms<ROOMS_MAX>, dim3(grid_for(n, lanes)), dim3(64), dyn, s, g, idx, n, occ, err,
                       lanes);
  else
    hipLaunchKernelGGL(k_map_generate_rooms<17>, dim3(grid_for(n, lanes)), dim3(64), dyn, s, g, idx, n, occ, err,
                       lanes);
  return check_launch("k_map_generate");
}

// Dynamic LDS of a k_lidar_step instance: windows + staged lidar rows + walk queue; fused rooms resets
// use the same bytes first for the primitives and each wave's map rows.
size_t step_lds_bytes(int epb, int beams, bool p4 = false) {
  size_t b = ((size_t)epb * WIN_STRIDE + 8) * sizeof(uint32_t);  // + RowsWindow::or_rows's over-read
  if (beams <= MAX_STAGED_BEAMS)
    b += (size_t)epb * (beams + 1) * sizeof(float) + (size_t)epb * beams * sizeof(uint16_t) + EMPTY_TAB * sizeof(float);
  if (p4 && beams <= MAX_STAGED_BEAMS) b += (size_t)epb * WIN_STRIDE * sizeof(uint32_t);  // s_win4
  return b;
}
constexpr size_t STEP_LDS_P4_MAX = 144 * 1024;  // the 4-row table only while the dynamic LDS stays below this

bool big_rooms(const apg_lidar_config *c) {
  return c->map_kind == APG_MAP_ROOMS && !c->is_static && (c->max_rooms > 17 || c->height > MAX_MAP_ROWS);
}

int step_gen(const Geo &g) {
  if (g.is_static) return GEN_NONE;
  if (g.kind == APG_MAP_POOL) return GEN_POOL;
  return GEN_ROOMS;  // mazes: GEN_PF (prefetched), or k_maze (autoresets) + the unfused step kernel
}

// Mazes whose next maps can be prefetched and installed by the fused step kernel: rows <= MAX_MAP_ROWS (one wave's
// LDS row copy, k_pf_paint's one row per thread), two row words, the staged-window step instance.
bool pf_supported(const apg_lidar_config *c) {
  return c->map_kind == APG_MAP_MAZE && !c->is_static && c->height <= MAX_MAP_ROWS && c->width <= 128 &&
         (int)ceilf(c->lidar_range) <= MAX_WIN_RANGE;
}

int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// Envs per step workgroup: 256 (1024 threads, one workgroup per CU: the CU's walks are balanced over
// its 16 waves) when that still gives every CU a workgroup, else 64 (256 threads).  APG_STEP_EPB=64|256
// overrides (tuning).
int step_epb(int n) {
  static int forced = -1;
  if (forced < 0) {
    const char *s = getenv("APG_STEP_EPB");
    forced = s ? atoi(s) : 0;
  }
  if (forced == 64 || forced == 256) return forced;  // (128: measured slower in r02, no longer instantiated)
  return (int64_t)n >= (int64_t)256 * cu_count() ? 256 : 64;
}

template <int GEN, bool FUSED, int EPB, bool GR = false>
int launch_step_t(const StepParams &P_in, const Geo &g, const apg_lidar_state *st, const float *act, const float *pred,
                  const apg_lidar_outputs *out, hipStream_t s, const PfView &V) {
  StepParams P = P_in;
  static const int p4_knob = getenv("APG_STEP_P4") ? atoi(getenv("APG_STEP_P4")) : 1;  // (A/B knob)
  P.p4 = !GR && P.pretest && p4_knob && P.beams <= MAX_STAGED_BEAMS &&
         step_lds_bytes(EPB, P.beams, true) <= STEP_LDS_P4_MAX;
  size_t lds = step_lds_bytes(EPB, P.beams, P.p4 != 0);
  if (FUSED && GEN == GEN_ROOMS && RoomsLds<EPB>::bytes > lds) lds = RoomsLds<EPB>::bytes;
  if (FUSED && GEN == GEN_PF) lds = std::max(lds, (size_t)(4 * EPB / 64) * PF_WAVE_WORDS * sizeof(uint64_t));
  auto kern = P.row ? k_lidar_step<GEN, FUSED, EPB, GR, true> : k_lidar_step<GEN, FUSED, EPB, GR, false>;
  if (int rc = opt_in_lds((const void *)kern, lds)) return rc;
  hipLaunchKernelGGL(kern, dim3(grid_for(P.n, EPB)), dim3(4 * EPB), lds, s, P, g, *st, act, pred, *out, V);
  return check_launch("k_lidar_step");
}

// pf: the prefetch view (its host_slot set) when the autoresets install prefetched mazes (GEN_PF), else NULL
template <int EPB>
int launch_step_epb(const StepParams &P, const Geo &g, const apg_lidar_state *st, const float *act, const float *pred,
                    const apg_lidar_outputs *out, hipStream_t s, bool fused, const PfView *pf) {
  PfView V{};
  if (pf) V = *pf;
  if (P.R > MAX_WIN_RANGE) {  // scans longer than the staged window covers: rows from global memory (EPB 64)
    if (!fused) return launch_step_t<GEN_NONE, false, 64, true>(P, g, st, act, pred, out, s, V);
    switch (step_gen(g)) {
      case GEN_ROOMS: return launch_step_t<GEN_ROOMS, true, 64, true>(P, g, st, act, pred, out, s, V);
      case GEN_POOL: return launch_step_t<GEN_POOL, true, 64, true>(P, g, st, act, pred, out, s, V);
      default: return launch_step_t<GEN_NONE, true, 64, true>(P, g, st, act, pred, out, s, V);
    }
  }
  if (!fused) return launch_step_t<GEN_NONE, false, EPB>(P, g, st, act, pred, out, s, V);
  if (pf) return launch_step_t<GEN_PF, true, EPB>(P, g, st, act, pred, out, s, V);
  switch (step_gen(g)) {
    case GEN_ROOMS: return launch_step_t<GEN_ROOMS, true, EPB>(P, g, st, act, pred, out, s, V);
    case GEN_POOL: return launch_step_t<GEN_POOL, true, EPB>(P, g, st, act, pred, out, s, V);
    default: return launch_step_t<GEN_NONE, true, EPB>(P, g, st, act, pred, out, s, V);
  }
}

// ActiveRegressionLogWrapper's episode-end stats of the episodes longer than PW_PTR_MAX_N steps that ended
// this step (the step kernel wrote their stats_len): one thread per env, after the step kernel.
__global__ __launch_bounds__(256) void k_episode_stats(StepParams P, const float *hist, apg_lidar_outputs O) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= P.n) return;
  const int len = oat(O.stats_len, P.row, e, 1);
  if (len > PW_PTR_MAX_N) log_episode_stats<true>(P, O, e, hist, len);
}

int launch_step_kernel(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *act,
                       const float *pred, const apg_lidar_outputs *out, hipStream_t s, bool fused,
                       const PfView *pf = nullptr) {
  StepParams P;
  P.n = cfg->num_envs;
  P.h = cfg->height;
  P.w = cfg->width;
  P.wpr = (cfg->width + 63) / 64;
  P.beams = cfg->beams;
  P.step_limit = cfg->step_limit;
  P.log_stats = cfg->log_stats ? 1 : 0;
  P.sparse = cfg->sparse ? 1 : 0;
  P.row = cfg->out_row_bytes;
  P.is_static = cfg->is_static;
  P.R = (int)ceilf(cfg->lidar_range);
  P.wrows = MAX_WIN_ROWS;
  // window rows a step can read (see load_windows): map rows [floor(p0) - R - 5, floor(p0) + R + 5] are the cells
  // of its scans, plus two rows for the walk's one-crossing-ahead row reads past the segment's end
  P.wlo = std::max(0, 15 - (P.R + 5) - 2);
  P.whi = std::min(MAX_WIN_ROWS, 15 + (P.R + 5) + 2 + 1);
  static int forced_pt = -2;  // APG_STEP_PRETEST=0|1 (tuning A/B only: the outputs do not depend on it)
  if (forced_pt == -2) {
    const char *e = getenv("APG_STEP_PRETEST");
    forced_pt = e ? atoi(e) : -1;
  }
  P.pretest = forced_pt >= 0 ? forced_pt : (cfg->map_kind == APG_MAP_MAZE ? 0 : 1);
  P.lidar16 = (P.beams & 3) == 0 && (reinterpret_cast<uintptr_t>(out->lidar) & 15) == 0;
  P.range = cfg->lidar_range;
  P.loss_scale = cfg->loss_scale;
  P.loss_offset = cfg->loss_offset;
  const Geo g = make_geo(cfg);
  int rc;
  switch (step_epb(P.n)) {
    case 256: rc = launch_step_epb<256>(P, g, st, act, pred, out, s, fused, pf); break;
    default: rc = launch_step_epb<64>(P, g, st, act, pred, out, s, fused, pf); break;
  }
  if (rc || !P.log_stats || P.step_limit <= PW_PTR_MAX_N) return rc;
  hipLaunchKernelGGL(k_episode_stats, dim3(grid_for(P.n, 256)), dim3(256), 0, s, P, st->stats_hist, *out);
  return check_launch("k_episode_stats");
}

// One prefetch batch on the prefetcher's side stream (k_pf_select .. k_pf_paint), after `after` (an event of the
// env's stream): the next mazes of every env whose record is stale by then.
// Streamed maps (apgym_capi.h, apg_lidar_peek_map_index): the dataset index the NEXT reset of each selected env
// will draw, integers(0, len) of a copy of its DatasetIterator stream (dataset_iterator.py:26-32), or (use_seed) of
// the stream reset(seed) gives it (the _np_random setter, lidar_localization2d.py:547-557).  Nothing is advanced.
// out_env NULL: out_idx[e] for every selected env; else the selected envs compacted (any order) with their count.
__global__ __launch_bounds__(256) void k_peek_map_index(int n, const apg_pcg64 *it_state, int64_t len, uint64_t seed,
                                                        int use_seed, const uint8_t *mask, int mask_stride,
                                                        int64_t *out_idx, int32_t *out_env, int32_t *count) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const bool sel = e < n && (!mask || mask[(size_t)e * mask_stride]);
  int64_t idx = 0;
  if (sel) {
    Pcg64 it;
    if (use_seed) {
      Pcg64 r = seed_pcg64(seed + (uint64_t)e);
      it = seed_pcg64(bounded_u64(r, 0x100000000ULL));  // integers(0, 2**32, endpoint=True)
    } else {
      it = *reinterpret_cast<const Pcg64 *>(&it_state[e]);
    }
    idx = integers(it, 0, len);
  }
  if (!out_env) {
    if (sel) out_idx[e] = idx;
    return;
  }
  const unsigned long long m = __ballot(sel);
  if (m == 0ULL) return;
  const int lane = threadIdx.x & 63, first = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == first) base = atomicAdd(count, __popcll(m));
  base = __shfl(base, first);
  if (sel) {
    const int k = base + __popcll(m & ((1ULL << lane) - 1ULL));
    out_env[k] = e;
    out_idx[k] = idx;
  }
}

int pf_batch_kernels(const apg_lidar_config *cfg, const apg_lidar_state *st, const apg_lidar_outputs *out,
                     hipStream_t side) {
  const Geo g = make_geo(cfg);
  const int n = g.n;
  PfView V = pf_view(st->prefetch, n, g.h, g.wpr);
  uint8_t *scratch = reinterpret_cast<uint8_t *>(st->stack);
  const MazeGeom m = maze_geom(g.h, g.w);
  const int ng = maze_ng(g), lanes = maze_lanes(n);
  if (!scratch) return fail(APG_E_INVALID, "maze prefetch needs the maze scratch buffer (stack)");
  if (ng / MZ_ITEM_GROUPS > MZ_MAX_ITEMS) return fail(APG_E_INVALID, "maze stream too long");
  const size_t dyn = maze_wg_lds_bytes(g.h, g.w);
  const bool onew = m.ncx <= 63;
  const void *kern = onew ? (const void *)k_pf_dfs<true> : (const void *)k_pf_dfs<false>;
  if (int rc = opt_in_lds(kern, dyn)) return rc;
  if (hipMemsetAsync(&V.ctl[0], 0, sizeof(unsigned long long), side) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipMemsetAsync (prefetch count)");
  hipLaunchKernelGGL(k_pf_select, dim3(grid_for(n, 256)), dim3(256), 0, side, n, V);
  if (int rc = check_launch("k_pf_select")) return rc;
  hipLaunchKernelGGL(k_pf_stream, dim3(grid_for(n, MZS_MAZES)), dim3(MZS_THREADS), 0, side, g, V, scratch, ng);
  if (int rc = check_launch("k_pf_stream")) return rc;
  if (onew)
    hipLaunchKernelGGL(k_pf_dfs<true>, dim3(grid_for(n, lanes)), dim3(64), dyn, side, g, V, scratch, out->err, lanes, ng);
  else
    hipLaunchKernelGGL(k_pf_dfs<false>, dim3(grid_for(n, lanes)), dim3(64), dyn, side, g, V, scratch, out->err, lanes,
                       ng);
  if (int rc = check_launch("k_pf_dfs")) return rc;
  hipLaunchKernelGGL(k_pf_paint, dim3(grid_for(n, MP_ENVS)), dim3(MP_THREADS), (size_t)g.h * g.wpr * sizeof(uint64_t),
                     side, g, V, scratch, ng, out->err);
  return check_launch("k_pf_paint");
}

}  // namespace

// The host side of the map prefetch (apgym_capi.h).  Steps are numbered from the last reset (step 0: every env
// reset); step c's kernel writes its reset count to host_ring[c % R] and c's completion event is main_ev[c % R].
struct apg_lidar_prefetcher {
  struct Batch {
    int64_t rmin, s;  // covers the resets of steps rmin .. s (rmin: the first of them)
    hipEvent_t ev;    // recorded on the side stream after the batch
  };
  int device = -1;
  int n = 0, h = 0, w = 0, L = 0, R = 0;
  hipStream_t side = nullptr;
  uint32_t *host_ring = nullptr, *dev_ring = nullptr;
  std::vector<hipEvent_t> main_ev;
  std::deque<Batch> batches;
  std::vector<hipEvent_t> spare;
  int64_t c = 0;            // step calls since the last reset
  int64_t observed = 0;     // reset counts read for steps <= observed
  int64_t pending_rmin = -1;  // first observed reset step not in a batch yet (-1: none)
  bool dirty = true;        // no reset yet, or steps ran outside the protocol (stream capture)
  int64_t stats[4] = {0, 0, 0, 0};
};

namespace {

hipEvent_t pf_take_event(apg_lidar_prefetcher *p) {
  if (!p->spare.empty()) {
    hipEvent_t e = p->spare.back();
    p->spare.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

// completed batches off the front of the list (their events back to the spares)
void pf_retire(apg_lidar_prefetcher *p) {
  while (!p->batches.empty() && hipEventQuery(p->batches.front().ev) == hipSuccess) {
    p->spare.push_back(p->batches.front().ev);
    p->batches.pop_front();
  }
}

// a batch after `after` (an event of the env's stream) covering the resets of steps rmin .. s
int pf_launch(apg_lidar_prefetcher *p, const apg_lidar_config *cfg, const apg_lidar_state *st,
              const apg_lidar_outputs *out, hipEvent_t after, int64_t rmin, int64_t s) {
  if (hipStreamWaitEvent(p->side, after, 0) != hipSuccess) return fail(APG_E_LAUNCH, "hipStreamWaitEvent (prefetch)");
  if (int rc = pf_batch_kernels(cfg, st, out, p->side)) return rc;
  hipEvent_t ev = pf_take_event(p);
  if (!ev || hipEventRecord(ev, p->side) != hipSuccess) return fail(APG_E_LAUNCH, "hipEventRecord (prefetch)");
  p->batches.push_back({rmin, s, ev});
  p->pending_rmin = -1;
  p->stats[0]++;
  return APG_OK;
}

// read the reset count of step o (its completion event has been seen)
void pf_observe(apg_lidar_prefetcher *p, int64_t o) {
  const uint32_t cnt = *reinterpret_cast<volatile uint32_t *>(&p->host_ring[o % p->R]);
  p->stats[2] += cnt;
  if (cnt && p->pending_rmin < 0) p->pending_rmin = o;
  p->observed = o;
}

// Before step c (p->c already incremented) on the env's stream `s`: observe the finished steps' reset counts,
// launch a batch for new resets, and make `s` wait for the batches covering the resets at steps <= c - L - 1.
int pf_before_step(apg_lidar_prefetcher *p, const apg_lidar_config *cfg, const apg_lidar_state *st,
                   const apg_lidar_outputs *out, hipStream_t s) {
  const int64_t c = p->c;
  if (p->dirty) {  // the records may be stale for any env: one batch after everything queued so far, waited for
    hipEvent_t mark = p->main_ev[(c - 1 + p->R) % p->R];
    if (hipEventRecord(mark, s) != hipSuccess) return fail(APG_E_LAUNCH, "hipEventRecord (prefetch)");
    if (int rc = pf_launch(p, cfg, st, out, mark, 0, c - 1)) return rc;
    if (hipStreamWaitEvent(s, p->batches.back().ev, 0) != hipSuccess)
      return fail(APG_E_LAUNCH, "hipStreamWaitEvent (prefetch)");
    p->stats[1]++;
    p->observed = c - 1;
    p->pending_rmin = -1;
    p->dirty = false;
    return APG_OK;
  }
  while (p->observed < c - 1) {  // non-blocking: steps the GPU has finished
    const hipError_t q = hipEventQuery(p->main_ev[(p->observed + 1) % p->R]);
    if (q == hipErrorNotReady) break;
    if (q != hipSuccess) return fail(APG_E_LAUNCH, "hipEventQuery (prefetch)");
    pf_observe(p, p->observed + 1);
  }
  const int64_t d = c - p->L - 1;  // resets at steps <= d may autoreset again at step c
  while (p->observed < d) {  // the GPU is more than a whole episode behind: block on the step's event
    if (hipEventSynchronize(p->main_ev[(p->observed + 1) % p->R]) != hipSuccess)
      return fail(APG_E_LAUNCH, "hipEventSynchronize (prefetch)");
    pf_observe(p, p->observed + 1);
  }
  if (p->pending_rmin >= 0) {
    if (int rc = pf_launch(p, cfg, st, out, p->main_ev[p->observed % p->R], p->pending_rmin, p->observed)) return rc;
  }
  pf_retire(p);
  // the last batch holding a reset at a step <= d (the side stream is in order: it implies the earlier ones)
  const apg_lidar_prefetcher::Batch *need = nullptr;
  for (const auto &b : p->batches)
    if (b.rmin <= d) need = &b;
  if (need) {
    if (hipStreamWaitEvent(s, need->ev, 0) != hipSuccess) return fail(APG_E_LAUNCH, "hipStreamWaitEvent (prefetch)");
    p->stats[1]++;
  }
  return APG_OK;
}

apg_lidar_prefetcher *prefetcher_of(const apg_lidar_config *cfg, const apg_lidar_state *st) {
  if (!st->prefetcher || !st->prefetch || !pf_supported(cfg)) return nullptr;
  auto *p = reinterpret_cast<apg_lidar_prefetcher *>(st->prefetcher);
  if (p->n != cfg->num_envs || p->h != cfg->height || p->w != cfg->width || p->L != cfg->step_limit) return nullptr;
  return p;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

}  // namespace

extern "C" {

const char *apg_version(void) { return "apgym-mi355x 0.3.0 (gfx950)"; }
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
  // (maze scratch: apg_maze.hpp's carve log + spilled DFS frames, maze_frames u16 per map)
  o->prefetch_bytes = pf_supported(cfg) ? pf_layout(g.n, g.h, g.wpr).bytes : 0;
  return APG_OK;
}

int apg_lidar_init(const apg_lidar_config *cfg, const apg_lidar_state *st, apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (cfg->map_kind == APG_MAP_POOL && (!st->pool_occ || !st->pool_free))
    return fail(APG_E_INVALID, "pool maps need the pool_occ and pool_free buffers");
  if (!cfg->is_static) return APG_OK;
  // One map for every env: generate dataset[static_map_index] once.
  Geo g = make_geo(cfg);
  hipStream_t s = (hipStream_t)stream;
  if (cfg->map_kind == APG_MAP_POOL) {  // dataset[static_map_index] is pool map static_map_index
    const size_t bytes = (size_t)g.h * g.wpr * sizeof(uint64_t);
    if (hipMemcpyAsync(st->occ, st->pool_occ + (size_t)cfg->static_map_index * g.h * g.wpr, bytes,
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
      return fail(APG_E_LAUNCH, "hipMemcpyAsync (static pool map)");
    return APG_OK;
  }
  // map_idx[0] already holds static_map_index (the host fills the state before init)
  return launch_map_generate_any(g, (const uint64_t *)st->map_idx, 1, st->occ, st->stack, nullptr, s);
}

int apg_lidar_reset(const apg_lidar_config *cfg, const apg_lidar_state *st, uint64_t seed, int use_seed,
                    const apg_lidar_outputs *out, apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (cfg->map_kind == APG_MAP_POOL && (!st->pool_occ || !st->pool_free))
    return fail(APG_E_INVALID, "pool maps need the pool_occ and pool_free buffers");
  hipStream_t s = (hipStream_t)stream;
  Geo g = make_geo(cfg);
  apg_lidar_prefetcher *p = prefetcher_of(cfg, st);
  if (p && !p->batches.empty() && hipStreamWaitEvent(s, p->batches.back().ev, 0) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipStreamWaitEvent (prefetch)");  // the batches use the maze scratch too
  if (g.kind == APG_MAP_MAZE && !g.is_static) {
    const bool pf = st->prefetch && pf_supported(cfg);
    const PfView pv = pf ? pf_view(st->prefetch, g.n, g.h, g.wpr) : PfView{};
    rc = launch_maze(g, *st, nullptr, g.n, nullptr, reinterpret_cast<uint8_t *>(st->stack), MZ_RESET, seed, use_seed,
                     1, out->map_idx, out->map_obs, out->err, s, pf ? &pv : nullptr);
  } else {
    rc = launch_reset(g, st, seed, use_seed, 1, out, s);
  }
  if (rc) return rc;
  apg_lidar_outputs o2 = *out;
  if (g.kind == APG_MAP_MAZE && !g.is_static) o2.map_obs = nullptr;  // written by k_maze
  if ((rc = launch_step_kernel(cfg, st, nullptr, nullptr, &o2, s, false))) return rc;
  if (p && !capturing(s)) {  // step 0: every env reset; its next maps are prefetched from here
    for (auto &b : p->batches) p->spare.push_back(b.ev);  // the env's stream waited for them above
    p->batches.clear();
    p->c = 0;
    p->observed = 0;
    p->pending_rmin = -1;
    if (hipEventRecord(p->main_ev[0], s) != hipSuccess) return fail(APG_E_LAUNCH, "hipEventRecord (prefetch)");
    if ((rc = pf_launch(p, cfg, st, out, p->main_ev[0], 0, 0))) return rc;
    p->dirty = false;
  } else if (p) {
    p->dirty = true;
  }
  return APG_OK;
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
  if (cfg->map_kind == APG_MAP_POOL && (!st->pool_occ || !st->pool_free))
    return fail(APG_E_INVALID, "pool maps need the pool_occ and pool_free buffers");
  hipStream_t s = (hipStream_t)stream;
  // rooms / static maps: one launch per step, the fused step kernel performs the NEXT_STEP autoresets itself;
  // mazes with a prefetcher: one launch per step, the fused step kernel installs the prefetched next maps;
  // other mazes: k_maze resets the envs with an autoreset pending (its waves exit at once when there are none),
  // then the unfused step kernel
  apg_lidar_prefetcher *p = prefetcher_of(cfg, st);
  const bool use_pf = p && !capturing(s);
  PfView V{};
  if (use_pf) {
    p->c++;
    if ((rc = pf_before_step(p, cfg, st, out, s))) return rc;
    V = pf_view(st->prefetch, cfg->num_envs, cfg->height, (cfg->width + 63) / 64);
    V.host_slot = p->dev_ring + p->c % p->R;
  } else if (p) {
    p->dirty = true;  // (stream capture) this step generates its mazes synchronously
  }
  if (ev_begin && hipEventRecord((hipEvent_t)ev_begin, s) != hipSuccess) return fail(APG_E_LAUNCH, "hipEventRecord");
  if (use_pf) {
    rc = launch_step_kernel(cfg, st, action, prediction, out, s, true, &V);
  } else if (big_rooms(cfg)) {
    // rooms the fused step kernel's LDS generator does not hold (max_rooms > 17, maps > 128): the pending
    // autoresets in k_lidar_reset, then the unfused step kernel (it writes their map obs)
    rc = launch_reset_gen<GEN_ROOMS>(make_geo(cfg), st, 0, 0, 0, out, s);
    if (rc == APG_OK) rc = launch_step_kernel(cfg, st, action, prediction, out, s, false);
  } else if (cfg->map_kind == APG_MAP_MAZE && !cfg->is_static) {
    const Geo g = make_geo(cfg);
    const bool pf = st->prefetch && pf_supported(cfg);
    const PfView pv = pf ? pf_view(st->prefetch, g.n, g.h, g.wpr) : PfView{};
    rc = launch_maze(g, *st, nullptr, g.n, nullptr, reinterpret_cast<uint8_t *>(st->stack), MZ_RESET, 0, 0, 0,
                     out->map_idx, out->map_obs, out->err, s, pf ? &pv : nullptr);
    apg_lidar_outputs o2 = *out;
    o2.map_obs = nullptr;  // written by k_maze
    if (rc == APG_OK) rc = launch_step_kernel(cfg, st, action, prediction, &o2, s, false);
  } else {
    rc = launch_step_kernel(cfg, st, action, prediction, out, s, true);
  }
  if (rc == APG_OK && ev_end && hipEventRecord((hipEvent_t)ev_end, s) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipEventRecord");
  if (rc == APG_OK && use_pf && hipEventRecord(p->main_ev[p->c % p->R], s) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipEventRecord (prefetch)");
  return rc;
}

int apg_lidar_prefetcher_create(const apg_lidar_config *cfg, apg_lidar_prefetcher **out) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!out) return fail(APG_E_INVALID, "null output");
  if (!pf_supported(cfg))
    return fail(APG_E_INVALID, "map prefetch needs dynamic maze maps of <= 128 x 128 cells and lidar_range <= 10");
  auto *p = new apg_lidar_prefetcher();
  p->n = cfg->num_envs;
  p->h = cfg->height;
  p->w = cfg->width;
  p->L = cfg->step_limit;
  p->R = cfg->step_limit + 2;
  int least = 0, greatest = 0;
  bool ok = hipGetDevice(&p->device) == hipSuccess && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
            hipStreamCreateWithPriority(&p->side, hipStreamNonBlocking, least) == hipSuccess;
  void *ring = nullptr;
  ok = ok && hipHostMalloc(&ring, (size_t)p->R * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
  if (ok) {
    p->host_ring = static_cast<uint32_t *>(ring);
    memset(p->host_ring, 0, (size_t)p->R * sizeof(uint32_t));
    void *dptr = nullptr;
    ok = hipHostGetDevicePointer(&dptr, ring, 0) == hipSuccess;
    p->dev_ring = static_cast<uint32_t *>(dptr);
  }
  p->main_ev.assign(p->R, nullptr);
  for (int i = 0; ok && i < p->R; i++) ok = hipEventCreateWithFlags(&p->main_ev[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    apg_lidar_prefetcher_destroy(p);
    return fail(APG_E_LAUNCH, "prefetcher: stream / pinned ring / event creation failed");
  }
  *out = p;
  return APG_OK;
}

int apg_lidar_prefetcher_destroy(apg_lidar_prefetcher *p) {
  if (!p) return APG_OK;
  int dev = -1;
  hipGetDevice(&dev);
  if (p->device >= 0) hipSetDevice(p->device);
  if (p->side) hipStreamSynchronize(p->side);
  for (auto &b : p->batches) hipEventDestroy(b.ev);
  for (auto e : p->spare) hipEventDestroy(e);
  for (auto e : p->main_ev)
    if (e) hipEventDestroy(e);
  if (p->side) hipStreamDestroy(p->side);
  if (p->host_ring) hipHostFree(p->host_ring);
  if (dev >= 0) hipSetDevice(dev);
  delete p;
  return APG_OK;
}

int apg_lidar_peek_map_index(const apg_lidar_config *cfg, const apg_lidar_state *st, uint64_t seed, int use_seed,
                             const uint8_t *mask, int64_t *out_idx, int32_t *out_env, int32_t *out_count,
                             apg_stream_t stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (cfg->map_kind != APG_MAP_POOL || cfg->is_static || cfg->stream_len <= 0)
    return fail(APG_E_INVALID, "peek_map_index: streamed pool maps only (stream_len > 0, dynamic maps)");
  if (!st || !out_idx || (!use_seed && !st->it_rng) || (out_env && !out_count))
    return fail(APG_E_INVALID, "peek_map_index: null buffer");
  hipStream_t s = (hipStream_t)stream;
  if (out_env && hipMemsetAsync(out_count, 0, sizeof(int32_t), s) != hipSuccess)
    return fail(APG_E_LAUNCH, "hipMemsetAsync (peek count)");
  const int n = cfg->num_envs;
  hipLaunchKernelGGL(k_peek_map_index, dim3(grid_for(n, 256)), dim3(256), 0, s, n, st->it_rng, cfg->stream_len, seed,
                     use_seed, mask, cfg->out_row_bytes ? cfg->out_row_bytes : 1, out_idx, out_env, out_count);
  return check_launch("k_peek_map_index");
}

int apg_lidar_prefetcher_stats(const apg_lidar_prefetcher *p, int64_t out[4]) {
  if (!p || !out) return fail(APG_E_INVALID, "null prefetcher / output");
  for (int i = 0; i < 3; i++) out[i] = p->stats[i];
  out[3] = p->c;
  return APG_OK;
}

int apg_lidar_step(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *action,
                   const float *prediction, const apg_lidar_outputs *out, apg_stream_t stream) {
  return apg_lidar_step_profiled(cfg, st, action, prediction, out, stream, nullptr, nullptr);
}

int apg_maze_frames(int h, int w) { return (int)(maze_scratch_bytes(h, w) / 2); }

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
  if (n <= 0 || h <= 0 || w <= 0 || w > 255) return fail(APG_E_INVALID, "bad scan batch arguments");
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
  P.row = cfg->out_row_bytes;
  hipLaunchKernelGGL(k_lidar_render_track, dim3(rs->num_tracked), dim3(RT_THREADS), 0, (hipStream_t)stream, P, *st,
                     prediction, *out, *rs);
  return check_launch("k_lidar_render_track");
}

int apg_rng_draws(const uint64_t *seeds, int m, int kind, int64_t a, int64_t b, int n, double *out,
                  apg_stream_t stream) {
  if (m <= 0 || n <= 0 || kind < 0 || kind > 5) return fail(APG_E_INVALID, "bad rng draw arguments");
  if (kind == 5 && (a < 0 || a > 15)) return fail(APG_E_INVALID, "binomial n must be in [0, 15]");
  hipLaunchKernelGGL(k_rng_draws, dim3(grid_for(m, 64)), dim3(64), 0, (hipStream_t)stream, seeds, m, kind, a, b,
                     n, out);
  return check_launch("k_rng_draws");
}

#ifdef APG_STEP_PROFILE
int apg_debug_step_profile(void *dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_step_prof), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int apg_debug_step_profile_waves(void *dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_step_prof_w), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
}  // extern "C"
