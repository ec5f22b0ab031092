/*
 * apgym_capi.h — C ABI of the MI355X (gfx950) backend for ap_gym's data-parallel hot path.
 *
 * Library: active-perception-gym_amd/ap_gym_amd/_lib/libapgym_hip.so (hipcc --offload-arch=gfx950)
 * All pointers are DEVICE pointers owned by the caller unless stated otherwise.  Every entry point
 * is stream-ordered on `stream` (a hipStream_t passed as void*, NULL = default stream), allocates
 * nothing, never synchronises the host, and returns APG_OK or a negative APG_E_* code.  Device-side
 * failures the reference raises as Python exceptions are reported through the `err` word (bit
 * flags APG_ERR_*), which the host layer turns into the reference's ValueError /
 * NotImplementedError lazily.
 *
 * Reference interfaces replaced (ap_gym 0.5.0, /root/reference):
 *   apg_lidar_reset / apg_lidar_step
 *       gymnasium SyncVectorEnv.reset/step over TimeLimit(ActiveRegressionLogWrapper-free)
 *       LIDARLocalization2DEnv, i.e. ap_gym/envs/lidar_localization2d.py:293-389 (reset, _step),
 *       :238-277 (__get_obs), :496-536 (__lidar_scan), :547-557 (_np_random setter),
 *       ap_gym/time_limit.py:113-139, ap_gym/active_perception_env.py:101-121 (step + loss),
 *       ap_gym/envs/registration.py:319-356 (wrapper composition of the LIDARLoc* ids).
 *   apg_map_generate
 *       FloorMapDatasetRooms.get_data_point  ap_gym/envs/floor_map/floor_map_dataset_rooms.py:25-89
 *       FloorMapDatasetMaze.get_data_point   ap_gym/envs/floor_map/floor_map_dataset_maze.py:24-55
 *   apg_lidar_scan_batch
 *       LIDARLocalization2DEnv.__lidar_scan  ap_gym/envs/lidar_localization2d.py:496-536
 *   apg_lidar_render_track
 *       the render-only state of LIDARLocalization2DEnv (observation_map, trajectory, last readings)
 *       ap_gym/envs/lidar_localization2d.py:239-261, 312-313, 326-327, 377-380 used by render() :391-494.
 *   apg_rng_draws
 *       numpy Generator(PCG64(SeedSequence(seed))) draws as used by the above (test entry point).
 *   apg_rng_fill
 *       one vector-level numpy Generator drawing a whole batch: Generator.integers(lo, hi, n)
 *       (numpy distributions.c random_bounded_uint64_fill, Lemire on next_uint32) and
 *       Generator.uniform(low, high, (n, cols)) (random_uniform) as used by
 *       DatasetBatchIterator.__next__ ap_gym/envs/dataset/dataset_iterator.py:52-57 and
 *       ImagePerceptionModule ap_gym/envs/image/image_perception_module.py:105-118, 130-161, 278-291.
 *   apg_image_seed / apg_image_reset / apg_image_step
 *       ImageClassificationVectorEnv  ap_gym/envs/image_classification.py:107-151 (reset, _step,
 *       _np_random setter) and ImageLocalizationVectorEnv ap_gym/envs/image_localization.py:131-181,
 *       237-246 over ImagePerceptionModule ap_gym/envs/image/image_perception_module.py:105-251
 *       (seed, reset, step, _get_obs), with ActivePerceptionVectorEnv.step
 *       ap_gym/active_perception_vector_env.py:84-111 and the normalized CE / MSE losses
 *       ap_gym/loss_fn.py:69-83, 207-267.
 *   apg_image_glimpse
 *       ImagePerceptionModule.get_glimpse  image_perception_module.py:294-331 (scipy
 *       RegularGridInterpolator "linear", bounds_error=True; clip(0, 1); float32).
 *   apg_image_unique_top_k
 *       ImagePerceptionModule.sample_unique_glimpse_positions  image_perception_module.py:253-277.
 *   apg_loss_ce / apg_loss_mse
 *       CrossEntropyLossFn.numpy / MSELossFn.numpy + LossFnAffineTransformation (loss_fn.py).
 *   apg_circle_square_pool
 *       CircleSquareDataset / DoubleCircleSquareDataset get_data_point_batch
 *       ap_gym/envs/image/circle_square_dataset.py:32-178 (+ _process_imgs_np float64 -> float32).
 *   apg_hide_and_seek_reward
 *       CircleSquareHideAndSeekVectorWrapper.step  ap_gym/envs/circle_square_catch_or_flee.py:69-98.
 *   apg_light_dark_reset / apg_light_dark_step
 *       SyncVectorEnv over ActiveRegressionLogWrapper(TimeLimit(50)(LightDarkEnv)) as registered at
 *       ap_gym/envs/registration.py:640-647; LightDarkEnv.reset/_step/__get_obs
 *       ap_gym/envs/light_dark.py:93-155.
 *   apg_standard_normal_draws
 *       numpy Generator.standard_normal (ziggurat, distributions.c) as LightDarkEnv draws it (test entry).
 */
#ifndef APGYM_CAPI_H
#define APGYM_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define APG_OK 0
#define APG_E_INVALID (-1)     /* bad argument / unsupported configuration */
#define APG_E_LAUNCH (-2)      /* kernel launch failed (see apg_last_error) */

#define APG_ERR_NAN_ACTION 1u     /* "NaN values detected in action." */
#define APG_ERR_NAN_PREDICTION 2u /* "NaN values detected in prediction." */
#define APG_ERR_MAPGEN 4u         /* internal map-generation bound exceeded */
#define APG_ERR_OOB_Y 8u          /* "One of the requested xi is out of bounds in dimension 0" */
#define APG_ERR_OOB_X 16u         /* "One of the requested xi is out of bounds in dimension 1" */
#define APG_ERR_PREFETCH 32u      /* a maze autoreset found no prefetched map (prefetch protocol violated) */
#define APG_ERR_NO_FREE_CELL 64u  /* a pool map without a free cell was drawn: numpy's integers(0, 0) raises
                                     ValueError("high <= 0") in reset (lidar_localization2d.py:302-303) */

#define APG_MAP_ROOMS 0
#define APG_MAP_MAZE 1
#define APG_MAP_POOL 2 /* maps of any FloorMapDataset, read once into a resident pool (state.pool_occ):
                          ap_gym/envs/floor_map/floor_map_dataset.py:10-22, drawn per episode as
                          DatasetIterator does, ap_gym/envs/dataset/dataset_iterator.py:26-32 */

typedef void *apg_stream_t; /* hipStream_t */

/* numpy PCG64 stream with next_uint32 half-buffer; 40 bytes, 8-byte aligned */
typedef struct apg_pcg64 {
  uint64_t state_hi, state_lo, inc_hi, inc_lo;
  uint32_t has_uint32, uinteger;
} apg_pcg64;

typedef struct apg_lidar_config {
  int32_t num_envs;
  int32_t height, width;        /* map size in cells, 3 .. 511 each (pool maps 1 .. 511); rooms maps must be square,
                                   mazes odd; pool maps any H x W */
  int32_t map_kind;             /* APG_MAP_ROOMS | APG_MAP_MAZE | APG_MAP_POOL */
  int32_t is_static;            /* 1: one map for all envs (static_map=True) */
  int32_t static_map_index;     /* dataset index of the static map */
  int32_t beams;                /* lidar_beam_count */
  int32_t step_limit;           /* TimeLimit max_episode_steps (issue_termination=True) */
  int32_t max_rooms, door_width;/* FloorMapDatasetRooms parameters (max_rooms 1 .. 64) */
  float lidar_range;
  float loss_scale, loss_offset;/* normalized MSE affine, as float32 (NEP 50) */
  double branching_prob;        /* FloorMapDatasetMaze parameter */
  int32_t log_stats;            /* 1: ActiveRegressionLogWrapper episode statistics (registered ids) */
  int32_t sparse;               /* 1: the -sparse ids (SparsifyWrapper, sparsify_wrapper.py:93-161):
                                   reward = base_reward - loss * (terminated ? 1 : 0) */
  int32_t out_row_bytes;        /* 0: dense outputs.  > 0 (a multiple of 8): packed rows — the per-env outputs
                                   lidar, odometry, time_step, reward, terminated, truncated, base_reward,
                                   target, loss, info_mask, map_idx, reset_mask, stats, stats_len, weight of
                                   env e are at their pointer + e * out_row_bytes (element j of a field at
                                   + j * element size; stats as [N][4]), i.e. the pointers are field offsets
                                   into one [N][out_row_bytes] buffer that a sharded run all-gathers as is.
                                   It must hold every enabled field (apg_lidar_step rejects a row smaller than
                                   16 + 4 * beams + 36 bytes, + 8 with sparse, + 20 with log_stats, rounded up to
                                   a multiple of 8).  Added in ABI 0.2 (apg_version): callers built against 0.1
                                   must zero it. */
  int32_t pool_len;             /* APG_MAP_POOL: len(dataset), 1 .. 2**31 - 1 maps in state.pool_occ; the episode's
                                   map is pool map integers(0, pool_len) of the env's DatasetIterator stream
                                   (dataset_iterator.py:26-32), the static map pool map static_map_index.
                                   Other kinds: ignored (ABI 0.3) */
  int64_t stream_len;           /* APG_MAP_POOL, dynamic maps: 0 = the pool holds every map of the dataset (above).
                                   > 0 = streamed maps (ABI 0.4): len(dataset) (any size, e.g. 2**32); the episode's
                                   map index is integers(0, stream_len) of the env's DatasetIterator stream and its
                                   map is pool slot e (pool_len == num_envs), which the host filled with
                                   dataset.get_data_point(that index) before the reset -- the reference's per-draw
                                   fetch (dataset_iterator.py:26-32) through its prefetch thread
                                   (buffered_iterator.py:11-61).  apg_lidar_peek_map_index tells the host which index
                                   each env's next reset draws.  Callers built against ABI <= 0.3 must zero it. */
} apg_lidar_config;

/* Persistent per-env state.  Sizes come from apg_lidar_query_sizes(). */
typedef struct apg_lidar_state {
  float *pos;          /* [N][2] */
  float *init_pos;     /* [N][2] */
  int32_t *elapsed;    /* [N]   TimeLimit._elapsed_steps */
  uint8_t *flags;      /* [N]   bit0 autoreset pending, bit1 reset this step, bit2 pos aliases init_pos */
  apg_pcg64 *rng;      /* [N]   env np_random */
  apg_pcg64 *it_rng;   /* [N]   DatasetIterator rng (dynamic maps) */
  uint64_t *occ;       /* [N or 1][H][wpr] bit-packed occupancy, wpr = ceil(W/64) */
  uint64_t *scratch;   /* reserved, unused (may be NULL; query_sizes reports scratch_bytes = 0) */
  uint16_t *stack;     /* [N or 1][maze_frames] maze scratch (carve log + spilled DFS frames), contiguous
                          per map, 64-byte aligned (mazes only) */
  uint64_t *map_idx;   /* [N]   dataset index of the current map */
  const float *beam_dirs; /* [beams][2] lidar_directions (f32, computed by the host like the reference) */
  float *stats_hist;   /* [2][step_limit][N] per-step euclidean_distance, mse of the episode (log_stats) */
  uint8_t *prefetch;   /* prefetch_bytes (apg_lidar_query_sizes) of zeroed device memory, or NULL: the next map of
                          every env, generated ahead of its autoreset (mazes up to 128 rows) */
  void *prefetcher;    /* apg_lidar_prefetcher_create() handle owning the side stream that fills `prefetch`, or
                          NULL (then mazes are generated synchronously by the autoreset step) */
  const uint64_t *pool_occ;  /* APG_MAP_POOL: [pool_len][H][wpr] bit-packed maps (bit x % 64 of word x / 64 of row
                                y is map[y, x]; bits past W zero), i.e. dataset.get_data_point(i) for every i;
                                NULL for the procedural kinds (ABI 0.3) */
  const int32_t *pool_free;  /* APG_MAP_POOL: [pool_len] free cells of each pool map (the start-cell draw's
                                integers(0, nfree), lidar_localization2d.py:302-304) */
} apg_lidar_state;

typedef struct apg_lidar_outputs {
  float *lidar;        /* [N][beams] (any 4-byte alignment; 16-byte aligned rows take vector stores) */
  float *odometry;     /* [N][2] */
  float *time_step;    /* [N] */
  float *map_obs;      /* [N][H][W] (dynamic maps; rewritten only for envs that reset) or NULL */
  double *reward;      /* [N] float64 like SyncVectorEnv */
  uint8_t *terminated; /* [N] */
  uint8_t *truncated;  /* [N] */
  float *base_reward;  /* [N] info["base_reward"] */
  float *target;       /* [N][2] info["prediction"]["target"] */
  float *loss;         /* [N] info["prediction"]["loss"] */
  uint8_t *info_mask;  /* [N] 1 where the step info carries base_reward/prediction (0 on autoreset) */
  uint64_t *map_idx;   /* [N] info["map_idx"] of envs that reset this step (others untouched) or NULL */
  uint8_t *reset_mask; /* [N] 1 where the env auto-reset this step (info["_map_idx"]) or NULL */
  uint32_t *err;       /* [1] OR-ed APG_ERR_* bits (never cleared by the library) */
  float *stats;        /* [4][N] avg_euclidean_distance, avg_mse, final_euclidean_distance, final_mse
                          of the episodes that ended this step (log_stats) */
  int32_t *stats_len;  /* [N] length of the episode that ended this step, 0 = no stats (log_stats) */
  double *weight;      /* [N] sparse: info["prediction"]["target"]["weight"] (1.0 where terminated) or NULL */
} apg_lidar_outputs;

typedef struct apg_lidar_state_sizes {
  size_t occ_bytes, scratch_bytes, stack_bytes; /* bytes of the variable-size buffers (scratch_bytes: reserved, 0) */
  int32_t wpr, maze_frames;
  size_t prefetch_bytes;                        /* apg_lidar_state.prefetch (0: the configuration has no prefetch) */
} apg_lidar_state_sizes;

const char *apg_version(void);
const char *apg_last_error(void);

int apg_lidar_query_sizes(const apg_lidar_config *cfg, apg_lidar_state_sizes *out);

/* Build the static map (is_static) into state->occ; no-op for dynamic maps. */
int apg_lidar_init(const apg_lidar_config *cfg, const apg_lidar_state *st, apg_stream_t stream);

/* reset(seed=seed): sub-env i reseeded with seed+i when use_seed (else streams continue, like
 * reset(seed=None)); draws maps / start cells; writes obs (lidar, odometry, time_step, map_obs)
 * and map_idx. */
int apg_lidar_reset(const apg_lidar_config *cfg, const apg_lidar_state *st, uint64_t seed,
                    int use_seed, const apg_lidar_outputs *out, apg_stream_t stream);

/* step({"action": action, "prediction": prediction}) with NEXT_STEP autoreset. */
int apg_lidar_step(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *action,
                   const float *prediction, const apg_lidar_outputs *out, apg_stream_t stream);

/* apg_lidar_step, additionally recording hipEvent_t `ev_begin` / `ev_end` (may be NULL) on `stream`
 * immediately before and after the fused step kernel (k_lidar_step) — used by bench.py to time the
 * dominant kernel live. */
int apg_lidar_step_profiled(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *action,
                            const float *prediction, const apg_lidar_outputs *out, apg_stream_t stream,
                            void *ev_begin, void *ev_end);

/* ---------------------------------------------------------------- map prefetch (dynamic mazes)
 * The reference builds each sub-env's DataLoader(prefetch=True, prefetch_buffer_size=128): a background thread
 * generates the next maps while the env steps (ap_gym/envs/lidar_localization2d.py:130-131, 296-298;
 * ap_gym/envs/dataset/buffered_iterator.py:11-61).  Here every env's next maze (map index, occupancy rows, start
 * cell and its streams after that reset, all independent of the actions) is generated on a low-priority side
 * stream right after the env's reset, into apg_lidar_state.prefetch, and the fused step kernel's autoreset only
 * copies it in (occupancy rows, f32 map obs, state).  The prefetcher is the host side of that protocol, driven by
 * apg_lidar_reset / apg_lidar_step on the env's stream: after a step with autoresets (it reads the per-step reset
 * count the step kernel writes to pinned host memory, without synchronizing) it launches a prefetch batch on the
 * side stream, and before step c it makes the step's stream wait for the batches covering every reset at steps
 * <= c - step_limit - 1 (the earliest an env can reset again), so an autoreset never waits on a map unless the
 * side stream fell that far behind.  Create it after apg_lidar_init on the env's device; one prefetcher per env
 * state; not thread-safe.  Steps captured into a hipGraph (stream capture) generate their mazes synchronously. */
typedef struct apg_lidar_prefetcher apg_lidar_prefetcher;
int apg_lidar_prefetcher_create(const apg_lidar_config *cfg, apg_lidar_prefetcher **out);
int apg_lidar_prefetcher_destroy(apg_lidar_prefetcher *p); /* synchronizes its side stream first */
/* per-prefetcher counters: [0] batches launched, [1] steps whose main stream had to wait for a batch that was still
 * running, [2] resets observed, [3] step calls since the last reset (diagnostics, host memory) */
int apg_lidar_prefetcher_stats(const apg_lidar_prefetcher *p, int64_t out[4]);

/* ---------------------------------------------------------------- streamed maps (APG_MAP_POOL, stream_len > 0)
 * The dataset index the NEXT reset of each selected env will draw (integers(0, stream_len) of a copy of its
 * DatasetIterator stream, dataset_iterator.py:26-32; use_seed: of the stream reset(seed=seed) gives sub-env e, i.e.
 * default_rng(seed + e).integers(0, 2**32, endpoint=True), the _np_random setter of lidar_localization2d.py:547-557).
 * No stream is advanced.  mask: NULL = every env, else the envs whose reset_mask output is 1 (the step that just ran
 * reset them: their slots were consumed; mask is read with the output row stride when out_row_bytes > 0).
 * out_env NULL: out_idx[e] for every selected env.  Else the selected envs compacted (in no particular order) into
 * out_env[k] / out_idx[k], k < *out_count (zeroed by the call).  Replaces next(DataLoader(DatasetIterator)) of
 * lidar_localization2d.py:296-298 on the host side: the host fetches get_data_point(idx) into the env's slot. */
int apg_lidar_peek_map_index(const apg_lidar_config *cfg, const apg_lidar_state *st, uint64_t seed, int use_seed,
                             const uint8_t *mask, int64_t *out_idx, int32_t *out_env, int32_t *out_count,
                             apg_stream_t stream);

/* u16 units of maze scratch per map (apg_lidar_state.stack / apg_map_generate's stack) for an h x w maze;
 * replaces the reference's recursion stack of carve() (floor_map_dataset_maze.py:31-45). */
int apg_maze_frames(int h, int w);

/* n maps from dataset indices idx[n] into occ[n][h][wpr]; stack [n][apg_maze_frames(h, w)] (mazes only);
 * scratch is reserved and unused (may be NULL). */
int apg_map_generate(int map_kind, const uint64_t *idx, int n, int h, int w, int max_rooms,
                     int door_width, double branching_prob, uint64_t *occ, uint64_t *scratch,
                     uint16_t *stack, uint32_t *err, apg_stream_t stream);

/* n segments seg[n][4] = (px, py, qx, qy) against map map_index[n] of occ[*][h][wpr]. */
int apg_lidar_scan_batch(const uint64_t *occ, const int32_t *map_index, int h, int w,
                         const float *seg, int n, float *dist, int32_t *kind, apg_stream_t stream);

/* ---------------------------------------------------------------- LIDAR render path (not the hot path)
 * Render-only state of the tracked sub-envs: what LIDARLocalization2DEnv keeps for render()
 * (ap_gym/envs/lidar_localization2d.py:391-494) — observation_map (:239-261, :301), the trajectory deque
 * (:312, :327, :377-380), the last lidar readings (:242) and last pos / prediction (:313, :326-327). */
typedef struct apg_lidar_render_state {
  int32_t num_tracked;       /* T */
  int32_t scan_points;       /* P = len(np.arange(0, lidar_range, 0.05)) */
  const int32_t *env;        /* [T] tracked sub-env indices (< num_envs) */
  const double *scan_xy;     /* [beams][P][2] scan_points (float64, computed by the host like :188-191) */
  const double *scan_norm;   /* [beams][P] np.linalg.norm(scan_points, axis=-1) */
  uint32_t *obs_map;         /* [T][H][ceil(W/32)] observation_map, bit x%32 of word x/32 */
  float *traj;               /* [T][step_limit][3] trajectory rows: last_pos x, y, min(prediction_quality, 1) */
  int32_t *traj_len;         /* [T] */
  float *pose;               /* [T][6] last_pos (x, y), last_pred (x, y), pos (x, y) */
  int32_t *has_last;         /* [T] 0 after a reset (last_pos = last_pred = None) */
  float *lidar_dist;         /* [T][beams] distances of the last observation */
} apg_lidar_render_state;

/* After apg_lidar_reset (prediction = NULL) or apg_lidar_step (its prediction): update the render state
 * of the tracked sub-envs from st->pos, out->reset_mask and out->target (both required). */
int apg_lidar_render_track(const apg_lidar_config *cfg, const apg_lidar_state *st, const float *prediction,
                           const apg_lidar_outputs *out, const apg_lidar_render_state *rs, apg_stream_t stream);

/* n draws of `kind` (0 next64, 1 next32, 2 random, 3 integers(a,b), 4 integers(0,2**32,endpoint),
 * 5 binomial(a, 0.3)) from default_rng(seed[i]) for each of m seeds; out[m][n] as float64. */
int apg_rng_draws(const uint64_t *seeds, int m, int kind, int64_t a, int64_t b, int n, double *out,
                  apg_stream_t stream);

/* ---------------------------------------------------------------- vector-level numpy streams */
#define APG_DRAW_UNIFORM 0 /* out f64[n][cols] = low[c] + range[c] * next_double   (Generator.uniform) */
#define APG_DRAW_INTEGERS 1 /* out i64[n] = lo + bounded(hi - lo - 1)               (Generator.integers) */

/* n draws (n x cols for uniform, cols <= 2) from the ONE stream *state (device), advancing it
 * exactly as numpy would.  integers: bound = hi - lo (exclusive range, 1 <= bound <= 2**32) and
 * `work` holds apg_rng_fill_work_elems(n, bound) int64 (device), zeroed before its first use and left zeroed
 * (work[0] counts the finished workgroups, so the last one advances the generator state in the same launch);
 * uniform draws use only work[0] and accept work == NULL (then a second launch advances the state). */
int64_t apg_rng_fill_work_elems(int64_t n, uint64_t bound);
int apg_rng_fill(apg_pcg64 *state, int kind, int64_t n, int cols, const double *low, const double *range,
                 int64_t lo, uint64_t bound, void *out, int64_t *work, apg_stream_t stream);

/* ---------------------------------------------------------------- image glimpse envs */
#define APG_IMAGE_CLASSIFY 0 /* ImageClassificationVectorEnv */
#define APG_IMAGE_LOCALIZE 1 /* ImageLocalizationVectorEnv */
#define APG_POOL_U8 0        /* pool values v -> float32(v) / 255 (_process_imgs_np) */
#define APG_POOL_F32 1
#define APG_POOL_U8_TILED 2  /* u8 RGB pools (pool_channels 3) as RGBX, 4 bytes per pixel (the 4th unused), in tiles of
                                8 x 4 pixels = one 128-byte line, tiles row-major: pixel (y, x) of an image at byte
                                (y / 4) * ceil(W / 8) * 128 + (y % 4) * 32 + (x / 8) * 128 + (x % 8) * 4 + channel;
                                an image takes ceil(H / 4) * ceil(W / 8) * 128 bytes.  A
                                glimpse's tap box then spans ~40 % fewer cache lines than in row-major HWC, and every tap
                                is one aligned dword.  Same values as APG_POOL_U8 (v -> float32(v) / 255) (ABI 0.4) */

typedef struct apg_image_config {
  int32_t num_envs;
  int32_t kind;               /* APG_IMAGE_CLASSIFY | APG_IMAGE_LOCALIZE */
  int32_t height, width;      /* image size of the dataset */
  int32_t pool_channels;      /* channels stored in the pool (1 or 3) */
  int32_t channels;           /* observation channels (1 or 3; 1 -> 3 repeats the grey channel) */
  int32_t pool_dtype;         /* APG_POOL_U8 | APG_POOL_F32 | APG_POOL_U8_TILED */
  int32_t sensor_h, sensor_w; /* sensor_size[0], sensor_size[1] */
  int32_t step_limit;
  int32_t num_classes;
  int32_t invert_labels;      /* randomly_invert_labels */
  int32_t top_k;              /* unique_sampling_top_k */
  int32_t unique_points;      /* P: sampling grid points of sample_unique_glimpse_positions */
  int32_t num_envs_total;     /* envs of the whole (sharded) batch: every vector-level draw has this size */
  int32_t env_offset;         /* first env of this shard: the shard uses draws [offset, offset + num_envs) */
  int64_t pool_len;           /* len(dataset) */
  double sensor_scale;
  double max_step[2];         /* max_step_length broadcast to (2,) */
  double cell[2];             /* unique sampling max_grid_cell_size_norm */
  double ce_scale, ce_offset; /* normalized CrossEntropyLossFn affine (float64) */
  float mse_scale, mse_offset;/* normalized MSELossFn affine (float32, NEP 50) */
  int32_t log_stats;          /* 1: the registered ids' vector log wrapper statistics */
  int32_t sparse;             /* 1: the -sparse ids (SparsifyVectorWrapper, sparsify_wrapper.py:23-92):
                                 reward = base_reward - loss * terminated */
  int32_t out_row_bytes;      /* 0: dense outputs.  > 0 (a multiple of 8): packed rows — the per-env outputs glimpse,
                                 glimpse_pos, time_step, reward, base_reward, target, label_target, loss_f64,
                                 loss_f32, stats (as [N][4]) and stats_idx (as [N][2]) of env e are at their
                                 pointer + e * out_row_bytes, i.e. the pointers are field offsets into one
                                 [N][out_row_bytes] buffer that a sharded run all-gathers as is (ABI 0.2; the row
                                 must hold the enabled fields: apg_image_* reject a smaller one).  target_glimpse
                                 stays dense [N][G0][G1][C] either way: it changes only with the batch */
} apg_image_config;

/* u8 pools are read with whole-dword loads that may run up to APG_U8_POOL_PAD - 1 bytes past the last image: the
 * allocation must extend APG_U8_POOL_PAD readable bytes beyond [pool_len][H][W][pool_channels] */
#define APG_U8_POOL_PAD 16

typedef struct apg_image_state {
  const void *pool;           /* [pool_len][H][W][pool_channels] u8 (+ APG_U8_POOL_PAD bytes) or f32 */
  const int32_t *pool_labels; /* [pool_len] */
  const double *unique_grid;  /* [P][2] sampling positions (localize) */
  int64_t *index;             /* [N] data point index of each env (info["index"]) */
  int32_t *label;             /* [N] current label (after inversion) */
  int32_t *inverted;          /* [N] 0/1 label inverted this episode */
  double *pos;                /* [N][2] sensor position, normalized (float64 like the reference) */
  float *target;              /* [N][2] localization target */
  apg_pcg64 *rng;             /* [3] env np_random, module current_rng, DatasetBatchIterator rng */
  int64_t *scratch_i64;       /* [2][N_total] batch draws */
  double *scratch_f64;        /* [N_total][2] batch draws */
  int32_t *top_k;             /* [N][top_k] unique-sampling ranking (localize) */
  int64_t *rng_work;          /* apg_rng_fill_work_elems(N, max(pool_len, top_k, 2)) int64 */
  float *stats_hist;          /* [N][2][step_limit] per-step metrics of the episode (log_stats):
                                 classify: correct_label_prob; localize: euclidean_distance, mse */
  int64_t *ahead_i64;         /* [2][N_total] the next batch's index and inversion draws (apg_image_draw_ahead) or NULL */
  double *ahead_f64;          /* [2][N_total][2] the next batch's start positions and (localize) refreshed targets */
  apg_pcg64 *rng_saved;       /* [3] the streams before the draws made ahead (apg_image_discard_ahead) */
} apg_image_state;

typedef struct apg_image_outputs {
  float *glimpse;             /* [N][sensor_h][sensor_w][C] */
  float *glimpse_pos;         /* [N][2] */
  float *time_step;           /* [N] */
  float *target_glimpse;      /* [N][sensor_h][sensor_w][C] (localize) */
  double *reward;             /* [N] base_reward - loss; a float32 value whenever the reference's is */
  float *base_reward;         /* [N] (the reference's are float64 zeros on the autoreset step) */
  float *target;              /* [N][2] localize: info["prediction"]["target"] (pre-update copy) */
  int32_t *label_target;      /* [N] classify: info["prediction"]["target"] */
  double *loss_f64;           /* [N] classify: normalized cross entropy (float64) */
  float *loss_f32;            /* [N] localize: normalized MSE (float32) */
  uint32_t *err;              /* [1] OR-ed APG_ERR_* bits */
  float *stats;               /* [4][N] on the episode's last step (log_stats): classify final/avg of
                                 correct_label_prob, accuracy; localize final/avg of euclidean_distance, mse
                                 (order: final m0, final m1, avg m0, avg m1) */
  int32_t *stats_idx;         /* [2][N] classify: first_correct, last_incorrect (-1: none) */
} apg_image_outputs;

/* reset(seed=seed) seeding chain: np_random = default_rng(seed); module.seed(np_random.integers(0,
 * 2**32-1, endpoint=True)); iterator seed = current_rng.integers(0, 2**32-1, endpoint=True). */
int apg_image_seed(const apg_image_config *cfg, const apg_image_state *st, uint64_t seed, apg_stream_t stream);

/* ImagePerceptionModule.reset (+ ImageLocalizationVectorEnv unique targets): draws the batch,
 * positions and labels; writes glimpse / glimpse_pos / time_step (and target_glimpse). */
int apg_image_reset(const apg_image_config *cfg, const apg_image_state *st, const apg_image_outputs *out,
                    apg_stream_t stream);

/* One vector step.  t = time step before the step; prev_done bit 0 = the previous step terminated all envs (the
 * module then resets instead of moving; the host tracks both, they are batch-global), bit 1 = that reset's draws
 * were made ahead by apg_image_draw_ahead (the step then only installs them: one launch). */
int apg_image_step(const apg_image_config *cfg, const apg_image_state *st, const float *action,
                   const float *prediction, int32_t t, int32_t prev_done, const apg_image_outputs *out,
                   apg_stream_t stream);

/* The next batch autoreset's draws, made ahead (typically on a second stream right after a reset, while the episode
 * steps; they depend only on the streams, not on actions): DatasetBatchIterator indices, label inversions, start
 * positions (image_perception_module.py:120-139, dataset_iterator.py:52-57) and, localize, the refreshed targets
 * (image_localization.py:151-158), into ahead_i64 / ahead_f64, advancing the streams as the autoreset step would;
 * the streams before them are kept in rng_saved.  The stream of the step that consumes them must wait for them. */
int apg_image_draw_ahead(const apg_image_config *cfg, const apg_image_state *st, apg_stream_t stream);
/* Undo apg_image_draw_ahead (restores the streams from rng_saved): before a reset() that replaces the batch. */
int apg_image_discard_ahead(const apg_image_config *cfg, const apg_image_state *st, apg_stream_t stream);

/* Glimpses of npos positions per env: pos (f64 or f32, pos_is_f32) [N][npos][2] -> out
 * [N][npos][sensor_h][sensor_w][C]; index[N] selects the pool image of each env (u8 pools: + APG_U8_POOL_PAD). */
int apg_image_glimpse(const apg_image_config *cfg, const void *pool, const int64_t *index, const void *pos,
                      int pos_is_f32, int32_t npos, float *out, uint32_t *err, apg_stream_t stream);

/* Uniqueness ranking of sample_unique_glimpse_positions: top_k[N][k] grid indices by descending
 * min_{b != a} mean((g_b - g_a)^2) (exact ties: ascending index); uniq[N][P] (float, may be NULL). */
int apg_image_unique_top_k(const apg_image_config *cfg, const void *pool, const int64_t *index,
                           const double *grid, int32_t npoints, int32_t k, int32_t *top_k, float *uniq,
                           apg_stream_t stream);

/* Normalized losses over n rows: CE on logits [n][k] vs int32 targets -> f64; MSE on [n][d] -> f32. */
int apg_loss_ce(const float *logits, const int32_t *target, int32_t n, int32_t k, double scale, double offset,
                double *out, apg_stream_t stream);
int apg_loss_mse(const float *pred, const float *target, int32_t n, int32_t d, float scale, float offset,
                 float *out, apg_stream_t stream);

/* ---------------------------------------------------------------- procedural CircleSquare datasets */
#define APG_DS_CIRCLE_SQUARE 0        /* CircleSquareDataset        circle_square_dataset.py:79-113 */
#define APG_DS_DOUBLE_CIRCLE_SQUARE 1 /* DoubleCircleSquareDataset  circle_square_dataset.py:116-178 */

typedef struct apg_circle_square_config {
  int32_t kind;                       /* APG_DS_* */
  int32_t height, width;              /* image_shape */
  int32_t show_gradient_a;            /* CircleSquare: show_gradient; Double: show_gradient_a */
  int32_t show_gradient_b;            /* Double: show_gradient_b */
  int32_t pad_;
  int64_t num_positions;              /* Double: len(positions) (valid coordinate pairs) */
  double half_extent;                 /* object_extents / 2 */
  double max_dist;                    /* np.sqrt(np.sum(np.array(image_shape) ** 2)) */
} apg_circle_square_config;

/* Data points [first, first + count) rendered into pool[count][H][W] (float32, one channel) and
 * labels[count] (int32), i.e. get_data_point_batch(arange(first, first + count)).  Double:
 * positions[num_positions][2][2] int16 (row, col) pairs in the reference's order. */
int apg_circle_square_pool(const apg_circle_square_config *cfg, const int16_t *positions, int64_t first,
                           int64_t count, float *pool, int32_t *labels, apg_stream_t stream);

/* CircleSquareHideAndSeekVectorWrapper.step (circle_square_catch_or_flee.py:69-98) on the inner
 * ImageClassificationVectorEnv's step outputs (+ SparsifyVectorWrapper for the -sparse ids). */
typedef struct apg_hide_and_seek_args {
  int32_t num_envs;
  int32_t height, width;              /* CircleSquareDataset image_shape */
  int32_t resetting;                  /* the inner step was the batch autoreset (base_reward = f64 zeros) */
  int32_t terminated;                 /* the inner step terminated the batch */
  int32_t mask_prediction;            /* NoPrediction variant: reward = base_reward */
  int32_t sparse;                     /* -sparse ids: reward = base_reward - loss * terminated */
  int32_t pad_;
  double lim[2];                      /* sensor_pos_lim_pixels (x, y) */
  const int64_t *index;               /* [N] info["index"] */
  const float *glimpse_pos;           /* [N][2] obs["glimpse_pos"] */
  const float *base_reward_in;        /* [N] inner info["base_reward"] (unused when resetting) */
  const double *reward_in;            /* [N] inner reward */
  const double *loss;                 /* [N] inner normalized CE (sparse) */
  double *base_reward_out;            /* [N] new info["base_reward"] (float32 values unless resetting) */
  double *reward_out;                 /* [N] new reward */
  double *additional;                 /* [N] sign * distance */
} apg_hide_and_seek_args;

int apg_hide_and_seek_reward(const apg_hide_and_seek_args *args, apg_stream_t stream);

/* ---------------------------------------------------------------- LightDark-v0 */
typedef struct apg_light_dark_config {
  int32_t num_envs;
  int32_t step_limit;                 /* TimeLimit max_episode_steps (50 for LightDark-v0) */
  int32_t log_stats;                  /* 1: ActiveRegressionLogWrapper episode statistics */
  int32_t sparse;                     /* 1: LightDark-sparse-v0 (SparsifyWrapper): reward = base - loss * terminated */
  float loss_scale, loss_offset;      /* normalized MSE affine, as float32 (NEP 50) */
} apg_light_dark_config;

typedef struct apg_light_dark_state {
  float *pos;                         /* [N][2] agent position */
  int32_t *elapsed;                   /* [N] TimeLimit._elapsed_steps */
  uint8_t *flags;                     /* [N] bit0: the env is reset by the next step (NEXT_STEP autoreset) */
  apg_pcg64 *rng;                     /* [N] env np_random */
  float *stats_hist;                  /* [N][2][step_limit] per-step euclidean_distance, mse (log_stats) */
} apg_light_dark_state;

typedef struct apg_light_dark_outputs {
  float *noisy_position;              /* [N][2] obs["noisy_position"] */
  float *time_step;                   /* [N] obs["time_step"] */
  double *reward;                     /* [N] float64 like SyncVectorEnv */
  uint8_t *terminated, *truncated;    /* [N] */
  float *base_reward;                 /* [N] info["base_reward"] */
  float *target;                      /* [N][2] info["prediction"]["target"] (the pre-move position) */
  float *loss;                        /* [N] info["prediction"]["loss"] */
  uint8_t *info_mask;                 /* [N] 1 where the step info carries base_reward/prediction */
  uint8_t *reset_mask;                /* [N] 1 where the env auto-reset this step */
  uint32_t *err;                      /* [1] OR-ed APG_ERR_* bits */
  float *stats;                       /* [4][N] avg/avg/final/final (euclidean_distance, mse) of ended episodes */
  int32_t *stats_len;                 /* [N] episode length where an episode ended this step, else 0 */
  double *weight;                     /* [N] sparse: 1.0 where terminated */
} apg_light_dark_outputs;

/* reset(seed): sub-env i seeded with seed + i when use_seed (else the streams continue). */
int apg_light_dark_reset(const apg_light_dark_config *cfg, const apg_light_dark_state *st, uint64_t seed,
                         int use_seed, const apg_light_dark_outputs *out, apg_stream_t stream);
/* step({"action", "prediction"}) with NEXT_STEP autoreset. */
int apg_light_dark_step(const apg_light_dark_config *cfg, const apg_light_dark_state *st, const float *action,
                        const float *prediction, const apg_light_dark_outputs *out, apg_stream_t stream);
/* n draws of Generator.standard_normal from default_rng(seeds[i]) for each of m seeds -> out[m][n]. */
int apg_standard_normal_draws(const uint64_t *seeds, int m, int n, double *out, apg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
