// apg_circle_square.hip — gfx950 kernels + C ABI for the procedural CircleSquare datasets and the
// CircleSquareHideAndSeek reward (ap_gym/envs/image/circle_square_dataset.py,
// ap_gym/envs/circle_square_catch_or_flee.py).
//
//   k_cs_pool         one thread per pixel: the whole dataset rendered into the device-resident f32
//                     pool the glimpse kernels read (CircleSquareDataset._get_data_point :98-107,
//                     DoubleCircleSquareDataset._get_data_point :149-172, _draw_object :32-55),
//                     evaluated in float64 in numpy's operation order, then cast to float32
//                     (_process_imgs_np, image_classification_dataset.py:66-70).  The pool is written
//                     once per env construction (2.8 GB for DoubleCircleSquare 28x28, HBM-write bound).
//   k_hide_and_seek   one thread per env: the additional reward sign(label) * |glimpse_pos - object|
//                     of CircleSquareHideAndSeekVectorWrapper.step (:69-98), folded into
//                     info["base_reward"] and the reward, with the -sparse ids' SparsifyVectorWrapper
//                     (sparsify_wrapper.py:72-83) applied on top when requested.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/apgym_capi.h"
#include "apg_host.hpp"

using namespace apg;

namespace {

struct CsGeo {
  int kind, h, w, grad_a, grad_b;
  double half_extent, max_dist;
  int64_t num_positions;
};

// |(r0, c0) - (r1, c1)| as np.linalg.norm over the last axis of an int64 difference: the squares and
// their sum are exact in float64, one correctly rounded sqrt.
__device__ __forceinline__ double int_norm(int64_t dr, int64_t dc) {
  return __dsqrt_rn(__dadd_rn((double)(dr * dr), (double)(dc * dc)));
}

// _draw_object (:32-55): label 0 = rectangle (closed box of half side e/2), 1 = circle (norm <= e/2)
__device__ __forceinline__ bool on_object(const CsGeo &g, int label, int64_t pr, int64_t pc, int i, int j,
                                          double norm) {
  if (label == 0)
    return __dsub_rn((double)pr, g.half_extent) <= (double)i && (double)i <= __dadd_rn((double)pr, g.half_extent) &&
           __dsub_rn((double)pc, g.half_extent) <= (double)j && (double)j <= __dadd_rn((double)pc, g.half_extent);
  return norm <= g.half_extent;
}

__global__ __launch_bounds__(256) void k_cs_pool(CsGeo g, const int16_t *__restrict__ positions, int64_t first,
                                                 int64_t count, float *__restrict__ pool, int32_t *__restrict__ labels) {
  const int64_t px_per_img = (int64_t)g.h * g.w;
  const int64_t total = count * px_per_img;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / px_per_img;
    const int p = (int)(t - k * px_per_img);
    const int i = p / g.w, j = p - (p / g.w) * g.w;
    const int64_t idx = first + k;
    double v;
    int label;
    if (g.kind == APG_DS_CIRCLE_SQUARE) {
      // _unpack with max_vals [2, W, H] (:57-64, :85-86); position = (pos_y, pos_x) = (row, col)
      label = (int)(idx % 2);
      const int64_t rest = idx / 2;
      const int64_t pcol = rest % g.w, prow = (rest / g.w) % g.h;
      const double n = int_norm(prow - i, pcol - j);
      v = g.grad_a ? __dsub_rn(1.0, __ddiv_rn(n, g.max_dist)) : 0.0;
      if (on_object(g, label, prow, pcol, i, j, n)) v = 1.0;
    } else {
      // _unpack with max_vals [2, 2, len(positions)] (:174-175)
      const int l1 = (int)(idx % 2), l2 = (int)((idx / 2) % 2);
      const int64_t pi = (idx / 4) % g.num_positions;
      const int64_t r1 = positions[4 * pi], c1 = positions[4 * pi + 1];
      const int64_t r2 = positions[4 * pi + 2], c2 = positions[4 * pi + 3];
      const double n1 = int_norm(r1 - i, c1 - j), n2 = int_norm(r2 - i, c2 - j);
      // 1 - minimum(n1 * show_gradient_a, n2 * show_gradient_b) / max_dist   (:156-163)
      const double m = fmin(__dmul_rn(n1, g.grad_a ? 1.0 : 0.0), __dmul_rn(n2, g.grad_b ? 1.0 : 0.0));
      v = __dsub_rn(1.0, __ddiv_rn(m, g.max_dist));
      if (on_object(g, l1, r1, c1, i, j, n1) || on_object(g, l2, r2, c2, i, j, n2)) v = 1.0;
      label = l1 == l2 ? l1 : 2;
    }
    __builtin_nontemporal_store(__double2float_rn(v), pool + t);
    if (p == 0) labels[k] = label;
  }
}

__global__ __launch_bounds__(256) void k_hide_and_seek(apg_hide_and_seek_args a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.num_envs) return;
  // CircleSquareDataset.get_object_position_and_label (:109-113): label, pos_x, pos_y
  const int64_t idx = a.index[e];
  const int64_t label = idx % 2, rest = idx / 2;
  const int64_t pcol = rest % a.width, prow = (rest / a.width) % a.height;
  // normalize_coords(flip(positions)) - 1 = (pos_x, pos_y) / sensor_pos_lim_pixels - 1
  const double nx = __dsub_rn(__ddiv_rn((double)pcol, a.lim[0]), 1.0);
  const double ny = __dsub_rn(__ddiv_rn((double)prow, a.lim[1]), 1.0);
  const double dx = __dsub_rn((double)a.glimpse_pos[2 * e], nx), dy = __dsub_rn((double)a.glimpse_pos[2 * e + 1], ny);
  const double dist = __dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)));
  const double add = __dmul_rn((double)(label * 2 - 1), dist);
  // info["base_reward"] += additional_reward: float32 storage except on the autoreset step (float64 zeros)
  const double base = a.resetting ? __dadd_rn(0.0, add)
                                  : (double)__double2float_rn(__dadd_rn((double)a.base_reward_in[e], add));
  a.base_reward_out[e] = base;
  a.additional[e] = add;
  double r;
  if (a.mask_prediction) {
    r = base;  // reward = info["base_reward"] (the sparse wrapper then subtracts float32 zeros)
  } else if (a.sparse) {
    // SparsifyVectorWrapper: base_reward - CE(prediction, target) * weight, weight = float32(terminated)
    r = __dsub_rn(base, __dmul_rn(a.loss[e], a.terminated ? 1.0 : 0.0));
  } else {
    r = __dadd_rn(a.reward_in[e], add);  // reward += additional_reward
  }
  a.reward_out[e] = r;
}

int cs_validate(const apg_circle_square_config *c) {
  if (!c) return fail(APG_E_INVALID, "null config");
  if (c->kind != APG_DS_CIRCLE_SQUARE && c->kind != APG_DS_DOUBLE_CIRCLE_SQUARE)
    return fail(APG_E_INVALID, "unknown circle-square dataset kind");
  if (c->height <= 0 || c->width <= 0 || c->height > 4096 || c->width > 4096)
    return fail(APG_E_INVALID, "image_shape must be positive (<= 4096)");
  if (c->kind == APG_DS_DOUBLE_CIRCLE_SQUARE && c->num_positions <= 0)
    return fail(APG_E_INVALID, "DoubleCircleSquareDataset needs at least one position pair");
  return APG_OK;
}

}  // namespace

extern "C" {

int apg_circle_square_pool(const apg_circle_square_config *cfg, const int16_t *positions, int64_t first,
                           int64_t count, float *pool, int32_t *labels, apg_stream_t stream) {
  int rc = cs_validate(cfg);
  if (rc) return rc;
  if (first < 0 || count <= 0) return fail(APG_E_INVALID, "bad data point range");
  if (!pool || !labels || (cfg->kind == APG_DS_DOUBLE_CIRCLE_SQUARE && !positions))
    return fail(APG_E_INVALID, "null pool / labels / positions");
  CsGeo g;
  g.kind = cfg->kind;
  g.h = cfg->height;
  g.w = cfg->width;
  g.grad_a = cfg->show_gradient_a != 0;
  g.grad_b = cfg->show_gradient_b != 0;
  g.half_extent = cfg->half_extent;
  g.max_dist = cfg->max_dist;
  g.num_positions = cfg->num_positions;
  const int64_t total = count * cfg->height * cfg->width;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 256 * 64) blocks = 256 * 64;  // grid-stride beyond 64 workgroups per CU
  hipLaunchKernelGGL(k_cs_pool, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, g, positions, first,
                     count, pool, labels);
  return check_launch("k_cs_pool");
}

int apg_hide_and_seek_reward(const apg_hide_and_seek_args *args, apg_stream_t stream) {
  if (!args || args->num_envs <= 0 || args->width <= 0 || args->height <= 0)
    return fail(APG_E_INVALID, "bad hide-and-seek arguments");
  if (!args->index || !args->glimpse_pos || !args->base_reward_out || !args->reward_out || !args->additional ||
      (!args->resetting && !args->base_reward_in) || (!args->mask_prediction && !args->sparse && !args->reward_in) ||
      (!args->mask_prediction && args->sparse && !args->loss))
    return fail(APG_E_INVALID, "null hide-and-seek buffer");
  hipLaunchKernelGGL(k_hide_and_seek, dim3((args->num_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, *args);
  return check_launch("k_hide_and_seek");
}

}  // extern "C"
