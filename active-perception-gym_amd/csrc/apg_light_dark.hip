// apg_light_dark.hip — gfx950 kernels + C ABI for the LightDark-v0 id as one batched env.
//
// Reference (ap_gym 0.5.0): `make_vec("LightDark-v0", N)` = gymnasium SyncVectorEnv over N x
// ActiveRegressionLogWrapper(TimeLimit(50, issue_termination=True)(LightDarkEnv))
// (ap_gym/envs/registration.py:640-647, ap_gym/envs/light_dark.py:14-155, ap_gym/time_limit.py:113-139,
// ap_gym/active_perception_env.py:101-121, ap_gym/active_regression_env.py:131-159).
//
//   k_light_dark_reset   one thread per env: sub-env i seeded with seed + i (SyncVectorEnv.reset),
//                        start position uniform(-1, 1) (float64 -> float32), noisy observation.
//   k_light_dark_step    one thread per env: NEXT_STEP autoreset (rng continues), NaN checks, base
//                        reward, move (project to the unit disc, x 0.15), out-of-bounds termination +
//                        clip, TimeLimit, normalized MSE loss vs the pre-move position, episode stats,
//                        noisy observation pos + N(0, 1) * (1 - brightness(pos)) * 0.3 clipped to [-2, 2].
// The normal draws are numpy's Generator.normal: loc + scale * random_standard_normal (ziggurat over
// PCG64, distributions.c), with numpy's own tables (apg_ziggurat.hpp).  All arithmetic is float32 in
// numpy's NEP 50 order (python-float constants rounded to float32), no FMA contraction.
// Per env-step the kernel moves ~160 bytes (state 53 B in + out, action/prediction 16 B, outputs
// 52 B): HBM-bound, one launch per step.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py).
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/apgym_capi.h"
#include "apg_device.hpp"
#include "apg_host.hpp"
#include "apg_pairwise.hpp"
#include "apg_ziggurat.hpp"

using namespace apg;

namespace {

constexpr uint8_t LD_AUTORESET = 1;  // the env terminated/truncated: the next step resets it

// glibc's log1p (sysdeps/ieee754/dbl-64/s_log1p.c: fdlibm's reduction with the Estrin-grouped
// polynomial), which numpy's npy_log1p calls on the reference's host; restated operation by
// operation so the ziggurat's tail draws (NOR_R + xx) round like the reference's.  Checked against
// the host libm on 350k inputs (tools/gen_ziggurat.py's companion check in DESIGN.md §2).
APG_DEV double glibc_log1p(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  const int32_t hx = (int32_t)(__double_as_longlong(x) >> 32), ax = hx & 0x7fffffff;
  int k = 1, hu = 0;
  double f = 0.0, c = 0.0;
  if (hx < 0x3FDA827A) {
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_huge_val() : __builtin_nan("");
    if (ax < 0x3e200000) {
      if (ax < 0x3c900000) return x;
      return __dsub_rn(x, __dmul_rn(__dmul_rn(x, x), 0.5));
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {
      k = 0;
      f = x;
      hu = 1;
    }
  }
  if (hx >= 0x7ff00000) return __dadd_rn(x, x);
  if (k != 0) {
    double u;
    if (hx < 0x43400000) {
      u = __dadd_rn(1.0, x);
      hu = (int32_t)(__double_as_longlong(u) >> 32);
      k = (hu >> 20) - 1023;
      c = k > 0 ? __dsub_rn(1.0, __dsub_rn(u, x)) : __dsub_rn(x, __dsub_rn(u, 1.0));
      c = __ddiv_rn(c, u);
    } else {
      u = x;
      hu = (int32_t)(__double_as_longlong(u) >> 32);
      k = (hu >> 20) - 1023;
      c = 0.0;
    }
    hu &= 0x000fffff;
    const uint64_t lo = (uint64_t)__double_as_longlong(u) & 0xffffffffULL;
    if (hu < 0x6a09e) {
      u = __longlong_as_double((long long)(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo));
    } else {
      k += 1;
      u = __longlong_as_double((long long)(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo));
      hu = (0x00100000 - hu) >> 2;
    }
    f = __dsub_rn(u, 1.0);
  }
  const double hfsq = __dmul_rn(__dmul_rn(0.5, f), f);
  const double dk = (double)k;
  if (hu == 0) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c = __dadd_rn(c, __dmul_rn(dk, ln2_lo));
      return __dadd_rn(__dmul_rn(dk, ln2_hi), c);
    }
    const double R = __dmul_rn(hfsq, __dsub_rn(1.0, __dmul_rn(0.66666666666666666, f)));
    if (k == 0) return __dsub_rn(f, R);
    return __dsub_rn(__dmul_rn(dk, ln2_hi), __dsub_rn(__dsub_rn(R, __dadd_rn(__dmul_rn(dk, ln2_lo), c)), f));
  }
  const double s = __ddiv_rn(f, __dadd_rn(2.0, f)), z = __dmul_rn(s, s);
  const double R1 = __dmul_rn(z, Lp1), z2 = __dmul_rn(z, z), R2 = __dadd_rn(Lp2, __dmul_rn(z, Lp3));
  const double z4 = __dmul_rn(z2, z2), R3 = __dadd_rn(Lp4, __dmul_rn(z, Lp5)), z6 = __dmul_rn(z4, z2);
  const double R4 = __dadd_rn(Lp6, __dmul_rn(z, Lp7));
  const double R = __dadd_rn(__dadd_rn(__dadd_rn(R1, __dmul_rn(z2, R2)), __dmul_rn(z4, R3)), __dmul_rn(z6, R4));
  if (k == 0) return __dsub_rn(f, __dsub_rn(hfsq, __dmul_rn(s, __dadd_rn(hfsq, R))));
  return __dsub_rn(__dmul_rn(dk, ln2_hi),
                   __dsub_rn(__dsub_rn(hfsq, __dadd_rn(__dmul_rn(s, __dadd_rn(hfsq, R)),
                                                       __dadd_rn(__dmul_rn(dk, ln2_lo), c))),
                             f));
}

// random_standard_normal (numpy distributions.c): 99.3 % of draws return after one table lookup.
// The wedge test compares against exp(): the device libm's exp may differ from the host's by an
// ulp, which flips the accept decision only when the uniform lands within that ulp (p ~ 1e-16).
APG_DEV double standard_normal(Pcg64 &r) {
  for (;;) {
    uint64_t v = next64(r);
    const int idx = (int)(v & 0xff);
    v >>= 8;
    const int sign = (int)(v & 1);
    const uint64_t rabs = (v >> 1) & 0x000fffffffffffffULL;
    double x = __dmul_rn((double)rabs, zig_wi[idx]);
    if (sign) x = -x;
    if (rabs < zig_ki[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = __dmul_rn(-ZIG_NOR_INV_R, glibc_log1p(-next_double(r)));
        const double yy = -glibc_log1p(-next_double(r));
        if (__dadd_rn(yy, yy) > __dmul_rn(xx, xx))
          return ((rabs >> 8) & 1) ? -__dadd_rn(ZIG_NOR_R, xx) : __dadd_rn(ZIG_NOR_R, xx);
      }
    }
    if (__dadd_rn(__dmul_rn(__dsub_rn(zig_fi[idx - 1], zig_fi[idx]), next_double(r)), zig_fi[idx]) <
        exp(__dmul_rn(__dmul_rn(-0.5, x), x)))
      return x;
  }
}

// light_dark.py:98-118: std = (1 - brightness(pos)) * 0.3, brightness = h^2 / (|pos - light|^2 + h^2)
// with light = float32([0, -0.7]), h = 0.2 (float32 scalar arithmetic, constants rounded to float32)
APG_DEV float light_std(float px, float py) {
  const float dx = __fsub_rn(px, 0.0f), dy = __fsub_rn(py, -0.7f);
  const float dsq = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), (float)(0.2 * 0.2));
  const float b = f32_div((float)(0.2 * 0.2), dsq);
  return __fmul_rn(__fsub_rn(1.0f, b), 0.3f);
}

// __get_obs (:97-101): pos + normal(size=2).astype(float32) * std, clipped to [-2, 2]
APG_DEV void noisy_obs(Pcg64 &r, float px, float py, float *out) {
  const float z0 = (float)__dadd_rn(0.0, __dmul_rn(1.0, standard_normal(r)));
  const float z1 = (float)__dadd_rn(0.0, __dmul_rn(1.0, standard_normal(r)));
  const float s = light_std(px, py);
  out[0] = fminf(fmaxf(__fadd_rn(px, __fmul_rn(z0, s)), -2.0f), 2.0f);
  out[1] = fminf(fmaxf(__fadd_rn(py, __fmul_rn(z1, s)), -2.0f), 2.0f);
}

// reset (:106-118): pos = uniform(-ones(2), ones(2), size=2).astype(float32), then the observation
APG_DEV void reset_env(Pcg64 &r, float &px, float &py, float *obs) {
  px = (float)__dadd_rn(-1.0, __dmul_rn(2.0, next_double(r)));
  py = (float)__dadd_rn(-1.0, __dmul_rn(2.0, next_double(r)));
  noisy_obs(r, px, py, obs);
}

__global__ __launch_bounds__(256) void k_light_dark_reset(apg_light_dark_config c, apg_light_dark_state S,
                                                          uint64_t seed, int use_seed, apg_light_dark_outputs O) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.num_envs) return;
  Pcg64 r = use_seed ? seed_pcg64(seed + (uint64_t)e) : *reinterpret_cast<const Pcg64 *>(&S.rng[e]);
  float px, py, obs[2];
  reset_env(r, px, py, obs);
  S.pos[2 * e] = px;
  S.pos[2 * e + 1] = py;
  S.elapsed[e] = 0;
  S.flags[e] = 0;
  *reinterpret_cast<Pcg64 *>(&S.rng[e]) = r;
  O.noisy_position[2 * e] = obs[0];
  O.noisy_position[2 * e + 1] = obs[1];
  O.time_step[e] = -1.0f;
}

APG_DEV void clear_info(const apg_light_dark_config &c, const apg_light_dark_outputs &O, int e) {
  O.reward[e] = 0.0;
  O.terminated[e] = 0;
  O.truncated[e] = 0;
  O.base_reward[e] = 0.0f;
  O.target[2 * e] = 0.0f;
  O.target[2 * e + 1] = 0.0f;
  O.loss[e] = 0.0f;
  O.info_mask[e] = 0;
  if (c.log_stats) O.stats_len[e] = 0;
  if (c.sparse) O.weight[e] = 0.0;
}

__global__ __launch_bounds__(256) void k_light_dark_step(apg_light_dark_config c, apg_light_dark_state S,
                                                         const float *__restrict__ act,
                                                         const float *__restrict__ pred, apg_light_dark_outputs O) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.num_envs) return;
  uint8_t f = S.flags[e];
  float px = S.pos[2 * e], py = S.pos[2 * e + 1];
  if (f & LD_AUTORESET) {  // NEXT_STEP autoreset: reset(seed=None), reward 0, no step info
    Pcg64 r = *reinterpret_cast<const Pcg64 *>(&S.rng[e]);
    float obs[2];
    reset_env(r, px, py, obs);
    *reinterpret_cast<Pcg64 *>(&S.rng[e]) = r;
    S.pos[2 * e] = px;
    S.pos[2 * e + 1] = py;
    S.elapsed[e] = 0;
    S.flags[e] = 0;
    clear_info(c, O, e);
    O.reset_mask[e] = 1;
    O.noisy_position[2 * e] = obs[0];
    O.noisy_position[2 * e + 1] = obs[1];
    O.time_step[e] = -1.0f;
    return;
  }
  O.reset_mask[e] = 0;
  float ax = act[2 * e], ay = act[2 * e + 1];
  const float prx = pred[2 * e], pry = pred[2 * e + 1];
  uint32_t errbits = 0;
  if (isnan(ax) || isnan(ay)) errbits |= APG_ERR_NAN_ACTION;
  if (isnan(prx) || isnan(pry)) errbits |= APG_ERR_NAN_PREDICTION;
  if (errbits) {  // the reference raises ValueError before touching this env's state
    clear_info(c, O, e);
    atomicOr(O.err, errbits);
    return;
  }
  const float lpx = px, lpy = py;  // __last_pos (the prediction target)
  // base_reward = 1.0 - 1e-3 * sum(action ** 2) (:127-129)
  const float br = __fsub_rn(1.0f, __fmul_rn(0.001f, __fadd_rn(__fmul_rn(ax, ax), __fmul_rn(ay, ay))));
  const float mag = norm_f32(ax, ay);
  if (mag > 1.0f) {
    ax = f32_div(ax, mag);
    ay = f32_div(ay, mag);
  }
  px = __fadd_rn(px, __fmul_rn(ax, 0.15f));
  py = __fadd_rn(py, __fmul_rn(ay, 0.15f));
  bool term = fabsf(px) >= 1.0f || fabsf(py) >= 1.0f;
  px = fminf(fmaxf(px, -1.0f), 1.0f);
  py = fminf(fmaxf(py, -1.0f), 1.0f);
  Pcg64 r = *reinterpret_cast<const Pcg64 *>(&S.rng[e]);
  float obs[2];
  noisy_obs(r, px, py, obs);
  *reinterpret_cast<Pcg64 *>(&S.rng[e]) = r;
  // TimeLimit(step_limit, issue_termination=True)
  const int el = S.elapsed[e] + 1;
  S.elapsed[e] = el;
  if (el >= c.step_limit) term = true;
  // normalized MSE vs the previous position (active_regression_env.py:29-52, loss_fn.py:261-267)
  const float ex = __fsub_rn(prx, lpx), ey = __fsub_rn(pry, lpy);
  const float mse = f32_div(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), 2.0f);
  const float loss = __fadd_rn(__fmul_rn(mse, c.loss_scale), c.loss_offset);
  if (c.log_stats) {  // ActiveRegressionLogWrapper (active_regression_env.py:131-159)
    float *hist = S.stats_hist + (size_t)e * 2 * c.step_limit;
    hist[el - 1] = norm_f32(ex, ey);
    hist[c.step_limit + el - 1] = mse;
    if (term) {
      for (int m = 0; m < 2; m++) {
        const float *h = hist + m * c.step_limit;
        O.stats[(size_t)m * c.num_envs + e] = f32_div(__fadd_rn(0.0f, pw_sum_ptr(h, el)), (float)el);
        O.stats[(size_t)(2 + m) * c.num_envs + e] = h[el - 1];
      }
      O.stats_len[e] = el;
    } else {
      O.stats_len[e] = 0;
    }
  }
  O.base_reward[e] = br;
  O.target[2 * e] = lpx;
  O.target[2 * e + 1] = lpy;
  O.loss[e] = loss;
  if (c.sparse) {  // SparsifyWrapper (sparsify_wrapper.py:93-161): base_reward - loss * weight
    O.weight[e] = term ? 1.0 : 0.0;
    O.reward[e] = (double)__fsub_rn(br, __fmul_rn(loss, term ? 1.0f : 0.0f));
  } else {
    O.reward[e] = (double)__fsub_rn(br, loss);
  }
  O.terminated[e] = term;
  O.truncated[e] = 0;
  O.info_mask[e] = 1;
  S.pos[2 * e] = px;
  S.pos[2 * e + 1] = py;
  S.flags[e] = term ? LD_AUTORESET : 0;
  O.noisy_position[2 * e] = obs[0];
  O.noisy_position[2 * e + 1] = obs[1];
  O.time_step[e] = (float)(2.0 * (double)el / (double)c.step_limit - 1.0);
}

__global__ void k_standard_normal(const uint64_t *seeds, int m, int n, double *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  Pcg64 r = seed_pcg64(seeds[i]);
  for (int k = 0; k < n; k++) out[(size_t)i * n + k] = standard_normal(r);
}

int ld_validate(const apg_light_dark_config *c) {
  if (!c) return fail(APG_E_INVALID, "null config");
  if (c->num_envs <= 0) return fail(APG_E_INVALID, "num_envs must be positive");
  if (c->step_limit <= 0) return fail(APG_E_INVALID, "step_limit must be positive");
  if (c->log_stats && c->step_limit > PW_PTR_MAX_N) return fail(APG_E_INVALID, "log_stats needs step_limit <= 968");
  return APG_OK;
}

}  // namespace

extern "C" {

int apg_light_dark_reset(const apg_light_dark_config *cfg, const apg_light_dark_state *st, uint64_t seed,
                         int use_seed, const apg_light_dark_outputs *out, apg_stream_t stream) {
  int rc = ld_validate(cfg);
  if (rc) return rc;
  hipLaunchKernelGGL(k_light_dark_reset, dim3((cfg->num_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, *cfg,
                     *st, seed, use_seed, *out);
  return check_launch("k_light_dark_reset");
}

int apg_light_dark_step(const apg_light_dark_config *cfg, const apg_light_dark_state *st, const float *action,
                        const float *prediction, const apg_light_dark_outputs *out, apg_stream_t stream) {
  int rc = ld_validate(cfg);
  if (rc) return rc;
  if (!action || !prediction) return fail(APG_E_INVALID, "null action/prediction");
  if (cfg->log_stats && (!st->stats_hist || !out->stats || !out->stats_len))
    return fail(APG_E_INVALID, "log_stats needs stats_hist, stats and stats_len buffers");
  if (cfg->sparse && !out->weight) return fail(APG_E_INVALID, "sparse needs the weight buffer");
  hipLaunchKernelGGL(k_light_dark_step, dim3((cfg->num_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, *cfg,
                     *st, action, prediction, *out);
  return check_launch("k_light_dark_step");
}

int apg_standard_normal_draws(const uint64_t *seeds, int m, int n, double *out, apg_stream_t stream) {
  if (m <= 0 || n <= 0 || !seeds || !out) return fail(APG_E_INVALID, "bad standard normal draw arguments");
  hipLaunchKernelGGL(k_standard_normal, dim3((m + 63) / 64), dim3(64), 0, (hipStream_t)stream, seeds, m, n, out);
  return check_launch("k_standard_normal");
}

}  // extern "C"
