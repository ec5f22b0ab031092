// apg_torch_ops.cpp — PyTorch custom ops (TORCH_LIBRARY(apgym, ...)) over the C ABI of libapgym_hip.so.
//
// The envs' hot path calls these instead of marshalling the C-ABI structs through ctypes on every
// step: an env handle (torch.classes.apgym.LidarEnv / ImageEnv) is built once from the env's config
// fields and its persistent device buffers, and the ops launch on PyTorch's current HIP stream, so
// they are stream-ordered with the caller's tensors and can be captured into a torch.cuda.CUDAGraph
// (hipGraph) like any ATen op.
//
//   torch.ops.apgym.lidar_reset(LidarEnv env, int seed, bool use_seed) -> ()
//   torch.ops.apgym.lidar_step(LidarEnv env, Tensor action, Tensor prediction) -> ()
//   torch.ops.apgym.image_reset(ImageEnv env) -> ()
//   torch.ops.apgym.image_step(ImageEnv env, Tensor action, Tensor prediction, int t, int prev_done) -> ()
//
// Replaces, like the C ABI below it (include/apgym_capi.h): SyncVectorEnv.reset/step over
// TimeLimit(LIDARLocalization2DEnv) (ap_gym/envs/lidar_localization2d.py:293-389) and
// Image{Classification,Localization}VectorEnv reset/step (ap_gym/envs/image_classification.py:107-151,
// image_localization.py:131-181, image/image_perception_module.py:105-251).
// Build: hipcc (host code only) against torch's headers, linked to libapgym_hip.so (build.py).
#include <ATen/Tensor.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/apgym_capi.h"

namespace {

void *ptr(const at::Tensor &t) { return t.defined() && t.numel() > 0 ? t.data_ptr() : nullptr; }

void check(int rc, const char *what) {
  TORCH_CHECK(rc == APG_OK, what, " failed (", rc, "): ", apg_last_error());
}

apg_stream_t stream_of(const at::Device &d) { return (apg_stream_t)c10::hip::getCurrentHIPStream(d.index()).stream(); }

void check_io(const at::Tensor &t, const at::Device &d, int64_t numel, const char *name) {
  TORCH_CHECK(t.device() == d, name, " must be on ", d, ", got ", t.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() == numel, name, " must have ", numel, " elements, got ", t.numel());
}

// Buffers are passed in the C struct's field order; a 0-element tensor stands for NULL.  The handle
// keeps them alive for its lifetime.
template <class S>
void fill_ptrs(S &s, const std::vector<at::Tensor> &ts, const char *what) {
  constexpr size_t n = sizeof(S) / sizeof(void *);
  static_assert(sizeof(S) == n * sizeof(void *), "pointer-only struct");
  TORCH_CHECK(ts.size() == n, what, ": expected ", n, " buffers, got ", ts.size());
  void *p[n];
  for (size_t i = 0; i < n; i++) p[i] = ptr(ts[i]);
  std::memcpy(&s, p, sizeof(S));
}

struct LidarEnv : torch::CustomClassHolder {
  apg_lidar_config cfg{};
  apg_lidar_state st{};
  apg_lidar_outputs out{};
  std::vector<at::Tensor> keep;
  at::Device dev = at::Device(at::kCUDA, 0);

  // ints: num_envs, height, width, map_kind, is_static, static_map_index, beams, step_limit, max_rooms,
  // door_width, log_stats, sparse, out_row_bytes, prefetcher handle (apg_lidar_prefetcher_create's pointer or 0:
  // owned by the Python env), pool_len, stream_len; reals: lidar_range, loss_scale, loss_offset, branching_prob.  The state
  // buffers are the struct's fields in order: ..., the prefetch buffer, a 0-element placeholder for the prefetcher
  // field, the map pool (pool_occ, pool_free: 0-element tensors for the procedural kinds).
  LidarEnv(std::vector<int64_t> ints, std::vector<double> reals, std::vector<at::Tensor> state,
           std::vector<at::Tensor> outputs) {
    TORCH_CHECK(ints.size() == 16 && reals.size() == 4, "LidarEnv: 16 ints and 4 reals expected");
    cfg.num_envs = (int32_t)ints[0];
    cfg.height = (int32_t)ints[1];
    cfg.width = (int32_t)ints[2];
    cfg.map_kind = (int32_t)ints[3];
    cfg.is_static = (int32_t)ints[4];
    cfg.static_map_index = (int32_t)ints[5];
    cfg.beams = (int32_t)ints[6];
    cfg.step_limit = (int32_t)ints[7];
    cfg.max_rooms = (int32_t)ints[8];
    cfg.door_width = (int32_t)ints[9];
    cfg.log_stats = (int32_t)ints[10];
    cfg.sparse = (int32_t)ints[11];
    cfg.out_row_bytes = (int32_t)ints[12];
    cfg.pool_len = (int32_t)ints[14];
    cfg.stream_len = ints[15];
    cfg.lidar_range = (float)reals[0];
    cfg.loss_scale = (float)reals[1];
    cfg.loss_offset = (float)reals[2];
    cfg.branching_prob = reals[3];
    fill_ptrs(st, state, "LidarEnv state");
    fill_ptrs(out, outputs, "LidarEnv outputs");
    st.prefetcher = reinterpret_cast<void *>(static_cast<uintptr_t>(ints[13]));
    for (auto &t : state)
      if (t.defined() && t.numel() > 0) dev = t.device();
    keep = state;
    keep.insert(keep.end(), outputs.begin(), outputs.end());
  }
};

struct ImageEnv : torch::CustomClassHolder {
  apg_image_config cfg{};
  apg_image_state st{};
  apg_image_outputs out{};
  std::vector<at::Tensor> keep;
  at::Device dev = at::Device(at::kCUDA, 0);

  // ints: the 16 int32 fields of apg_image_config up to env_offset, pool_len, log_stats, sparse, out_row_bytes;
  // reals: sensor_scale, max_step[2], cell[2], ce_scale, ce_offset, mse_scale, mse_offset
  ImageEnv(std::vector<int64_t> ints, std::vector<double> reals, std::vector<at::Tensor> state,
           std::vector<at::Tensor> outputs) {
    TORCH_CHECK(ints.size() == 20 && reals.size() == 9, "ImageEnv: 20 ints and 9 reals expected");
    int32_t *f = &cfg.num_envs;  // num_envs .. env_offset: 16 consecutive int32 fields
    for (int i = 0; i < 16; i++) f[i] = (int32_t)ints[i];
    cfg.pool_len = ints[16];
    cfg.log_stats = (int32_t)ints[17];
    cfg.sparse = (int32_t)ints[18];
    cfg.out_row_bytes = (int32_t)ints[19];
    cfg.sensor_scale = reals[0];
    cfg.max_step[0] = reals[1];
    cfg.max_step[1] = reals[2];
    cfg.cell[0] = reals[3];
    cfg.cell[1] = reals[4];
    cfg.ce_scale = reals[5];
    cfg.ce_offset = reals[6];
    cfg.mse_scale = (float)reals[7];
    cfg.mse_offset = (float)reals[8];
    fill_ptrs(st, state, "ImageEnv state");
    fill_ptrs(out, outputs, "ImageEnv outputs");
    for (auto &t : state)
      if (t.defined() && t.numel() > 0) dev = t.device();
    keep = state;
    keep.insert(keep.end(), outputs.begin(), outputs.end());
  }
};
static_assert(offsetof(apg_image_config, env_offset) == 15 * sizeof(int32_t), "apg_image_config int32 prefix");

void lidar_reset(const c10::intrusive_ptr<LidarEnv> &e, int64_t seed, bool use_seed) {
  const c10::DeviceGuard guard(e->dev);
  check(apg_lidar_reset(&e->cfg, &e->st, (uint64_t)seed, use_seed ? 1 : 0, &e->out, stream_of(e->dev)),
        "apg_lidar_reset");
}

void lidar_step(const c10::intrusive_ptr<LidarEnv> &e, const at::Tensor &action, const at::Tensor &prediction) {
  const c10::DeviceGuard guard(e->dev);
  const int64_t n2 = 2 * (int64_t)e->cfg.num_envs;
  check_io(action, e->dev, n2, "action");
  check_io(prediction, e->dev, n2, "prediction");
  check(apg_lidar_step(&e->cfg, &e->st, action.data_ptr<float>(), prediction.data_ptr<float>(), &e->out,
                       stream_of(e->dev)),
        "apg_lidar_step");
}

void image_reset(const c10::intrusive_ptr<ImageEnv> &e) {
  const c10::DeviceGuard guard(e->dev);
  check(apg_image_reset(&e->cfg, &e->st, &e->out, stream_of(e->dev)), "apg_image_reset");
}

// prev_done: bit 0 the previous step terminated the batch, bit 1 its draws were made ahead (apg_image_step)
void image_step(const c10::intrusive_ptr<ImageEnv> &e, const at::Tensor &action, const at::Tensor &prediction,
                int64_t t, int64_t prev_done) {
  const c10::DeviceGuard guard(e->dev);
  const int64_t n = e->cfg.num_envs;
  check_io(action, e->dev, 2 * n, "action");
  const int64_t pw = e->cfg.kind == APG_IMAGE_CLASSIFY ? (int64_t)e->cfg.num_classes : 2;
  check_io(prediction, e->dev, pw * n, "prediction");
  check(apg_image_step(&e->cfg, &e->st, action.data_ptr<float>(), prediction.data_ptr<float>(), (int32_t)t,
                       (int32_t)prev_done, &e->out, stream_of(e->dev)),
        "apg_image_step");
}

}  // namespace

TORCH_LIBRARY(apgym, m) {
  m.class_<LidarEnv>("LidarEnv")
      .def(torch::init<std::vector<int64_t>, std::vector<double>, std::vector<at::Tensor>, std::vector<at::Tensor>>());
  m.class_<ImageEnv>("ImageEnv")
      .def(torch::init<std::vector<int64_t>, std::vector<double>, std::vector<at::Tensor>, std::vector<at::Tensor>>());
  m.def("lidar_reset(__torch__.torch.classes.apgym.LidarEnv env, int seed, bool use_seed) -> ()", lidar_reset);
  m.def("lidar_step(__torch__.torch.classes.apgym.LidarEnv env, Tensor action, Tensor prediction) -> ()", lidar_step);
  m.def("image_reset(__torch__.torch.classes.apgym.ImageEnv env) -> ()", image_reset);
  m.def("image_step(__torch__.torch.classes.apgym.ImageEnv env, Tensor action, Tensor prediction, int t, "
        "int prev_done) -> ()",
        image_step);
}
