// maze_bench.hip — tuning tool (not shipped): times the parts of apg_maze.hpp's generator on BASELINE config 3
// (262144 mazes of 127 x 127) in isolation, with HIP events:
//   k_stream the precomputed random stream of every maze (one thread per item, as k_maze_stream)
//   k_dfs    the DFS of every maze (vis / ring / log / spills), logs left in scratch: the general-width path
//            (maze_dfs_words) and the ncx <= 63 path (maze_dfs_rows), whose logs must agree (FNV hash per maze)
//   k_paint  each maze's occupancy rows painted from its log (one wave paints its 64 mazes in turn)
// and runs each twice (the second time is reported).  For PMC passes: rocprofv3 --pmc ... -- tools/maze_bench
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I active-perception-gym_amd/csrc \
//       -o tools/maze_bench tools/maze_bench.hip
//   tools/maze_bench [num_mazes] [size] [lanes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "apg_maze.hpp"

using namespace apg;

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ __launch_bounds__(256) void k_stream(int n, int h, int w, uint8_t *scratch, int ng) {
  const int nitems = ng / MZ_ITEM_GROUPS;
  const long q = blockIdx.x * 256L + threadIdx.x;
  if (q >= (long)n * nitems) return;
  const int i = (int)(q / nitems), c = (int)(q % nitems);
  const Pcg64 r = seed_pcg64((uint64_t)i * 2654435761ULL + 12345ULL);
  const MzJump j = mz_jump((uint64_t)c * MZ_ITEM_GROUPS * MZ_GROUP);
  maze_stream_item(r.s_hi, r.s_lo, r.i_hi, r.i_lo, j, 1.0, c, scratch + (size_t)i * maze_scratch_bytes(h, w) +
                   maze_stream_off(h, w), ng);
}

// V = 1: maze_dfs_rows (the shipped path for ncx <= 63); V = 0: maze_dfs_words (the general path) on the same
// mazes, as the A/B reference: both must write the same carve logs
template <int V>
__global__ __launch_bounds__(64) void k_dfs(int n, int h, int w, uint8_t *scratch, int *nlog, int lanes, int ng) {
  extern __shared__ uint64_t s_mz[];
  const int lane = threadIdx.x, i = blockIdx.x * lanes + lane;
  const bool active = lane < lanes && i < n;
  const MazeGeom m = maze_geom(h, w);
  const size_t sb = maze_scratch_bytes(h, w), lb = maze_log_bytes(h, w);
  Pcg64 r{};
  if (active) r = seed_pcg64((uint64_t)i * 2654435761ULL + 12345ULL);
  uint8_t *my = scratch + (size_t)(active ? i : 0) * sb;
  char *lds = reinterpret_cast<char *>(s_mz);
  maze_table_init<V == 1>(lds, lane);
  __syncthreads();
  bool bad = false;
  const int nl = V == 1 ? maze_dfs_rows<true>(r, my + maze_stream_off(h, w), ng, active, m, 1.0, lds, lane, my + lb,
                                        reinterpret_cast<uint32_t *>(my), bad)
                        : maze_dfs_words(r, my + maze_stream_off(h, w), ng, active, m, 1.0, lds, lane, my + lb,
                                         reinterpret_cast<uint32_t *>(my), bad);
  if (active) nlog[i] = bad ? -1 : nl;
}

// per-maze FNV-1a of the carve log (nlog entries), entries decoded to (x, y, direction): the two paths log in
// their own formats (cx | cy << 7 | d << 14, resp. pos | d << 13 with pos = cy * 64 + cx)
__global__ void k_loghash(int n, int h, int w, const uint8_t *scratch, const int *nlog, uint64_t *hash, int rows_fmt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint16_t *lg = reinterpret_cast<const uint16_t *>(scratch + (size_t)i * maze_scratch_bytes(h, w));
  uint64_t x = 1469598103934665603ULL;
  for (int e = 0; e < nlog[i]; e++) {
    const uint32_t v = lg[e];
    const uint32_t c = v == MZ_LOG_PAD ? 0xFFFFFFFFu
                       : rows_fmt ? (v & 63u) | (((v >> 6) & 127u) << 7) | ((v >> 13) << 14) : v;
    x = (x ^ c) * 1099511628211ULL;
  }
  hash[i] = x ^ (uint64_t)nlog[i];
}

__global__ __launch_bounds__(64) void k_paint(int n, int h, int w, const uint8_t *scratch, const int *nlog,
                                              uint64_t *occ, float *mo, int lanes) {
  extern __shared__ uint64_t s_mz[];
  const int lane = threadIdx.x;
  const MazeGeom m = maze_geom(h, w);
  const int wpr = (w + 63) / 64;
  const size_t sb = maze_scratch_bytes(h, w);
  for (int j = 0; j < lanes; j++) {
    const int e = blockIdx.x * lanes + j;
    if (e >= n) break;
    maze_paint(m, wpr, reinterpret_cast<const uint32_t *>(scratch + (size_t)e * sb), nlog[e], s_mz, lane);
    for (int y = lane; y < h; y += 64)
      for (int k = 0; k < wpr; k++) occ[((size_t)e * h + y) * wpr + k] = s_mz[y * wpr + k];
    if (mo) bitmap_map_obs(s_mz, h, w, wpr, mo + (size_t)e * h * w, lane, s_mz + h * wpr);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 262144;
  const int size = argc > 2 ? atoi(argv[2]) : 127;
  const int lanes = argc > 3 ? atoi(argv[3]) : 64;
  const size_t sb = maze_scratch_bytes(size, size);
  const int wpr = (size + 63) / 64;
  const MazeGeom mg = maze_geom(size, size);
  if (!maze_onew(mg)) {
    fprintf(stderr, "maze_bench compares the ncx <= 63 path: size <= 127\n");
    return 1;
  }
  uint8_t *scratch;
  int *nlog;
  uint64_t *occ, *hash;
  float *mo;
  CHECK(hipMalloc(&scratch, (size_t)n * sb));
  CHECK(hipMalloc(&mo, (size_t)n * size * size * sizeof(float)));
  CHECK(hipMalloc(&nlog, (size_t)n * sizeof(int)));
  CHECK(hipMalloc(&hash, (size_t)2 * n * sizeof(uint64_t)));
  CHECK(hipMalloc(&occ, (size_t)n * size * wpr * 8));
  const size_t lds = maze_wg_lds_bytes(size, size);
  const size_t lds_p = ((size_t)size * wpr + bitmap_lin_words(size, size)) * 8;
  CHECK(hipFuncSetAttribute((const void *)k_dfs<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHECK(hipFuncSetAttribute((const void *)k_dfs<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int occ0 = 0, occ1 = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, (const void *)k_dfs<0>, 64, lds));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, (const void *)k_dfs<1>, 64, lds));
  hipEvent_t a, b, c;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventCreate(&c));
  const int grid = (n + lanes - 1) / lanes;
  float t_dfs[2] = {0, 0}, t_paint = 0, t_obs = 0, t_stream = 0;
  const int ng = maze_stream_groups(size, size);
  const long items = (long)n * (ng / MZ_ITEM_GROUPS);
  for (int rep = 0; rep < 2; rep++) {
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_stream, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, 0, n, size, size, scratch, ng);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&t_stream, a, b));
    for (int v = 0; v < 2; v++) {
      CHECK(hipEventRecord(a, 0));
      if (v == 0)
        hipLaunchKernelGGL(k_dfs<0>, dim3(grid), dim3(64), lds, 0, n, size, size, scratch, nlog, lanes, ng);
      else
        hipLaunchKernelGGL(k_dfs<1>, dim3(grid), dim3(64), lds, 0, n, size, size, scratch, nlog, lanes, ng);
      CHECK(hipEventRecord(b, 0));
      hipLaunchKernelGGL(k_loghash, dim3((n + 255) / 256), dim3(256), 0, 0, n, size, size, scratch, nlog,
                         hash + (size_t)v * n, v);
      CHECK(hipEventSynchronize(b));
      CHECK(hipEventElapsedTime(&t_dfs[v], a, b));
    }
    CHECK(hipEventRecord(b, 0));
    hipLaunchKernelGGL(k_paint, dim3(grid), dim3(64), lds_p, 0, n, size, size, scratch, nlog, occ, (float *)nullptr,
                       lanes);
    CHECK(hipEventRecord(c, 0));
    CHECK(hipEventSynchronize(c));
    CHECK(hipEventElapsedTime(&t_paint, b, c));
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_paint, dim3(grid), dim3(64), lds_p, 0, n, size, size, scratch, nlog, occ, mo, lanes);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&t_obs, a, b));
  }
  uint64_t *hh = (uint64_t *)malloc((size_t)2 * n * sizeof(uint64_t));
  CHECK(hipMemcpy(hh, hash, (size_t)2 * n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  int diff = 0, first = -1;
  for (int i = 0; i < n; i++)
    if (hh[i] != hh[n + i]) {
      diff++;
      if (first < 0) first = i;
    }
  int nl0 = 0;
  CHECK(hipMemcpy(&nl0, nlog, sizeof(int), hipMemcpyDeviceToHost));
  printf("{\"mazes\": %d, \"size\": %d, \"lanes\": %d, \"lds_per_wg\": %zu, \"wg_per_cu\": [%d, %d], "
         "\"stream_ms\": %.3f, \"dfs_words_ms\": %.3f, \"dfs_rows_ms\": %.3f, \"paint_ms\": %.3f, "
         "\"paint_map_obs_ms\": %.3f, \"log0\": %d, \"log_mismatch\": %d, \"first_mismatch\": %d}\n",
         n, size, lanes, lds, occ0, occ1, t_stream, t_dfs[0], t_dfs[1], t_paint, t_obs, nl0, diff, first);
  free(hh);
  return diff ? 2 : 0;
}
