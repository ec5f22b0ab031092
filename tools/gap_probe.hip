// Inter-dispatch gap probe (tuning tool, not product code): back-to-back launches of a kernel that writes
// `mb` MB with ordinary or non-temporal stores (or only reads them), wall time per launch from hipEvents
// around the whole loop; run under rocprofv3 --kernel-trace to split wall into kernel duration + gap.
//   hipcc --offload-arch=gfx950 -O3 tools/gap_probe.hip -o tools/gap_probe && tools/gap_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0: ordinary stores, 1: non-temporal stores, 2: reads only, 3: nothing
__global__ __launch_bounds__(256) void k_probe(f4 *buf, size_t n, float v, float *sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  f4 acc = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (MODE == 0) buf[i] = f4{v, v, v, v};
    if constexpr (MODE == 1) __builtin_nontemporal_store(f4{v, v, v, v}, buf + i);
    if constexpr (MODE == 2) acc += buf[i];
  }
  if constexpr (MODE == 2)
    if (acc.x == 12345.0f) sink[0] = acc.y;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int MODE>
double run(f4 *buf, size_t n, float *sink, int reps, hipStream_t s) {
  const int grid = 256 * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 10; i++) k_probe<MODE><<<grid, 256, 0, s>>>(buf, n, (float)i, sink);
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; i++) k_probe<MODE><<<grid, 256, 0, s>>>(buf, n, (float)i, sink);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1000.0 * ms / reps;
}

int main() {
  const int reps = 200;
  const size_t mbs[] = {0, 1, 8, 24, 64};
  f4 *buf;
  float *sink;
  CK(hipMalloc(&buf, (size_t)64 << 20));
  CK(hipMalloc(&sink, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char *names[] = {"store", "nt_store", "read", "empty"};
  for (size_t mb : mbs) {
    const size_t n = (mb << 20) / sizeof(f4);
    double us[4] = {run<0>(buf, n, sink, reps, s), run<1>(buf, n, sink, reps, s), run<2>(buf, n, sink, reps, s),
                    run<3>(buf, n, sink, reps, s)};
    for (int m = 0; m < 4; m++) printf("{\"mb\": %zu, \"mode\": \"%s\", \"us_per_launch\": %.2f}\n", mb, names[m], us[m]);
  }
  return 0;
}
