// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns the
// backend's kernels use (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a 16-B/lane streaming read; other widths
// are uncalibrated).  Each kernel moves a known number of bytes over a 1 GiB buffer (past the 256 MiB Infinity
// Cache, which a 1 GiB streaming kernel evicts between patterns) and is run once:
//   k_stream16  16 B per lane, coalesced, every byte once          (the guide's reference pattern)
//   k_stream8    8 B per lane, coalesced (state loads, occupancy rows of one env read by consecutive lanes)
//   k_stream4    4 B per lane, coalesced
//   k_seg256_8   8 B per lane, half a wave per 256-B segment, segments in a bijective hashed order
//                (k_lidar_step's 32-row occupancy windows: 32 lanes x 8 B of one env's rows)
//   k_seg64_4    4 B per lane, 16 lanes per 64-B segment, hashed order (u8 glimpse taps: dword row gathers)
//   k_store16 / k_store8 / k_store4   coalesced stores of every byte once
// Each read kernel also writes one dword per wave (64 MiB / 16 / ... of the buffer: tiny, listed as
// known_write).  The program prints one JSON line with the known bytes per kernel; tools/fetch_calib.py joins
// it with the PMC pass (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE) into profiles/<round>/fetch_calibration.json.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr size_t kBytes = (size_t)1 << 30;  // 1 GiB per pattern

__global__ void k_stream16(const uint4 *__restrict__ src, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = acc;
}

__global__ void k_stream8(const uint64_t *__restrict__ src, size_t n, uint32_t *out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[i];
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = (uint32_t)(acc ^ (acc >> 32));
}

__global__ void k_stream4(const uint32_t *__restrict__ src, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[i];
  if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = acc;
}

// segment s of `nseg` (a power of two) -> a bijective hash of it: odd multiplier and xor-shift mod 2^k
__device__ inline uint32_t seg_hash(uint32_t s, uint32_t mask) {
  s = (s * 2654435761u) & mask;
  s ^= s >> 7;
  return (s * 2246822519u) & mask;
}

// one thread per 8-B word: 32 lanes per 256-B segment, segment order hashed
__global__ void k_seg256_8(const uint64_t *__restrict__ src, uint32_t nseg, uint32_t *out) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const uint32_t seg = (uint32_t)(t >> 5), lane = (uint32_t)(t & 31);
  uint64_t v = 0;
  if (seg < nseg) v = src[(size_t)seg_hash(seg, nseg - 1) * 32 + lane];
  if ((threadIdx.x & 63) == 0) out[t >> 6] = (uint32_t)(v ^ (v >> 32));
  else if (v == 0x0123456789abcdefULL) out[t >> 6] = 1u;  // keeps every load live
}

// one thread per dword: 16 lanes per 64-B segment, segment order hashed
__global__ void k_seg64_4(const uint32_t *__restrict__ src, uint32_t nseg, uint32_t *out) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const uint32_t seg = (uint32_t)(t >> 4), lane = (uint32_t)(t & 15);
  uint32_t v = 0;
  if (seg < nseg) v = src[(size_t)seg_hash(seg, nseg - 1) * 16 + lane];
  if ((threadIdx.x & 63) == 0) out[t >> 6] = v;
  else if (v == 0x89abcdefu) out[t >> 6] = 1u;
}

template <class T>
__global__ void k_store(T *dst, size_t n, T v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = v;
}
__global__ void k_store16(uint4 *dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void k_evict(uint4 *dst, size_t n) {  // streams another 1 GiB between patterns (Infinity Cache)
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4(0u, 0u, 0u, (uint32_t)i);
}

int main() {
  uint8_t *buf, *ev;
  uint32_t *out;
  CHECK(hipMalloc(&buf, kBytes));
  CHECK(hipMalloc(&ev, kBytes));
  CHECK(hipMalloc(&out, kBytes / 16));
  const int grid = 256 * 8, block = 256;  // 8 workgroups per CU, grid-stride
  auto evict = [&]() { hipLaunchKernelGGL(k_evict, dim3(grid), dim3(block), 0, 0, (uint4 *)ev, kBytes / 16); };
  hipLaunchKernelGGL(k_store16, dim3(grid), dim3(block), 0, 0, (uint4 *)buf, kBytes / 16);  // initialise
  const size_t waves_stream = (size_t)grid * block / 64;
  evict();
  hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(block), 0, 0, (const uint4 *)buf, kBytes / 16, out);
  evict();
  hipLaunchKernelGGL(k_stream8, dim3(grid), dim3(block), 0, 0, (const uint64_t *)buf, kBytes / 8, out);
  evict();
  hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(block), 0, 0, (const uint32_t *)buf, kBytes / 4, out);
  evict();
  const uint32_t nseg256 = (uint32_t)(kBytes / 256), nseg64 = (uint32_t)(kBytes / 64);
  hipLaunchKernelGGL(k_seg256_8, dim3((unsigned)(kBytes / 8 / block)), dim3(block), 0, 0, (const uint64_t *)buf,
                     nseg256, out);
  evict();
  hipLaunchKernelGGL(k_seg64_4, dim3((unsigned)(kBytes / 4 / block)), dim3(block), 0, 0, (const uint32_t *)buf,
                     nseg64, out);
  evict();
  hipLaunchKernelGGL(k_store16, dim3(grid), dim3(block), 0, 0, (uint4 *)buf, kBytes / 16);
  evict();
  hipLaunchKernelGGL(k_store<uint64_t>, dim3(grid), dim3(block), 0, 0, (uint64_t *)buf, kBytes / 8, (uint64_t)7);
  evict();
  hipLaunchKernelGGL(k_store<uint32_t>, dim3(grid), dim3(block), 0, 0, (uint32_t *)buf, kBytes / 4, 7u);
  CHECK(hipDeviceSynchronize());
  const size_t w8 = kBytes / 8 / 64 * 4, w4 = kBytes / 4 / 64 * 4;  // seg kernels: one dword per wave
  printf("{\"bytes\": %zu, \"known\": {"
         "\"k_stream16\": {\"read\": %zu, \"write\": %zu}, \"k_stream8\": {\"read\": %zu, \"write\": %zu}, "
         "\"k_stream4\": {\"read\": %zu, \"write\": %zu}, \"k_seg256_8\": {\"read\": %zu, \"write\": %zu}, "
         "\"k_seg64_4\": {\"read\": %zu, \"write\": %zu}, \"k_store16\": {\"read\": 0, \"write\": %zu}, "
         "\"k_store8\": {\"read\": 0, \"write\": %zu}, \"k_store4\": {\"read\": 0, \"write\": %zu}, "
         "\"k_evict\": {\"read\": 0, \"write\": %zu}}}\n",
         kBytes, kBytes, waves_stream * 4, kBytes, waves_stream * 4, kBytes, waves_stream * 4, kBytes, w8, kBytes, w4,
         kBytes, kBytes, kBytes, kBytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(ev));
  CHECK(hipFree(out));
  return 0;
}
