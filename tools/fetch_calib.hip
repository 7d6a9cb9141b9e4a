// Diagnostic (not part of the product): calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against known
// byte counts for the access shapes of the engine's kernels (MI355X_MICROARCH.md: the 2x FETCH
// correction is measured for wide coalesced streaming reads only; other widths uncalibrated).
// Every kernel below touches an exactly known number of bytes, once, from a buffer far larger
// than the 256 MiB Infinity Cache; the summary line per kernel gives the bytes it moved, and
// FETCH_SIZE x 1024 / bytes (from the PMC pass) is that shape's counter factor.
//   stream16   coalesced 16 B / lane streaming read (the guide's calibrated shape)
//   stream4    coalesced 4 B / lane streaming read (narrow lane = word loads: k_gw_p / k_gw_grad)
//   rows512    random 512-B rows, 16 lanes x 2 float4 per row (k_wide_last_ws / k_wide_tgt gathers)
//   rows512w   random 512-B rows, one wave x 2 float4 per lane-pair... (64 lanes x 8 B: k_wide_l1s)
//   word4      random 4-B words, one per lane (keep words mT0[u], CSR entries)
//   wstream16  coalesced 16 B / lane streaming store
//   wrows512   random 512-B rows stored, 16 lanes x 2 float4 per row (h1 tiles)
// hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
// rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d OUT -o run -- ./tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

__global__ __launch_bounds__(256) void stream16(const float4* __restrict__ a, int64_t n, float* out) {
  float s = 0.f;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(256) void stream4(const uint32_t* __restrict__ a, int64_t n, float* out) {
  uint32_t s = 0;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s ^= a[i];
  if (s == 0x12345u) out[0] = 1.f;
}

// nrows random rows of 128 floats (512 B) from a table of n_tab rows; 16-lane group = one row
__global__ __launch_bounds__(256) void rows512(const float* __restrict__ tab, int64_t n_tab, int64_t nrows,
                                               float* out) {
  const int gl = threadIdx.x & 15;
  float s = 0.f;
  for (int64_t r = (blockIdx.x * 256LL + threadIdx.x) >> 4; r < nrows; r += (int64_t)gridDim.x * 16) {
    const int64_t row = mix(r * 0x9E3779B97F4A7C15ULL + 7) % n_tab;
    const float4* p = reinterpret_cast<const float4*>(tab + row * 128) + gl * 2;
    const float4 u = p[0], v = p[1];
    s += u.x + u.y + u.z + u.w + v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}

// nrows random rows of 128 floats, one wave per row, 2 floats (8 B) per lane
__global__ __launch_bounds__(256) void rows512w(const float* __restrict__ tab, int64_t n_tab, int64_t nrows,
                                                float* out) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int64_t r = (blockIdx.x * 256LL + threadIdx.x) >> 6; r < nrows; r += (int64_t)gridDim.x * 4) {
    const int64_t row = mix(r * 0x9E3779B97F4A7C15ULL + 11) % n_tab;
    const float2 u = reinterpret_cast<const float2*>(tab + row * 128)[lane];
    s += u.x + u.y;
  }
  if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(256) void word4(const uint32_t* __restrict__ a, int64_t n, int64_t nreads, float* out) {
  uint32_t s = 0;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < nreads; i += (int64_t)gridDim.x * 256)
    s ^= a[mix(i * 0x9E3779B97F4A7C15ULL + 3) % n];
  if (s == 0x12345u) out[0] = 1.f;
}

__global__ __launch_bounds__(256) void wstream16(float4* __restrict__ a, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

// nrows DISTINCT rows (a bijection of the first nrows rows), 16-lane group = one row
__global__ __launch_bounds__(256) void wrows512(float* __restrict__ tab, int64_t nrows) {
  const int gl = threadIdx.x & 15;
  for (int64_t r = (blockIdx.x * 256LL + threadIdx.x) >> 4; r < nrows; r += (int64_t)gridDim.x * 16) {
    const int64_t row = (r * 2654435761LL) % nrows;  // nrows odd and coprime: a permutation
    float4* p = reinterpret_cast<float4*>(tab + row * 128) + gl * 2;
    p[0] = make_float4(1.f, 2.f, 3.f, 4.f);
    p[1] = make_float4(5.f, 6.f, 7.f, 8.f);
  }
}

int main() {
  const int64_t big = 8LL << 30;  // 8 GiB buffer
  char* buf = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&buf, big));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, big));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 16;
  const int64_t n_tab = big / 512;
  const int64_t nrows = 4LL << 20;        // 4 Mi random rows = 2 GiB
  const int64_t wrows = (4LL << 20) + 1;  // odd
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), (int64_t)(2LL << 30) / 16, out);
    hipLaunchKernelGGL(stream4, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(buf), (int64_t)(2LL << 30) / 4, out);
    hipLaunchKernelGGL(rows512, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const float*>(buf), n_tab, nrows, out);
    hipLaunchKernelGGL(rows512w, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const float*>(buf), n_tab, nrows, out);
    hipLaunchKernelGGL(word4, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(buf), big / 4, (int64_t)(64LL << 20), out);
    hipLaunchKernelGGL(wstream16, dim3(grid), dim3(256), 0, 0, reinterpret_cast<float4*>(buf), (int64_t)(2LL << 30) / 16);
    hipLaunchKernelGGL(wrows512, dim3(grid), dim3(256), 0, 0, reinterpret_cast<float*>(buf), wrows);
    CK(hipDeviceSynchronize());
  }
  printf("bytes stream16 %lld stream4 %lld rows512 %lld rows512w %lld word4 %lld (64-B sectors: %lld) "
         "wstream16 %lld wrows512 %lld\n",
         2LL << 30, 2LL << 30, nrows * 512, nrows * 512, (64LL << 20) * 4, (64LL << 20) * 64, 2LL << 30,
         wrows * 512);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
