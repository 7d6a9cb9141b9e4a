// Diagnostic (not part of the product): the HBM read rate of the c3 layer-2 access shape, i.e.
// the ceiling k_wide_last_ws's gathers run against.  Layer 2 reads, per
// target and sample, the 512-B h1 row [node][sample][128 fp32] of each kept in-edge's source:
// random rows of a 16 GB node-major buffer, one 16-lane group per sample, up to RP rows in flight
// per group.  Here the row ids come from a hash (no index traffic), every loaded dword is summed
// (no dead loads), and each variant reads the same bytes:
//   rows<RB, RP>   : random RB-byte rows, a 16-lane group per row stream, RP rows in flight
//   stream         : the same buffer read contiguously, 16 B per lane (the streaming rate)
// Grid: G workgroups of 512 threads (8 waves = 32 groups), persistent over the rows.
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_probe tools/gather_probe.hip && ./tools/gather_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// RB bytes per row (512: the layer-2 h1 row), RP rows in flight per 16-lane group
template <int RB, int RP>
__global__ __launch_bounds__(512) void rows(const float4* __restrict__ buf, int64_t nrows_buf, int64_t total,
                                            uint32_t seed, float* __restrict__ out) {
  constexpr int V = RB / 16 / 16;  // float4 per lane per row
  const int lane16 = threadIdx.x & 15;
  const int64_t group = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 4);
  const int64_t groups = (int64_t)gridDim.x * 32;
  float acc = 0.f;
  for (int64_t r0 = group * RP; r0 < total; r0 += groups * RP) {
    float4 v[RP][V];
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const uint32_t h = mix(static_cast<uint32_t>(r0 + j) ^ seed);
      const int64_t row = (int64_t)(h % static_cast<uint32_t>(nrows_buf));
      const float4* p = buf + row * (RB / 16) + lane16;
#pragma unroll
      for (int u = 0; u < V; ++u) v[j][u] = p[u * 16];
    }
#pragma unroll
    for (int j = 0; j < RP; ++j)
#pragma unroll
      for (int u = 0; u < V; ++u) acc += v[j][u].x + v[j][u].y + v[j][u].z + v[j][u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ void fill(float4* p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = mix(static_cast<uint32_t>(i));
    p[i] = make_float4(h * 1e-9f, (h >> 3) * 1e-9f, (h >> 7) * 1e-9f, (h >> 11) * 1e-9f);
  }
}

__global__ __launch_bounds__(512) void stream(const float4* __restrict__ p, int64_t n4, float* __restrict__ out) {
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 512;
  for (int64_t i = (int64_t)blockIdx.x * 512 + threadIdx.x; i < n4; i += stride * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = i + u * stride;
      v[u] = k < n4 ? p[k] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const int64_t bytes = 16LL << 30;  // the c3 h1 buffer: 1M nodes x 32 samples x 512 B
  float4* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  fill<<<4096, 256>>>(buf, bytes / 16);  // random-looking values (a zero buffer can clock differently)
  hipDeviceSynchronize();
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int64_t read = 8LL << 30;  // bytes read per launch
  auto run = [&](const char* name, int grid, auto launch) {
    launch(grid, 1u);
    hipDeviceSynchronize();
    const int reps = 3;
    hipEventRecord(a);
    for (int s = 0; s < reps; ++s) launch(grid, 7u + s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-22s grid %5d  %8.3f ms/launch  %7.0f GB/s\n", name, grid, ms / reps, read / (ms * 1e-3 / reps) / 1e9);
    fflush(stdout);
  };
#define ROWS(RB, RP, G)                                                                                     \
  run("rows<" #RB "," #RP ">", (G), [&](int g, uint32_t seed) {                                               \
    rows<RB, RP><<<g, 512>>>(buf, bytes / (RB), read / (RB), seed, out);                                      \
  })
  for (int per : {1, 2}) {
    const int G = cus * per;
    ROWS(512, 1, G);
    ROWS(512, 2, G);
    ROWS(512, 4, G);
    ROWS(512, 8, G);
    ROWS(512, 16, G);
    ROWS(1024, 4, G);
    ROWS(2048, 2, G);
    ROWS(256, 8, G);
    run("stream", G, [&](int g, uint32_t) { stream<<<g, 512>>>(buf, read / 16, out); });
  }
  return 0;
}
