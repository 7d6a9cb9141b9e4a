// Diagnostic (not part of the product): HBM read rate of the access shapes the many-column
// surrogate fit can use on a [rows][words] uint32 bit matrix (one 512-row step batch).
//   slab<SW>: workgroup = SW-word column slab x 512 rows, lane = word, 32 rows per load round
//   contig  : workgroup = one contiguous 128 KB block
// hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip && ./tools/bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <int SW>
__global__ __launch_bounds__(512) void slab(const uint32_t* __restrict__ bits, int64_t words, int rows,
                                            uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * SW;
  uint32_t acc = 0;
  for (int sw = 0; sw < SW / 64; ++sw) {
    const int64_t wd = w0 + sw * 64 + lane;
    if (wd >= words) break;
    for (int rb = wave; rb * 32 < rows; rb += 8) {
      uint32_t x[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) x[i] = bits[(int64_t)(rb * 32 + i) * words + wd];
#pragma unroll
      for (int i = 0; i < 32; ++i) acc ^= x[i] * (i + 1);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(512) void contig(const uint4* __restrict__ p, int64_t n4, uint32_t* __restrict__ out) {
  const int64_t per = 128 * 1024 / 16;  // uint4 per workgroup
  const int64_t base = (int64_t)blockIdx.x * per;
  uint32_t acc = 0;
  for (int64_t i = threadIdx.x; i < per; i += 512 * 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = base + i + u * 512;
      v[u] = k < n4 ? p[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int rows = 512;
  const int64_t words = 31250;
  const int64_t n = (int64_t)rows * words;
  uint32_t *bits, *out;
  hipMalloc(&bits, n * 4 * 50);  // 50 step batches: a fresh batch per launch (no cache reuse)
  hipMalloc(&out, 64);
  hipMemset(bits, 0x5a, n * 4 * 50);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int s = 0; s < 5; ++s) launch(s);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int s = 0; s < 50; ++s) launch(s);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-10s %8.2f us/launch  %7.0f GB/s\n", name, ms * 1e3 / 50, n * 4.0 / (ms * 1e-3 / 50) / 1e9);
  };
  run("slab64", [&](int s) { slab<64><<<dim3((words + 63) / 64), 512>>>(bits + s * n, words, rows, out); });
  run("slab128", [&](int s) { slab<128><<<dim3((words + 127) / 128), 512>>>(bits + s * n, words, rows, out); });
  run("slab256", [&](int s) { slab<256><<<dim3((words + 255) / 256), 512>>>(bits + s * n, words, rows, out); });
  run("contig", [&](int s) {
    const int64_t n4 = n / 4;
    contig<<<dim3((n * 4 + 128 * 1024 - 1) / (128 * 1024)), 512>>>(reinterpret_cast<const uint4*>(bits + s * n), n4, out);
  });
  return 0;
}
