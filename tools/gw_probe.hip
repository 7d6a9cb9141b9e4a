// Diagnostic (not part of the product): launch-level timings of the many-column surrogate
// kernels (k_gw_p, k_gw_grad) against the batch size B at S = 1M columns, to separate the
// per-row cost from fixed per-launch costs.
// hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o tools/gw_probe tools/gw_probe.hip
#include "../bikg_graph_explainability_public_amd/csrc/xpgnn.hip"

#include <cstdio>

int main() {
  const int64_t cols = 1000000, words = (cols + 31) / 32;
  const int maxB = 1024;
  uint32_t* bits;
  float *w, *m, *v, *g, *p_part;
  double* aw;
  WlmStep* stp;
  hipMalloc(&bits, (size_t)maxB * words * 4 * 8);
  hipMemset(bits, 0x5a, (size_t)maxB * words * 4 * 8);
  hipMalloc(&w, cols * 4);
  hipMalloc(&m, cols * 4);
  hipMalloc(&v, cols * 4);
  hipMemset(w, 0, cols * 4);
  hipMemset(m, 0, cols * 4);
  hipMemset(v, 0, cols * 4);
  hipMalloc(&g, maxB * 4);
  hipMemset(g, 0, maxB * 4);
  const int n_wg = static_cast<int>((words + kGwWords - 1) / kGwWords);
  hipMalloc(&p_part, (size_t)n_wg * maxB * 4);
  hipMalloc(&aw, (size_t)n_wg * 64 * 8);
  hipMalloc(&stp, sizeof(WlmStep) * 64);
  hipMemset(stp, 0, sizeof(WlmStep) * 64);
  xpg_wlm_params P{0.01f, 1e-4f, 0.9f, 0.999f, 1e-8f, 1e-2f};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int B : {32, 64, 128, 256, 512, 1024}) {
    const int64_t rows = (int64_t)B * 8;  // 8 steps, a fresh batch per launch
    const size_t lds_g = sizeof(float) * (size_t)(((16 * (((B + 31) / 32) * 8 | 1) + 3) & ~3) + 32 * 65);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gw_grad), hipFuncAttributeMaxDynamicSharedMemorySize,
                        static_cast<int>(lds_g));
    float tp = 0, tg = 0;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      for (int t = 0; t < 8; ++t)
        hipLaunchKernelGGL(k_gw_p, dim3(n_wg, 1), dim3(kGpWaves * 64), 0, 0, bits, rows, cols, words, B, t, w, p_part);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&tp, a, b);
      hipEventRecord(a);
      for (int t = 0; t < 8; ++t)
        hipLaunchKernelGGL(k_gw_grad, dim3(n_wg, 1), dim3(kGgWaves * 64), lds_g, 0, bits, rows, cols, words, B, t, g,
                           stp, (int64_t)8, P, w, m, v, aw);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&tg, a, b);
    }
    const double mb = (double)B * words * 4 / 1e6;
    printf("B=%5d  bits %7.1f MB  k_gw_p %8.2f us (%6.0f GB/s)  k_gw_grad %8.2f us (%6.0f GB/s)\n", B, mb,
           tp * 1e3 / 8, mb / (tp / 8), tg * 1e3 / 8, mb / (tg / 8));
  }
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
