// Diagnostic harness (not part of the product): per-phase cycle counts of k_wlm_fit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DXPG_WLM_STAMPS tools/wlm_probe.cpp -o /tmp/wlm_probe
#include "../bikg_graph_explainability_public_amd/csrc/xpgnn.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>


int main(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 1193, R = argc > 2 ? atoll(argv[2]) : 12800,
                batch = argc > 3 ? atoll(argv[3]) : 256;
  const int words = (int)((S + 31) / 32);
  std::mt19937 rng(0);
  std::vector<uint32_t> bits(R * words);
  for (auto& x : bits) x = rng();
  for (int64_t r = 0; r < R; ++r)
    if (S % 32) bits[r * words + words - 1] &= (1u << (S % 32)) - 1;
  std::vector<float> y(R), w(S, 0.f), z(S, 0.f);
  std::vector<double> k(R);
  for (auto& v : y) v = (rng() % 1000) / 1000.f;
  for (auto& v : k) v = 1e-3 * (1 + rng() % 100);
  uint32_t* d_bits; float *d_y, *d_w, *d_m, *d_v; double *d_k, *d_l; int32_t* d_b; void* ws;
  size_t wsb = 0;
  xpg_wlm_workspace(1, R, S, batch, &wsb);
  hipMalloc(&d_bits, bits.size() * 4); hipMalloc(&d_y, R * 4); hipMalloc(&d_k, R * 8);
  hipMalloc(&d_w, S * 4); hipMalloc(&d_m, S * 4); hipMalloc(&d_v, S * 4);
  hipMalloc(&d_l, (R / batch + 2) * 8); hipMalloc(&d_b, 4); hipMalloc(&ws, wsb);
  hipMemcpy(d_bits, bits.data(), bits.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_y, y.data(), R * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_k, k.data(), R * 8, hipMemcpyHostToDevice);
  xpg_wlm_params P{0.01f, 1e-4f, 0.9f, 0.999f, 1e-8f, 1e-2f};
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) {
    hipMemcpy(d_w, w.data(), S * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_m, z.data(), S * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_v, z.data(), S * 4, hipMemcpyHostToDevice);
    hipEventRecord(a, 0);
    int rc = xpg_wlm_fit(1, d_bits, R, S, batch, d_y, d_k, &P, 0, d_w, d_m, d_v, d_l, d_b, nullptr, ws, wsb, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    if (rc) printf("rc=%d %s\n", rc, xpg_last_error());
    uint64_t st[2][8];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_wlm_stamps), sizeof(st));
    const int64_t steps = (R + batch - 1) / batch;
    printf("S=%ld R=%ld batch=%ld: fit chain %.1f us (%.2f us/step); cycles/step per segment:\n", (long)S, (long)R,
           (long)batch, ms * 1e3, ms * 1e3 / steps);
    const bool mc = getenv("XPG_WLM") == nullptr || strcmp(getenv("XPG_WLM"), "single") != 0;
    const char* nm1[8] = {"B lookups", "syncA", "G + COLS_ST", "sync1", "D lookups", "syncD", "Adam+T+ROWS", "sync2"};
    const char* nm2[8] = {"B+publish", "stage issue", "poll+g+G", "bar1", "D+Adam+T", "stage store", "bar2", "plain path"};
    const char* const* nm = mc ? nm2 : nm1;
    for (int q = 0; q < 8; ++q) printf("  %-12s wave0 %8.0f  last %8.0f\n", nm[q], (double)st[0][q] / steps, (double)st[1][q] / steps);
  }
  return 0;
}
