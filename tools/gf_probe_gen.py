"""Generate tools/gf_probe.hip: the fused many-column fit kernel (k_gw_fused) cut out of
csrc/xpgnn.hip with the helpers it uses, plus a host main that times it at the c3
graph_prediction shape (S = 1M columns, 25,600 rows, batch 512) and prints per-phase
s_memtime cycles (-DXPG_GF_STAMPS).  Diagnostics only; the product kernel is the one in
xpgnn.hip.

    python tools/gf_probe_gen.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 \\
        -fno-slp-vectorize -DXPG_GF_STAMPS -o tools/gf_probe tools/gf_probe.hip
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "bikg_graph_explainability_public_amd", "csrc", "xpgnn.hip")
s = open(SRC).read()


def seg(start, end):
    i = s.index(start)
    return s[i:s.index(end, i)]


parts = ['#include <hip/hip_runtime.h>\n#include <cstdint>\n#include <cstdio>\n#include <cstdlib>\n'
         '#include <vector>\n#include "../include/xpgnn.h"\nnamespace {\n',
         seg("typedef float f32x2", "// Workgroup barrier that orders LDS only"),
         seg("__device__ __forceinline__ void lds_barrier()", "__device__ __forceinline__ bool bit_of"),
         seg("// In-register 32 x 32 bit transpose", "// ---------------------------------------------"
             "--------------------------------------- masks"),
         seg("struct WlmStep {", "// Also clears the multi"),
         seg("constexpr uint32_t kMcSpinLimit", "// WlmStep from the 12 dwords"),
         seg("constexpr int kGwWords", "// grid (n_chunks, n_fits), kGpWaves"),
         seg("// ------------------------------------------------------------ surrogate, fused many-column fit",
             "// Also hands the fit's status word"),
         "}  // namespace\n", r'''
__global__ void fill_bits(uint32_t* b, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    b[i] = x;
  }
}
#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)
int main(int argc, char** argv) {
  const int cols = argc > 1 ? atoi(argv[1]) : 1000000, rows = argc > 2 ? atoi(argv[2]) : 25600;
  const int batch = argc > 3 ? atoi(argv[3]) : 512, reps = argc > 4 ? atoi(argv[4]) : 3;
  const int words = (cols + 31) / 32, steps = (rows + batch - 1) / batch;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int n_chunks = (words + kGwWords - 1) / kGwWords;
  const int nrb = (batch + 31) / 32, nrbp = (nrb + kGfTpw - 1) / kGfTpw * kGfTpw;
  const int ch = (n_chunks + cus - 1) / cus, nwg = (n_chunks + ch - 1) / ch;
  const GfLds L = gf_lds(ch, nrbp);
  size_t lds = sizeof(float) * L.total + 2 * kGfWaves * sizeof(double) + sizeof(double);
  if (lds < 81 * 1024) lds = 81 * 1024;
  printf("cols %d rows %d batch %d steps %d: ch %d nrbp %d nwg %d lds %zu\n", cols, rows, batch, steps, ch, nrbp, nwg, lds);
  uint32_t* bits; double* kern; WlmStep* stp; float *w, *m, *v, *ph; double *tk, *aw; uint64_t* xp; uint32_t* err;
  CK(hipMalloc(&bits, sizeof(uint32_t) * (size_t)rows * words));
  CK(hipMalloc(&kern, sizeof(double) * rows));
  CK(hipMalloc(&stp, sizeof(WlmStep) * steps));
  CK(hipMalloc(&w, 4 * (size_t)cols)); CK(hipMalloc(&m, 4 * (size_t)cols)); CK(hipMalloc(&v, 4 * (size_t)cols));
  CK(hipMalloc(&ph, 4 * (size_t)rows));
  CK(hipMalloc(&tk, 8 * (size_t)steps * nwg)); CK(hipMalloc(&aw, 8 * (size_t)steps * nwg));
  const size_t n_xp = (size_t)batch * ((size_t)nwg + 1);  // [batch][workgroup slots] + g granules
  CK(hipMalloc(&xp, 8 * n_xp)); CK(hipMalloc(&err, 4));
  hipLaunchKernelGGL(fill_bits, dim3(4096), dim3(256), 0, 0, bits, (size_t)rows * words, 7u);
  std::vector<double> hk(rows, 1e-3);
  CK(hipMemcpy(kern, hk.data(), 8 * rows, hipMemcpyHostToDevice));
  std::vector<WlmStep> hs(steps);
  for (int t = 0; t < steps; ++t) {
    WlmStep& q = hs[t];
    q.ybar = 0.5; q.ksum = batch * 1e-3; q.vy = 1.0; q.cg = 2.0 / (batch * q.ksum);
    q.step_size = 0.01f; q.bc2_sqrt = 0.05f; q.inv_bc2 = 20.f; q.pad = 0.f;
  }
  CK(hipMemcpy(stp, hs.data(), sizeof(WlmStep) * steps, hipMemcpyHostToDevice));
  hipFuncAttributes fa;
  CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_gw_fused)));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gw_fused), hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024 - static_cast<int>(fa.sharedSizeBytes)));
  GfArgs a;
  a.bits = bits; a.kern = kern; a.stp = stp; a.wg = w; a.mg = m; a.vg = v; a.p_hist = ph; a.tk_part = tk;
  a.aw_part = aw; a.xp = xp; a.err = err;
  a.P.lr = 0.01f; a.P.beta1 = 0.9f; a.P.beta2 = 0.999f; a.P.eps = 1e-8f; a.P.weight_decay = 1e-2f; a.P.l1_lambda = 1e-4f;
  a.rows = rows; a.cols = cols; a.words = words; a.steps = steps; a.batch = batch; a.ch = ch; a.nrbp = nrbp;
  a.nwg = nwg; a.fault_wg = -1; a.spin_limit = kMcSpinLimit;
#ifdef XPG_GF_STAMPS
  a.dbg = argc > 5 ? atoi(argv[5]) : 0;
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < reps; ++r) {
    CK(hipMemset(w, 0, 4 * (size_t)cols)); CK(hipMemset(m, 0, 4 * (size_t)cols)); CK(hipMemset(v, 0, 4 * (size_t)cols));
    CK(hipMemset(xp, 0, 8 * n_xp)); CK(hipMemset(err, 0, 4));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_gw_fused, dim3(nwg), dim3(kGfThreads), lds, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t he = 0;
    CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
#ifdef XPG_GF_STAMPS
    std::vector<uint64_t> st(1024 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_gf_stamps), sizeof(uint64_t) * 1024 * 8));
    double ph8[8] = {0};
    for (int g = 0; g < nwg; ++g) for (int i = 0; i < 8; ++i) ph8[i] += st[g * 8 + i] / (double)nwg / steps;
    printf("rep %d: %.3f ms (%.2f us/step) err %u | cycles/step: p1 %.0f reduce %.0f gpoll %.0f Gbuild %.0f p3 %.0f tree %.0f adam %.0f wtab %.0f\n",
           r, ms, 1e3 * ms / steps, he, ph8[0], ph8[1], ph8[2], ph8[3], ph8[4], ph8[5], ph8[6], ph8[7]);
#else
    printf("rep %d: %.3f ms (%.2f us/step) err %u\n", r, ms, 1e3 * ms / steps, he);
#endif
  }
  return 0;
}
''']
open(os.path.join(HERE, "gf_probe.hip"), "w").write("".join(parts))
