// Diagnostic (not part of the product): where the many-column surrogate kernels (k_gw_p,
// k_gw_grad at S = 1M columns, B = 512 rows per step) spend their time.  Copies of the two kernels
// with ablation modes (0 full, 1 no LDS lookups, 2 no global bit loads) and wave counts, beside
// pure streaming reads of the same bytes (dword and dwordx4 per lane).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -o tools/gw2_probe tools/gw2_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kGwWords = 64;

__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
#pragma unroll
  for (int j = 16, s = 0; j != 0; j >>= 1, ++s) {
    const uint32_t m = s == 0 ? 0x0000FFFFu : s == 1 ? 0x00FF00FFu : s == 2 ? 0x0F0F0F0Fu
                     : s == 3 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & m;
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

__device__ __forceinline__ float wave_transpose_reduce32(float (&v)[32], int lane) {
#pragma unroll
  for (int st = 0; st < 5; ++st) {
    const int half = 16 >> st;
    const int xm = 32 >> st;
    const bool hi = (lane & xm) != 0;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      float lo_v = v[k], hi_v = v[k + half];
      asm volatile("" : "+v"(lo_v), "+v"(hi_v));
      const float keep = hi ? hi_v : lo_v;
      const float send = hi ? lo_v : hi_v;
      float r = keep + __shfl_xor(send, xm);
      asm volatile("" : "+v"(r));
      v[k] = r;
    }
  }
  return v[0] + __shfl_xor(v[0], 1);
}

template <int MODE>
__device__ __forceinline__ void gw_load32(const uint32_t* __restrict__ bits, int64_t words, int64_t row0, int nr,
                                          uint32_t wd, uint32_t (&x)[32]) {
  typedef const __attribute__((address_space(1))) uint32_t gu32;
  gu32* base = (gu32*)(bits + row0 * words);
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    if (MODE == 2) x[i] = (wd * 2654435761u) ^ (uint32_t)(row0 + i) * 40503u;
    else x[i] = i < nr ? base[(int64_t)i * words + wd] : 0u;
  }
}

template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void p_kernel(const uint32_t* __restrict__ bits, int64_t rows, int64_t cols,
                                                       int64_t words, int batch, int64_t t,
                                                       const float* __restrict__ wg, float* __restrict__ p_part) {
  __shared__ float T[8 * 16 * kGwWords];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  p_part += (int64_t)blockIdx.x * batch;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  if (wv * 32 < B) gw_load32<MODE>(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);
  for (int task = tid; task < 8 * kGwWords; task += WAVES * 64) {
    const int j = task & (kGwWords - 1), q = task >> 6;
    const int64_t c = (w0 + j) * 32 + 4 * q;
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = c + b < cols ? wg[c + b] : 0.f;
    float* Tq = T + q * 16 * kGwWords + j;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      Tq[v * kGwWords] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                         ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  const float* Tl = T + lane;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += WAVES) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];
    const int rbn = rb + WAVES;
    if (rbn * 32 < B) gw_load32<MODE>(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
    float c[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t xi = i < nr ? (x[i] & lmask) : 0u;
      float s = 0.f;
      if (MODE == 1) {
        s = __uint_as_float((xi & 0x007FFFFFu) | 0x3F800000u);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) s += Tl[(q * 16 + ((xi >> (4 * q)) & 15u)) * kGwWords];
      }
      c[i] = s;
    }
    const float tot = wave_transpose_reduce32(c, lane);
    const int i = (lane >> 1) & 31;
    if (!(lane & 1) && i < nr) p_part[rb * 32 + i] = tot;
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
}

template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void grad_kernel(const uint32_t* __restrict__ bits, int64_t rows,
                                                          int64_t cols, int64_t words, int batch, int64_t t,
                                                          const float* __restrict__ g, float* __restrict__ wg,
                                                          float* __restrict__ mg, float* __restrict__ vg) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int ngrp = ((B + 31) / 32) * 8;
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  if (wv * 32 < B) gw_load32<MODE>(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);
  const int gp = ngrp | 1;
  float* G = gsm;
  float* colsum = gsm + ((16 * gp + 3) & ~3);
  for (int grp = tid; grp < ngrp; grp += WAVES * 64) {
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = 4 * grp + b < B ? g[4 * grp + b] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      G[v * gp + grp] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                        ((v & 8) ? a[3] : 0.f);
  }
  for (int e = tid; e < 32 * 65; e += WAVES * 64) colsum[e] = 0.f;
  __syncthreads();
  float acc[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) acc[b] = 0.f;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += WAVES) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];
    const int rbn = rb + WAVES;
    if (rbn * 32 < B) gw_load32<MODE>(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = i < nr ? (x[i] & lmask) : 0u;
    transpose32(x);
    const float* Gb = G + rb * 8;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      float s = 0.f;
      if (MODE == 1) {
        s = __uint_as_float((x[b] & 0x007FFFFFu) | 0x3F800000u);
      } else {
#pragma unroll
        for (int n = 0; n < 8; ++n) s += Gb[((x[b] >> (4 * n)) & 15u) * gp + n];
      }
      acc[b] += s;
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int b = 0; b < 32; ++b) colsum[b * 65 + lane] += acc[b];
    }
    __syncthreads();
  }
  for (int e = tid; e < 32 * kGwWords; e += WAVES * 64) {
    const int64_t c = w0 * 32 + e;
    if (c < cols) {
      const float gsum = colsum[(e & 31) * 65 + (e >> 5)];
      float w = wg[c], m = mg[c], v = vg[c];
      m = fmaf(0.1f, gsum - m, m);
      v = fmaf(0.001f, gsum * gsum, v * 0.999f);
      w = w - 0.01f * (m / (sqrtf(v) + 1e-8f));
      wg[c] = w;
      mg[c] = m;
      vg[c] = v;
    }
  }
}

// grad4: grad_kernel with the next row block prefetch optional and a waves-per-EU floor
template <int WAVES, int MODE, bool PF, int MINW>
__global__ __launch_bounds__(WAVES * 64, MINW) void grad4_kernel(const uint32_t* __restrict__ bits, int64_t rows,
                                                          int64_t cols, int64_t words, int batch, int64_t t,
                                                          const float* __restrict__ g, float* __restrict__ wg,
                                                          float* __restrict__ mg, float* __restrict__ vg) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int ngrp = ((B + 31) / 32) * 8;
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  if (wv * 32 < B) gw_load32<MODE>(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);
  const int gp = ngrp | 1;
  float* G = gsm;
  float* colsum = gsm + ((16 * gp + 3) & ~3);
  for (int grp = tid; grp < ngrp; grp += WAVES * 64) {
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = 4 * grp + b < B ? g[4 * grp + b] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      G[v * gp + grp] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                        ((v & 8) ? a[3] : 0.f);
  }
  for (int e = tid; e < 32 * 65; e += WAVES * 64) colsum[e] = 0.f;
  __syncthreads();
  float acc[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) acc[b] = 0.f;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += WAVES) {
    const int nr = min(32, B - rb * 32);
    if (!PF && rb != wv) gw_load32<MODE>(bits, words, r0 + rb * 32, nr, wd, x);
    uint32_t xn[32];
    const int rbn = rb + WAVES;
    if (PF && rbn * 32 < B) gw_load32<MODE>(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = i < nr ? (x[i] & lmask) : 0u;
    transpose32(x);
    const float* Gb = G + rb * 8;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      float s = 0.f;
      if (MODE == 1) {
        s = __uint_as_float((x[b] & 0x007FFFFFu) | 0x3F800000u);
      } else {
#pragma unroll
        for (int n = 0; n < 8; ++n) s += Gb[((x[b] >> (4 * n)) & 15u) * gp + n];
      }
      acc[b] += s;
    }
    if (PF) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x[k] = xn[k];
    }
  }
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int b = 0; b < 32; ++b) colsum[b * 65 + lane] += acc[b];
    }
    __syncthreads();
  }
  for (int e = tid; e < 32 * kGwWords; e += WAVES * 64) {
    const int64_t c = w0 * 32 + e;
    if (c < cols) {
      const float gsum = colsum[(e & 31) * 65 + (e >> 5)];
      float w = wg[c], m = mg[c], v = vg[c];
      m = fmaf(0.1f, gsum - m, m);
      v = fmaf(0.001f, gsum * gsum, v * 0.999f);
      w = w - 0.01f * (m / (sqrtf(v) + 1e-8f));
      wg[c] = w;
      mg[c] = m;
      vg[c] = v;
    }
  }
}

// v2 candidates: the lookups of two rows (16 table reads) issued before any of them is summed,
// the rows of the batch split over gridDim.y workgroups (balanced grids), 16 lookups per round
template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void p2_kernel(const uint32_t* __restrict__ bits, int64_t rows, int64_t cols,
                                                        int64_t words, int batch, int64_t t,
                                                        const float* __restrict__ wg, float* __restrict__ p_part) {
  __shared__ float T[8 * 16 * kGwWords];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  p_part += (int64_t)blockIdx.x * batch;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int rper = (((B + gridDim.y - 1) / gridDim.y) + 31) & ~31;  // rows of this workgroup's share
  const int rlo = blockIdx.y * rper, rhi = min(B, rlo + rper);
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  int rb = rlo + wv * 32;
  if (rb < rhi) gw_load32<MODE>(bits, words, r0 + rb, min(32, rhi - rb), wd, x);
  for (int task = tid; task < 8 * kGwWords; task += WAVES * 64) {
    const int j = task & (kGwWords - 1), q = task >> 6;
    const int64_t c = (w0 + j) * 32 + 4 * q;
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = c + b < cols ? wg[c + b] : 0.f;
    float* Tq = T + q * 16 * kGwWords + j;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      Tq[v * kGwWords] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                         ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  const float* Tl = T + lane;
#pragma unroll 1
  for (; rb < rhi; rb += WAVES * 32) {
    const int nr = min(32, rhi - rb);
    uint32_t xn[32];
    const int rbn = rb + WAVES * 32;
    if (rbn < rhi) gw_load32<MODE>(bits, words, r0 + rbn, min(32, rhi - rbn), wd, xn);
    float c[32];
#pragma unroll
    for (int i = 0; i < 32; i += 2) {
      const uint32_t x0 = i < nr ? (x[i] & lmask) : 0u, x1 = i + 1 < nr ? (x[i + 1] & lmask) : 0u;
      float a0[8], a1[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a0[q] = Tl[(q * 16 + ((x0 >> (4 * q)) & 15u)) * kGwWords];
        a1[q] = Tl[(q * 16 + ((x1 >> (4 * q)) & 15u)) * kGwWords];
      }
      c[i] = ((a0[0] + a0[1]) + (a0[2] + a0[3])) + ((a0[4] + a0[5]) + (a0[6] + a0[7]));
      c[i + 1] = ((a1[0] + a1[1]) + (a1[2] + a1[3])) + ((a1[4] + a1[5]) + (a1[6] + a1[7]));
    }
    const float tot = wave_transpose_reduce32(c, lane);
    const int i = (lane >> 1) & 31;
    if (!(lane & 1) && i < nr) p_part[rb + i] = tot;
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
}

template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void grad2_kernel(const uint32_t* __restrict__ bits, int64_t rows,
                                                           int64_t cols, int64_t words, int batch, int64_t t,
                                                           const float* __restrict__ g, float* __restrict__ wg,
                                                           float* __restrict__ mg, float* __restrict__ vg) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int ngrp = ((B + 31) / 32) * 8;
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  if (wv * 32 < B) gw_load32<MODE>(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);
  // the chunk's Adam state, in flight during the whole sweep (8 columns per thread at 4 waves)
  constexpr int CPT = 32 * kGwWords / (WAVES * 64);
  float wr[CPT], mr[CPT], vr[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int64_t c = w0 * 32 + tid + k * WAVES * 64;
    wr[k] = c < cols ? wg[c] : 0.f;
    mr[k] = c < cols ? mg[c] : 0.f;
    vr[k] = c < cols ? vg[c] : 0.f;
  }
  const int gp = ngrp | 1;
  float* G = gsm;
  float* part = gsm + ((16 * gp + 3) & ~3);  // [WAVES][32 bit][65]
  for (int grp = tid; grp < ngrp; grp += WAVES * 64) {
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = 4 * grp + b < B ? g[4 * grp + b] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      G[v * gp + grp] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                        ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  float acc[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) acc[b] = 0.f;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += WAVES) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];
    const int rbn = rb + WAVES;
    if (rbn * 32 < B) gw_load32<MODE>(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = i < nr ? (x[i] & lmask) : 0u;
    transpose32(x);
    const float* Gb = G + rb * 8;
#pragma unroll
    for (int b = 0; b < 32; b += 2) {
      float a0[8], a1[8];
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        a0[n] = Gb[((x[b] >> (4 * n)) & 15u) * gp + n];
        a1[n] = Gb[((x[b + 1] >> (4 * n)) & 15u) * gp + n];
      }
      acc[b] += ((a0[0] + a0[1]) + (a0[2] + a0[3])) + ((a0[4] + a0[5]) + (a0[6] + a0[7]));
      acc[b + 1] += ((a1[0] + a1[1]) + (a1[2] + a1[3])) + ((a1[4] + a1[5]) + (a1[6] + a1[7]));
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
  // every wave's column partials to LDS at once, one barrier, summed in wave order
#pragma unroll
  for (int b = 0; b < 32; ++b) part[(wave * 32 + b) * 65 + lane] = acc[b];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int e = tid + k * WAVES * 64;
    const int64_t c = w0 * 32 + e;
    float gsum = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) gsum += part[(w * 32 + (e & 31)) * 65 + (e >> 5)];
    if (c < cols) {
      float w = wr[k], m = mr[k], v = vr[k];
      m = fmaf(0.1f, gsum - m, m);
      v = fmaf(0.001f, gsum * gsum, v * 0.999f);
      w = w - 0.01f * (m / (sqrtf(v) + 1e-8f));
      wg[c] = w;
      mg[c] = m;
      vg[c] = v;
    }
  }
}

// v3: coalesced table build (the chunk's w staged through LDS), lookup addresses by one
// v_perm_b32 each (nibble byte -> address byte 1: T entry (q, v, lane) at byte lane*4 + v*256 +
// q*4096), 32x32 transposes by bitfield inserts, G tables at a 64-float pitch per 4-row group
// (entry v of group n at byte n*256 + v*4: one v_perm_b32 per lookup as well)
__device__ __forceinline__ void transpose32_bfi(uint32_t (&a)[32]) {
#pragma unroll
  for (int j = 16, s = 0; j != 0; j >>= 1, ++s) {
    const uint32_t m = s == 0 ? 0x0000FFFFu : s == 1 ? 0x00FF00FFu : s == 2 ? 0x0F0F0F0Fu
                     : s == 3 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t lo = a[k], hi = a[k + j];
      a[k + j] = ((lo >> j) & m) | (hi & ~m);
      a[k] = ((hi << j) & ~m) | (lo & m);  // (m << j) == ~m for these masks
    }
  }
}

template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void p3_kernel(const uint32_t* __restrict__ bits, int64_t rows, int64_t cols,
                                                        int64_t words, int batch, int64_t t,
                                                        const float* __restrict__ wg, float* __restrict__ p_part) {
  __shared__ float T[8 * 16 * kGwWords];
  __shared__ float Wc[kGwWords * 33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  p_part += (int64_t)blockIdx.x * batch;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int rper = (((B + gridDim.y - 1) / gridDim.y) + 31) & ~31;
  const int rlo = blockIdx.y * rper, rhi = min(B, rlo + rper);
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  int rb = rlo + wv * 32;
  if (rb < rhi && MODE != 3) gw_load32<MODE>(bits, words, r0 + rb, min(32, rhi - rb), wd, x);
  if (MODE == 3) {
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = (wd * 2654435761u) ^ (uint32_t)(rb + i) * 40503u;
  }
  // the chunk's 2048 weights: 4 consecutive columns per thread (one 16-B load), word j's
  // columns at Wc[j * 33 ..] (odd pitch: conflict-free stores and table-build reads)
  for (int e = tid; e < 8 * kGwWords; e += WAVES * 64) {
    const int64_t c = w0 * 32 + 4 * e;
    float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 3) v4 = make_float4(1e-3f * e, 2e-3f, 3e-3f, 4e-3f);
    else if (c + 3 < cols) v4 = *reinterpret_cast<const float4*>(wg + c);
    else {
      if (c < cols) v4.x = wg[c];
      if (c + 1 < cols) v4.y = wg[c + 1];
      if (c + 2 < cols) v4.z = wg[c + 2];
    }
    float* d = Wc + (e >> 3) * 33 + (e & 7) * 4;
    d[0] = v4.x; d[1] = v4.y; d[2] = v4.z; d[3] = v4.w;
  }
  __syncthreads();
  for (int task = tid; task < 8 * kGwWords; task += WAVES * 64) {
    const int j = task & (kGwWords - 1), q = task >> 6;
    const float* a = Wc + j * 33 + 4 * q;
    float* Tq = T + q * 16 * kGwWords + j;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      Tq[v * kGwWords] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                         ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  const char* Tb = reinterpret_cast<const char*>(T);
  const uint32_t base = static_cast<uint32_t>(lane) * 4u;
#pragma unroll 1
  for (; rb < rhi; rb += WAVES * 32) {
    const int nr = min(32, rhi - rb);
    uint32_t xn[32];
    const int rbn = rb + WAVES * 32;
    if (rbn < rhi && MODE != 3) gw_load32<MODE>(bits, words, r0 + rbn, min(32, rhi - rbn), wd, xn);
    float c[32];
#pragma unroll
    for (int i = 0; i < 32; i += 2) {
      float a[16];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t xi = i + h < nr ? (x[i + h] & lmask) : 0u;
        const uint32_t xe = xi & 0x0F0F0F0Fu, xo = (xi >> 4) & 0x0F0F0F0Fu;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t sel = 0x0C0C0000u | ((4u + (q >> 1)) << 8);  // byte1 = nibble byte, byte0 = base
          const uint32_t ad = __builtin_amdgcn_perm((q & 1) ? xo : xe, base, sel);
          a[8 * h + q] = *reinterpret_cast<const float*>(Tb + q * 4096 + ad);
        }
      }
      c[i] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      c[i + 1] = ((a[8] + a[9]) + (a[10] + a[11])) + ((a[12] + a[13]) + (a[14] + a[15]));
    }
    const float tot = wave_transpose_reduce32(c, lane);
    const int i = (lane >> 1) & 31;
    if (!(lane & 1) && i < nr) p_part[rb + i] = tot;
    if (MODE != 3) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x[k] = xn[k];
    }
  }
}

template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void grad3_kernel(const uint32_t* __restrict__ bits, int64_t rows,
                                                           int64_t cols, int64_t words, int batch, int64_t t,
                                                           const float* __restrict__ g, float* __restrict__ wg,
                                                           float* __restrict__ mg, float* __restrict__ vg) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int ngrp = ((B + 31) / 32) * 8;
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t x[32];
  if (wv * 32 < B) gw_load32<MODE>(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);
  constexpr int CPT = 32 * kGwWords / (WAVES * 64);
  float wr[CPT], mr[CPT], vr[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int64_t c = w0 * 32 + tid + k * WAVES * 64;
    wr[k] = c < cols ? wg[c] : 0.f;
    mr[k] = c < cols ? mg[c] : 0.f;
    vr[k] = c < cols ? vg[c] : 0.f;
  }
  float* G = gsm;                       // [ngrp][64]: entry v of 4-row group n at n * 64 + v
  float* part = gsm + 64 * ngrp;        // [WAVES][32 bit][65]
  for (int grp = tid; grp < ngrp; grp += WAVES * 64) {
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = 4 * grp + b < B ? g[4 * grp + b] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      G[grp * 64 + v] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                        ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  float acc[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) acc[b] = 0.f;
  const char* Gbase = reinterpret_cast<const char*>(G);
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += WAVES) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];
    const int rbn = rb + WAVES;
    if (rbn * 32 < B) gw_load32<MODE>(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = i < nr ? (x[i] & lmask) : 0u;
    transpose32_bfi(x);
    const uint32_t rbase = static_cast<uint32_t>(rb) * 2048u;  // group rb * 8 at byte rb * 8 * 256
#pragma unroll
    for (int b = 0; b < 32; b += 2) {
      float a[16];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t xb = x[b + h];
        const uint32_t xe = (xb << 2) & 0x3C3C3C3Cu, xo = (xb >> 2) & 0x3C3C3C3Cu;  // nibble * 4 per byte
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          // byte0 = nibble * 4, bytes 1-2 = the block's group base (a multiple of 256)
          const uint32_t sel = 0x0C020100u & 0xFFFFFF00u | (4u + (n >> 1));
          const uint32_t ad = __builtin_amdgcn_perm((n & 1) ? xo : xe, rbase, sel);
          a[8 * h + n] = *reinterpret_cast<const float*>(Gbase + n * 256 + ad);
        }
      }
      acc[b] += ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      acc[b + 1] += ((a[8] + a[9]) + (a[10] + a[11])) + ((a[12] + a[13]) + (a[14] + a[15]));
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
#pragma unroll
  for (int b = 0; b < 32; ++b) part[(wave * 32 + b) * 65 + lane] = acc[b];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int e = tid + k * WAVES * 64;
    const int64_t c = w0 * 32 + e;
    float gsum = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) gsum += part[(w * 32 + (e & 31)) * 65 + (e >> 5)];
    if (c < cols) {
      float w = wr[k], m = mr[k], v = vr[k];
      m = fmaf(0.1f, gsum - m, m);
      v = fmaf(0.001f, gsum * gsum, v * 0.999f);
      w = w - 0.01f * (m / (sqrtf(v) + 1e-8f));
      wg[c] = w;
      mg[c] = m;
      vg[c] = v;
    }
  }
}

// pure streaming read of the step's rows: lane = VEC words of a 64 * VEC word chunk (blockIdx.x),
// the rows of the batch split over gridDim.y workgroups and their WAVES waves in blocks of RIF
// rows (all RIF loads of a block in flight); one xor-sum per lane written
template <int VEC, int WAVES, int RIF>
__global__ __launch_bounds__(WAVES * 64) void stream_kernel(const uint32_t* __restrict__ bits, int64_t words, int batch,
                                                            int64_t t, uint32_t* __restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * 64 * VEC + lane * VEC;
  const int rows_wg = batch / gridDim.y, rbase = blockIdx.y * rows_wg;
  uint32_t acc = 0;
  if (w0 + VEC <= words) {
    const uint32_t* base = bits + (t * batch + rbase) * words + w0;
    for (int r0 = wave * RIF; r0 < rows_wg; r0 += WAVES * RIF) {
#pragma unroll
      for (int i = 0; i < RIF; ++i) {
        if (VEC == 4) {
          const uint4 v = *reinterpret_cast<const uint4*>(base + (int64_t)(r0 + i) * words);
          acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else if (VEC == 2) {
          const uint2 v = *reinterpret_cast<const uint2*>(base + (int64_t)(r0 + i) * words);
          acc ^= v.x ^ v.y;
        } else {
          acc ^= base[(int64_t)(r0 + i) * words];
        }
      }
    }
  }
  out[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + tid] = acc;
}

// contiguous read of the same byte count (the achievable streaming rate): grid-stride uint4
__global__ __launch_bounds__(256) void contig_kernel(const uint4* __restrict__ p, int64_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int64_t cols = 1000000, words = (cols + 31) / 32;  // 31,250 words: a multiple of 2, not of 4
  const int B = 512, steps = 8;
  const int64_t rows = (int64_t)B * steps;
  uint32_t* bits;
  float *w, *m, *v, *g, *p_part;
  uint32_t* sout;
  const int64_t words_pad = (words + 15) & ~int64_t(15);  // 16-B aligned rows for the dwordx4 stream
  hipMalloc(&bits, (size_t)rows * words_pad * 4 + 64);
  hipMemset(bits, 0x5a, (size_t)rows * words_pad * 4);
  hipMalloc(&w, cols * 4);
  hipMalloc(&m, cols * 4);
  hipMalloc(&v, cols * 4);
  hipMemset(w, 0, cols * 4);
  hipMemset(m, 0, cols * 4);
  hipMemset(v, 0, cols * 4);
  hipMalloc(&g, B * 4);
  hipMemset(g, 0, B * 4);
  const int n_wg = static_cast<int>((words + kGwWords - 1) / kGwWords);
  hipMalloc(&p_part, (size_t)n_wg * B * 4);
  hipMalloc(&sout, (size_t)8 * 4096 * 1024 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = (double)B * words * 4;
  auto timeit = [&](const char* name, auto launch) {
    for (int t = 0; t < steps; ++t) launch(t);  // warm
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
      for (int t = 0; t < steps; ++t) launch(t);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / (reps * steps);
    printf("%-28s %8.2f us  %7.2f TB/s (step bytes %.1f MB)\n", name, us, bytes / (us * 1e-6) / 1e12, bytes / 1e6);
  };
  const size_t lds_g = sizeof(float) * (size_t)(((16 * (((B + 31) / 32) * 8 | 1) + 3) & ~3) + 32 * 65);
#define P(WV, MD)                                                                                          \
  timeit("p<" #WV "," #MD ">", [&](int t) {                                                                \
    hipLaunchKernelGGL((p_kernel<WV, MD>), dim3(n_wg), dim3(WV * 64), 0, 0, bits, rows, cols, words, B, t, w, \
                       p_part);                                                                            \
  });
#define G(WV, MD)                                                                                          \
  hipFuncSetAttribute(reinterpret_cast<const void*>(&grad_kernel<WV, MD>),                                 \
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_g));                \
  timeit("grad<" #WV "," #MD ">", [&](int t) {                                                             \
    hipLaunchKernelGGL((grad_kernel<WV, MD>), dim3(n_wg), dim3(WV * 64), lds_g, 0, bits, rows, cols, words, B, \
                       t, g, w, m, v);                                                                     \
  });
  P(8, 0) P(8, 1) P(8, 2) P(4, 0) P(16, 0)
  G(4, 0) G(4, 1) G(4, 2) G(8, 0) G(16, 0)
#define G4(WV, PF, MINW)                                                                                  \
  hipFuncSetAttribute(reinterpret_cast<const void*>(&grad4_kernel<WV, 0, PF, MINW>),                       \
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_g));                \
  timeit("grad4<" #WV ",pf" #PF ",minw" #MINW ">", [&](int t) {                                             \
    hipLaunchKernelGGL((grad4_kernel<WV, 0, PF, MINW>), dim3(n_wg), dim3(WV * 64), lds_g, 0, bits, rows, cols, \
                       words, B, t, g, w, m, v);                                                           \
  });
  G4(4, true, 1) G4(4, false, 4) G4(4, true, 4) G4(8, false, 4) G4(8, true, 4) G4(8, false, 2) G4(16, false, 4)
#define P2(WV, MD, SPLIT)                                                                                  \
  timeit("p2<" #WV "," #MD "> x" #SPLIT, [&](int t) {                                                      \
    hipLaunchKernelGGL((p2_kernel<WV, MD>), dim3(n_wg, SPLIT), dim3(WV * 64), 0, 0, bits, rows, cols, words, B, \
                       t, w, p_part);                                                                      \
  });
  P2(8, 0, 1) P2(8, 2, 1) P2(4, 0, 2) P2(4, 2, 2) P2(8, 0, 2) P2(4, 0, 4)
  const size_t lds_g2 = sizeof(float) * (size_t)(((16 * (((B + 31) / 32) * 8 | 1) + 3) & ~3) + 8 * 32 * 65);
#define G2(WV, MD)                                                                                         \
  hipFuncSetAttribute(reinterpret_cast<const void*>(&grad2_kernel<WV, MD>),                                \
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_g2));               \
  timeit("grad2<" #WV "," #MD ">", [&](int t) {                                                            \
    hipLaunchKernelGGL((grad2_kernel<WV, MD>), dim3(n_wg), dim3(WV * 64), lds_g2, 0, bits, rows, cols, words, \
                       B, t, g, w, m, v);                                                                  \
  });
  G2(4, 0) G2(4, 2) G2(8, 0) G2(8, 2)
#define P3(WV, MD, SPLIT)                                                                                  \
  timeit("p3<" #WV "," #MD "> x" #SPLIT, [&](int t) {                                                      \
    hipLaunchKernelGGL((p3_kernel<WV, MD>), dim3(n_wg, SPLIT), dim3(WV * 64), 0, 0, bits, rows, cols, words, B, \
                       t, w, p_part);                                                                      \
  });
  P3(8, 0, 1) P3(8, 2, 1) P3(8, 3, 1) P3(4, 0, 2) P3(4, 3, 2) P3(8, 0, 2)
  const size_t lds_g3 = sizeof(float) * (size_t)(64 * (((B + 31) / 32) * 8) + 8 * 32 * 65);
#define G3(WV, MD)                                                                                         \
  hipFuncSetAttribute(reinterpret_cast<const void*>(&grad3_kernel<WV, MD>),                                \
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_g3));               \
  timeit("grad3<" #WV "," #MD ">", [&](int t) {                                                            \
    hipLaunchKernelGGL((grad3_kernel<WV, MD>), dim3(n_wg), dim3(WV * 64), lds_g3, 0, bits, rows, cols, words, \
                       B, t, g, w, m, v);                                                                  \
  });
  G3(4, 0) G3(4, 2) G3(8, 0) G3(8, 2)
#define SK(VEC, WV, RIF, SPLIT)                                                                            \
  timeit("stream<" #VEC "," #WV "," #RIF "> x" #SPLIT, [&](int t) {                                        \
    hipLaunchKernelGGL((stream_kernel<VEC, WV, RIF>), dim3((words + 64 * VEC - 1) / (64 * VEC), SPLIT),     \
                       dim3(WV * 64), 0, 0, bits, VEC > 1 ? words_pad : words, B, t, sout);                \
  });
  SK(1, 8, 32, 1) SK(1, 4, 32, 2) SK(1, 4, 16, 2) SK(1, 4, 8, 4) SK(1, 8, 8, 2)
  SK(2, 4, 32, 2) SK(2, 4, 16, 4) SK(2, 8, 8, 4)
  SK(4, 16, 32, 1) SK(4, 4, 32, 4) SK(4, 4, 16, 4) SK(4, 8, 8, 4) SK(4, 4, 8, 8) SK(4, 4, 16, 8)
  for (int nb : {1024, 2048, 4096})
    timeit(nb == 1024 ? "contig x1024" : nb == 2048 ? "contig x2048" : "contig x4096", [&](int t) {
      hipLaunchKernelGGL(contig_kernel, dim3(nb), dim3(256), 0, 0,
                         reinterpret_cast<const uint4*>(bits + (int64_t)t * B * words_pad), (int64_t)B * words / 4, sout);
    });
  return 0;
}
