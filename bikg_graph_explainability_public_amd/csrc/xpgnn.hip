// xpgnn.hip — MI355X (gfx950, CDNA4) kernels + C-ABI of the XP-GNN perturbation-scoring engine.
//
// Hot path: mask rows (bit-packed) -> masked k-hop message passing restricted to
// the query's receptive field (frontiers F_L ⊆ ... ⊆ F_0) -> dense head -> per-row query logit;
// KernelSHAP weights from row popcounts; the weighted linear surrogate's whole Adam epoch loop in
// one persistent workgroup.  See include/xpgnn.h for the interface and DESIGN.md for layouts.
//
// Conventions: wave64; 256-thread blocks unless noted; fp32 activations/weights, fp64 kernel
// weights and loss (as the reference); dense contractions on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32 fma chains, no reduced-precision path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/xpgnn.h"
#include "host_rng.h"
#include "plan_host.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define XPG_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(XPG_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define XPG_LAUNCHED() XPG_HIP(hipGetLastError())

// A kernel's dynamic-LDS limit is raised once, to all the CU's LDS its static LDS leaves (a launch
// still reserves only the bytes it asks for).  Set per launch to a new plan's size, the attribute
// call cost ~6 ms of host time in the HIP runtime on every new plan size (k_rows_forward,
// k_wlm_fit_mc: profiles/r4_api_first_calls.log).
hipError_t lds_limit(const void* f) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.count(f)) return hipSuccess;
  hipFuncAttributes fa;
  hipError_t e = hipFuncGetAttributes(&fa, f);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024 - static_cast<int>(fa.sharedSizeBytes));
  if (e == hipSuccess) done.insert(f);
  return e;
}

// Diagnostics switches (ablations that change results: XPG_WIDE_DBG, XPG_L1_DBG) are honoured
// only together with XPG_DIAGNOSTICS=1; set without it they are an error, so a variable leaked
// into a production environment cannot silently change outputs.
int diag_env(const char* name, int* out) {
  const char* v = getenv(name);
  *out = 0;
  if (!v || !*v || std::strcmp(v, "0") == 0) return 0;
  const char* d = getenv("XPG_DIAGNOSTICS");
  if (!d || std::strcmp(d, "1") != 0)
    return fail(XPG_EINVAL, std::string(name) + " is a diagnostics switch that changes results: "
                            "set XPG_DIAGNOSTICS=1 to use it, or unset it");
  *out = atoi(v);
  return 0;
}

#define XPG_REQ(cond, msg)                          \
  do {                                              \
    if (!(cond)) return fail(XPG_EINVAL, (msg));    \
  } while (0)

inline hipStream_t S(xpg_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int words_of(int64_t cols) { return static_cast<int>((cols + 31) / 32); }

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup fence on every address
// space: it waits for vmcnt(0), i.e. for every global load still in flight (prefetches of the
// next item) and every global store.  Where a workgroup shares data only through LDS the fence is
// narrowed to LDS ("local"), so the barrier waits for lgkmcnt(0) alone and register prefetches
// stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ bool bit_of(const uint32_t* row, int c) {
  return (row[c >> 5] >> (c & 31)) & 1u;
}

__device__ __forceinline__ float act_apply(float x, int act) {
  switch (act) {
    case XPG_ACT_RELU: return x > 0.f ? x : 0.f;
    case XPG_ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    case XPG_ACT_TANH: return tanhf(x);
    case XPG_ACT_LEAKY_RELU: return x > 0.f ? x : 0.01f * x;
    case XPG_ACT_ELU: return x > 0.f ? x : expm1f(x);
    default: return x;
  }
}

// In-register 32 x 32 bit transpose: in a[i] bit b = M[i][b], out a[b] bit i = M[i][b].
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

// transpose32 with its 16- and 8-bit stages as byte permutes (v_perm_b32: two per pair instead of
// the shift / xor / mask sequence); the 4-, 2- and 1-bit stages as in transpose32
__device__ __forceinline__ void transpose32_perm(uint32_t (&a)[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {  // j = 16: halves
    const uint32_t x = a[k], y = a[k + 16];
    a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);
    a[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
  }
#pragma unroll
  for (int k = 0; k < 32; k = (k + 9) & ~8) {  // j = 8: bytes
    const uint32_t x = a[k], y = a[k + 8];
    a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);
    a[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
  }
#pragma unroll
  for (int j = 4, s = 2; j != 0; j >>= 1, ++s) {
    const uint32_t m = s == 2 ? 0x0F0F0F0Fu : s == 3 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & m;
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

// ------------------------------------------------------------------------------------ masks
__global__ void k_pack(const uint8_t* __restrict__ m, int64_t rows, int64_t cols, int words,
                       uint32_t* __restrict__ bits) {
  int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= rows * words) return;
  int64_t r = idx / words;
  int w = static_cast<int>(idx - r * words);
  const uint8_t* p = m + r * cols + (int64_t)w * 32;
  int n = static_cast<int>(cols - (int64_t)w * 32);
  n = n > 32 ? 32 : n;
  uint32_t v = 0;
  for (int i = 0; i < n; ++i) v |= (p[i] ? 1u : 0u) << i;
  bits[idx] = v;
}

__global__ void k_unpack(const uint32_t* __restrict__ bits, int64_t rows, int64_t cols, int words,
                         uint8_t* __restrict__ m) {
  int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  int64_t r = idx / cols;
  int64_t c = idx - r * cols;
  m[idx] = (bits[r * words + (c >> 5)] >> (c & 31)) & 1u;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based, so any row range can be regenerated
// independently (multi-GPU shards draw disjoint global rows).
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// grid (ceil(quads / 256), min(rows, 65535)); thread = one 16-byte quad (4 words) of a row.
// ALIGN: 4 -> rows start 16-B aligned (words % 4 == 0): one dwordx4 store; 2 -> 8-B aligned
// (words even): two dwordx2 stores; 1 -> four dword stores.  counts != nullptr: the row's
// popcount is accumulated (one atomic per block and row; the caller zeroes counts first), which
// spares KernelSHAP a second pass over the bits (kernels.py:144 row sums).
template <int ALIGN>
__global__ __launch_bounds__(256) void k_shapley(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols,
                                                 int words, uint32_t* __restrict__ bits,
                                                 int32_t* __restrict__ counts, const uint64_t* __restrict__ seed_dev) {
  __shared__ int red[4];
  if (seed_dev) seed = *seed_dev;  // device-resident seed (graph replays draw new rows)
  const int quads = (words + 3) / 4;
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int tail = static_cast<int>(cols & 31);
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    int pc = 0;
    if (q < quads) {
      const uint64_t gr = static_cast<uint64_t>(row_offset + r);
      const uint4 o = philox4x32_10(make_uint4(static_cast<uint32_t>(q), static_cast<uint32_t>(gr),
                                               static_cast<uint32_t>(gr >> 32), 0x58504721u),
                                    static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
      uint32_t v[4] = {o.x, o.y, o.z, o.w};
      const int w0 = q * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (w0 + j >= words) v[j] = 0u;
        else if (w0 + j == words - 1 && tail) v[j] &= (1u << tail) - 1u;
        pc += __popc(v[j]);
      }
      uint32_t* dst = bits + r * words + w0;
      if (ALIGN == 4 && w0 + 4 <= words) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(v[0], v[1], v[2], v[3]);
      } else if (ALIGN == 2 && w0 + 4 <= words) {
        reinterpret_cast<uint2*>(dst)[0] = make_uint2(v[0], v[1]);
        reinterpret_cast<uint2*>(dst)[1] = make_uint2(v[2], v[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (w0 + j < words) dst[j] = v[j];
      }
    }
    if (counts) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) pc += __shfl_xor(pc, off, 64);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pc;
      __syncthreads();
      if (threadIdx.x == 0) atomicAdd(counts + r, red[0] + red[1] + red[2] + red[3]);
      __syncthreads();
    }
  }
}

// Short rows (fewer than 64 quads of words, e.g. a 1,193-column subgraph: 10 quads): one lane
// per (row, quad) over a flat index, so a 256-lane block covers many rows instead of leaving
// 246 of its lanes idle on one row.  Same Philox counters (quad, global row) — bit-identical
// rows; per-row popcounts by one atomic add per lane.
template <int ALIGN>
__global__ __launch_bounds__(256) void k_shapley_flat(uint64_t seed, int64_t row_offset, int64_t rows,
                                                      int64_t cols, int words, uint32_t* __restrict__ bits,
                                                      int32_t* __restrict__ counts,
                                                      const uint64_t* __restrict__ seed_dev) {
  if (seed_dev) seed = *seed_dev;
  const int quads = (words + 3) / 4;
  const int tail = static_cast<int>(cols & 31);
  const int64_t n = rows * quads;
  for (int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gid < n;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = gid / quads;
    const int q = static_cast<int>(gid - r * quads);
    const uint64_t gr = static_cast<uint64_t>(row_offset + r);
    const uint4 o = philox4x32_10(make_uint4(static_cast<uint32_t>(q), static_cast<uint32_t>(gr),
                                             static_cast<uint32_t>(gr >> 32), 0x58504721u),
                                  static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
    uint32_t v[4] = {o.x, o.y, o.z, o.w};
    const int w0 = q * 4;
    int pc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (w0 + j >= words) v[j] = 0u;
      else if (w0 + j == words - 1 && tail) v[j] &= (1u << tail) - 1u;
      pc += __popc(v[j]);
    }
    uint32_t* dst = bits + r * words + w0;
    if (ALIGN == 4 && w0 + 4 <= words) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(v[0], v[1], v[2], v[3]);
    } else if (ALIGN == 2 && w0 + 4 <= words) {
      reinterpret_cast<uint2*>(dst)[0] = make_uint2(v[0], v[1]);
      reinterpret_cast<uint2*>(dst)[1] = make_uint2(v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (w0 + j < words) dst[j] = v[j];
    }
    if (counts && pc) atomicAdd(counts + r, pc);
  }
}

// ------------------------------------------------------------------ community-aware masks
// Device restatement of the community sampler (masks.py:81-194 + pathways.py:234-385): the
// host lays out one block per community in length-descending order, blocks[b] = {row_start,
// size, size_internal, own, off}: `own` is the community whose members get internal random
// bits in every row of the block (masks.py:330), `off` the community column the reference
// switches off in the external coalitions (it passes the sorted position, masks.py:168).
// Row k >= size_internal of a block is an external coalition: the first h = ext/2 rows draw
// community flags, the next h are their complements (antithetic, pathways.py:267-271), an odd
// ext adds one more random row (:273-281); a lone external row with no flag on gets one other
// community switched on (activate_dead_mask — with h >= 1 a pair can never be all-off).  The
// active communities' members are switched on, the own members overwritten by the internal bits.
// Row shuffle (masks.py:380): a seeded Feistel bijection of [0, 4^hb) cycle-walked into
// [0, src_rows).  Every draw is a Philox word keyed by (block, row, word), so rows regenerate
// independently of the launch shape.
constexpr int kCommMaxWords = 1024;  // up to 32,768 communities (flag bitset in LDS)

__device__ __forceinline__ uint32_t comm_mix(uint32_t x, uint32_t k) {
  x ^= k;
  x *= 0x9E3779B1u;
  x ^= x >> 16;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ uint32_t comm_permute(uint32_t x, uint32_t n, int hb, uint32_t k0, uint32_t k1) {
  const uint32_t m = (1u << hb) - 1u;  // hb <= 16
  do {  // terminates: x's cycle under the bijection contains the start, which is < n
    uint32_t L = x >> hb, R = x & m;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t t = L ^ (comm_mix(R, ((i & 1) ? k1 : k0) + 0x632BE5ABu * i) & m);
      L = R;
      R = t;
    }
    x = (L << hb) | R;
  } while (x >= n);
  return x;
}

// One wave per output row (4 rows per 256-thread workgroup).  SMALL (<= 64 communities): the
// row's community flags live in one 64-bit register (word w drawn by lane w, shuffled to all);
// else in a per-wave LDS bitset.  Columns are lane-parallel (lane = column within a 64-column
// slice): each lane looks up its column's communities, the slice's bits come out of one ballot,
// and lane j keeps slice j's ballot until 64 slices are ready, then they are stored together.
// STAGED (cols <= kCommStageCols): each workgroup first stages every column's community as one
// int16 in LDS (-1: none, -2: several -> the CSR in global memory), so the per-slice lookups are
// LDS reads instead of two dependent L2 loads; the block plan is staged beside it.
// CM (SMALL and STAGED, n_comm x words fit LDS): the staging builds one column bitmask per
// community instead (cm[j] = the columns of community j), and a row is assembled a word per lane:
// OR of the active communities' masks outside the own community, the own community's columns
// from the internal random word -- the same bits as the per-column rule (a column of several
// communities: internal bit when it is in the own one, else the OR of its communities' flags),
// for ~10 LDS reads per word instead of a lookup + ballot per 64 columns.
constexpr int kCommStageCols = 16384;
template <bool SMALL, bool STAGED, bool CM = false>
// row0: the launch writes global rows [row0, row0 + rows) to bits / prow rows 0.. (a rank's shard).
__global__ __launch_bounds__(256) void k_communities(uint64_t seed, int64_t row0, int64_t rows, int64_t cols, int words,
                                                     int n_comm, const int32_t* __restrict__ blocks,
                                                     int n_blocks, uint32_t src_rows, int hb, int shuffle,
                                                     const int32_t* __restrict__ col_ptr,
                                                     const int32_t* __restrict__ col_comm,
                                                     uint32_t* __restrict__ bits, int32_t* __restrict__ prow) {
  // dynamic LDS, sized by the launcher: [4 x fw flag words (!SMALL)] [5 x n_blocks plan (STAGED)]
  // [cols x int16 column community (STAGED)] — a few KB at subgraph sizes, so occupancy stays high
  extern __shared__ uint32_t comm_lds[];
  const int fw = (n_comm + 31) >> 5;
  uint32_t* lflags = comm_lds;
  int32_t* lblk = reinterpret_cast<int32_t*>(comm_lds + (SMALL ? 0 : 4 * fw));
  int16_t* lone = reinterpret_cast<int16_t*>(lblk + (STAGED ? 5 * n_blocks : 0));
  uint32_t* cm = reinterpret_cast<uint32_t*>(lblk + (STAGED ? 5 * n_blocks : 0));  // CM: [n_comm][words]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (CM) {
    for (int i = threadIdx.x; i < n_comm * words; i += blockDim.x) cm[i] = 0u;
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += blockDim.x)
      for (int i = col_ptr[c]; i < col_ptr[c + 1]; ++i) atomicOr(&cm[col_comm[i] * words + (c >> 5)], 1u << (c & 31));
  } else if (STAGED) {
    for (int c = threadIdx.x; c < cols; c += blockDim.x) {
      const int p0 = col_ptr[c], n = col_ptr[c + 1] - p0;
      lone[c] = static_cast<int16_t>(n == 0 ? -1 : (n == 1 ? col_comm[p0] : -2));
    }
  }
  if (STAGED) {
    for (int i = threadIdx.x; i < 5 * n_blocks; i += blockDim.x) lblk[i] = blocks[i];
    __syncthreads();
    blocks = lblk;
  }
  uint32_t* flags = lflags + (SMALL ? 0 : wv * fw);
  const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * 4; base < rows; base += static_cast<int64_t>(gridDim.x) * 4) {
    const int64_t r = base + wv;
    const bool active = r < rows;  // inactive waves still reach every barrier
    uint32_t src = 0u;
    int b = 0;
    if (active) {
      const uint32_t rg = static_cast<uint32_t>(row0 + r);  // the global row
      src = shuffle ? comm_permute(rg, src_rows, hb, k0 ^ 0x5EED1234u, k1 ^ 0x0F00D321u) : rg;
      int lo = 0, hi = n_blocks - 1;  // last block whose row_start <= src (wave-uniform)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (static_cast<uint32_t>(blocks[mid * 5]) <= src) lo = mid;
        else hi = mid - 1;
      }
      b = lo;
    }
    const int* blk = blocks + b * 5;
    const int size_int = active ? blk[2] : 0, own = active ? blk[3] : -1, off = active ? blk[4] : 0;
    const int h = active ? (blk[1] - size_int) >> 1 : 0;
    const int k = active ? static_cast<int>(src) - blk[0] - size_int : -1;  // < 0: internal-only row
    // external coalition flags (antithetic pair / extra row), sorted-position column off
    int any = 0;
    uint64_t f64 = 0;
    for (int w0 = 0; w0 < fw; w0 += 64) {
      const int w = w0 + lane;
      uint32_t v = 0u;
      if (k >= 0 && w < fw) {
        const int kk = k < h ? k : (k < 2 * h ? k - h : 2 * h);
        v = philox4x32_10(make_uint4(static_cast<uint32_t>(w), static_cast<uint32_t>(b), static_cast<uint32_t>(kk),
                                     0x434F4D31u), k0, k1).x;
        if (k >= h && k < 2 * h) v = ~v;
        if (w == fw - 1 && (n_comm & 31)) v &= (1u << (n_comm & 31)) - 1u;
        if (w == (off >> 5)) v &= ~(1u << (off & 31));
      }
      any |= v != 0u;
      if (SMALL) f64 = static_cast<uint64_t>(__shfl(v, 0, 64)) | (static_cast<uint64_t>(__shfl(v, 1, 64)) << 32);
      else if (w < fw) flags[w] = v;
    }
    // activate_dead_mask: only a lone external row can be all-off (a pair never is)
    int extra = -1;
    if (k >= 0 && h == 0 && n_comm > 1 && !__any(any)) {
      uint32_t pick = philox4x32_10(make_uint4(0u, static_cast<uint32_t>(b), static_cast<uint32_t>(k), 0x44454144u),
                                    k0, k1).x % static_cast<uint32_t>(n_comm - 1);
      if (static_cast<int>(pick) >= off) ++pick;
      extra = static_cast<int>(pick);
    }
    if (!SMALL) __syncthreads();
    if (CM && active) {
      uint64_t act = f64 & ~(own >= 0 ? 1ull << own : 0ull);
      if (extra >= 0 && extra != own) act |= 1ull << extra;
      uint32_t* dst = bits + r * words;
      for (int w0 = 0; w0 < words; w0 += 64) {  // uniform
        const int w = w0 + lane;
        // internal word w: the per-column path's Philox word for columns 32 w .. 32 w + 31
        const uint32_t iw = philox4x32_10(make_uint4(static_cast<uint32_t>(w), src, 0u, 0x494E5431u), k0, k1).x;
        if (w < words) {
          uint32_t acc = 0u;
          for (uint64_t m = act; m; m &= m - 1) acc |= cm[(__builtin_ctzll(m)) * words + w];  // uniform
          const uint32_t mine = own >= 0 ? cm[own * words + w] : 0u;
          dst[w] = (acc & ~mine) | (iw & mine);
        }
      }
      if (lane == 0 && prow) prow[r] = own;
    } else if (active) {
      uint64_t keep = 0;
      const int slices = static_cast<int>((cols + 63) >> 6);
      uint32_t* dst = bits + r * words;
      uint32_t inner = 0u;  // internal-bit words 2*(sl & ~31) .. +63, one Philox word per lane
      for (int sl = 0; sl < slices; ++sl) {
        const int64_t c = static_cast<int64_t>(sl) * 64 + lane;
        if ((sl & 31) == 0)
          inner = philox4x32_10(make_uint4(static_cast<uint32_t>((sl >> 5) * 64 + lane), src, 0u, 0x494E5431u), k0, k1).x;
        const uint32_t iw = __shfl(inner, ((sl & 31) << 1) + (lane >> 5), 64);  // word c >> 5
        uint32_t bit = 0u;
        const int one = (STAGED && c < cols) ? lone[c] : -2;
        if (one >= 0) {
          if (one == own) bit = (iw >> (c & 31)) & 1u;
          else if (one == extra) bit = 1u;
          else if (SMALL) bit = static_cast<uint32_t>(f64 >> one) & 1u;
          else bit = (flags[one >> 5] >> (one & 31)) & 1u;
        } else if (one == -2 && c < cols) {
          int i = col_ptr[c];
          const int e = col_ptr[c + 1];
          bool mine = false;
          for (; i < e; ++i) {
            const int cc = col_comm[i];
            if (cc == own) mine = true;
            else if (cc == extra) bit = 1u;
            else if (SMALL) bit |= static_cast<uint32_t>(f64 >> cc) & 1u;
            else bit |= (flags[cc >> 5] >> (cc & 31)) & 1u;
          }
          if (mine) bit = (iw >> (c & 31)) & 1u;
        }
        const uint64_t bal = __ballot(bit);
        if (lane == (sl & 63)) keep = bal;
        if ((sl & 63) == 63 || sl == slices - 1) {
          const int first = sl & ~63;
          if (lane <= (sl & 63)) {
            const int w = (first + lane) * 2;
            dst[w] = static_cast<uint32_t>(keep);
            if (w + 1 < words) dst[w + 1] = static_cast<uint32_t>(keep >> 32);
          }
        }
      }
      if (lane == 0 && prow) prow[r] = own;
    }
    if (!SMALL) __syncthreads();
  }
}

__global__ void k_edge_keep(const uint32_t* __restrict__ bits, int64_t rows, int words,
                            const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                            int64_t n_edges, uint8_t* __restrict__ keep) {
  int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= rows * n_edges) return;
  int64_t b = idx / n_edges;
  int64_t e = idx - b * n_edges;
  const uint32_t* row = bits + b * words;
  keep[idx] = static_cast<uint8_t>(bit_of(row, src[e]) && bit_of(row, dst[e]));
}

// ------------------------------------------------------------------------------------ KernelSHAP
// one wave per row: lanes stride the row's words, popcount, wave-reduce.
// Empty copies of the multi-node-type loop (model.py:213-215): out[r] = 1 iff mask row r keeps
// no edge (both endpoints set).  One wave per row, 64 edges per round, the row's words read from
// L1 / L2; the wave stops at the first round with a kept edge (most rows keep one early), so a
// row costs a few rounds instead of the rows x edges keep matrix of k_edge_keep + a reduction.
// rpw rows per wave, one after another (default 4, XPG_RNE_RPW; c5: 158 -> 143 us, 8 no better).
__global__ __launch_bounds__(256) void k_rows_no_edge(const uint32_t* __restrict__ bits, int64_t rows, int words,
                                                      const int* __restrict__ src, const int* __restrict__ dst,
                                                      int64_t n_edges, uint8_t* __restrict__ out, int rpw) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  for (int64_t r = w * rpw; r < rows && r < (w + 1) * rpw; ++r) {  // wave-uniform
    const uint32_t* row = bits + r * words;
    bool any = false;
    for (int64_t e0 = 0; e0 < n_edges && !any; e0 += 64) {
      const int64_t e = e0 + lane;
      bool k = false;
      if (e < n_edges) {
        const int a = src[e], b = dst[e];
        k = (((row[a >> 5] >> (a & 31)) & (row[b >> 5] >> (b & 31))) & 1u) != 0u;
      }
      any = __ballot(k) != 0ull;
    }
    if (lane == 0) out[r] = any ? 0 : 1;
  }
}

__global__ void k_popcount(const uint32_t* __restrict__ bits, int64_t rows, int words,
                           int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const uint32_t* row = bits + r * words;
  int c = 0, c1 = 0, c2 = 0, c3 = 0;
  int w = lane;
  for (; w + 192 < words; w += 256) {  // 4 independent loads in flight per lane
    c += __popc(row[w]);
    c1 += __popc(row[w + 64]);
    c2 += __popc(row[w + 128]);
    c3 += __popc(row[w + 192]);
  }
  for (; w < words; w += 64) c += __popc(row[w]);
  c += c1 + c2 + c3;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if (lane == 0) counts[r] = c;
}

// scipy.special.binom for integer-valued n >= 0, k (kernels.py:64,109 call sites): the product
// formula below 20 (bit-identical to scipy), the Gamma form otherwise (~1e-13 relative).
__device__ double binom_d(double n, double k) {
  if (k < 0.0 || k > n) return 0.0;
  double kx = k;
  if (kx > n / 2 && n > 0) kx = n - kx;
  if (kx >= 0 && kx < 20) {
    double num = 1.0, den = 1.0;
    const int kk = static_cast<int>(kx);
    for (int i = 1; i < 1 + kk; ++i) {
      num *= i + n - kx;
      den *= i;
      if (fabs(num) > 1e50) {
        num /= den;
        den = 1.0;
      }
    }
    return num / den;
  }
  return exp(lgamma(n + 1.0) - lgamma(k + 1.0) - lgamma(n - k + 1.0));
}

__device__ __forceinline__ double clean_inf(double v) { return (isinf(v) || isnan(v)) ? 0.0 : v; }

__device__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// Kernel.compute exact branch (M = S-1 <= 1000, kernels.py:83-113): thread per row.
__global__ void k_shap_exact(const int32_t* __restrict__ cnt, int64_t rows, int64_t cols,
                             double* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int64_t Mi = cols - 1;
  const double M = static_cast<double>(Mi);
  const int64_t k = cnt[r];
  const double choose = binom_d(M + 1.0, static_cast<double>(k));
  out[r] = clean_inf(M / (choose * static_cast<double>(Mi + 1 - k) * static_cast<double>(k)));
}

// Approximate branch (M > 1000, kernels.py:23-80): value of one row at reference size `ref`.
__device__ __forceinline__ double shap_approx_row(int64_t k, int64_t Mi, int ref) {
  const double M = static_cast<double>(Mi);
  int64_t idx = static_cast<int64_t>(static_cast<float>(k * 1000) / static_cast<float>(Mi));
  idx = idx < 0 ? 0 : (idx > ref - 1 ? ref - 1 : idx);
  const double choose = (binom_d(static_cast<double>(ref), static_cast<double>(idx)) + 1e-10) * M / 1000.0;
  return M / (choose * static_cast<double>(k) * static_cast<double>(Mi - k));
}

// pass 1 (grid): every row at ref = 1000 (raw values, +-inf kept for the sum test)
__global__ void k_shap_approx_rows(const int32_t* __restrict__ cnt, int64_t rows, int64_t cols,
                                   double* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r < rows) out[r] = shap_approx_row(cnt[r], cols - 1, 1000);
}

// pass 2 (one block): the reference's loop `while sum(kernel) == 0 and ref > 0` (kernels.py:
// 148-162).  Row values are >= 0, +inf, or negative for an all-active row (k = M + 1, quirk Q5),
// and a sum holding a NaN or an infinity is != 0: the block scans 1024-row chunks until one
// holds a value that is not == 0 (normally the first), instead of summing every row (the sum
// of non-zero values cancelling to exactly 0 is the only case this reads differently, and the
// reference's own float summation order would decide that case); the ref = int(0.9 ref)
// back-off recomputes rows in-block.
__global__ __launch_bounds__(1024) void k_shap_approx_finish(const int32_t* __restrict__ cnt,
                                                             int64_t rows, int64_t cols,
                                                             double* __restrict__ out) {
  const int64_t Mi = cols - 1;
  int ref = 1000;
  for (;;) {
    bool found = false;
    for (int64_t base = 0; base < rows && !found; base += blockDim.x) {  // block-uniform
      const int64_t r = base + threadIdx.x;
      found = __syncthreads_or(r < rows && !(out[r] == 0.0)) != 0;
    }
    if (found) break;
    ref = static_cast<int>(0.9 * static_cast<double>(ref));
    if (!(ref > 0)) break;  // the sum is 0 here
    __syncthreads();
    for (int64_t r = threadIdx.x; r < rows; r += blockDim.x) out[r] = shap_approx_row(cnt[r], Mi, ref);
    __syncthreads();
  }
}

// pass 3 (grid): +-inf / NaN -> 0 (kernels.py:172)
__global__ void k_shap_clean(int64_t rows, double* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r < rows) out[r] = clean_inf(out[r]);
}

// Sum over the 32 lanes of each half of the wave (lanes l and l ^ 32 keep separate sums), on the
// VALU: quad DPP (xor 1, xor 2), row_ror 4 and 8 inside 16-lane rows, then v_permlane16_swap for
// the two rows of the half.  Every lane of the half ends with the same total.
__device__ __forceinline__ float half_wave_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));  // row_ror:4
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));  // row_ror:8
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ------------------------------------------------------------------------------------ dense
// C = act(A W^T + b) on v_mfma_f32_32x32x2_f32.  One wave owns 32 rows x (NT*32) columns
// (column group cg of n_groups: consecutive waves take the column groups of one 32-row block, so
// a workgroup's waves share its A rows in L1 and a wide layer spreads over n_groups x as many
// waves); the k loop advances 8 at a time: each lane loads one float4 of its A row and one
// float4 of each W row, feeding 4 MFMAs whose 2 k-slots map to k = kc + 4*h + s (h = lane >> 5),
// identically for A and B, so the contraction is exact.  C/D map: col = lane & 31,
// row = (reg & 3) + 8 * (reg >> 2) + 4 * h.
// HEAD: the network's output column is one more linear layer of this one, y[m] =
// hact(sum_c v[m][c] hw[c] + hb[0]) over this layer's outputs v (bias + activation applied, padding
// columns 0).  v is not stored: each lane multiplies its column's values by hw, the 32 columns of a
// tile are summed across the half-wave, the column groups of a 32-row block (the workgroup's 4
// waves when n_groups = 4) add their partials in group order through LDS.  This replaces the
// 1-column head's own dense launch (a 32-wide padded tile) and the column pick.
template <int NT, bool HEAD = false>
__global__ __launch_bounds__(256) void k_dense(const float* __restrict__ A, int64_t M, int64_t lda,
                                               const float* __restrict__ W, int64_t ldw, int k_pad,
                                               const float* __restrict__ bias, int n_real, int act,
                                               float* __restrict__ C, int64_t ldc,
                                               const int32_t* __restrict__ row_type, int64_t type_mod,
                                               int bias_ld, int n_groups, const float* __restrict__ hw = nullptr,
                                               const float* __restrict__ hb = nullptr, int hact = 0,
                                               float* __restrict__ y = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  const int cg = static_cast<int>(wv % n_groups);
  const int64_t m0 = (wv / n_groups) * 32;
  if (m0 >= M) return;
  const int c0 = cg * NT * 32;  // first column of this wave's group
  W += (int64_t)c0 * ldw;
  bias += c0;
  C += c0;
  if (HEAD) hw += c0;
  n_real -= c0;
  const int i = lane & 31, h = lane >> 5;
  const int64_t arow = m0 + i;
  const bool a_ok = arow < M;
  const float* ap = A + (a_ok ? arow : 0) * lda + 4 * h;
  const uint32_t amask = a_ok ? 0xffffffffu : 0u;  // rows past M contribute +0
  f32x16 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[nt][q] = 0.f;
  // D k-steps per iteration: all their loads are issued before their MFMAs (one step per
  // iteration waited out a full L2 latency per 4 x NT MFMAs).  Steps past k_pad are skipped
  // (uniform branches), so the MFMA sequence per accumulator is unchanged.
  constexpr int D = NT == 1 ? 4 : NT == 2 ? 2 : 1;
  for (int kc = 0; kc < k_pad; kc += 8 * D) {
    float4 a[D], w[D][NT];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int k = kc + 8 * u;
      if (k < k_pad) {
        // ap is row 0 for rows past M: the load stays unconditional, masked to +0 below
        a[u] = *reinterpret_cast<const float4*>(ap + k);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          w[u][nt] = *reinterpret_cast<const float4*>(W + (int64_t)(nt * 32 + i) * ldw + k + 4 * h);
      }
    }
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if (kc + 8 * u < k_pad) {
        a[u].x = __uint_as_float(__float_as_uint(a[u].x) & amask);
        a[u].y = __uint_as_float(__float_as_uint(a[u].y) & amask);
        a[u].z = __uint_as_float(__float_as_uint(a[u].z) & amask);
        a[u].w = __uint_as_float(__float_as_uint(a[u].w) & amask);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].x, w[u][nt].x, acc[nt], 0, 0, 0);
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].y, w[u][nt].y, acc[nt], 0, 0, 0);
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].z, w[u][nt].z, acc[nt], 0, 0, 0);
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].w, w[u][nt].w, acc[nt], 0, 0, 0);
        }
      }
    }
  }
  float part[HEAD ? 16 : 1];
  if (HEAD) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) part[reg] = 0.f;
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = nt * 32 + i;
    const float bv = col < n_real ? bias[col] : 0.f;
    const float hwc = HEAD && col < n_real ? hw[col] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int64_t m = m0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      // multi-node-type layers: the bias of the row's target type (rows are (mask row, target))
      const float b = (row_type && m < M && col < n_real) ? bias[(int64_t)row_type[m % type_mod] * bias_ld + col]
                                                          : bv;
      const float v = col < n_real ? act_apply(acc[nt][reg] + b, act) : 0.f;
      if (HEAD) part[reg] = fmaf(v, hwc, part[reg]);
      else if (m < M) C[m * ldc + col] = v;
    }
  }
  if (HEAD) {
    __shared__ float hp[4][32];  // [wave][row of the 32-row block]
    const int wl = threadIdx.x >> 6;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) part[reg] = half_wave_sum(part[reg]);
    if (i == 0) {  // lanes 0 and 32: the totals of their half's 16 rows
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) hp[wl][(reg & 3) + 8 * (reg >> 2) + 4 * h] = part[reg];
    }
    if (n_groups > 1) {
      __syncthreads();  // the workgroup's waves are the n_groups column groups of one block
      if (cg != 0) return;
    } else {
      __builtin_amdgcn_wave_barrier();
    }
    if (lane < 32 && m0 + lane < M) {
      float t = hp[wl][lane];
      for (int g = 1; g < n_groups; ++g) t += hp[wl + g][lane];
      y[m0 + lane] = act_apply(t + hb[0], hact);
    }
  }
}

// ------------------------------------------------------------------------------------ forward
// kin[(b * n_rel + r) * n0 + p] = kept in-degree of F_0 node p under relation r for mask row b
// (self-loops excluded), or -1 when the node itself is masked out (then it keeps only the
// GCN self-loop / an empty SAGE neighbourhood).
// Edge masks (deg_eid != NULL, Data.perturb_edge): every node is active and an in-edge counts iff
// its own column bit is set.
// n_deg: the F_0 prefix whose degrees are kept (kin [rows][n_rel][n_deg]): every F_0 node when
// some term needs its sources' degrees (GCN) or edges carry the mask bits, else only the targets
// (F_1, a prefix of F_0: k_agg then tests a MEAN source's own mask bit)
__global__ void k_degree(const uint32_t* __restrict__ bits, int64_t rows, int words, int n0, int n_deg,
                         int n_rel, const int32_t* __restrict__ f0_node,
                         const int32_t* __restrict__ deg_ptr, const int32_t* __restrict__ deg_src,
                         const int32_t* __restrict__ deg_eid, float* __restrict__ kin) {
  const int64_t per_row = (int64_t)n_rel * n_deg;
  int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= rows * per_row) return;
  const int64_t b = idx / per_row;
  const int rem = static_cast<int>(idx - b * per_row);
  const int r = rem / n_deg, p = rem - r * n_deg;
  const uint32_t* row = bits + b * words;
  const int* pp = deg_ptr + (int64_t)r * (n0 + 1);
  float out = -1.f;
  if (deg_eid) {
    int c = 0;
    for (int e = pp[p]; e < pp[p + 1]; ++e) c += bit_of(row, deg_eid[e]);
    out = static_cast<float>(c);
  } else if (bit_of(row, f0_node[p])) {
    int c = 0;
    for (int e = pp[p]; e < pp[p + 1]; ++e) c += bit_of(row, deg_src[e]);
    out = static_cast<float>(c);
  }
  kin[idx] = out;
}

struct AggArgs {
  int64_t rows;
  int n0, n_rel, n_tgt, n_prev;
  const float* kin;
  const int32_t* tgt_prev;
  const int32_t* tgt_f0;
  const int32_t* agg_ptr;
  const int32_t* agg_src;
  const int32_t* agg_f0;
  const int32_t* self_mult;
  int n_terms;
  int kind[XPG_MAX_TERMS];
  int rel[XPG_MAX_TERMS];
  const float* table[XPG_MAX_TERMS];
  const float* hprev;   // layer >= 2 source rows [rows][n_prev][width]
  int width;            // source row width (floats, % 32 == 0)
  float* out;
  int64_t out_ld;
  const float* bias;    // layer 1 epilogue ([n_types][width] with tgt_type)
  int act;
  int f_real;
  const int32_t* tgt_type;      // multi-node-type plans: node type of each target (else null)
  int dst_type[XPG_MAX_TERMS];  // term k reaches only targets of this type (-1: every target)
  // edge masks (agg_eid != null): in-edge e kept iff bit agg_eid[e] of the row; MEAN self term =
  // number of kept self-loop edges (self_ptr / self_eid)
  const uint32_t* bits;
  int words;
  const int32_t* agg_eid;
  const int32_t* self_ptr;
  const int32_t* self_eid;
  // kin row pitch per relation (k_degree's n_deg); mbits / f0_node (non-null when kin holds only
  // the targets' degrees): a MEAN source is active iff its own mask bit is set
  int kpitch;
  const uint32_t* mbits;
  const int32_t* f0_node;
  int rows_blk;  // (diagnostics, XPG_L1_DBG) k_agg_l1_rows: 1 every source kept, 2 every source = the self row, 4 no output stores
};

__device__ __forceinline__ float inv_sqrt_deg(float kin) {
  return 1.f / sqrtf(1.f + (kin > 0.f ? kin : 0.f));
}

__device__ __forceinline__ void fma4(float4& a, float c, const float4 v) {
  a.x = fmaf(c, v.x, a.x);
  a.y = fmaf(c, v.y, a.y);
  a.z = fmaf(c, v.z, a.z);
  a.w = fmaf(c, v.w, a.w);
}

// Masked aggregation for one conv layer.  Item = (mask row b, target t); LPS lanes per item,
// each lane owns NV float4 feature chunks.  L1: sources are the shared pre-transformed F_0
// tables (X W^T computed once per query: features are never masked, data.py:582) and the
// epilogue applies bias + activation; otherwise sources are the previous layer's per-row
// outputs and each term's aggregate is written to its slice of the GEMM input.
template <bool L1, int LPS, int NV>
__global__ __launch_bounds__(256) void k_agg(AggArgs a) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t item = gid / LPS;
  const int sub = static_cast<int>(gid - item * LPS);
  if (item >= a.rows * a.n_tgt) return;
  const int64_t b = item / a.n_tgt;
  const int t = static_cast<int>(item - b * a.n_tgt);
  const float* kb = a.kin + b * (int64_t)a.n_rel * a.kpitch;
  const uint32_t* mrow = a.mbits ? a.mbits + b * a.words : nullptr;
  const int t0 = a.tgt_f0[t];
  const int tp = a.tgt_prev[t];
  float4 tot[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int k = 0; k < a.n_terms; ++k) {
    const int kind = a.kind[k];
    const int r = a.rel[k];
    const float* base = L1 ? a.table[k] : a.hprev + b * (int64_t)a.n_prev * a.width;
    const int self_pos = L1 ? t0 : tp;
    const float4* selfrow = reinterpret_cast<const float4*>(base + (int64_t)self_pos * a.width);
    float4 s[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    // HeteroConv on several node types: a relation's conv only produces rows of its
    // destination type (hetero_conv.py sums per destination), so other targets get 0
    if (a.tgt_type && a.dst_type[k] >= 0 && a.tgt_type[t] != a.dst_type[k]) {
    } else if (kind == XPG_TERM_ROOT) {
#pragma unroll
      for (int j = 0; j < NV; ++j) s[j] = selfrow[sub + j * LPS];
    } else {
      const float kt = kb[(int64_t)r * a.kpitch + t0];
      const int* pp = a.agg_ptr + (int64_t)r * (a.n_tgt + 1);
      const uint32_t* brow = a.agg_eid ? a.bits + b * a.words : nullptr;
      if (kind == XPG_TERM_GCN) {
        const float dt = inv_sqrt_deg(kt);
        const float cself = dt * dt;
#pragma unroll
        for (int j = 0; j < NV; ++j) fma4(s[j], cself, selfrow[sub + j * LPS]);
        if (kt >= 0.f) {
          for (int e = pp[t]; e < pp[t + 1]; ++e) {
            const int u0 = a.agg_f0[e];
            const float ku = kb[(int64_t)r * a.kpitch + u0];
            if (brow ? bit_of(brow, a.agg_eid[e]) : ku >= 0.f) {
              const float c = inv_sqrt_deg(ku) * dt;
              const int up = L1 ? u0 : a.agg_src[e];
              const float4* src = reinterpret_cast<const float4*>(base + (int64_t)up * a.width);
#pragma unroll
              for (int j = 0; j < NV; ++j) fma4(s[j], c, src[sub + j * LPS]);
            }
          }
        }
      } else {  // MEAN
        if (kt >= 0.f) {
          int sm = 0;
          if (brow) {
            const int* sp = a.self_ptr + (int64_t)r * (a.n_tgt + 1);
            for (int e = sp[t]; e < sp[t + 1]; ++e) sm += bit_of(brow, a.self_eid[e]);
          } else {
            sm = a.self_mult[(int64_t)r * a.n_tgt + t];
          }
          const float cnt = kt + static_cast<float>(sm);
#pragma unroll
          for (int j = 0; j < NV; ++j) fma4(s[j], static_cast<float>(sm), selfrow[sub + j * LPS]);
          // EB in-edges at a time: their keep tests, then the kept sources' rows, are all issued
          // before the first add (one edge at a time each edge waited out its whole
          // edge -> keep word -> row chain); the adds stay in edge order
          constexpr int EB = NV >= 4 ? 2 : NV == 2 ? 4 : 8;
          const int e_end = pp[t + 1];
          for (int eb = pp[t]; eb < e_end; eb += EB) {
            bool kp[EB];
            int up[EB], kx[EB];
            // stage by stage over the EB edges (the keep source is uniform: edge bits, the
            // source's own mask bit, or its kin entry), so each stage's loads go out together
#pragma unroll
            for (int q = 0; q < EB; ++q) {
              const int e = eb + q < e_end ? eb + q : eb;
              up[q] = a.agg_f0[e];
              kx[q] = brow ? a.agg_eid[e] : 0;
            }
            if (brow) {
#pragma unroll
              for (int q = 0; q < EB; ++q) kp[q] = bit_of(brow, kx[q]);
            } else if (mrow) {
#pragma unroll
              for (int q = 0; q < EB; ++q) kx[q] = a.f0_node[up[q]];
#pragma unroll
              for (int q = 0; q < EB; ++q) kp[q] = bit_of(mrow, kx[q]);
            } else {
#pragma unroll
              for (int q = 0; q < EB; ++q) kp[q] = kb[(int64_t)r * a.kpitch + up[q]] >= 0.f;
            }
#pragma unroll
            for (int q = 0; q < EB; ++q) {
              kp[q] = kp[q] && eb + q < e_end;
              if (!L1) up[q] = a.agg_src[eb + q < e_end ? eb + q : eb];
            }
#pragma unroll
            for (int q = 0; q < EB; ++q) asm volatile("" ::"v"(up[q]));  // issued here, not sunk into the branches
            float4 v[EB][NV];
#pragma unroll
            for (int q = 0; q < EB; ++q) {
              const float4* src = reinterpret_cast<const float4*>(base + (int64_t)up[q] * a.width);
#pragma unroll
              for (int j = 0; j < NV; ++j) v[q][j] = kp[q] ? src[sub + j * LPS] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int q = 0; q < EB; ++q) {
              if (kp[q]) {
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                  s[j].x += v[q][j].x; s[j].y += v[q][j].y; s[j].z += v[q][j].z; s[j].w += v[q][j].w;
                }
              }
            }
          }
          const float inv = 1.f / (cnt > 1.f ? cnt : 1.f);
#pragma unroll
          for (int j = 0; j < NV; ++j) { s[j].x *= inv; s[j].y *= inv; s[j].z *= inv; s[j].w *= inv; }
        }
      }
    }
    if (L1) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        tot[j].x += s[j].x; tot[j].y += s[j].y; tot[j].z += s[j].z; tot[j].w += s[j].w;
      }
    } else {
      float4* o = reinterpret_cast<float4*>(a.out + item * a.out_ld + (int64_t)k * a.width);
#pragma unroll
      for (int j = 0; j < NV; ++j) o[sub + j * LPS] = s[j];
    }
  }
  if (L1) {
    float4* o = reinterpret_cast<float4*>(a.out + item * a.out_ld);
    const float* bias = a.bias + (a.tgt_type ? (int64_t)a.tgt_type[t] * a.width : 0);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int f = (sub + j * LPS) * 4;
      float v[4] = {tot[j].x, tot[j].y, tot[j].z, tot[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = (f + q < a.f_real) ? act_apply(v[q] + bias[f + q], a.act) : 0.f;
      o[sub + j * LPS] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// One term of k_agg_l1_rows for the wave's 64 rows and W features: s (all 0 on entry) gets the
// term's value, in k_agg<true>'s operation order.  Features are handled in pairs (f32x2: packed
// fp32 add / fma / mul, two features per VALU instruction; each lane's operations per feature are
// unchanged).
template <int W>
__device__ __forceinline__ void l1_rows_term(const AggArgs& a, int k, int t, int t0, int fo, const float* kb,
                                             const uint32_t* mrow, f32x2 (&s)[W / 2]) {
  const int kind = a.kind[k];
  const int r = a.rel[k];
  const float* __restrict__ T = a.table[k] + fo;
  const f32x2* __restrict__ selfrow = reinterpret_cast<const f32x2*>(T + (int64_t)t0 * a.width);
  if (kind == XPG_TERM_ROOT) {
#pragma unroll
    for (int j = 0; j < W / 2; ++j) s[j] = selfrow[j];
    return;
  }
  const float kt = kb[(int64_t)r * a.kpitch + t0];
  const int* pp = a.agg_ptr + (int64_t)r * (a.n_tgt + 1);
  const int e0 = pp[t], e1 = pp[t + 1];
  if (kind == XPG_TERM_GCN) {
    const float dt = inv_sqrt_deg(kt);
    const f32x2 cself = dt * dt;
#pragma unroll
    for (int j = 0; j < W / 2; ++j) s[j] = fma2(cself, selfrow[j], s[j]);
    for (int e = e0; e < e1; ++e) {  // uniform
      const int u0 = a.agg_f0[e];
      const float ku = kb[(int64_t)r * a.kpitch + u0];
      if (kt >= 0.f && ku >= 0.f) {
        const f32x2 c = inv_sqrt_deg(ku) * dt;
        const f32x2* __restrict__ src = reinterpret_cast<const f32x2*>(T + (int64_t)u0 * a.width);
#pragma unroll
        for (int j = 0; j < W / 2; ++j) s[j] = fma2(c, src[j], s[j]);
      }
    }
  } else {  // MEAN
    const int sm = a.self_mult[(int64_t)r * a.n_tgt + t];
    const float cnt = kt + static_cast<float>(sm);
    if (kt >= 0.f) {
      const f32x2 smf = static_cast<float>(sm);
#pragma unroll
      for (int j = 0; j < W / 2; ++j) s[j] = fma2(smf, selfrow[j], s[j]);
    }
    // 8 in-edges at a time: their sources and keep words are loaded stage by stage before the
    // first add (one edge at a time each edge waited out its edge -> node -> keep word chain)
    for (int eb = e0; eb < e1; eb += 8) {  // uniform
      int uu[8];
      bool kw[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) uu[q] = a.agg_f0[eb + q < e1 ? eb + q : eb];
      if (mrow) {
        int nd[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) nd[q] = a.f0_node[uu[q]];
#pragma unroll
        for (int q = 0; q < 8; ++q) kw[q] = bit_of(mrow, nd[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) kw[q] = kb[(int64_t)r * a.kpitch + uu[q]] >= 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (eb + q >= e1) break;  // uniform
        const bool keep = kt >= 0.f && ((a.rows_blk & 1) ? true : kw[q]);
        if (keep) {
          const f32x2* __restrict__ src =
              (a.rows_blk & 2) ? selfrow : reinterpret_cast<const f32x2*>(T + (int64_t)uu[q] * a.width);
#pragma unroll
          for (int j = 0; j < W / 2; ++j) s[j] += src[j];
        }
      }
    }
    if (kt >= 0.f) {
      const f32x2 inv = 1.f / (cnt > 1.f ? cnt : 1.f);
#pragma unroll
      for (int j = 0; j < W / 2; ++j) s[j] *= inv;
    }
  }
}

// Layer-1 aggregation with lanes = mask rows (no edge masks): wave = (block of 64 mask rows, one
// target, one W-feature slice of the layer's a.width = W, 2W, 4W features).  The tables are shared
// by every mask row, so each in-edge's table slice is a wave-uniform read (scalar loads) added to
// the lanes that keep the edge; only the per-row keep bits / degrees are per-lane loads.
// k_agg<true> instead gives each (row, target) item 16-32 lanes that fetch every kept row's table
// slice themselves: for small frontiers and many rows (the c5 shape; c3 node_prediction's 128-wide
// SAGE tables) that re-reads the same table rows from L2 once per mask row.  Same operations per
// value in the same order as k_agg<true> (bitwise the same h1).
// ONE (host-checked): term 0 is the only non-ROOT term (SAGE: [MEAN, ROOT]).  Its value then
// builds in tot itself (0 + s: the generic order's +0 for a -0 sum kept) and the ROOT terms add
// their rows straight in, so no second W-float array is live: 157 -> 111 VGPRs at W = 64.
template <int W, bool ONE>
__global__ __launch_bounds__(256) void k_agg_l1_rows(AggArgs a) {
  const int64_t wid = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (a.rows + 63) / 64;
  const int nsl = a.width / W;  // feature slices (host-checked: a.width = nsl * W)
  if (wid >= nblk * a.n_tgt * nsl) return;  // wave-uniform
  const int fo = static_cast<int>(wid % nsl) * W;
  const int64_t wt = wid / nsl;
  const int t = static_cast<int>(wt % a.n_tgt);
  const int64_t b0 = (wt / a.n_tgt) * 64, b = b0 + lane;
  const int64_t bb = b < a.rows ? b : b0;
  const float* kb = a.kin + bb * (int64_t)a.n_rel * a.kpitch;
  const uint32_t* mrow = a.mbits ? a.mbits + bb * a.words : nullptr;
  const int t0 = a.tgt_f0[t];
  f32x2 tot2[W / 2];
#pragma unroll
  for (int j = 0; j < W / 2; ++j) tot2[j] = 0.f;
  auto skip = [&](int k) { return a.tgt_type && a.dst_type[k] >= 0 && a.tgt_type[t] != a.dst_type[k]; };
  if (ONE) {
    if (!skip(0)) {  // uniform
      l1_rows_term<W>(a, 0, t, t0, fo, kb, mrow, tot2);
#pragma unroll
      for (int j = 0; j < W / 2; ++j) tot2[j] = 0.f + tot2[j];
    }
    for (int k = 1; k < a.n_terms; ++k) {
      if (skip(k)) continue;  // uniform
      const f32x2* __restrict__ selfrow = reinterpret_cast<const f32x2*>(a.table[k] + fo + (int64_t)t0 * a.width);
#pragma unroll
      for (int j = 0; j < W / 2; ++j) tot2[j] += selfrow[j];
    }
  } else {
    for (int k = 0; k < a.n_terms; ++k) {
      if (skip(k)) continue;  // uniform
      f32x2 s[W / 2];
#pragma unroll
      for (int j = 0; j < W / 2; ++j) s[j] = 0.f;
      l1_rows_term<W>(a, k, t, t0, fo, kb, mrow, s);
#pragma unroll
      for (int j = 0; j < W / 2; ++j) tot2[j] += s[j];
    }
  }
  float tot[W];
#pragma unroll
  for (int j = 0; j < W / 2; ++j) {
    tot[2 * j] = tot2[j].x;
    tot[2 * j + 1] = tot2[j].y;
  }
  // epilogue: bias + activation, then the 64 rows x W tile leaves through this wave's LDS slice
  // in 32-float column chunks, so every store instruction writes whole 128-B lines (8 rows x
  // 128 B).  Stored straight from the lanes (each lane its own 256-B row, 16 B per instruction,
  // 64 lines per instruction), the lines sat half-written in L2 and HBM saw ~2.4x the bytes.
  const float* bias = a.bias + (a.tgt_type ? (int64_t)a.tgt_type[t] * a.width : 0) + fo;
#pragma unroll
  for (int f = 0; f < W; ++f) tot[f] = (fo + f < a.f_real) ? act_apply(tot[f] + bias[f], a.act) : 0.f;
  __shared__ float l1o[4][64 * 33];
  float* tile = l1o[threadIdx.x >> 6];
  const int rr = lane >> 3, q = lane & 7;  // store phase: row rr + 8 i, float4 q of the chunk
#pragma unroll
  for (int c = 0; c < W / 32; ++c) {
#pragma unroll
    for (int f = 0; f < 32; ++f) tile[lane * 33 + f] = tot[32 * c + f];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = rr + 8 * i;
      const float* src = tile + row * 33 + 4 * q;
      const float4 v = make_float4(src[0], src[1], src[2], src[3]);
      if (b0 + row < a.rows && !(a.rows_blk & 4))
        *reinterpret_cast<float4*>(a.out + ((b0 + row) * a.n_tgt + t) * a.out_ld + fo + 32 * c + 4 * q) = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void k_take_col(const float* __restrict__ C, int64_t M, int64_t ldc, int col,
                           float* __restrict__ y) {
  int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (m < M) y[m] = C[m * ldc + col];
}

// Link decoder of edge problems: y[r] = act(sum_f C[r][a][f] C[r][b][f]) over the n real columns
// of the last layer (the query edge's endpoint rows a, b of mask row r), fixed fma order.
__global__ void k_edge_dot(const float* __restrict__ C, int64_t rows, int n_tgt, int64_t ldc, int n, int ta,
                           int tb, int act, float* __restrict__ y) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* ca = C + (r * n_tgt + ta) * ldc;
  const float* cb = C + (r * n_tgt + tb) * ldc;
  float s = 0.f;
  for (int f = 0; f < n; ++f) s = fmaf(ca[f], cb[f], s);
  y[r] = act_apply(s, act);
}

// ------------------------------------------------------------------------------ fused forward
// The whole masked forward of a small plan (a query's receptive field) in ONE launch: one wave
// per mask row, lanes = feature chunks.  The layer-1 tables (X W^T of the F_0 nodes) and the
// weights of layers >= 2 are copied into LDS once per workgroup; the row's mask words, kept
// in-degrees and layer outputs live in the wave's own LDS slice, so nothing per row touches HBM
// except the mask words read and the output written.  Same arithmetic per target as k_agg.
constexpr int kFusedMaxLayers = 4;
constexpr int kFusedMaxHead = 4;

struct FusedLayer {
  int n_tgt, n_terms, act, f_in_pad, f_out, f_out_pad, K, w_ld, lds_w;
  const int32_t* tgt_prev;
  const int32_t* tgt_f0;
  const int32_t* agg_ptr;
  const int32_t* agg_src;
  const int32_t* agg_f0;
  const int32_t* self_mult;
  const float* weight;
  const float* bias;
  int kind[XPG_MAX_TERMS], rel[XPG_MAX_TERMS], lds_tab[XPG_MAX_TERMS];
  const float* table[XPG_MAX_TERMS];
};

struct FusedHead {
  int k_pad, n_real, n_pad, act;
  const float* weight;
  const float* bias;
};

struct FusedArgs {
  int64_t rows;
  const uint32_t* bits;
  float* y;
  int words, n0, n_rel, n_layers, n_head, out_col, n_last;
  const int32_t* f0_node;
  const int32_t* deg_ptr;
  const int32_t* deg_src;
  int shared_floats, wave_floats, o_kin, o_h0, o_h1, o_a;
  FusedLayer L[kFusedMaxLayers];
  FusedHead H[kFusedMaxHead];
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void add4(float4& a, const float4 b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

template <int WPB>
__global__ __launch_bounds__(WPB * 64) void k_fused_forward(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) float fl[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {  // prologue: layer-1 tables and the weights of layers >= 2 into LDS
    const FusedLayer& L0 = a.L[0];
    const int n4 = a.n0 * L0.f_out_pad / 4;
    for (int k = 0; k < L0.n_terms; ++k) {
      const float4* src = reinterpret_cast<const float4*>(L0.table[k]);
      float4* dst = reinterpret_cast<float4*>(fl + L0.lds_tab[k]);
      for (int i = tid; i < n4; i += WPB * 64) dst[i] = src[i];
    }
    for (int l = 1; l < a.n_layers; ++l) {
      const FusedLayer& L = a.L[l];
      const int k4 = L.K / 4;
      for (int i = tid; i < L.f_out_pad * k4; i += WPB * 64) {
        const int o = i / k4, c = i - o * k4;
        reinterpret_cast<float4*>(fl + L.lds_w + o * L.w_ld)[c] =
            reinterpret_cast<const float4*>(L.weight + (int64_t)o * L.K)[c];
      }
    }
  }
  __syncthreads();
  float* wv = fl + a.shared_floats + wave * a.wave_floats;
  uint32_t* mb = reinterpret_cast<uint32_t*>(wv);
  float* kin = wv + a.o_kin;
  float* Ab = wv + a.o_a;

  for (int64_t row = (int64_t)blockIdx.x * WPB + wave; row < a.rows; row += (int64_t)gridDim.x * WPB) {
    const uint32_t* rb = a.bits + row * a.words;
    for (int w = lane; w < a.words; w += 64) mb[w] = rb[w];
    wave_sync();
    // kept in-degree per (relation, F_0 node), -1 when the node is masked out
    for (int idx = lane; idx < a.n_rel * a.n0; idx += 64) {
      const int r = idx / a.n0, p = idx - r * a.n0;
      float out = -1.f;
      if (bit_of(mb, a.f0_node[p])) {
        const int32_t* pp = a.deg_ptr + r * (a.n0 + 1);
        const int e0 = pp[p], e1 = pp[p + 1];
        int c = 0;
        for (int e = e0; e < e1; ++e) c += bit_of(mb, a.deg_src[e]);
        out = static_cast<float>(c);
      }
      kin[idx] = out;
    }
    wave_sync();
    float* hcur = wv + a.o_h0;
    float* hprev = wv + a.o_h1;
    for (int l = 0; l < a.n_layers; ++l) {
      const FusedLayer& L = a.L[l];
      const bool l1 = l == 0;
      const int width = l1 ? L.f_out_pad : L.f_in_pad;
      const int CH = width >> 2, TPP = 64 / CH;
      for (int t0 = 0; t0 < L.n_tgt; t0 += TPP) {
        const int tt = lane / CH, ch = lane - tt * CH, t = t0 + tt;
        if (tt < TPP && t < L.n_tgt) {
          const int tf0 = L.tgt_f0[t], tp = L.tgt_prev[t];
          float4 tot = f4zero();
          for (int k = 0; k < L.n_terms; ++k) {
            const int kind = L.kind[k], r = L.rel[k];
            const float* base = l1 ? fl + L.lds_tab[k] : hprev;
            const float4 selfv = reinterpret_cast<const float4*>(base + (l1 ? tf0 : tp) * width)[ch];
            float4 s = f4zero();
            if (kind == XPG_TERM_ROOT) {
              s = selfv;
            } else {
              const float* kr = kin + r * a.n0;
              const float kt = kr[tf0];
              const int32_t* pp = L.agg_ptr + r * (L.n_tgt + 1);
              const int e0 = pp[t], e1 = pp[t + 1];
              if (kind == XPG_TERM_GCN) {
                const float dt = inv_sqrt_deg(kt);
                fma4(s, dt * dt, selfv);
                if (kt >= 0.f) {
                  for (int e = e0; e < e1; ++e) {
                    const int u0 = L.agg_f0[e];
                    const float ku = kr[u0];
                    if (ku >= 0.f) {
                      const int up = l1 ? u0 : L.agg_src[e];
                      fma4(s, inv_sqrt_deg(ku) * dt, reinterpret_cast<const float4*>(base + up * width)[ch]);
                    }
                  }
                }
              } else {  // MEAN
                if (kt >= 0.f) {
                  const int sm = L.self_mult[r * L.n_tgt + t];
                  fma4(s, static_cast<float>(sm), selfv);
                  for (int e = e0; e < e1; ++e) {
                    const int u0 = L.agg_f0[e];
                    if (kr[u0] >= 0.f) add4(s, reinterpret_cast<const float4*>(base + (l1 ? u0 : L.agg_src[e]) * width)[ch]);
                  }
                  const float cnt = kt + static_cast<float>(sm);
                  const float inv = 1.f / (cnt > 1.f ? cnt : 1.f);
                  s.x *= inv; s.y *= inv; s.z *= inv; s.w *= inv;
                }
              }
            }
            if (l1) add4(tot, s);
            else reinterpret_cast<float4*>(Ab + tt * L.K + k * width)[ch] = s;
          }
          if (l1) {
            const int f = ch * 4;
            float v[4] = {tot.x, tot.y, tot.z, tot.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = (f + q < L.f_out) ? act_apply(v[q] + L.bias[f + q], L.act) : 0.f;
            reinterpret_cast<float4*>(hcur + t * L.f_out_pad)[ch] = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
        if (!l1) {  // dense: h[t][o] = act(sum_k A[t][k] W[o][k] + b[o]) for this pass's targets
          wave_sync();
          const float* W = fl + L.lds_w;
          const int nq = min(TPP, L.n_tgt - t0);
          for (int o = lane; o < L.f_out_pad; o += 64) {
            const float bo = o < L.f_out ? L.bias[o] : 0.f;
            const float4* wr = reinterpret_cast<const float4*>(W + o * L.w_ld);
            for (int q = 0; q < nq; ++q) {
              const float4* ar = reinterpret_cast<const float4*>(Ab + q * L.K);
              float acc = 0.f;
              for (int k = 0; k < L.K / 4; ++k) {
                const float4 x = ar[k], wq = wr[k];
                acc = fmaf(x.x, wq.x, acc);
                acc = fmaf(x.y, wq.y, acc);
                acc = fmaf(x.z, wq.z, acc);
                acc = fmaf(x.w, wq.w, acc);
              }
              hcur[(t0 + q) * L.f_out_pad + o] = o < L.f_out ? act_apply(acc + bo, L.act) : 0.f;
            }
          }
        }
        wave_sync();
      }
      float* tmp = hcur;
      hcur = hprev;
      hprev = tmp;
    }
    // dense head on the last layer's targets (ping-pong through the free H buffer)
    const float* cur = hprev;
    int cur_w = a.L[a.n_layers - 1].f_out_pad;
    float* nxt = hcur;
    for (int i = 0; i < a.n_head; ++i) {
      const FusedHead& hd = a.H[i];
      for (int o = lane; o < hd.n_pad; o += 64) {
        const float bo = o < hd.n_real ? hd.bias[o] : 0.f;
        const float4* wr = reinterpret_cast<const float4*>(hd.weight + (int64_t)o * hd.k_pad);
        for (int t = 0; t < a.n_last; ++t) {
          const float4* ar = reinterpret_cast<const float4*>(cur + t * cur_w);
          float acc = 0.f;
          if (o < hd.n_real) {
            for (int k = 0; k < hd.k_pad / 4; ++k) {
              const float4 x = ar[k], wq = wr[k];
              acc = fmaf(x.x, wq.x, acc);
              acc = fmaf(x.y, wq.y, acc);
              acc = fmaf(x.z, wq.z, acc);
              acc = fmaf(x.w, wq.w, acc);
            }
          }
          nxt[t * hd.n_pad + o] = o < hd.n_real ? act_apply(acc + bo, hd.act) : 0.f;
        }
      }
      wave_sync();
      float* tmp = const_cast<float*>(cur);
      cur = nxt;
      nxt = tmp;
      cur_w = hd.n_pad;
    }
    for (int t = lane; t < a.n_last; t += 64) a.y[row * a.n_last + t] = cur[t * cur_w + a.out_col];
    wave_sync();
  }
}

#ifdef XPG_WLM_STAMPS  // diagnostic build only (tools/wlm_probe.cpp): per-phase cycle counts
#define XPG_STAMP(k)                                                       \
  {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                     \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                    \
    stamp_acc[k] += now_ - stamp_last;                                     \
    stamp_last = now_;                                                     \
    __builtin_amdgcn_sched_barrier(0);                                     \
  }
__device__ uint64_t g_wlm_stamps[2][8];
#else
#define XPG_STAMP(k)
#endif

// ------------------------------------------------------------- fused forward, lanes = mask rows
// For plans of one or two conv layers (the query's receptive field): one 1024-thread workgroup
// per 64 mask rows, lane = row.  The 16 waves split the F_0 nodes for the degree pass and the
// feature columns (FS = f1_pad / 16 each) for the layer passes.  Control flow and every index
// are uniform across a wave: CSR arrays sit in LDS and are pulled 64 at a time into a VGPR and
// handed out with v_readlane; the per-lane work is mask-word tests, one kept/degree factor per
// edge (dv = 1/sqrt(1+kin) of kept nodes, computed once per node and row) and FS FMAs against
// broadcast LDS reads of the layer-1 table row.  Layer-1 outputs are recomputed for each layer-2
// use instead of stored (a single-query plan uses each once); the layer-2 aggregate stays in
// registers until the wave-split dense layer and head.
// Per-XCD count of resident multi-workgroup fit workgroups (k_wlm_fit_mc registers each working
// workgroup while it holds its CU): the rows forward sizes its per-XCD worker count by it.
__device__ int g_xcd_busy[16];

__device__ __forceinline__ int xcc_id() { return static_cast<int>(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu); }

struct RowsFwdArgs {
  int64_t rows;
  // XCD-aware block scheduling (nullable): ctl[0] = next 64-row block, ctl[1 + x] = workgroups
  // started on XCD x (zeroed before the launch); cus_per_xcd = CUs per XCD
  int* ctl;
  int cus_per_xcd, n_blocks;
  const uint32_t* bits;
  float* y;
  int words, n0, n_rel, n_layers, out_col, n_last, n_deg_edges, n1_edges, n2_edges;
  const int32_t* f0_node;
  const int32_t* deg_ptr;
  const int32_t* deg_src;
  // layer 1 (tables in LDS)
  int n1, n_terms1, act1, f1_out, f1_pad;
  const int32_t* l1_ptr;
  const int32_t* l1_f0;
  const int32_t* l1_smul;
  const int32_t* l1_tgt_f0;
  int kind1[XPG_MAX_TERMS], rel1[XPG_MAX_TERMS];
  const float* tab1[XPG_MAX_TERMS];
  const float* bias1;
  // layer 2 (aggregate then dense)
  int n2, n_terms2, act2, f2_out, f2_pad;
  const int32_t* l2_ptr;
  const int32_t* l2_src;
  const int32_t* l2_f0;
  const int32_t* l2_smul;
  const int32_t* l2_tgt_f0;
  const int32_t* l2_tgt_prev;
  int kind2[XPG_MAX_TERMS], rel2[XPG_MAX_TERMS];
  const float* w2;
  const float* bias2;
  int n_head;
  FusedHead H[kFusedMaxHead];
  // LDS image (4-byte units)
  int stage_bits, mb_pitch, w2_lds, o_tab, o_mb, o_dv, o_kt, o_a2, o_h0, o_h1, o_w2;
  int o_dptr, o_f0n, o_dsrc, o_l1ptr, o_l1f0, o_l1smul, o_l1tgt, o_l2ptr, o_l2src, o_l2f0, o_l2smul, o_l2tgt, o_l2prev;
  int o_hw[kFusedMaxHead];  // head weights in LDS (-1: read from global)
};

constexpr int kRowsWaves = 16;

__device__ __forceinline__ int rdl(int v, int i) { return __builtin_amdgcn_readlane(v, i); }

__device__ __forceinline__ uint32_t row_word(const RowsFwdArgs& a, const uint32_t* mb, int64_t row, int lane,
                                             int node) {
  return a.stage_bits ? mb[lane * a.mb_pitch + (node >> 5)] : a.bits[row * a.words + (node >> 5)];
}

template <int FS>
__device__ __forceinline__ void ld_fs(const float* p, float (&v)[FS]) {
  if constexpr (FS % 4 == 0) {
#pragma unroll
    for (int i = 0; i < FS / 4; ++i) {
      const float4 x = reinterpret_cast<const float4*>(p)[i];
      v[4 * i] = x.x;
      v[4 * i + 1] = x.y;
      v[4 * i + 2] = x.z;
      v[4 * i + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < FS / 2; ++i) {
      const float2 x = reinterpret_cast<const float2*>(p)[i];
      v[2 * i] = x.x;
      v[2 * i + 1] = x.y;
    }
  }
}

// out[o][lane] = act(sum_k A[k][lane] W[o][k] + b[o]) for o < n_pad (0 beyond n_real); wave w
// takes outputs w, w + 16, ...  W rows are wave-uniform (broadcast) reads; K % 4 == 0.
__device__ __forceinline__ void rows_dense(const float* A, int K, const float* W, int ldw,
                                           const float* __restrict__ bias, int n_real, int n_pad, int act,
                                           float* out, int wave, int lane) {
  for (int o0 = wave * 4; o0 < n_pad; o0 += 4 * kRowsWaves) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int kc = 0; kc < K; kc += 4) {
      float av[4];
      float4 wv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = A[(kc + i) * 64 + lane];
#pragma unroll
      for (int q = 0; q < 4; ++q) wv[q] = *reinterpret_cast<const float4*>(W + (int64_t)(o0 + q) * ldw + kc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q] = fmaf(av[0], wv[q].x, acc[q]);
        acc[q] = fmaf(av[1], wv[q].y, acc[q]);
        acc[q] = fmaf(av[2], wv[q].z, acc[q]);
        acc[q] = fmaf(av[3], wv[q].w, acc[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = o0 + q;
      if (o < n_pad) out[o * 64 + lane] = o < n_real ? act_apply(acc[q] + bias[o], act) : 0.f;
    }
  }
}

// Layer-1 output of F_1 target s for this wave's FS feature columns (lane = row).
template <int FS>
__device__ __forceinline__ void rows_h1(const RowsFwdArgs& a, const float* lds, int s, int fo, int lane,
                                        float (&h)[FS]) {
  const int* li = reinterpret_cast<const int*>(lds);
#pragma unroll
  for (int f = 0; f < FS; ++f) h[f] = 0.f;
  const int tf0 = li[a.o_l1tgt + s];
  for (int k = 0; k < a.n_terms1; ++k) {
    const int kind = a.kind1[k], r = a.rel1[k];
    const float* T = lds + a.o_tab + k * a.n0 * a.f1_pad + fo;
    const float* dvr = lds + a.o_dv + r * a.n0 * 64 + lane;
    float cself, cedge_t;  // self coefficient; per-edge factor (GCN: dt, MEAN: 1/cnt)
    if (kind == XPG_TERM_ROOT) {
      cself = 1.f;
      cedge_t = 0.f;
    } else {
      const float kt = lds[a.o_kt + (r * a.n1 + tf0) * 64 + lane];
      if (kind == XPG_TERM_GCN) {
        const float dt = inv_sqrt_deg(kt);
        cself = dt * dt;
        cedge_t = kt >= 0.f ? dt : 0.f;
      } else {
        const int sm = li[a.o_l1smul + r * a.n1 + s];
        const float cnt = kt + static_cast<float>(sm);
        const float inv = 1.f / (cnt > 1.f ? cnt : 1.f);
        cself = kt >= 0.f ? static_cast<float>(sm) * inv : 0.f;
        cedge_t = kt >= 0.f ? inv : 0.f;
      }
    }
    {
      float v[FS];
      ld_fs<FS>(T + tf0 * a.f1_pad, v);
#pragma unroll
      for (int f = 0; f < FS; ++f) h[f] = fmaf(cself, v[f], h[f]);
    }
    if (kind == XPG_TERM_ROOT) continue;
    const int* pp = li + a.o_l1ptr + r * (a.n1 + 1);
    const int e0 = pp[s], e1 = pp[s + 1];
    // GCN edge factor dv_u * dt; MEAN: [u kept] / cnt = min(dv_u * BIG, 1) * inv (dv > 0 iff kept)
    const float gmul = kind == XPG_TERM_GCN ? cedge_t : 0.f;
    const float mmul = kind == XPG_TERM_GCN ? 0.f : cedge_t;
    // in-edges per batch (their LDS reads in flight together); 8 and 16 measured slower at c2
    // (59.8 -> 62.1 / 64.5 us per forward), equal at c3node: profiles/r5_rows_edge_batch_ab.log
    constexpr int EB = 4;
    for (int wb = e0; wb < e1; wb += 64) {
      const int ne = min(64, e1 - wb);
      const int vsrc = li[a.o_l1f0 + wb + min(lane, ne - 1)];
      for (int i0 = 0; i0 < ne; i0 += EB) {
        int u[EB];
        float d[EB], v[EB][FS];
#pragma unroll
        for (int q = 0; q < EB; ++q) u[q] = rdl(vsrc, min(i0 + q, ne - 1));
#pragma unroll
        for (int q = 0; q < EB; ++q) d[q] = dvr[u[q] * 64];
#pragma unroll
        for (int q = 0; q < EB; ++q) ld_fs<FS>(T + u[q] * a.f1_pad, v[q]);
#pragma unroll
        for (int q = 0; q < EB; ++q) {
          const float valid = static_cast<float>(i0 + q < ne);
          const float c = valid * fmaf(d[q], gmul, fminf(d[q] * 1e30f, 1.f) * mmul);
#pragma unroll
          for (int f = 0; f < FS; ++f) h[f] = fmaf(c, v[q][f], h[f]);
        }
      }
    }
  }
#pragma unroll
  for (int f = 0; f < FS; ++f) {
    const int fg = fo + f;
    h[f] = fg < a.f1_out ? act_apply(h[f] + a.bias1[fg], a.act1) : 0.f;
  }
}

// Block scheduling.  Without a control block: workgroup b takes 64-row block b.  With one
// (a.ctl): the dispatcher deals workgroups round-robin over the XCDs, so an XCD that hosts a
// persistent fit (13 of its 32 CUs held for ~160 us) got as many blocks as the others and ran
// them in two rounds — the forward took twice as long beside a fit.  Here a workgroup first
// takes a worker slot on its XCD (at most its free CUs: CUs per XCD minus the fit workgroups
// registered there) or leaves, and the workers take 64-row blocks from one counter until none is
// left, so the blocks go where CUs are free.  Every block is taken exactly once either way.
template <int FS>
__global__ __launch_bounds__(1024) void k_rows_forward(const RowsFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  int* li = reinterpret_cast<int*>(lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ int blk_s;
  if (a.ctl) {
    if (tid == 0) {
      const int x = xcc_id();
      const int busy = __hip_atomic_load(g_xcd_busy + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int cap = a.cus_per_xcd - busy > 1 ? a.cus_per_xcd - busy : 1;
      const int slot = __hip_atomic_fetch_add(a.ctl + 1 + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      blk_s = slot < cap ? 0 : -1;
    }
    __syncthreads();
    if (blk_s < 0) return;  // workgroup-uniform: no worker slot left on this XCD
  }
#ifdef XPG_WLM_STAMPS
  uint64_t stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stamp_last = __builtin_amdgcn_s_memtime();
#endif
  {  // LDS image: layer-1 tables, CSR arrays, layer-2 weights
    const int n4 = a.n0 * a.f1_pad / 4;
    for (int k = 0; k < a.n_terms1; ++k) {
      const float4* src = reinterpret_cast<const float4*>(a.tab1[k]);
      float4* dst = reinterpret_cast<float4*>(lds + a.o_tab + k * a.n0 * a.f1_pad);
      for (int i = tid; i < n4; i += 1024) dst[i] = src[i];
    }
    auto cp = [&](int off, const int32_t* src, int n) {
      for (int i = tid; i < n; i += 1024) li[off + i] = src[i];
    };
    cp(a.o_dptr, a.deg_ptr, a.n_rel * (a.n0 + 1));
    cp(a.o_f0n, a.f0_node, a.n0);
    cp(a.o_dsrc, a.deg_src, a.n_deg_edges);
    cp(a.o_l1ptr, a.l1_ptr, a.n_rel * (a.n1 + 1));
    cp(a.o_l1f0, a.l1_f0, a.n1_edges);
    cp(a.o_l1smul, a.l1_smul, a.n_rel * a.n1);
    cp(a.o_l1tgt, a.l1_tgt_f0, a.n1);
    if (a.n_layers == 2) {
      cp(a.o_l2ptr, a.l2_ptr, a.n_rel * (a.n2 + 1));
      cp(a.o_l2src, a.l2_src, a.n2_edges);
      cp(a.o_l2f0, a.l2_f0, a.n2_edges);
      cp(a.o_l2smul, a.l2_smul, a.n_rel * a.n2);
      cp(a.o_l2tgt, a.l2_tgt_f0, a.n2);
      cp(a.o_l2prev, a.l2_tgt_prev, a.n2);
      if (a.w2_lds) {
        const int n = a.f2_pad * a.n_terms2 * a.f1_pad / 4;
        for (int i = tid; i < n; i += 1024)
          reinterpret_cast<float4*>(lds + a.o_w2)[i] = reinterpret_cast<const float4*>(a.w2)[i];
      }
    }
    for (int i = 0; i < a.n_head; ++i) {
      if (a.o_hw[i] < 0) continue;
      const int n = a.H[i].n_pad * a.H[i].k_pad / 4;
      for (int e = tid; e < n; e += 1024)
        reinterpret_cast<float4*>(lds + a.o_hw[i])[e] = reinterpret_cast<const float4*>(a.H[i].weight)[e];
    }
  }
  for (int it = 0;; ++it) {
  int64_t blk;
  if (a.ctl) {
    __syncthreads();  // blk_s of the previous block read by every thread
    if (tid == 0) blk_s = __hip_atomic_fetch_add(a.ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    blk = blk_s;
    if (blk >= a.n_blocks) break;
  } else {
    if (it > 0) break;
    blk = blockIdx.x;
  }
  const int64_t row0 = blk * 64, row = row0 + lane;
  const int nrow = static_cast<int>(a.rows - row0 < 64 ? a.rows - row0 : 64);
  if (a.stage_bits) {  // this block's mask rows
    uint32_t* mbw = reinterpret_cast<uint32_t*>(lds + a.o_mb);
    for (int e = tid; e < 64 * a.words; e += 1024) {
      const int r = e / a.words, w = e - r * a.words;
      mbw[r * a.mb_pitch + w] = r < nrow ? a.bits[(row0 + r) * a.words + w] : 0u;
    }
  }
  __syncthreads();
  XPG_STAMP(0)
  const uint32_t* mb = reinterpret_cast<const uint32_t*>(lds + a.o_mb);
  const int64_t rrow = row < a.rows ? row : row0;  // clamped row for unstaged bit reads
  {  // per (relation, F_0 node) and row: dv = 1/sqrt(1 + kept in-degree) for kept nodes, else 0;
     // kt = kept in-degree (or -1 when masked) for the F_1 targets (the first n1 F_0 nodes)
    const int Q = a.n_rel * a.n0;
    // split the flat (relation, node) range so every wave gets about the same number of edges
    // plus nodes: first q with ptr(q) + q >= target, by binary search over the LDS ptr array
    auto flat_ptr = [&](int q) {  // start offset of flat node q (ptr arrays hold absolute offsets)
      const int r = q / a.n0, p = q - r * a.n0;
      return li[a.o_dptr + r * (a.n0 + 1) + p];
    };
    auto split = [&](int w) {
      if (w == 0) return 0;
      if (w == kRowsWaves) return Q;
      const int64_t target = ((int64_t)(a.n_deg_edges + Q) * w) / kRowsWaves;
      int lo = 0, hi = Q;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)flat_ptr(mid) + mid < target) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    const int q_lo = split(wave), q_hi = split(wave + 1);
    for (int qb = q_lo; qb < q_hi; qb += 64) {
      const int nq = min(64, q_hi - qb);
      const int ql = qb + min(lane, nq - 1);
      const int rl = ql / a.n0, pl = ql - rl * a.n0;
      const int vp0 = li[a.o_dptr + rl * (a.n0 + 1) + pl], vp1 = li[a.o_dptr + rl * (a.n0 + 1) + pl + 1];
      const int vnd = li[a.o_f0n + pl];
      uint64_t kept = 0;  // bit j: node qb + j is kept in this lane's row
      for (int j0 = 0; j0 < nq; j0 += 8) {
        uint32_t wv[8];
        int nd[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          nd[q] = rdl(vnd, min(j0 + q, nq - 1));
          wv[q] = row_word(a, mb, rrow, lane, nd[q]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          kept |= static_cast<uint64_t>(((wv[q] >> (nd[q] & 31)) & 1u) & static_cast<uint32_t>(j0 + q < nq))
                  << (j0 + q);
      }
      auto finish = [&](int j, int c) {
        const int qq = qb + j, r = qq / a.n0, p = qq - r * a.n0;
        const bool kp = (kept >> j) & 1ull;
        const float kin = kp ? static_cast<float>(c) : -1.f;
        lds[a.o_dv + qq * 64 + lane] = kp ? inv_sqrt_deg(kin) : 0.f;
        if (p < a.n1) lds[a.o_kt + (r * a.n1 + p) * 64 + lane] = kin;
      };
      const int E_lo = rdl(vp0, 0), E_hi = rdl(vp1, nq - 1);
      int j = 0, a0 = rdl(vp0, 0), a1 = rdl(vp1, 0), c = 0;
      for (int wb = E_lo; wb < E_hi; wb += 64) {
        const int ne = min(64, E_hi - wb);
        const int vsrc = li[a.o_dsrc + wb + min(lane, ne - 1)];
        uint64_t kb = 0;  // bit i: edge wb + i's source kept in this lane's row
        for (int i0 = 0; i0 < ne; i0 += 8) {
          uint32_t wv[8];
          int sv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            sv[q] = rdl(vsrc, min(i0 + q, ne - 1));
            wv[q] = row_word(a, mb, rrow, lane, sv[q]);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q)
            kb |= static_cast<uint64_t>(((wv[q] >> (sv[q] & 31)) & 1u) & static_cast<uint32_t>(i0 + q < ne))
                  << (i0 + q);
        }
        while (j < nq) {  // hand the window's kept edges to the nodes whose segments overlap it
          const int lo = max(a0, wb) - wb, hi = min(a1, wb + ne) - wb;
          if (hi > lo) {
            const uint64_t seg = (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo;
            c += __popcll(kb & seg);
          }
          if (a1 > wb + ne) break;  // node continues in the next window
          finish(j, c);
          c = 0;
          ++j;
          if (j < nq) {
            a0 = rdl(vp0, j);
            a1 = rdl(vp1, j);
          }
        }
      }
      for (; j < nq; ++j) {  // nodes without (remaining) edges
        finish(j, c);
        c = 0;
      }
    }
  }
  XPG_STAMP(1)
  __syncthreads();
  XPG_STAMP(2)
  float* h0 = lds + a.o_h0;
  float* h1b = lds + a.o_h1;
  const int fo = wave * FS;
  for (int t = 0; t < a.n_last; ++t) {
    int cur_w;
    float h[FS];
    if (a.n_layers == 1) {
      rows_h1<FS>(a, lds, t, fo, lane, h);
#pragma unroll
      for (int f = 0; f < FS; ++f) h0[(fo + f) * 64 + lane] = h[f];
      cur_w = a.f1_pad;
      XPG_STAMP(3)
      __syncthreads();
      XPG_STAMP(4)
    } else {
      float* A2 = lds + a.o_a2;
      const int tf0 = li[a.o_l2tgt + t], tp = li[a.o_l2prev + t];
      for (int k = 0; k < a.n_terms2; ++k) {
        const int kind = a.kind2[k], r = a.rel2[k];
        const float* dvr = lds + a.o_dv + r * a.n0 * 64 + lane;
        float acc[FS];
#pragma unroll
        for (int f = 0; f < FS; ++f) acc[f] = 0.f;
        float cself, cedge_t;
        int sm = 1;
        if (kind == XPG_TERM_ROOT) {
          cself = 1.f;
          cedge_t = 0.f;
        } else {
          const float kt = lds[a.o_kt + (r * a.n1 + tf0) * 64 + lane];
          if (kind == XPG_TERM_GCN) {
            const float dt = inv_sqrt_deg(kt);
            cself = dt * dt;
            cedge_t = kt >= 0.f ? dt : 0.f;
          } else {
            sm = li[a.o_l2smul + r * a.n2 + t];
            const float cnt = kt + static_cast<float>(sm);
            const float inv = 1.f / (cnt > 1.f ? cnt : 1.f);
            cself = kt >= 0.f ? static_cast<float>(sm) * inv : 0.f;
            cedge_t = kt >= 0.f ? inv : 0.f;
          }
        }
        if (sm > 0) {
          rows_h1<FS>(a, lds, tp, fo, lane, h);
#pragma unroll
          for (int f = 0; f < FS; ++f) acc[f] = fmaf(cself, h[f], acc[f]);
        }
        if (kind != XPG_TERM_ROOT) {
          const int e0 = li[a.o_l2ptr + r * (a.n2 + 1) + t], e1 = li[a.o_l2ptr + r * (a.n2 + 1) + t + 1];
          for (int e = e0; e < e1; ++e) {
            const int s1 = li[a.o_l2src + e], s0 = li[a.o_l2f0 + e];
            const float d = dvr[s0 * 64];
            const float c = kind == XPG_TERM_GCN ? d * cedge_t : (d > 0.f ? cedge_t : 0.f);
            rows_h1<FS>(a, lds, s1, fo, lane, h);
#pragma unroll
            for (int f = 0; f < FS; ++f) acc[f] = fmaf(c, h[f], acc[f]);
          }
        }
#pragma unroll
        for (int f = 0; f < FS; ++f) A2[(k * a.f1_pad + fo + f) * 64 + lane] = acc[f];
      }
      XPG_STAMP(3)
      __syncthreads();  // A2 complete over all waves' feature columns
      XPG_STAMP(4)
      const int K2 = a.n_terms2 * a.f1_pad;
      if (a.w2_lds) rows_dense(A2, K2, lds + a.o_w2, K2, a.bias2, a.f2_out, a.f2_pad, a.act2, h0, wave, lane);
      else rows_dense(A2, K2, a.w2, K2, a.bias2, a.f2_out, a.f2_pad, a.act2, h0, wave, lane);
      cur_w = a.f2_pad;
      __syncthreads();
    }
    XPG_STAMP(5)
    const float* cur = h0;
    float* nxt = h1b;
    for (int i = 0; i < a.n_head; ++i) {
      const FusedHead& hd = a.H[i];
      if (a.o_hw[i] >= 0)
        rows_dense(cur, cur_w, lds + a.o_hw[i], hd.k_pad, hd.bias, hd.n_real, hd.n_pad, hd.act, nxt, wave, lane);
      else
        rows_dense(cur, cur_w, hd.weight, hd.k_pad, hd.bias, hd.n_real, hd.n_pad, hd.act, nxt, wave, lane);
      __syncthreads();
      const float* tmp = cur;
      cur = nxt;
      nxt = const_cast<float*>(tmp);
      cur_w = hd.n_pad;
    }
    if (wave == 0 && lane < nrow) a.y[row * a.n_last + t] = cur[a.out_col * 64 + lane];
    __syncthreads();
    XPG_STAMP(6)
  }
  }  // blocks
#ifdef XPG_WLM_STAMPS
  if (blockIdx.x == 0 && (tid == 0 || tid == 1023)) {
    for (int q = 0; q < 8; ++q) g_wlm_stamps[tid == 0 ? 0 : 1][q] = stamp_acc[q];
  }
#endif
}

// ------------------------------------------------------------------------------ wide forward
// Masked forward for LARGE frontiers (the full-graph regime: every node a target, SURVEY.md §8d
// (ii)), 2-layer plans, 32 mask rows ("samples") per pass:
//   k_wide_bits    row bits -> node-major words mT[node] (bit s = sample s), 32 x 32 register
//                  transposes; k_wide_f0 gathers them to F_0 order (mT0)
//   k_wide_degree  (GCN terms) kept in-degree of every F_0 node for all 32 samples: kinT
//   k_wide_l1      layer 1 for all 32 samples at once, wave = target: each kept in-edge's table
//                  row X W^T is read ONCE per 32 samples (features are never masked, data.py:582)
//                  and scattered into 32 per-sample accumulators with per-sample coefficients
//   k_wide_last    layer 2 + head, workgroup = (sample, 32 targets): 16-lane groups gather the
//                  kept h1 rows of their targets (4 rows in flight per group) into an LDS tile,
//                  v_mfma_f32_32x32x2_f32 against the layer weights, bias/act, the dense head
//                  on the tile, and the output column.
// Same arithmetic per target as k_agg / k_dense.
constexpr int kWideS = 32;  // samples per pass

__global__ __launch_bounds__(256) void k_wide_bits(const uint32_t* __restrict__ bits, int64_t row0, int nr,
                                                   int words, int64_t cols, uint32_t* __restrict__ mT) {
  const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (w >= words) return;
  uint32_t x[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) x[i] = i < nr ? bits[(row0 + i) * words + w] : 0u;
  transpose32(x);
#pragma unroll
  for (int b = 0; b < 32; ++b) {
    const int64_t c = w * 32 + b;
    if (c < cols) mT[c] = x[b];
  }
}

__global__ void k_wide_f0(const uint32_t* __restrict__ mT, const int32_t* __restrict__ f0_node, int n0,
                          uint32_t* __restrict__ mT0) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n0) mT0[p] = mT[f0_node[p]];
}

// kinT[(r * n0 + p) * 32 + s]: kept in-degree (self-loops out) of F_0 node p under relation r in
// sample s, -1 when the node is masked out in s.  Thread = (item (r, p), sample s).
__global__ __launch_bounds__(256) void k_wide_degree(const uint32_t* __restrict__ mT, const uint32_t* __restrict__ mT0,
                                                     int n0, int n_rel, const int32_t* __restrict__ deg_ptr,
                                                     const int32_t* __restrict__ deg_src, float* __restrict__ kinT) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t item = gid >> 5;
  const int sidx = static_cast<int>(gid & 31);
  if (item >= (int64_t)n_rel * n0) return;
  const int r = static_cast<int>(item / n0), p = static_cast<int>(item - (int64_t)r * n0);
  float out = -1.f;
  if ((mT0[p] >> sidx) & 1u) {
    const int32_t* pp = deg_ptr + (int64_t)r * (n0 + 1);
    int c = 0;
    for (int e = pp[p]; e < pp[p + 1]; ++e) c += (mT[deg_src[e]] >> sidx) & 1u;
    out = static_cast<float>(c);
  }
  kinT[item * 32 + sidx] = out;
}

struct WideArgs {
  int64_t row0;  // global index of the block's first mask row (output rows of the last layer)
  int nr, n0, n_src, n_tgt, n_rel, n_terms, w_row, f_real, act;
  int agg1;  // the only aggregating (non-ROOT) term, or -1 when there are several
  int64_t rstride;  // floats between consecutive source rows: w_row (tables) or 32 w_row (h1)
  int head1;  // the head is one Linear(f_out, 1) (+ act) read at column 0: fused epilogue
  int sort_samples;  // IDX layer 2: gather groups take the target's samples active-first (see k_wide_last_ws)
  int early_prefetch;  // IDX layer 2: the next target's rows are issued before the A tile is finished
  int dbg;   // diagnostics (XPG_WIDE_DBG): 1 skip dense + head, 2 skip row gathers, 4 head, 8 dense;
             // warp-specialised layer 2: 16 no MFMA, 32 no gathers, 64 no epilogue, 128 no products,
             // 512 MFMA waves without the raised issue priority
  int K, a_ld, f_out, f_out_pad, n_head, out_col, h_ld, o_h0, o_h1, o_e;
  int o_hw[kFusedMaxHead];
  const uint32_t* mT0;
  const float* kinT;
  const float* src;  // last layer: h1 [n_src][32][w_row]
  const float* table[XPG_MAX_TERMS];  // layer 1: X W_k^T [n0][w_row]
  const int32_t* tgt_prev;
  const int32_t* tgt_f0;
  const int32_t* agg_ptr;
  const int32_t* agg_src;
  const int32_t* agg_f0;
  const int32_t* self_mult;
  const float* weight;  // last layer: [f_out_pad][K]
  const float* bias;
  int kind[XPG_MAX_TERMS], rel[XPG_MAX_TERMS];
  FusedHead H[kFusedMaxHead];
  float* out;  // layer 1: h1 [n_tgt][32][w_row] (node-major); last layer: y [rows][n_tgt]
  // inactive-row table ctab [n1][w_row] (nullable): the layer-1 row of a target masked out in a
  // sample does not depend on the sample (no kept in-edges: GCN keeps only the weight-1 self loop,
  // MEAN is 0; the ROOT terms and bias are the node's own), so layer 1 stores h1 only for the
  // samples that keep the target plus this one row, and layer 2 reads the row for the others
  float* ctab;
};

constexpr int kWideCap = 256;  // staged in-edges per target (all terms, one per thread); more: in place

// Sum of coef * source row over the kept in-edges [e0, e1) of one term for sample sidx (4 rows in
// flight per 16-lane group): STAGED reads (row, F_0 position, keep word) from the LDS stage,
// otherwise from the CSR in place.  Returns the number of kept edges.
template <int NFI, bool STAGED>
__device__ __forceinline__ int wide_gather_rows(const WideArgs& a, int k, int e0, int e1, const int* rowv,
                                                const int* u0v, const uint32_t* mv, int sidx, int kind, int r,
                                                float dt, const float* base, int fo, float (&acc)[NFI]) {
  int cnt = 0;
  for (int e = e0; e < e1; e += 4) {
    int row[4], u0[4];
    uint32_t m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // indices of 4 edges first (independent loads)
      const int ee = e + j < e1 ? e + j : e0;
      row[j] = rowv[ee];
      u0[j] = u0v[ee];
      m[j] = STAGED ? mv[ee] : 0u;
    }
    if (!STAGED) {
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = a.mT0[u0[j]];
    }
    float cf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool kept = e + j < e1 && ((m[j] >> sidx) & 1u);
      cf[j] = !kept ? 0.f : (kind == XPG_TERM_GCN ? dt * inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + u0[j]) * 32 + sidx]) : 1.f);
    }
    float rr[4][NFI];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < NFI; ++i) rr[j][i] = 0.f;
      if (cf[j] != 0.f) {
        const float* sp = base + (int64_t)row[j] * a.rstride + fo;
        if (NFI % 4 == 0) {
#pragma unroll
          for (int i = 0; i < NFI / 4; ++i) {
            const float4 v = reinterpret_cast<const float4*>(sp)[i];
            rr[j][4 * i] = v.x;
            rr[j][4 * i + 1] = v.y;
            rr[j][4 * i + 2] = v.z;
            rr[j][4 * i + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int i = 0; i < NFI / 2; ++i) {
            const float2 v = reinterpret_cast<const float2*>(sp)[i];
            rr[j][2 * i] = v.x;
            rr[j][2 * i + 1] = v.y;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cnt += cf[j] != 0.f;
#pragma unroll
      for (int i = 0; i < NFI; ++i) acc[i] = fmaf(cf[j], rr[j][i], acc[i]);
    }
  }
  return cnt;
}

// Both samples of a 16-lane group over the staged in-edges [e0, e1) of one term: 16 edges per
// round are tested lane-parallel, the kept ones of either sample are compacted with ballots and
// fetched RIF rows at a time (a slot takes sample s0's next kept edge, else s1's).
template <int NFI, int RIF>
__device__ __forceinline__ void wide_gather2(const WideArgs& a, int e0, int e1, const int* Esrc, const int* Eu0,
                                             const uint32_t* Em, int s0, int s1, bool tk0, bool tk1, int kind, int r,
                                             float dt0, float dt1, const float* base0, const float* base1, int fo,
                                             int gl, int lb, float (&acc0)[NFI], float (&acc1)[NFI], int& cnt0,
                                             int& cnt1) {
  for (int c0 = e0; c0 < e1; c0 += 16) {
    const int e = c0 + gl;
    const uint32_t m = e < e1 ? Em[e] : 0u;
    uint32_t m0 = static_cast<uint32_t>(__ballot(tk0 && ((m >> s0) & 1u)) >> lb) & 0xFFFFu;
    uint32_t m1 = static_cast<uint32_t>(__ballot(tk1 && ((m >> s1) & 1u)) >> lb) & 0xFFFFu;
    cnt0 += __popc(m0);
    cnt1 += __popc(m1);
    while (m0 | m1) {
      float rr[RIF][NFI];
      float c0v[RIF], c1v[RIF];
#pragma unroll
      for (int q = 0; q < RIF; ++q) {
        int j = -1;
        bool first = false;
        if (m0) {
          j = __builtin_ctz(m0);
          m0 &= m0 - 1u;
          first = true;
        } else if (m1) {
          j = __builtin_ctz(m1);
          m1 &= m1 - 1u;
        }
        c0v[q] = c1v[q] = 0.f;
#pragma unroll
        for (int i = 0; i < NFI; ++i) rr[q][i] = 0.f;
        if (j >= 0) {
          const int ee = c0 + j;
          const float* bp = first ? base0 : base1;
          const float* sp = bp + (int64_t)Esrc[ee] * a.rstride + fo;
          const int sidx = first ? s0 : s1;
          const float c = kind == XPG_TERM_GCN
                              ? (first ? dt0 : dt1) * inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + Eu0[ee]) * 32 + sidx])
                              : 1.f;
          c0v[q] = first ? c : 0.f;
          c1v[q] = first ? 0.f : c;
          if (NFI % 4 == 0) {
#pragma unroll
            for (int i = 0; i < NFI / 4; ++i) {
              const float4 v = reinterpret_cast<const float4*>(sp)[i];
              rr[q][4 * i] = v.x;
              rr[q][4 * i + 1] = v.y;
              rr[q][4 * i + 2] = v.z;
              rr[q][4 * i + 3] = v.w;
            }
          } else {
#pragma unroll
            for (int i = 0; i < NFI / 2; ++i) {
              const float2 v = reinterpret_cast<const float2*>(sp)[i];
              rr[q][2 * i] = v.x;
              rr[q][2 * i + 1] = v.y;
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < RIF; ++q)
#pragma unroll
        for (int i = 0; i < NFI; ++i) {
          acc0[i] = fmaf(c0v[q], rr[q][i], acc0[i]);
          acc1[i] = fmaf(c1v[q], rr[q][i], acc1[i]);
        }
    }
  }
}





// One launch per conv layer of a 2-layer plan, persistent (target += gridDim.x).  Item = one
// target for all 32 samples of the pass.  Its in-edges of every term (source row, F_0 position,
// 32-sample keep word) are staged in LDS once; then the 16 lane-groups of 16 lanes own samples
// g and g + 16 and gather their sample's kept source rows (NFI = w_row / 16 floats per lane,
// 4 rows in flight per group), in a fixed order per (target, sample): bitwise reproducible.
//   LAST = false (layer 1): sources are the shared tables X W_k^T (features are never masked,
//     data.py:582); the sum over terms + bias + act is written to h1[s][t].
//   LAST = true (layer 2 + head): each term's aggregate fills the sample's row of the A tile
//     (32 samples x K), v_mfma_f32_32x32x2_f32 against the layer weights (KW > 0: held in
//     registers, K = 8 KW; else read from L2), bias + act, the dense head on the tile, and the
//     output column for the 32 samples.
template <int NFI, bool LAST, int KW>
__global__ __launch_bounds__(256, LAST ? (KW == 0 && NFI <= 8 ? 3 : 2) : (NFI >= 12 ? 2 : 3)) void k_wide_tgt(const WideArgs a) {
  constexpr int RIF = (LAST && KW > 0) || NFI >= 8 ? 4 : 8;  // rows in flight per 16-lane group
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  float* A = wsm;  // LAST: [32][a_ld]
  int* Esrc = reinterpret_cast<int*>(wsm + a.o_e);
  int* Eu0 = Esrc + kWideCap;
  uint32_t* Em = reinterpret_cast<uint32_t*>(Eu0 + kWideCap);
  __shared__ int seg[XPG_MAX_TERMS + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = tid >> 4, gl = tid & 15, fo = gl * NFI;
  const int i32 = lane & 31, h = lane >> 5;
  float4 wreg[KW > 0 ? KW : 1];
  if (LAST) {
    if (KW > 0 && wave * 32 < a.f_out_pad) {
      const float* wp = a.weight + (int64_t)(wave * 32 + i32) * a.K + 4 * h;
#pragma unroll
      for (int kk = 0; kk < (KW > 0 ? KW : 1); ++kk) wreg[kk] = *reinterpret_cast<const float4*>(wp + kk * 8);
    }
    for (int li = 0; li < a.n_head; ++li) {  // head weights: once per (persistent) workgroup
      const FusedHead& hd = a.H[li];
      for (int e = tid; e < hd.n_real * hd.k_pad; e += 256) wsm[a.o_hw[li] + e] = hd.weight[e];
    }
  }
  // Software pipeline over this workgroup's targets: the next target's CSR ranges and edge
  // indices are loaded while the current one gathers, its keep words while it computes; the
  // staged edges are committed to LDS at the top of the next iteration (one edge per thread).
  int pf_seg[XPG_MAX_TERMS + 1], pf_p0[XPG_MAX_TERMS];
  int pf_u0 = 0, pf_src = 0, pf_tf0 = 0, pf_tp = 0;
  uint32_t pf_m = 0u, pf_mv = 0u;
  auto prefetch_idx = [&](int tn) {
    int off = 0, e = 0;
    if (a.agg1 >= 0) {  // one aggregating term (homogeneous GCN / SAGE): one CSR range, no loop
      const int32_t* pp = a.agg_ptr + (int64_t)a.rel[a.agg1] * (a.n_tgt + 1);
      const int b0 = pp[tn], b1 = pp[tn + 1];
#pragma unroll
      for (int k = 0; k <= XPG_MAX_TERMS; ++k) pf_seg[k] = k <= a.agg1 ? 0 : b1 - b0;
      off = b1 - b0;
      e = b0 + tid;
    } else {
#pragma unroll
      for (int k = 0; k < XPG_MAX_TERMS; ++k) {
        pf_seg[k] = off;
        pf_p0[k] = 0;
        if (k < a.n_terms && a.kind[k] != XPG_TERM_ROOT) {
          const int32_t* pp = a.agg_ptr + (int64_t)a.rel[k] * (a.n_tgt + 1);
          pf_p0[k] = pp[tn];
          off += pp[tn + 1] - pf_p0[k];
        }
      }
      pf_seg[XPG_MAX_TERMS] = off;
#pragma unroll
      for (int k = 0; k < XPG_MAX_TERMS; ++k)
        if (k < a.n_terms && a.kind[k] != XPG_TERM_ROOT && tid >= pf_seg[k]) e = pf_p0[k] + (tid - pf_seg[k]);
    }
    pf_tf0 = a.tgt_f0[tn];
    pf_tp = LAST ? a.tgt_prev[tn] : pf_tf0;
    if (off <= kWideCap && tid < off) {
      pf_u0 = a.agg_f0[e];
      pf_src = LAST ? a.agg_src[e] : pf_u0;
    }
  };
  auto prefetch_m = [&]() {
    pf_mv = a.mT0[pf_tf0];
    if (pf_seg[XPG_MAX_TERMS] <= kWideCap && tid < pf_seg[XPG_MAX_TERMS]) pf_m = a.mT0[pf_u0];
  };
  if (blockIdx.x < a.n_tgt) {
    prefetch_idx(blockIdx.x);
    prefetch_m();
  }
  for (int t = blockIdx.x; t < a.n_tgt; t += gridDim.x) {
    const int tn = t + gridDim.x;
    lds_barrier();  // the previous item's readers of E / A / the head tiles are done
    const int total = pf_seg[XPG_MAX_TERMS];
    const bool staged = total <= kWideCap;
    if (staged && tid < total) {
      Esrc[tid] = pf_src;
      Eu0[tid] = pf_u0;
      Em[tid] = pf_m;
    }
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k <= XPG_MAX_TERMS; ++k) seg[k] = pf_seg[k];  // term k: [seg[k], seg[k + 1])
    }
    const int tf0 = pf_tf0, tp = pf_tp;
    const uint32_t mv = pf_mv;
    if (tn < a.n_tgt) prefetch_idx(tn);
    lds_barrier();
    // ---- gather: group g owns samples s0 = g and s1 = g + 16
    {
      const int s0 = g, s1 = g + 16;
      const bool v0 = s0 < a.nr, v1 = s1 < a.nr;
      const bool tk0 = v0 && ((mv >> s0) & 1u), tk1 = v1 && ((mv >> s1) & 1u);
      float tot0[NFI], tot1[NFI];
#pragma unroll
      for (int i = 0; i < NFI; ++i) tot0[i] = tot1[i] = 0.f;
      for (int k = 0; k < a.n_terms; ++k) {
        const int kind = a.kind[k], r = a.rel[k];
        const float* base0 = LAST ? a.src + (int64_t)(v0 ? s0 : 0) * a.w_row : a.table[k];
        const float* base1 = LAST ? a.src + (int64_t)(v1 ? s1 : 0) * a.w_row : a.table[k];
        float self0[NFI], self1[NFI];
        {
          const float* p0r = base0 + (int64_t)tp * a.rstride + fo;
          const float* p1r = base1 + (int64_t)tp * a.rstride + fo;
#pragma unroll
          for (int i = 0; i < NFI; ++i) {
            self0[i] = p0r[i];
            self1[i] = LAST ? p1r[i] : self0[i];
          }
        }
        float acc0[NFI], acc1[NFI];
        if (kind == XPG_TERM_ROOT) {
#pragma unroll
          for (int i = 0; i < NFI; ++i) {
            acc0[i] = self0[i];
            acc1[i] = self1[i];
          }
        } else {
          float dt0 = 1.f, dt1 = 1.f;
          if (kind == XPG_TERM_GCN) {
            dt0 = inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + tf0) * 32 + s0]);
            dt1 = inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + tf0) * 32 + s1]);
          }
#pragma unroll
          for (int i = 0; i < NFI; ++i) acc0[i] = acc1[i] = 0.f;
          int cnt0 = 0, cnt1 = 0;
          if (a.dbg & 2) {
          } else if (staged) {
            wide_gather2<NFI, RIF>(a, seg[k], seg[k + 1], Esrc, Eu0, Em, s0, s1, tk0, tk1, kind, r, dt0, dt1, base0,
                                   base1, fo, gl, (lane & 48), acc0, acc1, cnt0, cnt1);
          } else {
            const int32_t* pp = a.agg_ptr + (int64_t)r * (a.n_tgt + 1);
            if (tk0)
              cnt0 = wide_gather_rows<NFI, false>(a, k, pp[t], pp[t + 1], LAST ? a.agg_src : a.agg_f0, a.agg_f0,
                                                  nullptr, s0, kind, r, dt0, base0, fo, acc0);
            if (tk1)
              cnt1 = wide_gather_rows<NFI, false>(a, k, pp[t], pp[t + 1], LAST ? a.agg_src : a.agg_f0, a.agg_f0,
                                                  nullptr, s1, kind, r, dt1, base1, fo, acc1);
          }
          if (kind == XPG_TERM_GCN) {
#pragma unroll
            for (int i = 0; i < NFI; ++i) {
              acc0[i] = fmaf(dt0 * dt0, self0[i], acc0[i]);
              acc1[i] = fmaf(dt1 * dt1, self1[i], acc1[i]);
            }
          } else {  // MEAN: 0 when the target is masked out in the sample
            const int sm = a.self_mult[(int64_t)r * a.n_tgt + t];
            const float inv0 = tk0 ? 1.f / static_cast<float>(max(cnt0 + sm, 1)) : 0.f;
            const float inv1 = tk1 ? 1.f / static_cast<float>(max(cnt1 + sm, 1)) : 0.f;
#pragma unroll
            for (int i = 0; i < NFI; ++i) {
              acc0[i] = fmaf(static_cast<float>(sm), self0[i], acc0[i]) * inv0;
              acc1[i] = fmaf(static_cast<float>(sm), self1[i], acc1[i]) * inv1;
            }
          }
        }
        if (LAST) {
#pragma unroll
          for (int i = 0; i < NFI; ++i) {
            A[s0 * a.a_ld + k * a.w_row + fo + i] = v0 ? acc0[i] : 0.f;
            A[s1 * a.a_ld + k * a.w_row + fo + i] = v1 ? acc1[i] : 0.f;
          }
        } else {
#pragma unroll
          for (int i = 0; i < NFI; ++i) {
            tot0[i] += acc0[i];
            tot1[i] += acc1[i];
          }
        }
      }
      if (!LAST) {
        float o0[NFI], o1[NFI];
#pragma unroll
        for (int i = 0; i < NFI; ++i) {
          const int f = fo + i;
          const float bv = f < a.f_real ? a.bias[f] : 0.f;
          o0[i] = f < a.f_real ? act_apply(tot0[i] + bv, a.act) : 0.f;
          o1[i] = f < a.f_real ? act_apply(tot1[i] + bv, a.act) : 0.f;
        }
        if (v0) {
          float* o = a.out + ((int64_t)t * 32 + s0) * a.w_row + fo;
#pragma unroll
          for (int i = 0; i < NFI; ++i) o[i] = o0[i];
        }
        if (v1) {
          float* o = a.out + ((int64_t)t * 32 + s1) * a.w_row + fo;
#pragma unroll
          for (int i = 0; i < NFI; ++i) o[i] = o1[i];
        }
      }
    }
    if (tn < a.n_tgt) prefetch_m();
    if (!LAST || (a.dbg & 1)) continue;
    lds_barrier();
    // ---- dense: C[32 samples x f_out_pad] = act(A W^T + b), wave = 32-column blocks
    float* H0 = wsm + a.o_h0;
    for (int nb = wave; nb * 32 < a.f_out_pad && !(a.dbg & 8); nb += 4) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.f;
      const float* ap = A + i32 * a.a_ld + 4 * h;
      if (KW > 0) {
#pragma unroll
        for (int kk = 0; kk < (KW > 0 ? KW : 1); ++kk) {
          const float4 av = *reinterpret_cast<const float4*>(ap + kk * 8);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wreg[kk].x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wreg[kk].y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wreg[kk].z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wreg[kk].w, acc, 0, 0, 0);
        }
      } else {
        // weights streamed from L2 through a ring of 4 float4 per lane: each slot is refilled
        // right after its MFMAs with an unconditional (clamped) load, so no loop-carried copy
        // forces a wait — the load lands one iteration (16 MFMAs) later.  The A tile (LDS) is
        // read half an iteration ahead.  Two independent accumulation chains; K % 32 == 0.
        const float* wp = a.weight + (int64_t)(nb * 32 + i32) * a.K + 4 * h;
        const int klast = a.K - 8;
        auto ldw = [&](int k) { return *reinterpret_cast<const float4*>(wp + (k < klast ? k : klast)); };
        auto lda = [&](int k) { return *reinterpret_cast<const float4*>(ap + k); };
        float4 w0 = ldw(0), w1 = ldw(8), w2 = ldw(16), w3 = ldw(24);
        float4 a0 = lda(0), a1 = lda(8);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 acc2;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc2[q] = 0.f;
        for (int kc = 0; kc < a.K; kc += 32) {
          const float4 a2 = lda(kc + 16), a3 = lda(kc + 24);
          __builtin_amdgcn_sched_barrier(0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, w0.x, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, w1.x, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, w0.y, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, w1.y, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, w0.z, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, w1.z, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, w0.w, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, w1.w, acc2, 0, 0, 0);
          w0 = ldw(kc + 32);
          w1 = ldw(kc + 40);
          const int kn = kc + 32 < a.K ? kc + 32 : 0;
          a0 = lda(kn);
          a1 = lda(kn + 8);
          __builtin_amdgcn_sched_barrier(0);  // keep the refills here (the scheduler sinks them to the use)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.x, w2.x, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.x, w3.x, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.y, w2.y, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.y, w3.y, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.z, w2.z, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.z, w3.z, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.w, w2.w, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.w, w3.w, acc2, 0, 0, 0);
          w2 = ldw(kc + 48);
          w3 = ldw(kc + 56);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] += acc2[q];
      }
      const int col = nb * 32 + i32;
      const float bv = col < a.f_out ? a.bias[col] : 0.f;
      if (a.head1) {  // single-logit head: the dot with its weight row, reduced over the block's columns
        const float hwc = col < a.f_out ? wsm[a.o_hw[0] + col] : 0.f;
        float part[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          part[reg] = col < a.f_out ? act_apply(acc[reg] + bv, a.act) * hwc : 0.f;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) part[reg] = half_wave_sum(part[reg]);
        if (i32 == 0) {  // lanes 0 and 32 hold the 16 sample rows of their half
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) H0[nb * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h] = part[reg];
        }
      } else {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
          H0[row * a.h_ld + col] = col < a.f_out ? act_apply(acc[reg] + bv, a.act) : 0.f;
        }
      }
    }
    lds_barrier();
    if (a.head1) {  // y[s] = act(sum over column blocks + b)
      if (tid < a.nr) {
        float v = 0.f;
        for (int nb = 0; nb * 32 < a.f_out_pad; ++nb) v += H0[nb * 32 + tid];
        a.out[(a.row0 + tid) * a.n_tgt + t] = act_apply(v + a.H[0].bias[0], a.H[0].act);
      }
      continue;
    }
    // ---- head on the tile: out[s][n] = act(sum_k cur[s][k] W[n][k] + b[n]) (n < n_real; pad 0)
    float* cur = H0;
    float* nxt = wsm + a.o_h1;
    int cur_w = a.f_out_pad;
    for (int li = 0; li < a.n_head && !(a.dbg & 4); ++li) {
      const FusedHead& hd = a.H[li];
      const float* hw = wsm + a.o_hw[li];
      for (int e = tid; e < 32 * hd.n_pad; e += 256) {
        const int ss = e / hd.n_pad, n = e - ss * hd.n_pad;
        float v = 0.f;
        if (n < hd.n_real) {
          const float4* cr = reinterpret_cast<const float4*>(cur + ss * a.h_ld);
          const float4* wr = reinterpret_cast<const float4*>(hw + n * hd.k_pad);
          float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
          for (int kk = 0; kk < cur_w / 4; ++kk) {
            const float4 c = cr[kk], w = wr[kk];
            v0 = fmaf(c.x, w.x, v0);
            v1 = fmaf(c.y, w.y, v1);
            v2 = fmaf(c.z, w.z, v2);
            v3 = fmaf(c.w, w.w, v3);
          }
          v = act_apply((v0 + v1) + (v2 + v3) + hd.bias[n], hd.act);
        }
        nxt[ss * a.h_ld + n] = v;
      }
      lds_barrier();
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
      cur_w = hd.n_pad;
    }
    if (tid < a.nr) a.out[(a.row0 + tid) * a.n_tgt + t] = cur[tid * a.h_ld + a.out_col];
  }
}

// Layer 2 + single-logit head of the wide path, warp-specialised (SAGE / GCN plans with one
// aggregating term; the c3 shape).  The phase costs of k_wide_tgt<.., true, 0> barely overlap
// (XPG_WIDE_DBG ablation at c3: gathers alone 10.7 ms, MFMA + head alone 20.5 ms, both 30.4 ms
// per 32-row pass), so here the two run in different waves of ONE persistent workgroup per CU:
//   waves 0-3  gather: 16-lane groups own samples g and g + 16 of target t_i and fill A[i & 1];
//              each group reads its in-edges straight from the CSR (16 per chunk, lane = edge,
//              the next target's first chunk and keep words prefetched while the current one
//              gathers), compacts the kept ones with ballots and keeps 8 source rows in flight
//   waves 4-7  MFMA: column block (wave - 4) of act(A W^T + b) for target t_{i-1} from
//              A[(i - 1) & 1] (v_mfma_f32_32x32x2_f32, weights streamed from L2 through a
//              register ring, two accumulation chains), the head dot reduced over the block's
//              columns into H0[(i - 1) & 1]; wave 4 then finishes target t_{i-2}'s logits
// One LDS barrier per target (double-buffered A and H0).  Same arithmetic per target as
// k_wide_tgt (fp32, fixed summation order).
// B3 (K = 256, the c3 SAGE shape): the f32 products run as three bf16 products on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate per k): the gather waves store each A value
// as hi = bf16(a), lo = bf16(a - hi) (two bf16 tiles, rows of K + 8 elements: the ds_read_b128
// lane groups hit 16 distinct 16-B bank quads), the MFMA waves split their weight columns the
// same way once into registers, and acc += a_hi w_hi + a_hi w_lo + a_lo w_hi (fp32 accumulate).
// Each operand keeps ~16 significant bits and the dropped a_lo w_lo term is ~2^-16 of the
// product: relative error ~1e-5 per product, accumulated with random signs (the parity suites
// run both; XPG_WIDE_B3=0 selects the exact f32 MFMA).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split_bf16x8(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = static_cast<__bf16>(x[j]);
    lo[j] = static_cast<__bf16>(x[j] - static_cast<float>(hi[j]));
  }
}

// TEAMS = 2 (GW = 8): the gather waves form two teams of 4 that gather two different targets
// at once (a group owns samples g and g + 16 of its team's target), so a CU keeps twice the
// rows in flight; the MFMA waves then take both targets of the previous interval (four A
// buffers).  A group's own gather is one dependent chain (CSR -> keep bits -> rows), so more
// targets in flight, not more waves per target, is what raises the CU's memory parallelism.
// PIPE (B3 with one team, SAGE-shaped plans: one MEAN term + one ROOT term): the gather role is
// software-pipelined across its targets.  A group's gather of one target is a chain of four
// dependent loads (CSR range → edge list → keep words → kept rows), so each stage runs one
// interval ahead of the next: at the start of interval k the group issues the keep words of
// target k + 1, the edge list of k + 2 and the CSR range of k + 3; before the barrier of
// interval k it issues the first 4 kept rows (and the own row) of target k + 1.  Interval k then
// only consumes loads that were in flight during the previous interval; kept edges past the
// first 4 of the first 16-edge chunk, and chunks past the first, are gathered in place.
// Same summation order as the plain gather (bitwise the same A tile).
// IDX (with PIPE): the target's index work is done ONCE per workgroup instead of by each of the 32
// gather groups (they all read the same CSR range, edge list and keep words, which hold every
// sample's bit): MFMA wave 0 -- idle most of each interval -- runs that chain ahead of the
// gathers (CSR range -> first kIxEdges in-edges -> keep words, software-pipelined one stage per
// interval, each stage's loads consumed an interval after their issue) and leaves per target the edges' source rows and 32-sample kept masks
// (source keep word & target keep word) in an LDS ring of three lists.  A gather group then
// reads its kept edges from the list (ballots over the mask bits), so its own chain per target
// is LDS -> kept rows.  In-degrees past kIxEdges keep the in-place path.  Same summation order as
// the plain gather: bitwise the same A tile.
// XPG_WIDE_DIAG (a diagnostics build only, never the product library): XPG_WIDE_DBG 1024 reads
// every gathered h1 row from the first 64 nodes (L2-resident: the gather's cost without HBM),
// 2048 drops the kept edges past the prefetched ones (the in-place rounds' cost).
// XPG_WIDE_STAMPS (a diagnostics build only): per-wave cycle counts of the layer-2 phases
// (s_memtime), per workgroup, read back with xpg_debug_wide_stamps (tools/ws_stamps.py)
#ifdef XPG_WIDE_STAMPS
__device__ uint64_t g_wide_stamps[512][16][8];
#define XPG_WST_INIT                                                       \
  uint64_t wst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};                          \
  uint64_t wst_last = __builtin_amdgcn_s_memtime();
#define XPG_WST(k)                                                         \
  {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                     \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                    \
    wst_acc[k] += now_ - wst_last;                                         \
    wst_last = now_;                                                       \
    __builtin_amdgcn_sched_barrier(0);                                     \
  }
// lane-indexed (vector) stores of the wave's totals
#define XPG_WST_STORE                                                      \
  if (blockIdx.x < 512 && lane < 8) {                                      \
    uint64_t v_ = 0;                                                       \
    for (int q_ = 0; q_ < 8; ++q_) v_ = lane == q_ ? wst_acc[q_] : v_;     \
    g_wide_stamps[blockIdx.x][wave][lane] = v_;                            \
  }
#else
#define XPG_WST_INIT
#define XPG_WST(k)
#define XPG_WST_STORE
#endif
#ifdef XPG_WIDE_DIAG
#define XPG_WDIAG_ROW(r) ((a.dbg & 1024) ? ((r) & 63) : (r))
#define XPG_WDIAG_REST(m) ((a.dbg & 2048) ? 0u : (m))
#else
#define XPG_WDIAG_ROW(r) (r)
#define XPG_WDIAG_REST(m) (m)
#endif
constexpr int kIxEdges = 32;                 // listed in-edges per target (32-bit kept masks)
constexpr int kIxInts = 2 * kIxEdges + 8 + 32;  // src[32] | km[32] | b0 b1 tp sm mv + pad | order[32]
constexpr int kIxOrder = 2 * kIxEdges + 8;       // order[g]: the sample gather group g takes

// position of the n-th set bit of m (n < popc(m)): binary search on prefix popcounts
__device__ __forceinline__ int nth_set_bit(uint32_t m, int n) {
  int pos = 0;
#pragma unroll
  for (int w = 16; w > 0; w >>= 1) {
    const uint32_t low = pos + w >= 32 ? 0xFFFFFFFFu : ((1u << (pos + w)) - 1u);
    if (__popc(m & low) <= n) pos += w;
  }
  return pos;
}


template <int NFI, int KW, int GW, bool B3 = false, int TEAMS = 1, bool PIPE = false, int RPF = 4,
          bool IDX = false, bool TH = false>
__global__ __launch_bounds__(64 * (GW + 4), (GW + 4) / 4) void k_wide_last_ws(const WideArgs a) {
  constexpr int RIF = 8;
  // GW / TEAMS = 4 gather waves per target: a group owns samples g and g + 16; 8: sample g
  constexpr bool TWO = GW / TEAMS == 4;
  static_assert(TEAMS == 1 || (TEAMS == 2 && GW == 8), "two teams of four gather waves");
  static_assert(!B3 || (KW == 32 && NFI == 8), "B3: K = 256, 8 features per gather lane");
  constexpr int KB = B3 ? 8 * KW / 16 : 1;  // bf16 k-blocks of 16
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int aph = a.K + 8;  // B3: bf16 elements per A row
  const int abuf = B3 ? 32 * aph : 32 * a.a_ld;  // floats per A buffer (B3: hi + lo bf16 tiles)
  float* H0 = wsm + 2 * TEAMS * abuf;  // [2][TEAMS][f_out_pad]: head partials per (column block, sample)
  // WL (B3, one team): the weight lo pieces live in LDS ([kb][h][column][8] bf16: a ds_read_b128
  // lane group reads 16 distinct columns = 16 distinct bank quads), which frees 64 VGPRs of the
  // MFMA waves for A / weight fragments loaded two k-blocks ahead (with all pieces in registers
  // every A read waited for its LDS latency right before its MFMA)
  constexpr bool WL = B3 && TEAMS == 1;
  __bf16* WLs = reinterpret_cast<__bf16*>(H0 + 2 * TEAMS * a.f_out_pad);
  // IDX: three in-edge lists [kIxInts] after the weight lo pieces (16-B aligned)
  int* IX = reinterpret_cast<int*>(WLs + (WL ? (int64_t)a.K * a.f_out_pad : 0));
  const int ntgt_wg = a.n_tgt > (int)blockIdx.x ? (a.n_tgt - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nint = (ntgt_wg + TEAMS - 1) / TEAMS;  // intervals (one LDS barrier each)
  const int kagg = a.agg1;
  const int ragg = a.rel[kagg];
  const int32_t* aptr = a.agg_ptr + (int64_t)ragg * (a.n_tgt + 1);
  if constexpr (PIPE) {
    static_assert(!TWO && TEAMS == 1 && B3, "pipelined gather: one sample per group, one team, B3 tiles");
  }
  static_assert(!IDX || PIPE, "shared index lists: pipelined gather only");
  const int32_t* smul_all = a.self_mult + (int64_t)ragg * a.n_tgt;
  // ---- IDX index chain (MFMA wave 0, lane = listed edge): stage A = CSR range / target fields,
  // B = the first kIxEdges edges' sources, C = keep words -> the LDS list of the target.  Every
  // load is a vector load, also the target's own fields (lanes 0-4: CSR begin / end, first-layer
  // position, previous-layer position, self count; lane 32 of stage C: the target's keep word):
  // a wave-uniform address compiles to a scalar load, and lgkmcnt counts scalar loads together
  // with LDS accesses, so each LDS wait of the wave (the list stores, the logit reads, the MFMA
  // operand reads) waited for the chain's loads from HBM too
  int qa_v = 0, qb_v = 0, qb_src = 0, qb_u0 = 0, qc_v = 0, qc_src = 0;
  uint32_t qc_em = 0u;
  auto stA = [&](int k) {
    if (k >= ntgt_wg) return;
    const int t = blockIdx.x + k * gridDim.x;
    const int32_t* pa = lane < 2 ? aptr + t + lane : lane == 2 ? a.tgt_f0 + t : lane == 3 ? a.tgt_prev + t
                                                                                            : smul_all + t;
    qa_v = *pa;
  };
  auto stB = [&](int k) {
    if (k >= ntgt_wg) return;
    qb_v = qa_v;
    const int b0 = __builtin_amdgcn_readlane(qa_v, 0), b1 = __builtin_amdgcn_readlane(qa_v, 1);
    const int tf0 = __builtin_amdgcn_readlane(qa_v, 2);
    const int e = b0 + lane;
    qb_src = e < b1 && lane < kIxEdges ? a.agg_src[e] : 0;
    qb_u0 = lane < kIxEdges ? (e < b1 ? a.agg_f0[e] : 0) : tf0;  // lanes >= kIxEdges: the target
  };
  auto stC_load = [&](int k) {
    if (k >= ntgt_wg) return;
    qc_v = qb_v;
    qc_src = qb_src;
    qc_em = a.mT0[qb_u0];
  };
  auto stC_store = [&](int k) {
    if (k >= ntgt_wg) return;
    int* ix = IX + (k % 3) * kIxInts;
    const int b0 = __builtin_amdgcn_readlane(qc_v, 0), b1 = __builtin_amdgcn_readlane(qc_v, 1);
    const uint32_t qc_mv = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(qc_em), kIxEdges));
    if (lane < kIxEdges) {
      ix[lane] = qc_src;
      ix[kIxEdges + lane] = b0 + lane < b1 ? static_cast<int>(qc_em & qc_mv) : 0;
    }
    if (lane == 0) {
      ix[2 * kIxEdges] = b0;
      ix[2 * kIxEdges + 1] = b1;
      ix[2 * kIxEdges + 2] = __builtin_amdgcn_readlane(qc_v, 3);
      ix[2 * kIxEdges + 3] = __builtin_amdgcn_readlane(qc_v, 4);
      ix[2 * kIxEdges + 4] = static_cast<int>(qc_mv);
    }
    // sample order: the target's active samples (keep bit set) first, then the others, each in
    // sample order.  A gather wave's four groups then hold samples of alike activity: a wave of
    // masked-out samples issues no row slot at all, and a wave's slot count (the maximum over
    // its groups' kept edges) is not raised by a busy sample among idle ones.  Per sample the
    // edges are summed in the same order: the A tile is bitwise the same.  (Ordering by kept
    // count instead packs the slot loads fuller, 0.8 of their lanes against 0.6, but the index
    // wave's per-sample counts and sort cost more than the loads saved: profiles/r4_cntsort.log)
    if (lane < 32) {
      const int na = __popc(qc_mv);
      ix[kIxOrder + lane] = lane < na ? nth_set_bit(qc_mv, lane) : nth_set_bit(~qc_mv, lane - na);
    }
  };
  // the index wave: the last MFMA wave (MFMA wave 0 also writes the logits; per-wave stamps,
  // profiles/r4_ws_stamps_*.log: the MFMA waves past the first wait at the barrier for about half
  // of each interval)
  const bool ixw = IDX && wave == GW + 3 && !(a.dbg & 32);
  // TH (with IDX): the layer bias and the head's weight row in LDS after the lists ([f_out_pad]
  // each), read back four columns at a time by the transposed epilogue
  float* const HBW = reinterpret_cast<float*>(IX + 3 * kIxInts);
  if constexpr (TH) {
    static_assert(IDX && B3 && TEAMS == 1, "transposed head epilogue: B3 IDX kernel");
    for (int c = tid - 64 * GW; c >= 0 && c < a.f_out_pad; c += 256) {
      HBW[c] = c < a.f_out ? a.bias[c] : 0.f;
      HBW[a.f_out_pad + c] = c < a.f_out ? a.H[0].weight[c] : 0.f;
    }
  }
  if constexpr (IDX) {
    // prologue: the lists of targets 0 and 1, the chain state of targets 2 (C: stored at the
    // start of interval 0), 3 (B) and 4 (A)
    if (ixw) {
      stA(0); stB(0); stC_load(0); stC_store(0);
      stA(1); stB(1); stC_load(1); stC_store(1);
      stA(2); stB(2); stC_load(2);
      stA(3); stB(3); stA(4);
    }
    lds_barrier();
  }
  if (PIPE && IDX && wave < GW) {
    // ------------------------------------------------------------------ gather role, shared lists
    const int g = tid >> 4, gl = tid & 15, fo = gl * NFI, lb = lane & 48;
    // the group's sample of the current target (p_s0: the list's order with sort_samples, else
    // sample g) and of the prefetched one
    int s0 = g;
    bool v0 = s0 < a.nr;
    const float* base0 = a.src + (int64_t)(v0 ? s0 : 0) * a.w_row;
    int p_s0 = g;
    constexpr int64_t RS = 32 * 16 * NFI;  // h1 row stride (node-major: 32 samples x w_row floats)
    const int kroot = 1 - kagg;            // host-checked: terms {MEAN, ROOT}
    constexpr int RP = RPF;
    constexpr int RI = 4;
    __bf16* const Ab = reinterpret_cast<__bf16*>(wsm);
    uint32_t p_rest = 0u;
    int p_cnt = 0, p_sm = 0, p_b0 = 0, p_b1 = 0, p_fill = 0;
    bool p_tk = false;
    // the own rows of the current and the prefetched target alternate between two arrays (the
    // loop runs two targets per trip): a loaded array that is not the one the next trip reads
    // would be copied at the back edge, after a wait for every load in flight
    float p_cv[RP], p_row[RP][NFI], p_selfA[NFI], p_selfB[NFI];
#pragma unroll
    for (int jj = 0; jj < RP; ++jj)
#pragma unroll
      for (int x = 0; x < NFI; ++x) p_row[jj][x] = 0.f;  // slots keep finite values: 0 x stale row = 0
    XPG_WST_INIT
    // the next target's kept edges from its list (wave-uniform k: the ballots see every lane),
    // its first RP kept rows (slot jj loaded only by the groups with a jj-th kept edge, and only
    // while some group of the wave has one) and its own row in flight
    auto prefetch = [&](int k, float (&p_self)[NFI]) {
      if (k >= ntgt_wg) return;
      const int* ix = IX + (k % 3) * kIxInts;
      // every LDS read of the list is issued up front and waited for once: read one after another
      // behind the branches that use them, each paid the LDS latency in turn (the list header,
      // the sample order, each 16-edge chunk of kept masks, then each slot's source row)
      const int b0 = ix[2 * kIxEdges], b1 = ix[2 * kIxEdges + 1], tp = ix[2 * kIxEdges + 2];
      const int smk = ix[2 * kIxEdges + 3];
      const uint32_t mv = static_cast<uint32_t>(ix[2 * kIxEdges + 4]);
      const int ord = ix[kIxOrder + g];
      uint32_t kmc[kIxEdges / 16];
#pragma unroll
      for (int c = 0; c < kIxEdges / 16; ++c) kmc[c] = static_cast<uint32_t>(ix[kIxEdges + 16 * c + gl]);
#pragma unroll
      for (int c = 0; c < kIxEdges / 16; ++c) asm volatile("" ::"v"(kmc[c]));  // not sunk into the branches
      XPG_WST(6)
      const int sk = a.sort_samples ? ord : g;  // group-uniform
      const bool vk = sk < a.nr;
      const float* bk = a.src + (int64_t)(vk ? sk : 0) * a.w_row;
      p_s0 = sk;
      const bool tk = vk && ((mv >> sk) & 1u);
      const int ne = min(b1 - b0, kIxEdges);
      uint32_t M = 0u;
#pragma unroll
      for (int c = 0; c < kIxEdges / 16; ++c) {
        if (16 * c < ne) {  // workgroup-uniform
          const uint32_t km = 16 * c + gl < ne ? kmc[c] : 0u;
          M |= (static_cast<uint32_t>(__ballot(tk && ((km >> sk) & 1u)) >> lb) & 0xFFFFu) << (16 * c);
        }
      }
      p_cnt = __popc(M);
      p_tk = tk;
      p_sm = smk;
      p_b0 = b0;
      p_b1 = b1;
      const float* p0r = a.ctab && !((mv >> sk) & 1u) ? a.ctab + (int64_t)tp * a.w_row + fo
                                                       : bk + (int64_t)XPG_WDIAG_ROW(tp) * RS + fo;
      // the source rows of the group's first RP kept edges (slot jj: the jj-th set bit of M)
      int srcs[RP];
      {
        uint32_t Mx = M;
#pragma unroll
        for (int jj = 0; jj < RP; ++jj) {
          srcs[jj] = ix[Mx ? __builtin_ctz(Mx) : 0];
          Mx &= Mx - 1u;
        }
#pragma unroll
        for (int jj = 0; jj < RP; ++jj) asm volatile("" ::"v"(srcs[jj]));  // all reads issued here
      }
      XPG_WST(7)
      int fill = 0;
#pragma unroll
      for (int jj = 0; jj < RP; ++jj) {
        p_cv[jj] = M ? 1.f : 0.f;
        if (__ballot(M != 0u) != 0ull) {  // wave-uniform: some group has a jj-th kept edge
          fill = jj + 1;
          if (M) {
            const float* sp = bk + (int64_t)XPG_WDIAG_ROW(srcs[jj]) * RS + fo;
#pragma unroll
            for (int x = 0; x < NFI / 4; ++x) {
              const float4 v = reinterpret_cast<const float4*>(sp)[x];
              p_row[jj][4 * x] = v.x;
              p_row[jj][4 * x + 1] = v.y;
              p_row[jj][4 * x + 2] = v.z;
              p_row[jj][4 * x + 3] = v.w;
            }
          }
        }
        M &= M - 1u;
      }
      p_fill = fill;
      p_rest = M;
#pragma unroll
      for (int x = 0; x < NFI / 4; ++x) {
        const float4 v = reinterpret_cast<const float4*>(p0r)[x];
        p_self[4 * x] = v.x;
        p_self[4 * x + 1] = v.y;
        p_self[4 * x + 2] = v.z;
        p_self[4 * x + 3] = v.w;
      }
    };
    const bool run = !(a.dbg & 32);  // dbg 32 (diagnostics): no gathers
    if (run) prefetch(0, p_selfA);
    auto step = [&](int i, float (&p_self)[NFI], float (&p_next)[NFI]) {
      if (run && i < ntgt_wg) {
        s0 = p_s0;  // the sample of target i (set by its prefetch)
        v0 = s0 < a.nr;
        base0 = a.src + (int64_t)(v0 ? s0 : 0) * a.w_row;
        float acc[NFI];
#pragma unroll
        for (int x = 0; x < NFI; ++x) acc[x] = 0.f;
#pragma unroll
        for (int q = 0; q < RP; ++q)
          if (q < p_fill) {  // wave-uniform
#pragma unroll
            for (int x = 0; x < NFI; ++x) acc[x] = fmaf(p_cv[q], p_row[q][x], acc[x]);
          }
        XPG_WST(1)
        // listed kept edges past the prefetched ones, in place (ctz order), RI rows per round
        const int* ix = IX + (i % 3) * kIxInts;
        uint32_t m = XPG_WDIAG_REST(p_rest);
        while (m) {  // group-uniform
          float rr[RI][NFI];
          float cv[RI];
          // a round's empty slots re-read its first kept row: a row layer 1 wrote (h1 holds rows
          // only for the samples that keep the node; 0 x an unwritten row may be 0 x NaN)
          const int jf = __builtin_ctz(m);
#pragma unroll
          for (int q = 0; q < RI; ++q) {
            const int j = m ? __builtin_ctz(m) : jf;
            cv[q] = m ? 1.f : 0.f;
            m &= m - 1u;
            const float* sp = base0 + (int64_t)XPG_WDIAG_ROW(ix[j]) * RS + fo;
#pragma unroll
            for (int x = 0; x < NFI / 4; ++x) {
              const float4 v = reinterpret_cast<const float4*>(sp)[x];
              rr[q][4 * x] = v.x;
              rr[q][4 * x + 1] = v.y;
              rr[q][4 * x + 2] = v.z;
              rr[q][4 * x + 3] = v.w;
            }
          }
#pragma unroll
          for (int q = 0; q < RI; ++q)
#pragma unroll
            for (int x = 0; x < NFI; ++x) acc[x] = fmaf(cv[q], rr[q][x], acc[x]);
        }
        int cnt = p_cnt;
        // in-edges past the list (in-degree > kIxEdges): straight from the CSR, in place
        for (int c0 = p_b0 + kIxEdges; c0 < p_b1; c0 += 16) {
          const int e = c0 + gl;
          const int esrc = e < p_b1 ? a.agg_src[e] : 0;
          const int eu0 = e < p_b1 ? a.agg_f0[e] : 0;
          const uint32_t em = e < p_b1 ? a.mT0[eu0] : 0u;
          uint32_t mm = static_cast<uint32_t>(__ballot(p_tk && ((em >> s0) & 1u)) >> lb) & 0xFFFFu;
          cnt += __popc(mm);
          while (mm) {
            float rr[RI][NFI];
            float cv[RI];
            const int jf = __builtin_ctz(mm);  // empty slots: the round's first kept row (above)
#pragma unroll
            for (int q = 0; q < RI; ++q) {
              const int j = mm ? __builtin_ctz(mm) : jf;
              cv[q] = mm ? 1.f : 0.f;
              mm &= mm - 1u;
              const int srow = __shfl(esrc, lb + j, 64);
              const float* sp = base0 + (int64_t)XPG_WDIAG_ROW(srow) * RS + fo;
#pragma unroll
              for (int x = 0; x < NFI / 4; ++x) {
                const float4 v = reinterpret_cast<const float4*>(sp)[x];
                rr[q][4 * x] = v.x;
                rr[q][4 * x + 1] = v.y;
                rr[q][4 * x + 2] = v.z;
                rr[q][4 * x + 3] = v.w;
              }
            }
#pragma unroll
            for (int q = 0; q < RI; ++q)
#pragma unroll
              for (int x = 0; x < NFI; ++x) acc[x] = fmaf(cv[q], rr[q][x], acc[x]);
          }
        }
        // every load of target i has been consumed: the own row goes into the ROOT columns of the
        // A tile and into the mean's sum first, so no register of target i is live across the
        // next target's loads (a loaded register still live there costs a copy at the loop's back
        // edge, i.e. a wait for every load in flight before the barrier); with early_prefetch the
        // next target's rows then go out and the mean, the bf16 split and the A stores of the
        // aggregate run while they are in flight
        __bf16* A = Ab + (i & 1) * 2 * abuf;  // abuf floats = 2 abuf bf16
        const int sm_i = p_sm;
        const bool tk_i = p_tk;
        XPG_WST(2)
        {
          float self[NFI];
#pragma unroll
          for (int x = 0; x < NFI; ++x) {
            acc[x] = fmaf(static_cast<float>(sm_i), p_self[x], acc[x]);
            self[x] = v0 ? p_self[x] : 0.f;
          }
          bf16x8 hi, lo;
          split_bf16x8(self, hi, lo);
          const int er = s0 * aph + kroot * a.w_row + fo;
          *reinterpret_cast<bf16x8*>(A + er) = hi;
          *reinterpret_cast<bf16x8*>(A + 32 * aph + er) = lo;
        }
        XPG_WST(3)
        if (a.early_prefetch) prefetch(i + 1, p_next);  // list of target i + 1: written at interval i - 1
        XPG_WST(4)
        const float inv = tk_i ? 1.f / static_cast<float>(max(cnt + sm_i, 1)) : 0.f;
        {
          bf16x8 hi, lo;
#pragma unroll
          for (int x = 0; x < NFI; ++x) acc[x] = v0 ? acc[x] * inv : 0.f;
          split_bf16x8(acc, hi, lo);
          const int ea = s0 * aph + kagg * a.w_row + fo;
          *reinterpret_cast<bf16x8*>(A + ea) = hi;
          *reinterpret_cast<bf16x8*>(A + 32 * aph + ea) = lo;
        }
        XPG_WST(5)
        if (!a.early_prefetch) prefetch(i + 1, p_next);  // list of target i + 1: written at interval i - 1 (or the prologue)
        XPG_WST(4)
      }
      lds_barrier();
      XPG_WST(0)
    };
    for (int i = 0; i <= nint + 1; i += 2) {
      step(i, p_selfA, p_selfB);
      if (i + 1 <= nint + 1) step(i + 1, p_selfB, p_selfA);
    }
    XPG_WST_STORE
  } else if (PIPE && wave < GW) {
    // ------------------------------------------------------------------ pipelined gather role
    const int g = tid >> 4, gl = tid & 15, fo = gl * NFI, lb = lane & 48;
    const int s0 = g;
    const bool v0 = s0 < a.nr;
    const float* base0 = a.src + (int64_t)(v0 ? s0 : 0) * a.w_row;
    const int32_t* smul = a.self_mult + (int64_t)ragg * a.n_tgt;
    const int kroot = 1 - kagg;  // host-checked: terms {MEAN, ROOT}
    constexpr int RP = RPF;      // prefetched kept rows per target (~2.5 kept per 16-edge chunk)
    constexpr int RI = 4;        // rows per round of the in-place remainder
    __bf16* const Ab = reinterpret_cast<__bf16*>(wsm);
    // stage states: 1 = CSR range / node / prev position / self count, 2 = + this lane's edge,
    // 3 = + keep words, 4 = + the first kept rows and the own row (the current target)
    int q1_b0 = 0, q1_b1 = 0, q1_tf0 = 0, q1_tp = 0, q1_sm = 0;
    int q2_b0 = 0, q2_b1 = 0, q2_tf0 = 0, q2_tp = 0, q2_sm = 0, q2_src = 0, q2_u0 = 0;
    int q3_b0 = 0, q3_b1 = 0, q3_tp = 0, q3_sm = 0, q3_src = 0;
    uint32_t q3_mv = 0u, q3_em = 0u;
    int q4_b0 = 0, q4_b1 = 0, q4_sm = 0, q4_src = 0, q4_cnt = 0;
    uint32_t q4_rest = 0u;
    bool q4_tk = false;
    float q4_cv[RP], q4_row[RP][NFI], q4_self[NFI];
    auto st1 = [&](int k) {
      if (k >= ntgt_wg) return;
      const int t = blockIdx.x + k * gridDim.x;
      q1_b0 = aptr[t];
      q1_b1 = aptr[t + 1];
      q1_tf0 = a.tgt_f0[t];
      q1_tp = a.tgt_prev[t];
      q1_sm = smul[t];
    };
    auto st2 = [&](int k) {
      if (k >= ntgt_wg) return;
      q2_b0 = q1_b0; q2_b1 = q1_b1; q2_tf0 = q1_tf0; q2_tp = q1_tp; q2_sm = q1_sm;
      const int e = q1_b0 + gl;
      q2_src = e < q1_b1 ? a.agg_src[e] : 0;
      q2_u0 = e < q1_b1 ? a.agg_f0[e] : 0;
    };
    auto st3 = [&](int k) {
      if (k >= ntgt_wg) return;
      q3_b0 = q2_b0; q3_b1 = q2_b1; q3_tp = q2_tp; q3_sm = q2_sm; q3_src = q2_src;
      q3_mv = a.mT0[q2_tf0];
      q3_em = q2_b0 + gl < q2_b1 ? a.mT0[q2_u0] : 0u;
    };
    auto st4 = [&](int k) {  // wave-uniform k: the ballot sees every lane
      if (k >= ntgt_wg) return;
      q4_b0 = q3_b0; q4_b1 = q3_b1; q4_sm = q3_sm; q4_src = q3_src;
      q4_tk = v0 && ((q3_mv >> s0) & 1u);
      uint32_t m0 = static_cast<uint32_t>(__ballot(q4_tk && ((q3_em >> s0) & 1u)) >> lb) & 0xFFFFu;
      q4_cnt = __popc(m0);
      // the target's own row: its inactive-row table entry when the sample masks it out (ctab)
      const float* p0r = a.ctab && !((q3_mv >> s0) & 1u) ? a.ctab + (int64_t)q3_tp * a.w_row + fo
                                                          : base0 + (int64_t)q3_tp * a.rstride + fo;
#pragma unroll
      for (int jj = 0; jj < RP; ++jj) {
        const int j = m0 ? __builtin_ctz(m0) : 0;
        q4_cv[jj] = m0 ? 1.f : 0.f;
        m0 &= m0 - 1u;
        const int srow = __shfl(q3_src, lb + j, 64);
        // an empty slot re-reads the own row (a written row: 0 x row stays finite)
        const float* sp = q4_cv[jj] != 0.f ? base0 + (int64_t)srow * a.rstride + fo : p0r;
#pragma unroll
        for (int x = 0; x < NFI / 4; ++x) {
          const float4 v = reinterpret_cast<const float4*>(sp)[x];
          q4_row[jj][4 * x] = v.x;
          q4_row[jj][4 * x + 1] = v.y;
          q4_row[jj][4 * x + 2] = v.z;
          q4_row[jj][4 * x + 3] = v.w;
        }
      }
      q4_rest = m0;
#pragma unroll
      for (int x = 0; x < NFI / 4; ++x) {
        const float4 v = reinterpret_cast<const float4*>(p0r)[x];
        q4_self[4 * x] = v.x;
        q4_self[4 * x + 1] = v.y;
        q4_self[4 * x + 2] = v.z;
        q4_self[4 * x + 3] = v.w;
      }
    };
    // kept edges of mask m (group lanes = the chunk's edges, sources in esrc) in place, RI rows
    // per round, added in ctz order
    auto gather_in_place = [&](uint32_t m, int esrc, float (&acc)[NFI]) {
      while (m) {  // group-uniform
        float rr[RI][NFI];
        float cv[RI];
        // empty slots re-read the round's first kept row: a written row (h1 holds rows only for
        // the samples that keep the node; 0 x an unwritten row may be 0 x NaN)
        const int jf = __builtin_ctz(m);
#pragma unroll
        for (int q = 0; q < RI; ++q) {
          const int j = m ? __builtin_ctz(m) : jf;
          cv[q] = m ? 1.f : 0.f;
          m &= m - 1u;
          const int srow = __shfl(esrc, lb + j, 64);
          const float* sp = base0 + (int64_t)srow * a.rstride + fo;
#pragma unroll
          for (int x = 0; x < NFI / 4; ++x) {
            const float4 v = reinterpret_cast<const float4*>(sp)[x];
            rr[q][4 * x] = v.x;
            rr[q][4 * x + 1] = v.y;
            rr[q][4 * x + 2] = v.z;
            rr[q][4 * x + 3] = v.w;
          }
        }
#pragma unroll
        for (int q = 0; q < RI; ++q)
#pragma unroll
          for (int x = 0; x < NFI; ++x) acc[x] = fmaf(cv[q], rr[q][x], acc[x]);
      }
    };
    const bool run = !(a.dbg & 32);  // dbg 32 (diagnostics): no gathers
    if (run) {
      st1(0); st2(0); st3(0); st4(0);
      st1(1); st2(1); st1(2);
    }
    for (int i = 0; i <= nint + 1; ++i) {
      if (run && i < ntgt_wg) {
        st3(i + 1);  // q2 = stage 2 of i + 1 (issued one interval ago)
        st2(i + 2);  // q1 = stage 1 of i + 2
        st1(i + 3);
        float acc[NFI];
#pragma unroll
        for (int x = 0; x < NFI; ++x) acc[x] = 0.f;
#pragma unroll
        for (int q = 0; q < RP; ++q)
#pragma unroll
          for (int x = 0; x < NFI; ++x) acc[x] = fmaf(q4_cv[q], q4_row[q][x], acc[x]);
        gather_in_place(q4_rest, q4_src, acc);
        int cnt = q4_cnt;
        for (int c0 = q4_b0 + 16; c0 < q4_b1; c0 += 16) {  // in-degree > 16: later chunks in place
          const int e = c0 + gl;
          const int esrc = e < q4_b1 ? a.agg_src[e] : 0;
          const int eu0 = e < q4_b1 ? a.agg_f0[e] : 0;
          const uint32_t em = e < q4_b1 ? a.mT0[eu0] : 0u;
          const uint32_t m = static_cast<uint32_t>(__ballot(q4_tk && ((em >> s0) & 1u)) >> lb) & 0xFFFFu;
          cnt += __popc(m);
          gather_in_place(m, esrc, acc);
        }
        const float inv = q4_tk ? 1.f / static_cast<float>(max(cnt + q4_sm, 1)) : 0.f;
        float self[NFI];
#pragma unroll
        for (int x = 0; x < NFI; ++x) {
          self[x] = q4_self[x];
          acc[x] = fmaf(static_cast<float>(q4_sm), self[x], acc[x]) * inv;
        }
        __bf16* A = Ab + (i & 1) * 2 * abuf;  // abuf floats = 2 abuf bf16
        bf16x8 hi, lo;
#pragma unroll
        for (int x = 0; x < NFI; ++x) {
          acc[x] = v0 ? acc[x] : 0.f;
          self[x] = v0 ? self[x] : 0.f;
        }
        split_bf16x8(acc, hi, lo);
        const int ea = s0 * aph + kagg * a.w_row + fo;
        *reinterpret_cast<bf16x8*>(A + ea) = hi;
        *reinterpret_cast<bf16x8*>(A + 32 * aph + ea) = lo;
        split_bf16x8(self, hi, lo);
        const int er = s0 * aph + kroot * a.w_row + fo;
        *reinterpret_cast<bf16x8*>(A + er) = hi;
        *reinterpret_cast<bf16x8*>(A + 32 * aph + er) = lo;
        st4(i + 1);  // q3 = stage 3 of i + 1 (issued at the top of this interval)
      }
      lds_barrier();
    }
  } else if (wave < GW) {
    // ------------------------------------------------------------------ gather role
    const int team = TEAMS == 2 ? wave >> 2 : 0;
    const int g = (TEAMS == 2 ? tid & 255 : tid) >> 4, gl = tid & 15, fo = gl * NFI, lb = lane & 48;
    const int s0 = g, s1 = TWO ? g + 16 : g;
    const bool v0 = s0 < a.nr, v1 = TWO && s1 < a.nr;
    const float* base0 = a.src + (int64_t)(v0 ? s0 : 0) * a.w_row;
    const float* base1 = a.src + (int64_t)(v1 ? s1 : 0) * a.w_row;
    // prefetched state of the group's next target
    int pb0 = 0, pb1 = 0, psrc = 0, pu0 = 0, ptf0 = 0, ptp = 0;
    uint32_t pm = 0u, pmv = 0u;
    auto prefetch = [&](int tn) {
      pb0 = aptr[tn];
      pb1 = aptr[tn + 1];
      ptf0 = a.tgt_f0[tn];
      ptp = a.tgt_prev[tn];
      const int e = pb0 + gl;
      psrc = e < pb1 ? a.agg_src[e] : 0;
      pu0 = e < pb1 ? a.agg_f0[e] : 0;
    };
    auto prefetch_m = [&]() {
      pmv = a.mT0[ptf0];
      pm = pb0 + gl < pb1 ? a.mT0[pu0] : 0u;
    };
    if (team < ntgt_wg) {
      prefetch(blockIdx.x + team * gridDim.x);
      prefetch_m();
    }
    for (int i = 0; i <= nint + 1; ++i) {
      const int idx = TEAMS * i + team;  // the team's target of this interval
      if (idx < ntgt_wg && !(a.dbg & 32)) {  // dbg 32 (diagnostics): no gathers
        const int t = blockIdx.x + idx * gridDim.x;
        const int b0 = pb0, b1 = pb1, tf0 = ptf0, tp = ptp;
        int esrc = psrc, eu0 = pu0;
        uint32_t em = pm;
        const uint32_t mv = pmv;
        if (idx + TEAMS < ntgt_wg) prefetch(t + TEAMS * gridDim.x);
        const bool tk0 = v0 && ((mv >> s0) & 1u), tk1 = v1 && ((mv >> s1) & 1u);
        float* A = wsm + ((i & 1) * TEAMS + team) * abuf;
        float self0[NFI], self1[NFI];  // the target's own rows: the same for every term
        {
          // ctab: a sample that masks the target out reads its inactive-row table entry
          const float* p0r = a.ctab && !((mv >> s0) & 1u) ? a.ctab + (int64_t)tp * a.w_row + fo
                                                           : base0 + (int64_t)tp * a.rstride + fo;
          const float* p1r = a.ctab && !((mv >> s1) & 1u) ? a.ctab + (int64_t)tp * a.w_row + fo
                                                           : base1 + (int64_t)tp * a.rstride + fo;
#pragma unroll
          for (int q = 0; q < NFI; ++q) {
            self0[q] = p0r[q];
            self1[q] = TWO ? p1r[q] : 0.f;
          }
        }
        for (int k = 0; k < a.n_terms; ++k) {
          const int kind = a.kind[k], r = a.rel[k];
          float acc0[NFI], acc1[NFI];
          if (kind == XPG_TERM_ROOT) {
#pragma unroll
            for (int q = 0; q < NFI; ++q) {
              acc0[q] = self0[q];
              acc1[q] = self1[q];
            }
          } else {
            float dt0 = 1.f, dt1 = 1.f;
            if (kind == XPG_TERM_GCN) {
              dt0 = inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + tf0) * 32 + s0]);
              dt1 = inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + tf0) * 32 + s1]);
            }
#pragma unroll
            for (int q = 0; q < NFI; ++q) acc0[q] = acc1[q] = 0.f;
            int cnt0 = 0, cnt1 = 0;
            for (int c0 = b0; c0 < b1; c0 += 16) {
              if (c0 != b0) {  // chunks past the first (in-degree > 16): loaded in place
                const int e = c0 + gl;
                esrc = e < b1 ? a.agg_src[e] : 0;
                eu0 = e < b1 ? a.agg_f0[e] : 0;
                em = e < b1 ? a.mT0[eu0] : 0u;
              }
              uint32_t m0 = static_cast<uint32_t>(__ballot(tk0 && ((em >> s0) & 1u)) >> lb) & 0xFFFFu;
              uint32_t m1 = static_cast<uint32_t>(__ballot(tk1 && ((em >> s1) & 1u)) >> lb) & 0xFFFFu;
              cnt0 += __popc(m0);
              cnt1 += __popc(m1);
              while (m0 | m1) {  // group-uniform
                float rr[RIF][NFI];
                float c0v[RIF], c1v[RIF];
#pragma unroll
                for (int q = 0; q < RIF; ++q) {
                  int j = -1;
                  bool first = false;
                  if (m0) {
                    j = __builtin_ctz(m0);
                    m0 &= m0 - 1u;
                    first = true;
                  } else if (m1) {
                    j = __builtin_ctz(m1);
                    m1 &= m1 - 1u;
                  }
                  const int jj = j >= 0 ? j : 0;
                  const int srow = __shfl(esrc, lb + jj, 64);
                  const int su0 = __shfl(eu0, lb + jj, 64);
                  c0v[q] = c1v[q] = 0.f;
#pragma unroll
                  for (int x = 0; x < NFI; ++x) rr[q][x] = 0.f;
                  if (j >= 0) {
                    const float* sp = (first ? base0 : base1) + (int64_t)srow * a.rstride + fo;
                    const int sidx = first ? s0 : s1;
                    const float c = kind == XPG_TERM_GCN
                                        ? (first ? dt0 : dt1) * inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + su0) * 32 + sidx])
                                        : 1.f;
                    c0v[q] = first ? c : 0.f;
                    c1v[q] = first ? 0.f : c;
#pragma unroll
                    for (int x = 0; x < NFI / 4; ++x) {
                      const float4 v = reinterpret_cast<const float4*>(sp)[x];
                      rr[q][4 * x] = v.x;
                      rr[q][4 * x + 1] = v.y;
                      rr[q][4 * x + 2] = v.z;
                      rr[q][4 * x + 3] = v.w;
                    }
                  }
                }
#pragma unroll
                for (int q = 0; q < RIF; ++q)
#pragma unroll
                  for (int x = 0; x < NFI; ++x) {
                    acc0[x] = fmaf(c0v[q], rr[q][x], acc0[x]);
                    acc1[x] = fmaf(c1v[q], rr[q][x], acc1[x]);
                  }
              }
            }
            if (kind == XPG_TERM_GCN) {
#pragma unroll
              for (int q = 0; q < NFI; ++q) {
                acc0[q] = fmaf(dt0 * dt0, self0[q], acc0[q]);
                acc1[q] = fmaf(dt1 * dt1, self1[q], acc1[q]);
              }
            } else {  // MEAN: 0 when the target is masked out in the sample
              const int sm = a.self_mult[(int64_t)r * a.n_tgt + t];
              const float inv0 = tk0 ? 1.f / static_cast<float>(max(cnt0 + sm, 1)) : 0.f;
              const float inv1 = tk1 ? 1.f / static_cast<float>(max(cnt1 + sm, 1)) : 0.f;
#pragma unroll
              for (int q = 0; q < NFI; ++q) {
                acc0[q] = fmaf(static_cast<float>(sm), self0[q], acc0[q]) * inv0;
                acc1[q] = fmaf(static_cast<float>(sm), self1[q], acc1[q]) * inv1;
              }
            }
          }
          if constexpr (B3) {
            __bf16* Ah = reinterpret_cast<__bf16*>(A);
            bf16x8 hi, lo;
#pragma unroll
            for (int q = 0; q < NFI; ++q) acc0[q] = v0 ? acc0[q] : 0.f;
            split_bf16x8(acc0, hi, lo);
            const int e0 = s0 * aph + k * a.w_row + fo;
            *reinterpret_cast<bf16x8*>(Ah + e0) = hi;
            *reinterpret_cast<bf16x8*>(Ah + 32 * aph + e0) = lo;
            if (TWO) {
#pragma unroll
              for (int q = 0; q < NFI; ++q) acc1[q] = v1 ? acc1[q] : 0.f;
              split_bf16x8(acc1, hi, lo);
              const int e1 = s1 * aph + k * a.w_row + fo;
              *reinterpret_cast<bf16x8*>(Ah + e1) = hi;
              *reinterpret_cast<bf16x8*>(Ah + 32 * aph + e1) = lo;
            }
          } else {
          float* a0p = A + s0 * a.a_ld + k * a.w_row + fo;
          float* a1p = A + s1 * a.a_ld + k * a.w_row + fo;
#pragma unroll
          for (int q = 0; q < NFI; q += 4) {
            *reinterpret_cast<float4*>(a0p + q) = v0 ? make_float4(acc0[q], acc0[q + 1], acc0[q + 2], acc0[q + 3])
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            if (TWO)
              *reinterpret_cast<float4*>(a1p + q) = v1 ? make_float4(acc1[q], acc1[q + 1], acc1[q + 2], acc1[q + 3])
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
          }
          }
        }
        if (idx + TEAMS < ntgt_wg) prefetch_m();
      }
      lds_barrier();
    }
  } else {
    // ------------------------------------------------------------------ MFMA role
    // MFMA waves issue first when both roles are ready (c3 pass 17.0 -> 16.8 ms, repeated A/B in
    // profiles/r3_ws_prio_ab.log; XPG_WIDE_DBG 512 turns it off): a ready MFMA wave otherwise
    // waits behind gather waves issuing their address / keep-test VALU work
    if (!(a.dbg & 512)) __builtin_amdgcn_s_setprio(2);
    const int nb = wave - GW, i32 = lane & 31, h = lane >> 5;
    const bool active = nb * 32 < a.f_out_pad;
    const int col = nb * 32 + i32;
    const float bv = active && col < a.f_out ? a.bias[col] : 0.f;
    const float hwc = active && col < a.f_out ? a.H[0].weight[col] : 0.f;
    const float hb = a.H[0].bias[0];
    const int hact = a.H[0].act;
    const float* wp = a.weight + (int64_t)(active ? col : 0) * a.K + 4 * h;
    const int klast = a.K - 8;
    auto ldw = [&](int k) { return *reinterpret_cast<const float4*>(wp + (k < klast ? k : klast)); };
    float4 wreg[KW > 0 && !B3 ? KW : 1];  // KW > 0: the wave's 32 weight columns held in registers (K = 8 KW)
    bf16x8 whi[KB], wlo[WL ? 1 : KB];       // B3: the same columns as bf16 hi / lo pieces (k = 16 kb + 8 h + j)
    if (KW > 0 && !B3) {
#pragma unroll
      for (int kk = 0; kk < (KW > 0 ? KW : 1); ++kk) wreg[kk] = ldw(kk * 8);
    }
    if constexpr (B3) {
      const float* wb = a.weight + (int64_t)(active ? col : 0) * a.K + 8 * h;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        float x[8];
        const float4 u = *reinterpret_cast<const float4*>(wb + 16 * kb);
        const float4 v = *reinterpret_cast<const float4*>(wb + 16 * kb + 4);
        x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
        x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
        if constexpr (WL) {
          bf16x8 lo;
          split_bf16x8(x, whi[kb], lo);
          // each lane reads back only what it wrote: no barrier needed before the first use
          if (active) *reinterpret_cast<bf16x8*>(WLs + ((int64_t)(2 * kb + h) * a.f_out_pad + col) * 8) = lo;
        } else {
          split_bf16x8(x, whi[kb], wlo[WL ? 0 : kb]);
        }
      }
    }
    XPG_WST_INIT
    for (int i = 0; i <= nint + 1; ++i) {
      if (ixw) {
        // index chain, every stage's loads consumed one interval after they were issued: the
        // list of target i + 2 (its keep words loaded during interval i - 1; the slot held the
        // list of target i - 1, done with at the last barrier), then the keep words of i + 3,
        // the edges of i + 4 and the CSR range of i + 5
        stC_store(i + 2);
        // every value the new loads need (loaded during the last interval) is read before any of
        // them is issued: vmcnt counts in issue order, so a wait placed after a new load would
        // wait for that load's whole HBM latency too
        const int va = qa_v, vb = qb_v, srcb = qb_src, u0b = qb_u0;
        const int a_b0 = __builtin_amdgcn_readlane(va, 0), a_b1 = __builtin_amdgcn_readlane(va, 1);
        const int a_tf0 = __builtin_amdgcn_readlane(va, 2);
        asm volatile("" ::"v"(vb), "v"(srcb), "v"(u0b), "s"(a_b0), "s"(a_b1), "s"(a_tf0));
        if (i + 3 < ntgt_wg) {  // stage C of target i + 3: keep words
          qc_v = vb;
          qc_src = srcb;
          qc_em = a.mT0[u0b];
        }
        if (i + 4 < ntgt_wg) {  // stage B of target i + 4: in-edges
          qb_v = va;
          const int e = a_b0 + lane;
          qb_src = e < a_b1 && lane < kIxEdges ? a.agg_src[e] : 0;
          qb_u0 = lane < kIxEdges ? (e < a_b1 ? a.agg_f0[e] : 0) : a_tf0;
        }
        stA(i + 5);
      }
      XPG_WST(1)
#pragma unroll
      for (int j = 0; j < TEAMS; ++j) {  // targets of interval i - 2: y[s] = act(sum over blocks + b)
        const int idx = TEAMS * (i - 2) + j;
        if (nb == 0 && i >= 2 && idx < ntgt_wg && lane < a.nr) {
          // written at interval i - 1 into buffer (i - 2) & 1 = i & 1
          const float* hp = H0 + ((i & 1) * TEAMS + j) * a.f_out_pad;
          // the column blocks' partials read at once (f_out_pad <= 128: four MFMA waves of 32
          // columns), summed in block order
          float hv[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) hv[b] = hp[min(b * 32, a.f_out_pad - 32) + lane];
          float v = 0.f;
#pragma unroll
          for (int b = 0; b < 4; ++b) v = b * 32 < a.f_out_pad ? v + hv[b] : v;
          const int tf = blockIdx.x + idx * gridDim.x;
          a.out[(a.row0 + lane) * a.n_tgt + tf] = act_apply(v + hb, hact);
        }
      }
      XPG_WST(2)
      for (int j = 0; j < TEAMS; ++j) {
      const int slot = ((i - 1) & 1) * TEAMS + j;
      if (i >= 1 && TEAMS * (i - 1) + j < ntgt_wg && active && !(a.dbg & 16)) {  // dbg 16 (diagnostics): no MFMA
        const float* ap = wsm + slot * abuf + i32 * a.a_ld + 4 * h;
        auto lda = [&](int k) { return *reinterpret_cast<const float4*>(ap + k); };
        f32x16 acc, acc2;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = acc2[q] = 0.f;
        if (a.dbg & 128) {  // dbg 128 (diagnostics): epilogue only, no products
        } else if constexpr (WL) {
          const __bf16* ah = reinterpret_cast<const __bf16*>(wsm + slot * abuf) + i32 * aph + 8 * h;
          const __bf16* wl = WLs + ((int64_t)h * a.f_out_pad + col) * 8;
          const int wstep = 2 * a.f_out_pad * 8;  // bf16 per k-block of the lo pieces
          bf16x8 A1[3], A2[3], WW[3];             // ring: k-blocks kb, kb + 1, kb + 2
          auto ld = [&](int kb, int r) {
            A1[r] = *reinterpret_cast<const bf16x8*>(ah + 16 * kb);
            A2[r] = *reinterpret_cast<const bf16x8*>(ah + 32 * aph + 16 * kb);
            WW[r] = *reinterpret_cast<const bf16x8*>(wl + kb * wstep);
          };
          ld(0, 0);
          ld(1, 1);
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            if (kb + 2 < KB) ld(kb + 2, (kb + 2) % 3);
            __builtin_amdgcn_sched_barrier(0);  // keep the reads two k-blocks ahead of their MFMAs
            const int r = kb % 3;
            if constexpr (TH) {  // the transposed product: acc[reg] = out[sample i32][column row(reg)]
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[kb], A2[r], acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(WW[r], A1[r], acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[kb], A1[r], acc, 0, 0, 0);
            } else {
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2[r], whi[kb], acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1[r], WW[r], acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1[r], whi[kb], acc, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        } else if constexpr (B3) {
          const __bf16* ah = reinterpret_cast<const __bf16*>(wsm + slot * abuf) + i32 * aph + 8 * h;
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(ah + 16 * kb);
            const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(ah + 32 * aph + 16 * kb);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, whi[kb], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, wlo[WL ? 0 : kb], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, whi[kb], acc, 0, 0, 0);
          }
        } else if (KW > 0) {
#pragma unroll
          // one accumulation chain (f32 32x32x2: 64-cycle issue = 64-cycle dependent latency)
          for (int kk = 0; kk < (KW > 0 ? KW : 1); ++kk) {
            const float4 av = lda(kk * 8);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wreg[kk].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wreg[kk].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wreg[kk].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wreg[kk].w, acc, 0, 0, 0);
          }
        } else {
        float4 w0 = ldw(0), w1 = ldw(8), w2 = ldw(16), w3 = ldw(24);
        float4 a0 = lda(0), a1 = lda(8);
        __builtin_amdgcn_sched_barrier(0);
        for (int kc = 0; kc < a.K; kc += 32) {
          const float4 a2 = lda(kc + 16), a3 = lda(kc + 24);
          __builtin_amdgcn_sched_barrier(0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, w0.x, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, w1.x, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, w0.y, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, w1.y, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, w0.z, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, w1.z, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, w0.w, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, w1.w, acc2, 0, 0, 0);
          w0 = ldw(kc + 32);
          w1 = ldw(kc + 40);
          const int kn = kc + 32 < a.K ? kc + 32 : 0;
          a0 = lda(kn);
          a1 = lda(kn + 8);
          __builtin_amdgcn_sched_barrier(0);  // keep the refills here (the scheduler sinks them to the use)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.x, w2.x, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.x, w3.x, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.y, w2.y, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.y, w3.y, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.z, w2.z, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.z, w3.z, acc2, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.w, w2.w, acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a3.w, w3.w, acc2, 0, 0, 0);
          w2 = ldw(kc + 48);
          w3 = ldw(kc + 56);
          __builtin_amdgcn_sched_barrier(0);
        }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] += acc2[q];
        XPG_WST(3)
        if constexpr (TH) {
          // column c = nb * 32 + (reg & 3) + 8 (reg >> 2) + 4 h of sample i32 sits in acc[reg]:
          // the head dot over the wave's 32 columns is 16 in-lane FMAs plus one swap of the two
          // lane halves (the untransposed product needs a 32-lane reduction per register)
          const float* hb = HBW + nb * 32 + 4 * h;
          float v = 0.f;
          if (a.act == XPG_ACT_RELU) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float4 b4 = *reinterpret_cast<const float4*>(hb + 8 * q);
              const float4 w4 = *reinterpret_cast<const float4*>(hb + a.f_out_pad + 8 * q);
              v = fmaf(fmaxf(acc[4 * q] + b4.x, 0.f), w4.x, v);
              v = fmaf(fmaxf(acc[4 * q + 1] + b4.y, 0.f), w4.y, v);
              v = fmaf(fmaxf(acc[4 * q + 2] + b4.z, 0.f), w4.z, v);
              v = fmaf(fmaxf(acc[4 * q + 3] + b4.w, 0.f), w4.w, v);
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float4 b4 = *reinterpret_cast<const float4*>(hb + 8 * q);
              const float4 w4 = *reinterpret_cast<const float4*>(hb + a.f_out_pad + 8 * q);
              v = fmaf(act_apply(acc[4 * q] + b4.x, a.act), w4.x, v);
              v = fmaf(act_apply(acc[4 * q + 1] + b4.y, a.act), w4.y, v);
              v = fmaf(act_apply(acc[4 * q + 2] + b4.z, a.act), w4.z, v);
              v = fmaf(act_apply(acc[4 * q + 3] + b4.w, a.act), w4.w, v);
            }
          }
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          v = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);  // both halves: the same sum
          if (h == 0) H0[slot * a.f_out_pad + nb * 32 + i32] = v;
        } else {
        float part[16];
        if (a.dbg & 64) {  // dbg 64 (diagnostics): products only, no activation / head reduction
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) part[reg] = acc[reg];
        } else {
          // one scalar branch on the activation for all 16 values (per value, the runtime switch
          // and the column test were exec-mask branches: the epilogue cost more than the
          // products); padded columns hold hwc = 0 and zero weights, so they add 0
          if (a.act == XPG_ACT_RELU) {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) part[reg] = fmaxf(acc[reg] + bv, 0.f) * hwc;
          } else {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) part[reg] = act_apply(acc[reg] + bv, a.act) * hwc;
          }
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) part[reg] = half_wave_sum(part[reg]);
        }
        if (i32 == 0) {  // lanes 0 and 32 hold the 16 sample rows of their half
          float* hp = H0 + slot * a.f_out_pad;
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) hp[nb * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h] = part[reg];
        }
        }  // !TH
      }
      }
      XPG_WST(4)
      lds_barrier();
      XPG_WST(0)
    }
    XPG_WST_STORE
  }
}

// Layer 1 of the wide path, one wave per target and all 32 samples at once.  Features are never
// masked (data.py:582), so the table row T[u] of an in-edge is the same for every sample: the
// wave reads it once (lane = FPL features, 512 B coalesced at F = 128) and adds it to the
// accumulators of the samples that keep the edge (keep bits wave-uniform: v_readlane of the
// lane-per-edge keep words), instead of every 16-lane sample group fetching its own copy.
// Plans whose term 0 aggregates (GCN / MEAN) and whose other terms are ROOT (homogeneous GCN and
// SAGE layers); rows are fetched 8 edges ahead.  Per sample the edges (CSR order), self terms
// and ROOT terms are summed in k_wide_tgt's order, so h1 is bitwise the gather kernel's.
template <int FPL, bool GCN>
__global__ __launch_bounds__(256) void k_wide_l1s(const WideArgs a) {
  constexpr int RIF = 8;
  constexpr int RC = FPL >= 4 ? 4 : RIF;  // rows prefetched across targets (register budget)
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t valid = a.nr >= 32 ? 0xFFFFFFFFu : ((1u << a.nr) - 1u);
  const int r = a.rel[0];
  const float* T = a.table[0] + lane * FPL;
  const int32_t* pp = a.agg_ptr + (int64_t)r * (a.n_tgt + 1);
  // every per-target quantity below is wave-uniform and forced into SGPRs (readfirstlane): the
  // per-sample keep tests are then scalar bit tests + scalar branches (with the values in VGPRs
  // the compiler emitted an exec-mask branch of ~10 instructions per sample and edge).
  // Cross-target pipeline, three levels deep (vector memory ops complete in issue order, so a
  // load issued after this target's 32 row stores would first wait for every store's ack):
  //   A (target t + 2): CSR range and node                      issued at the top of t
  //   B (target t + 1): first edge chunk, keep word, own row    issued at the top of t (A(t+1) ready)
  //   C (target t + 1): first chunk's keep words, first 8 rows  issued before t's stores (B ready)
  int64_t t = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  int a_tf0 = 0, a_b0 = 0, a_b1 = 0;         // A state (lane copies of uniform values)
  int b_tf0 = 0, b_b0 = 0, b_b1 = 0, b_u0v = 0;  // B state
  uint32_t b_mv = 0u;
  int b_sm = 0;
  float b_self[FPL], b_root[FPL];  // own row of term 0 and of the ROOT term 1 (n_terms == 2)
  uint32_t c_kmv = 0u;                       // C state
  float c_row[RC][FPL];
#pragma unroll
  for (int q = 0; q < FPL; ++q) b_self[q] = b_root[q] = 0.f;
  const float* T1 = a.table[a.n_terms > 1 ? 1 : 0] + lane * FPL;
  float bv[FPL];  // loop-invariant (loaded once, not after every target's stores)
#pragma unroll
  for (int q = 0; q < FPL; ++q) bv[q] = lane * FPL + q < a.f_real ? a.bias[lane * FPL + q] : 0.f;
  int64_t a_t = 0;
  auto issueA = [&](int64_t tn) {
    a_t = tn;
    a_tf0 = a.tgt_f0[tn];
    a_b0 = pp[tn];
    a_b1 = pp[tn + 1];
  };
  auto issueB = [&]() {  // from A
    const int64_t tn_b = a_t;
    b_tf0 = a_tf0;
    b_b0 = a_b0;
    b_b1 = a_b1;
    const int e = b_b0 + lane;
    b_u0v = e < b_b1 ? a.agg_f0[e] : 0;
    b_mv = a.mT0[b_tf0];
    if (!GCN) b_sm = a.self_mult[(int64_t)r * a.n_tgt + tn_b];
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
      b_self[q] = T[(int64_t)b_tf0 * a.w_row + q];
      b_root[q] = a.n_terms == 2 ? T1[(int64_t)b_tf0 * a.w_row + q] : 0.f;
    }
  };
  auto issueC = [&]() {  // from B
    const int e = b_b0 + lane;
    c_kmv = e < b_b1 ? a.mT0[b_u0v] : 0u;
    const int ne = min(min(64, b_b1 - b_b0), RC);
#pragma unroll
    for (int jj = 0; jj < RC; ++jj) {
      const int u0 = __builtin_amdgcn_readlane(b_u0v, jj < ne ? jj : 0);
#pragma unroll
      for (int q = 0; q < FPL; ++q) c_row[jj][q] = T[(int64_t)u0 * a.w_row + q];
    }
  };
  if (t < a.n_tgt) {
    issueA(t);
    issueB();
    issueC();
    if (t + nw < a.n_tgt) issueA(t + nw);
  }
  for (; t < a.n_tgt; t += nw) {
    const int tf0 = __builtin_amdgcn_readfirstlane(b_tf0);
    const uint32_t mv = __builtin_amdgcn_readfirstlane(b_mv) & valid;
    const int b0 = __builtin_amdgcn_readfirstlane(b_b0), b1 = __builtin_amdgcn_readfirstlane(b_b1);
    const int u0v_first = b_u0v;
    const uint32_t kmv_first = c_kmv & mv;
    float row0[RC][FPL];
#pragma unroll
    for (int jj = 0; jj < RC; ++jj)
#pragma unroll
      for (int q = 0; q < FPL; ++q) row0[jj][q] = c_row[jj][q];
    float self[FPL], root[FPL];
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
      self[q] = b_self[q];
      root[q] = b_root[q];
    }
    const int sm = GCN ? 0 : __builtin_amdgcn_readfirstlane(b_sm);
    const bool more = t + nw < a.n_tgt;
    if (more) issueB();                          // target t + nw (A issued one iteration ago)
    if (t + 2 * nw < a.n_tgt) issueA(t + 2 * nw);
    float tot[32][FPL];
#pragma unroll
    for (int s = 0; s < 32; ++s)
#pragma unroll
      for (int q = 0; q < FPL; ++q) tot[s][q] = 0.f;
    // lane s (< 32): sample s's GCN target factor dt_s and kept in-edge count
    const float dt_l = GCN ? inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + tf0) * 32 + (lane & 31)]) : 1.f;
    int cnt_l = 0;
    for (int c0 = b0; c0 < b1; c0 += 64) {
      const int e = c0 + lane;
      const bool first = c0 == b0;
      const int u0v = first ? u0v_first : (e < b1 ? a.agg_f0[e] : 0);
      const uint32_t kmv = first ? kmv_first : (e < b1 ? (a.mT0[u0v] & mv) : 0u);
      const int ne = min(64, b1 - c0);
      for (int j0 = 0; j0 < ne; j0 += RIF) {
        float row[RIF][FPL];
        float c_l[RIF];
        uint32_t km[RIF];
#pragma unroll
        for (int jj = 0; jj < RIF; ++jj) {  // RIF rows in flight
          const int j = j0 + jj < ne ? j0 + jj : j0;
          km[jj] = j0 + jj < ne ? __builtin_amdgcn_readlane(kmv, j) : 0u;
          const int u0 = __builtin_amdgcn_readlane(u0v, j);
          if (first && j0 == 0 && jj < RC) {  // scalar: the rows prefetched before the previous stores
#pragma unroll
            for (int q = 0; q < FPL; ++q) row[jj][q] = row0[jj < RC ? jj : 0][q];
          } else {
#pragma unroll
            for (int q = 0; q < FPL; ++q) row[jj][q] = T[(int64_t)u0 * a.w_row + q];
          }
          c_l[jj] = GCN ? dt_l * inv_sqrt_deg(a.kinT[((int64_t)r * a.n0 + u0) * 32 + (lane & 31)]) : 1.f;
        }
#pragma unroll
        for (int jj = 0; jj < RIF; ++jj) {
          const uint32_t k = km[jj];
          if (k == 0u) continue;  // scalar
          cnt_l += (k >> (lane & 31)) & 1u;
#pragma unroll
          for (int s = 0; s < 32; ++s) {
            if ((k >> s) & 1u) {  // scalar
              if (GCN) {
                const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c_l[jj]), s));
#pragma unroll
                for (int q = 0; q < FPL; ++q) tot[s][q] = fmaf(c, row[jj][q], tot[s][q]);
              } else {
                // an empty asm with side effects keeps this a scalar branch: if-converted, every
                // sample cost 2 adds + 2 selects per edge whether its keep bit was set or not
                asm volatile("" ::: "memory");
#pragma unroll
                for (int q = 0; q < FPL; ++q) tot[s][q] = fmaf(1.f, row[jj][q], tot[s][q]);
              }
            }
          }
        }
      }
    }
    // MEAN: lane s computes sample s's 1 / (kept count + self count) once for all samples (the
    // division per sample on wave-uniform operands cost ~10 VALU instructions x 32 per target)
    const float inv_l = !GCN && ((mv >> (lane & 31)) & 1u) ? 1.f / static_cast<float>(max(cnt_l + sm, 1)) : 0.f;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (GCN) {
        const float dt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dt_l), s));
#pragma unroll
        for (int q = 0; q < FPL; ++q) tot[s][q] = fmaf(dt * dt, self[q], tot[s][q]);
      } else {
        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_l), s));
#pragma unroll
        for (int q = 0; q < FPL; ++q) tot[s][q] = fmaf(static_cast<float>(sm), self[q], tot[s][q]) * inv;
      }
    }
    // the row of a sample that masks the target out (ctab): no kept edge, GCN dt = 1 (the
    // weight-1 self loop), MEAN 0 — the values tot[s] holds for such a sample, bit for bit
    float cin[FPL];
#pragma unroll
    for (int q = 0; q < FPL; ++q) cin[q] = GCN ? fmaf(1.f, self[q], 0.f) : 0.f;
    for (int k = 1; k < a.n_terms; ++k) {  // ROOT terms (host-checked); term 1 prefetched
      float sk[FPL];
      if (k == 1 && a.n_terms == 2) {
#pragma unroll
        for (int q = 0; q < FPL; ++q) sk[q] = root[q];
      } else {
        const float* Tk = a.table[k] + lane * FPL;
#pragma unroll
        for (int q = 0; q < FPL; ++q) sk[q] = Tk[(int64_t)tf0 * a.w_row + q];
      }
#pragma unroll
      for (int s = 0; s < 32; ++s)
#pragma unroll
        for (int q = 0; q < FPL; ++q) tot[s][q] += sk[q];
#pragma unroll
      for (int q = 0; q < FPL; ++q) cin[q] += sk[q];
    }
    if (more) issueC();  // before the stores (see above)
    // ctab: store only the samples that keep the target, plus the inactive row once
    const uint32_t store_mask = a.ctab ? mv : 0xFFFFFFFFu;
    if (a.ctab && mv != 0xFFFFFFFFu) {
      float v[FPL];
#pragma unroll
      for (int q = 0; q < FPL; ++q)
        v[q] = lane * FPL + q >= a.f_real ? 0.f
               : a.act == XPG_ACT_RELU ? fmaxf(cin[q] + bv[q], 0.f) : act_apply(cin[q] + bv[q], a.act);
      float* co = a.ctab + (int64_t)t * a.w_row + lane * FPL;
#pragma unroll
      for (int q = 0; q < FPL; ++q) co[q] = v[q];
    }
    float* o = a.out + (int64_t)t * 32 * a.w_row + lane * FPL;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (s < a.nr && ((store_mask >> s) & 1u)) {
        float v[FPL];
        if (a.act == XPG_ACT_RELU) {  // one scalar branch, not a runtime switch per value
#pragma unroll
          for (int q = 0; q < FPL; ++q) v[q] = lane * FPL + q < a.f_real ? fmaxf(tot[s][q] + bv[q], 0.f) : 0.f;
        } else {
#pragma unroll
          for (int q = 0; q < FPL; ++q) v[q] = lane * FPL + q < a.f_real ? act_apply(tot[s][q] + bv[q], a.act) : 0.f;
        }
        if (FPL == 2) {
          *reinterpret_cast<float2*>(o + s * a.w_row) = make_float2(v[0], v[1]);
        } else {
#pragma unroll
          for (int q = 0; q < FPL; ++q) o[s * a.w_row + q] = v[q];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------ surrogate
// train_model (wlm.py:132-278) in three stages:
//  1. k_wlm_stats  (grid, block per Adam step): per-step constants that do not depend on w —
//     mean(y), sum(k), sum (y - mean)^2 — and the Adam bias corrections (step size, sqrt(bc2)).
//  2. k_wlm_colbits (grid, wave per (step, word, 64-row chunk)): transposes each step's mask
//     batch into per-column row bit vectors with 32 wave ballots, for the gradient M_b^T g.
//  3. k_wlm_fit (ONE persistent 1024-thread workgroup: the Adam steps are strictly sequential):
//     per step, 4-bit lookup tables of w (T[col/4][16]) turn p = M_b w into one LDS lookup per
//     nibble of a mask row; tables of g (G[row/4][16]) turn M_b^T g into one lookup per nibble of
//     a column's row vector; parameters and Adam moments stay in registers (CPT per thread).
//     The loss (closed form of the reference's [B] - [B,1] broadcast, quirk Q1) is computed
//     afterwards by k_wlm_loss_best from the recorded predictions and pre-step weights.
struct WlmStep {
  double ybar, ksum, vy;
  double cg;  // 2 / (B sum k): the per-row gradient factor g_j = k_j cg (p_j - ybar)
  float step_size, bc2_sqrt, inv_bc2;  // inv_bc2 = 1 / bc2_sqrt (multi-workgroup fit)
  float pad;
};

// Also clears the multi-workgroup fit's exchange slots (`clr`, n_clr granules) and error words
// (`clr32`, n_clr32), so the fit needs no memset launches (plain stores; the kernel boundary
// makes them visible to the fit).
// block (t, fit) of a (steps x n_fits) grid; nb / b: block count and this block's index for the
// slot clearing
__device__ __forceinline__ void wlm_stats_block(const float* __restrict__ y, const double* __restrict__ kern,
                                                int64_t rows, int batch, const xpg_wlm_params& P, int64_t step0,
                                                WlmStep* __restrict__ st, uint64_t* __restrict__ clr, int64_t n_clr,
                                                uint32_t* __restrict__ clr32, int n_clr32, int64_t t, int64_t fit,
                                                int64_t steps, int64_t nb, int64_t b) {
  __shared__ double red[16];
  {
    for (int64_t e = b * blockDim.x + threadIdx.x; e < n_clr; e += nb * blockDim.x) clr[e] = 0;
    if (b == 0)
      for (int e = threadIdx.x; e < n_clr32; e += blockDim.x) clr32[e] = 0u;
  }
  y += fit * rows;
  kern += fit * rows;
  st += fit * steps;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  double sy = 0.0, sk = 0.0;
  for (int j = threadIdx.x; j < B; j += blockDim.x) {
    sy += static_cast<double>(y[r0 + j]);
    sk += kern[r0 + j];
  }
  const double Sy = block_sum_d(sy, red);
  const double Sk = block_sum_d(sk, red);
  const double ybar = Sy / B;
  double vy = 0.0;
  for (int j = threadIdx.x; j < B; j += blockDim.x) {
    const double d = static_cast<double>(y[r0 + j]) - ybar;
    vy += d * d;
  }
  const double Vy = block_sum_d(vy, red);
  if (threadIdx.x == 0) {
    const double step = static_cast<double>(step0 + t + 1);
    const double bc1 = 1.0 - pow(static_cast<double>(P.beta1), step);
    const double bc2 = 1.0 - pow(static_cast<double>(P.beta2), step);
    WlmStep w;
    w.ybar = ybar;
    w.ksum = Sk;
    w.vy = Vy;
    w.cg = 2.0 / (static_cast<double>(B) * Sk);
    w.step_size = static_cast<float>(static_cast<double>(P.lr) / bc1);
    w.bc2_sqrt = static_cast<float>(sqrt(bc2));
    w.inv_bc2 = 1.f / w.bc2_sqrt;
    w.pad = 0.f;
    st[t] = w;
  }
}

__global__ __launch_bounds__(256) void k_wlm_stats(const float* __restrict__ y,
                                                   const double* __restrict__ kern, int64_t rows,
                                                   int batch, xpg_wlm_params P, int64_t step0,
                                                   WlmStep* __restrict__ st, uint64_t* __restrict__ clr,
                                                   int64_t n_clr, uint32_t* __restrict__ clr32, int n_clr32) {
  const int64_t nb = (int64_t)gridDim.x * gridDim.y;
  wlm_stats_block(y, kern, rows, batch, P, step0, st, clr, n_clr, clr32, n_clr32, blockIdx.x, blockIdx.y,
                  gridDim.x, nb, blockIdx.y * (int64_t)gridDim.x + blockIdx.x);
}

// colbits[(t * cols + c) * bw + jw] bit b = mask bit (row t*batch + 32*jw + b, column c)
// Lane = (step t, mask word wd, 32-row block jw), jw fastest: one in-register 32 x 32 bit
// transpose per lane; per load / store instruction a wave touches 8 contiguous 32-B pieces (8
// words of a row, 8 row blocks of a column) instead of 64 scattered 4-B column words (with wd
// fastest the stores wrote 3.4x the column bytes: WRITE_SIZE 7.2 MB for 2.1 MB per c2 fit).
__device__ __forceinline__ void wlm_colbits_lane(const uint32_t* __restrict__ bits, int64_t rows, int cols,
                                                 int words, int batch, int bw, int64_t steps,
                                                 uint32_t* __restrict__ colbits, int64_t gid, int64_t fit) {
  if (gid >= steps * bw * words) return;
  bits += fit * rows * words;
  colbits += fit * steps * cols * bw;
  const int jw = static_cast<int>(gid % bw);
  const int64_t tk = gid / bw;
  const int wd = static_cast<int>(tk % words);
  const int64_t t = tk / words;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  uint32_t x[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int j = 32 * jw + i;
    x[i] = j < B ? bits[(r0 + j) * words + wd] : 0u;
  }
  transpose32(x);
  uint32_t* dst = colbits + ((int64_t)t * cols + (int64_t)wd * 32) * bw + jw;
#pragma unroll
  for (int b = 0; b < 32; ++b)
    if (wd * 32 + b < cols) dst[(int64_t)b * bw] = x[b];
}

// The fit's two independent prologues in ONE launch (one kernel boundary less on the
// latency-bound chain): blocks [0, steps) of each fit row are k_wlm_stats' blocks, the rest
// k_wlm_colbits' 256-lane blocks.
__global__ __launch_bounds__(256) void k_wlm_prep(const float* __restrict__ y, const double* __restrict__ kern,
                                                  const uint32_t* __restrict__ bits, int64_t rows, int cols,
                                                  int words, int batch, int bw, int64_t steps, xpg_wlm_params P,
                                                  int64_t step0, WlmStep* __restrict__ st,
                                                  uint32_t* __restrict__ colbits, uint64_t* __restrict__ clr,
                                                  int64_t n_clr, uint32_t* __restrict__ clr32, int n_clr32,
                                                  uint32_t* __restrict__ ep, const float* __restrict__ w0,
                                                  float* __restrict__ w, float* __restrict__ m,
                                                  float* __restrict__ v, int64_t n_wmv) {
  const int64_t fit = blockIdx.y;
  if (w0) {  // fresh fit from w0 (xpg_wlm_fit_from): w = w0, Adam moments 0 — no separate launches
    const int64_t nb = (int64_t)gridDim.x * gridDim.y, b = fit * gridDim.x + blockIdx.x;
    for (int64_t e = b * blockDim.x + threadIdx.x; e < n_wmv; e += nb * blockDim.x) {
      w[e] = w0[e];
      m[e] = 0.f;
      v[e] = 0.f;
    }
  }
  // the exchange tags' device epoch advances once per fit chain (a replayed HIP graph carries
  // the host epoch of its capture; this word makes every replay's tags new)
  if (ep && blockIdx.x == 0 && fit == 0 && threadIdx.x == 0) *ep = *ep + 1u;
  if ((int64_t)blockIdx.x < steps) {
    wlm_stats_block(y, kern, rows, batch, P, step0, st, clr, n_clr, clr32, n_clr32, blockIdx.x, fit, steps,
                    steps * gridDim.y, fit * steps + blockIdx.x);
  } else {
    const int64_t gid = (blockIdx.x - steps) * (int64_t)blockDim.x + threadIdx.x;
    wlm_colbits_lane(bits, rows, cols, words, batch, bw, steps, colbits, gid, fit);
  }
}



constexpr int kTabPitch = 17;  // 16 entries + 1 pad (bank spread across tables)
constexpr int kStage = 10;     // staged words per thread per buffer (buffer <= 10K words)

// In-wave rebuild of the w nibble tables: the 4 columns of table g are owned by 4 adjacent
// lanes (column i = tid + 1024 c), so each lane shuffles its group's 4 weights and writes 4 of
// the 16 entries.  Columns >= cols hold w = 0, so tail tables are zero.
template <int CPT>
__device__ __forceinline__ void wlm_build_T(const float (&w)[CPT], float* T, int ntab) {
  const int lane = threadIdx.x & 63, q = lane & 3, base = lane & ~3;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    float wb[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) wb[b] = __shfl(w[c], base + b, 64);
    const int grp = (static_cast<int>(threadIdx.x) >> 2) + 256 * c;
    if (grp < ntab) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int vv = q * 4 + e;
        float s = 0.f;
        s += (vv & 1) ? wb[0] : 0.f;
        s += (vv & 2) ? wb[1] : 0.f;
        s += (vv & 4) ? wb[2] : 0.f;
        s += (vv & 8) ? wb[3] : 0.f;
        T[grp * kTabPitch + vv] = s;
      }
    }
  }
}

__device__ __forceinline__ float nib8(const float* tab, uint32_t word) {
  float a[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) a[nb] = tab[nb * kTabPitch + ((word >> (4 * nb)) & 15u)];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// One Adam step = four phases between four workgroup barriers.  Work is cut into WAVE items
// (64 rows or 64 columns x a slice of words) so that the 32 lanes of an LDS lane group always
// look up the SAME 16-entry nibble table at distinct rows/columns: every lookup is
// bank-conflict free, and the slices balance the work over the 16 waves.
//   B  item (64-row block, word slice): partial p_j over the slice -> bpart[slice][j]
//   -- barrier A --
//   G  entry (4-row group, nibble value): p_j = sum of partials, g_j, G tables, p_hist;
//      Cb(t) stored
//   -- barrier 1 --
//   D  item (64-column block, slice of the column bit vectors): partial (M_b^T g)_i -> dpart
//   -- barrier D --
//   Adam on owned columns (sum of partials), T rebuilt in-wave, Rb(t+1) / kbuf(t+1) stored
//   -- barrier 2 --
// STAGE: the step's mask rows ([batch][rp]), column bit vectors ([cols][cp]) and kernel weights
// live in LDS; the next copies are loaded into registers right after a barrier and written to
// LDS just before a later one, so their global latency hides behind a phase.
// Unstaged fits keep the w tables in global memory (t_glob), so their barriers fence it too.
template <bool STAGE>
__device__ __forceinline__ void wlm_barrier() {
  if (STAGE) lds_barrier();
  else __syncthreads();
}

template <int CPT, bool STAGE>
__global__ __launch_bounds__(1024) void k_wlm_fit(
    const uint32_t* __restrict__ bits, const uint32_t* __restrict__ colbits, int64_t rows,
    int cols, int words, int batch, int bw, int n_bs, int n_ds, const double* __restrict__ kern,
    const WlmStep* __restrict__ stp, xpg_wlm_params P, float* __restrict__ wg,
    float* __restrict__ mg, float* __restrict__ vg, float* __restrict__ p_hist,
    float* __restrict__ w_hist, float* __restrict__ t_glob) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntab = words * 8;        // one table per nibble of every word
  {  // independent fits: one workgroup each, fit-major arrays
    const int64_t f = blockIdx.x;
    const int64_t st_ = (rows + batch - 1) / batch;
    const int bw_ = (batch + 31) / 32;
    bits += f * rows * words;
    colbits += f * st_ * cols * bw_;
    kern += f * rows;
    stp += f * st_;
    wg += f * cols;
    mg += f * cols;
    vg += f * cols;
    p_hist += f * rows;
    w_hist += f * st_ * cols;
    if (t_glob) t_glob += f * (int64_t)ntab * kTabPitch;
  }
  const int ngrp_alloc = bw * 8;     // g tables cover every nibble of a column word
  const int rp = words | 1, cp = bw | 1;
  const int cpad = (cols + 63) & ~63;
  float* G = reinterpret_cast<float*>(smem);                          // [ngrp_alloc][17]
  float* bpart = G + ngrp_alloc * kTabPitch;                           // [n_bs][batch]
  float* dpart = bpart + n_bs * batch;                                 // [n_ds][cpad]
  const int kb_off = (ngrp_alloc * kTabPitch + n_bs * batch + n_ds * cpad + 1) & ~1;  // 8-B aligned
  double* kbuf = reinterpret_cast<double*>(G + kb_off);                // STAGE: [batch]
  float* T = STAGE ? reinterpret_cast<float*>(kbuf + batch) : t_glob;  // [ntab][17]
  uint32_t* Rb = reinterpret_cast<uint32_t*>(T + ntab * kTabPitch);   // STAGE: [batch][rp]
  uint32_t* Cb = Rb + batch * rp;                                      // STAGE: [cols][cp]

  const int nrb = (batch + 63) >> 6, ncb = (cols + 63) >> 6;
  const int bsw = (words + n_bs - 1) / n_bs, dsw = (bw + n_ds - 1) / n_ds;
  const float l1s = P.l1_lambda / static_cast<float>(cols);
  const int64_t nsteps = (rows + batch - 1) / batch;

  float w[CPT], m[CPT], v[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int i = tid + c * 1024;
    w[c] = i < cols ? wg[i] : 0.f;
    m[c] = i < cols ? mg[i] : 0.f;
    v[c] = i < cols ? vg[i] : 0.f;
  }
  for (int e = tid; e < ngrp_alloc * kTabPitch; e += 1024) G[e] = 0.f;
  wlm_build_T<CPT>(w, T, ntab);

  uint32_t stg[kStage] = {};  // loaded only where a stage has data; the rest are stored, never read
  double kst = 0.0;
  // stage-load helpers (flat element index q*1024 + tid over the buffer's logical extent)
#define XPG_ROWS_LOAD(TT)                                                               \
  {                                                                                     \
    const int64_t r0_ = (TT) * batch;                                                   \
    const int B_ = static_cast<int>((rows - r0_) < batch ? (rows - r0_) : batch);      \
    const uint32_t* src_ = bits + r0_ * words;                                          \
    const int n_ = B_ * words;                                                          \
    _Pragma("unroll") for (int q = 0; q < kStage; ++q) {                                \
      const int e_ = q * 1024 + tid;                                                    \
      if (q * 1024 < n_) stg[q] = src_[e_ < n_ ? e_ : n_ - 1];                          \
    }                                                                                   \
    kst = kern[r0_ + (tid < B_ ? tid : B_ - 1)];                                        \
  }
#define XPG_ROWS_STORE(TT)                                                              \
  {                                                                                     \
    _Pragma("unroll") for (int q = 0; q < kStage; ++q) {                                \
      const int e_ = q * 1024 + tid;                                                    \
      if (e_ < batch * words) Rb[(e_ / words) * rp + (e_ % words)] = stg[q];            \
    }                                                                                   \
    const int64_t r0_ = (TT) * batch;                                                   \
    const int B_ = static_cast<int>((rows - r0_) < batch ? (rows - r0_) : batch);      \
    if (tid < batch) kbuf[tid] = kst;                                                   \
    for (int e_ = tid + 1024; e_ < B_; e_ += 1024) kbuf[e_] = kern[r0_ + e_];           \
  }
#define XPG_COLS_LOAD(TT)                                                               \
  {                                                                                     \
    const uint32_t* src_ = colbits + (TT) * cols * bw;                                  \
    _Pragma("unroll") for (int q = 0; q < kStage; ++q) {                                \
      const int e_ = q * 1024 + tid;                                                    \
      if (q * 1024 < cols * bw) stg[q] = src_[e_ < cols * bw ? e_ : cols * bw - 1];     \
    }                                                                                   \
  }
#define XPG_COLS_STORE()                                                                \
  {                                                                                     \
    _Pragma("unroll") for (int q = 0; q < kStage; ++q) {                                \
      const int e_ = q * 1024 + tid;                                                    \
      if (e_ < cols * bw) Cb[(e_ / bw) * cp + (e_ % bw)] = stg[q];                      \
    }                                                                                   \
  }
  // schedule: Cb(t) is loaded at the start of phase B(t) and stored before barrier 1 (its
  // previous reader, D(t-1), finished at barrier D); Rb(t+1) and kbuf(t+1) are loaded after
  // barrier 1 and stored before barrier 2 (their readers, B(t) and G(t), finished at barrier 1).
  if (STAGE) {
    XPG_ROWS_LOAD(0)
    XPG_ROWS_STORE(0)
  }
  wlm_barrier<STAGE>();
#ifdef XPG_WLM_STAMPS
  uint64_t stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stamp_last = __builtin_amdgcn_s_memtime();
#endif

  for (int64_t t = 0; t < nsteps; ++t) {
    const int64_t r0 = t * batch;
    const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
    const WlmStep sc = stp[t];
    if (STAGE) XPG_COLS_LOAD(t)
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int i = tid + c * 1024;
      if (i < cols) w_hist[t * cols + i] = w[c];
    }
    // ---- B: partial predictions p_j = M_b[j] . w over a slice of words (lanes = rows)
    for (int it = wave; it < nrb * n_bs; it += 16) {
      const int rb = it % nrb, sl = it / nrb;
      const int j = rb * 64 + lane;
      const int wd0 = sl * bsw, wd1 = min(words, wd0 + bsw);
      float s = 0.f;
      if (j < B) {
        const uint32_t* row = STAGE ? (Rb + j * rp) : (bits + (r0 + j) * words);
        for (int k0 = wd0; k0 < wd1; k0 += 2) {  // 16 lookups in flight (lgkmcnt limit 15)
          uint32_t wv[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int wd = k0 + h;
            wv[h] = row[wd < wd1 ? wd : wd0];
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int wd = k0 + h;
            const float x = nib8(T + ((wd < wd1 ? wd : wd0) * 8) * kTabPitch, wv[h]);
            s += wd < wd1 ? x : 0.f;
          }
        }
      }
      if (j < batch) bpart[sl * batch + j] = s;
    }
    XPG_STAMP(0)
    wlm_barrier<STAGE>();  // bpart complete
    XPG_STAMP(1)
    // ---- G: g_j = 2 k_j (p_j - ybar) / (B sum k) and the nibble tables of g over 4-row groups
    {
      const int ngrp = (B + 3) >> 2;
      const double cg = 2.0 / (static_cast<double>(B) * sc.ksum);
      for (int e = tid; e < ngrp * 16; e += 1024) {
        const int grp = e >> 4, vv = e & 15;
        float acc = 0.f;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int j = 4 * grp + b;
          float g = 0.f;
          if (j < B) {
            float p = 0.f;
            for (int sl = 0; sl < n_bs; ++sl) p += bpart[sl * batch + j];
            const double kj = STAGE ? kbuf[j] : kern[r0 + j];
            g = static_cast<float>(kj * cg * (static_cast<double>(p) - sc.ybar));
            if (vv == b) p_hist[r0 + j] = p;
          }
          acc += ((vv >> b) & 1) ? g : 0.f;
        }
        G[grp * kTabPitch + vv] = acc;
      }
    }
    if (STAGE) XPG_COLS_STORE()
    XPG_STAMP(2)
    wlm_barrier<STAGE>();  // G and Cb(t) complete; Rb, kbuf free
    XPG_STAMP(3)
    if (STAGE && t + 1 < nsteps) XPG_ROWS_LOAD(t + 1)
    // ---- D: partial gradient (M_b^T g)_i over a slice of the column's row words (lanes = columns)
    for (int it = wave; it < ncb * n_ds; it += 16) {
      const int cbk = it % ncb, sl = it / ncb;
      const int i = cbk * 64 + lane;
      const int k0 = sl * dsw, k1 = min(bw, k0 + dsw);
      float s = 0.f;
      if (i < cols) {
        const uint32_t* cb = STAGE ? (Cb + i * cp) : (colbits + (t * cols + i) * bw);
        for (int kk = k0; kk < k1; kk += 2) {
          uint32_t wv[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = kk + h;
            wv[h] = cb[k < k1 ? k : k0];
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = kk + h;
            const float x = nib8(G + ((k < k1 ? k : k0) * 8) * kTabPitch, wv[h]);
            s += k < k1 ? x : 0.f;
          }
        }
      }
      dpart[sl * cpad + i] = s;
    }
    XPG_STAMP(4)
    wlm_barrier<STAGE>();  // dpart complete
    XPG_STAMP(5)
    // ---- L1 subgradient + L2 decay; Adam (torch single-tensor order) on the owned columns
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int i = tid + c * 1024;
      if (i < cols) {
        float s = 0.f;
        for (int sl = 0; sl < n_ds; ++sl) s += dpart[sl * cpad + i];
        const float sg = w[c] > 0.f ? 1.f : (w[c] < 0.f ? -1.f : 0.f);
        float g = fmaf(l1s, sg, s);
        g = fmaf(P.weight_decay, w[c], g);
        m[c] = fmaf(1.f - P.beta1, g - m[c], m[c]);
        v[c] = fmaf(1.f - P.beta2, g * g, v[c] * P.beta2);
        const float denom = sqrtf(v[c]) / sc.bc2_sqrt + P.eps;
        w[c] = w[c] - sc.step_size * (m[c] / denom);
      }
    }
    wlm_build_T<CPT>(w, T, ntab);
    if (STAGE && t + 1 < nsteps) XPG_ROWS_STORE(t + 1)
    XPG_STAMP(6)
    wlm_barrier<STAGE>();
    XPG_STAMP(7)
  }
#ifdef XPG_WLM_STAMPS
  if (tid == 0 || tid == 1023) {
    for (int k = 0; k < 8; ++k) g_wlm_stamps[tid == 0 ? 0 : 1][k] = stamp_acc[k];
  }
#endif
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int i = tid + c * 1024;
    if (i < cols) {
      wg[i] = w[c];
      mg[i] = m[c];
      vg[i] = v[c];
    }
  }
#undef XPG_ROWS_LOAD
#undef XPG_ROWS_STORE
#undef XPG_COLS_LOAD
#undef XPG_COLS_STORE
}

// Multi-workgroup fit (cols large enough to split): P workgroups per fit, one per CU, each
// owning a contiguous slice of mask words (its columns: w, Adam moments, T tables, column bit
// vectors).  Per Adam step the partial predictions over each slice are exchanged through memory
// (MI355X_MICROARCH.md inter-workgroup hand-off: 8-byte {value, step tag} granules, stored and
// polled with sc1) and summed in a fixed order, so every workgroup derives the same g; the
// gradient and Adam update of a column stay with its owner.  The poll is bounded: a grid that is
// not co-resident ends (with an error flag) instead of hanging.
//
// One Adam step = two workgroup barriers.  The step is issue-bound (4 waves share a SIMD), so
// every phase runs only in the waves that have work in it, all per-thread staging offsets are
// computed once, and reductions stay inside waves:
//   B     waves 0..nrb-1, lane = row j: partial p_j over the own words (w nibble tables T, rows
//         Rb(t)), published at once as a granule
//   stage every wave: the next step's rows, kernel weights and column bit vectors, and the step
//         constants (lanes 0..7, vector loads), into registers; the pre-step weights (w_hist)
//   poll  the B lanes again: the other parts' granules of row j (all loads in flight, then a
//         bounded spin on the untagged ones), p_j summed over parts 0..P-1 in order (the own
//         one from the register), g_j, and the 4 entries 4b..4b+3 of the group's 4-bit G table
//         (b = j & 3; the group's 4 g values by quad DPP moves)
//   -- barrier 1 --
//   D     lane = (column, slice of the column's row words): partial (M_b^T g)_i, xor-shuffle
//         reduction over the slices; the slice-0 lane owns the column: L1/L2 terms and Adam,
//         then the column quad's 4 T entries (quad DPP moves); staged registers -> LDS
//         (column vectors double-buffered: D(t) still reads Cb(t) while Cb(t+1) is stored)
//   -- barrier 2 --
constexpr uint32_t kMcSpinLimit = 1u << 21;
constexpr int kMcMaxP = 32;       // parts per fit (polled in rounds of kMcPollRound)
constexpr int kMcPollRound = 16;
constexpr int kMcMaxStage = 4;   // staged words per thread (rows and column vectors each; 8 spills)

__device__ __forceinline__ void st64_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64_sc1(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// WlmStep from the 12 dwords held by lanes 0..11 of the wave (v_readlane: no LDS, no scalar load)
constexpr int kStepDw = sizeof(WlmStep) / 4;
__device__ __forceinline__ WlmStep wlm_step_from_lanes(uint32_t v) {
  uint32_t d[kStepDw];
#pragma unroll
  for (int i = 0; i < kStepDw; ++i) d[i] = __builtin_amdgcn_readlane(v, i);
  WlmStep s;
  s.ybar = __hiloint2double(static_cast<int>(d[1]), static_cast<int>(d[0]));
  s.ksum = __hiloint2double(static_cast<int>(d[3]), static_cast<int>(d[2]));
  s.vy = __hiloint2double(static_cast<int>(d[5]), static_cast<int>(d[4]));
  s.cg = __hiloint2double(static_cast<int>(d[7]), static_cast<int>(d[6]));
  s.step_size = __uint_as_float(d[8]);
  s.bc2_sqrt = __uint_as_float(d[9]);
  s.inv_bc2 = __uint_as_float(d[10]);
  s.pad = 0.f;
  return s;
}

// value of lane (lane & ~3) + B of the quad (DPP quad_perm, no LDS)
template <int B>
__device__ __forceinline__ float quad_bcast(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), B | (B << 2) | (B << 4) | (B << 6), 0xF, 0xF, false));
}

// The 4 nibble-table entries vv = 4q..4q+3 (q = lane & 3) of the quad's 4 values x_0..x_3:
// entry vv = sum of x_b over the set bits b of vv, added in b order (as wlm_build_T / the G
// build of k_wlm_fit).
__device__ __forceinline__ void quad_table_entries(float x, float* dst) {
  const float x0 = quad_bcast<0>(x), x1 = quad_bcast<1>(x), x2 = quad_bcast<2>(x), x3 = quad_bcast<3>(x);
  const int q = threadIdx.x & 3;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int vv = 4 * q + i;
    float s = 0.f;
    s += (vv & 1) ? x0 : 0.f;
    s += (vv & 2) ? x1 : 0.f;
    s += (vv & 4) ? x2 : 0.f;
    s += (vv & 8) ? x3 : 0.f;
    dst[vv] = s;
  }
}

template <int CPL, int STG>
__global__ __launch_bounds__(1024) void k_wlm_fit_mc(
    const uint32_t* __restrict__ bits, const uint32_t* __restrict__ colbits, int64_t rows, int cols, int words,
    int batch, int bw, int P, int wpp, int n_ds, int64_t n_fits, int xcd_local,
    const double* __restrict__ kern,
    const WlmStep* __restrict__ stp, xpg_wlm_params Pm, float* __restrict__ wg, float* __restrict__ mg,
    float* __restrict__ vg, float* __restrict__ p_hist, float* __restrict__ w_hist, uint64_t* xp,
    uint32_t* err, uint32_t spin_limit, int fault_part, uint32_t epoch_host, int plain_ok,
    const uint32_t* __restrict__ ep_dev) {
  // granule tag epoch (16 bits, never 0): the host's per-call counter + the device word that
  // k_wlm_prep advances per chain, so replays of a captured launch get fresh tags too
  uint32_t epoch = (epoch_host + (ep_dev ? *ep_dev : 0u)) & 0xFFFFu;
  if (epoch == 0u) epoch = 1u;
  static_assert(sizeof(WlmStep) == 48, "WlmStep is read as 12 dwords");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int abort_s;  // set by any lane whose poll timed out (or saw the error word): leave the step loop
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) abort_s = 0;
  int64_t f;
  int part;
  if (xcd_local) {  // blocks b and b + 8 share an XCD (observed round-robin dealing, speed only)
    const int64_t k = blockIdx.x >> 3, g = k / P;
    part = static_cast<int>(k - g * P);
    f = g * 8 + (blockIdx.x & 7);
    if (f >= n_fits) return;  // filler block (whole workgroup)
  } else {
    f = blockIdx.x / P;
    part = static_cast<int>(blockIdx.x - f * P);
  }
  // this workgroup holds its CU until the fit ends: counted on its XCD (k_rows_forward)
  const int my_xcc = xcc_id();
  if (tid == 0) __hip_atomic_fetch_add(g_xcd_busy + my_xcc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t nsteps = (rows + batch - 1) / batch;
  const int w_lo = min(words, part * wpp), w_hi = min(words, w_lo + wpp);
  const int ow = w_hi - w_lo;                       // own words (>= 1: P = ceil(words / wpp))
  const int c_lo = w_lo * 32, ncol = max(0, min(cols, w_hi * 32) - c_lo);
  bits += f * rows * words + w_lo;
  colbits += f * nsteps * cols * bw + (int64_t)c_lo * bw;
  kern += f * rows;
  stp += f * nsteps;
  wg += f * cols + c_lo;
  mg += f * cols + c_lo;
  vg += f * cols + c_lo;
  p_hist += f * rows;
  w_hist += f * nsteps * cols + c_lo;
  xp += f * (2 * P * (int64_t)batch + P);  // [2][P][batch] step granules + [P] XCC granules
  const uint32_t* stp32 = reinterpret_cast<const uint32_t*>(stp);
  __shared__ int plain_s;

  const int rp = wpp | 1, cp = bw | 1;
  const int cbuf = wpp * 32 * cp;                                      // one Cb buffer (words)
  float* G = reinterpret_cast<float*>(smem);                           // [bw*8][17]
  const int kb_off = (bw * 8 * kTabPitch + 1) & ~1;
  double* kbuf = reinterpret_cast<double*>(G + kb_off);                // [batch]
  float* T = reinterpret_cast<float*>(kbuf + batch);                   // [wpp*8][17]
  uint32_t* Rb = reinterpret_cast<uint32_t*>(T + wpp * 8 * kTabPitch); // [batch][rp]
  uint32_t* Cb = Rb + batch * rp;                                      // [2][wpp*32][cp]

  const int nrb = (batch + 63) >> 6;
  const int cw = 64 / n_ds;                       // columns per wave chunk (power of 2, >= 4)
  const int dsw = (bw + n_ds - 1) / n_ds;         // row words per slice
  const int col_lo = lane & (cw - 1), sl = lane / cw;
  const int k0 = sl * dsw, k1 = min(bw, k0 + dsw);
  const int nchunk = (ow * 32 + cw - 1) / cw;  // chunks over the own words (tail columns: w = 0, zero T entries)
  const float l1s = Pm.l1_lambda / static_cast<float>(cols);

  // per-thread staging offsets (fixed for the whole fit).  With batch <= 512 the waves past the
  // B / poll waves do all the staging (ns stagers, sid < 0: a poll wave), so the next step's
  // loads are not issued between a poll wave's publish and its poll (the step's critical path)
  const bool split_stage = nrb <= 8;
  const int ns = split_stage ? 1024 - 64 * nrb : 1024;
  const int sid = split_stage ? tid - 64 * nrb : tid;
  int ro[STG], rl[STG], cl[STG];  // rows: global word offset (row * words + word), LDS offset | row << 16
  const int n_r = batch * ow, n_c = ncol * bw;
#pragma unroll
  for (int q = 0; q < STG; ++q) {
    const int e = sid < 0 ? n_r + n_c : q * ns + sid;
    const int rr = e < n_r ? e / ow : 0, wd = e < n_r ? e - rr * ow : 0;
    ro[q] = rr * words + wd;
    rl[q] = (rr * rp + wd) | (rr << 16);
    const int ce = e < n_c ? e : 0;
    cl[q] = (ce / bw) * cp + (ce % bw);
  }
  uint32_t sr[STG], sv[STG];
  double kst = 0.0;
#define XPG_MC_LOAD(TT)                                                                 \
  {                                                                                     \
    const int64_t r0_ = (TT) * batch;                                                   \
    const int B_ = static_cast<int>((rows - r0_) < batch ? (rows - r0_) : batch);      \
    const uint32_t* rs_ = bits + r0_ * words;                                           \
    const uint32_t* cs_ = colbits + (TT) * cols * bw;                                   \
    _Pragma("unroll") for (int q = 0; q < STG; ++q) {                                   \
      const int e_ = q * ns + sid;                                                      \
      if (sid >= 0 && e_ < n_r) {                                                       \
        const int rr_ = rl[q] >> 16;                                                    \
        sr[q] = rs_[rr_ < B_ ? ro[q] : ro[q] - rr_ * words];                            \
      }                                                                                 \
      if (sid >= 0 && e_ < n_c) sv[q] = cs_[e_];                                        \
    }                                                                                   \
    if (sid >= 0 && sid < B_) kst = kern[r0_ + sid];                                    \
  }
#define XPG_MC_STORE(TT)                                                                \
  {                                                                                     \
    uint32_t* cb_ = Cb + ((TT) & 1) * cbuf;                                             \
    _Pragma("unroll") for (int q = 0; q < STG; ++q) {                                   \
      const int e_ = q * ns + sid;                                                      \
      if (sid >= 0 && e_ < n_r) Rb[rl[q] & 0xFFFF] = sr[q];                             \
      if (sid >= 0 && e_ < n_c) cb_[cl[q]] = sv[q];                                     \
    }                                                                                   \
    if (sid >= 0 && sid < batch) kbuf[sid] = kst;                                       \
  }

  // own columns: column chunk (wave + 16 c), lane col_lo; the slice-0 lane holds w, m, v
  float w[CPL], m[CPL], v[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int i = (wave + 16 * c) * cw + col_lo;
    const bool own = sl == 0 && i < ncol;
    w[c] = own ? wg[i] : 0.f;
    m[c] = own ? mg[i] : 0.f;
    v[c] = own ? vg[i] : 0.f;
  }
  for (int e = tid; e < bw * 8 * kTabPitch; e += 1024) G[e] = 0.f;
  // initial T: quads of own columns (tail columns hold w = 0, so tail entries are 0)
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = wave + 16 * c;
    if (ch < nchunk && sl == 0) {
      const int i = ch * cw + col_lo;
      if (i < ow * 32) quad_table_entries(w[c], T + (i >> 2) * kTabPitch);
    }
  }
  XPG_MC_LOAD(0)
  uint32_t stw = lane < kStepDw ? stp32[lane] : 0u;
  // XCC handshake (once per fit): when every part of the fit runs on one XCD, the step granules
  // are published with workgroup-scope stores, which keep the line in that XCD's L2, so the
  // parts' sc1 polls are served from L2 instead of memory (speed only: the test is made at run
  // time, so any placement stays correct).  Tag epoch << 16 (step 0).
  if (wave == 0) {
    uint64_t* xc = xp + 2 * P * (int64_t)batch;
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu;  // HW_REG_XCC_ID[3:0]
    const uint32_t htag = epoch << 16;
    if (lane == 0) st64_sc1(xc + part, (static_cast<uint64_t>(htag) << 32) | xcc);
    bool same = true;
    if (lane < P && plain_ok) {
      uint64_t gx = ld64_sc1(xc + lane);
      uint32_t n = 0;
      while (static_cast<uint32_t>(gx >> 32) != htag && n <= spin_limit) {
        __builtin_amdgcn_s_sleep(1);
        gx = ld64_sc1(xc + lane);
        ++n;
      }
      same = static_cast<uint32_t>(gx >> 32) == htag && static_cast<uint32_t>(gx) == xcc;
    }
    const bool all = __ballot(!same) == 0ull && plain_ok;
    if (lane == 0) plain_s = all ? 1 : 0;
  }
  XPG_MC_STORE(0)
  lds_barrier();
  const bool plain = plain_s != 0;
#ifdef XPG_WLM_STAMPS
  uint64_t stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stamp_last = __builtin_amdgcn_s_memtime();
#endif

  for (int64_t t = 0; t < nsteps; ++t) {
    const int64_t r0 = t * batch;
    const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
    const WlmStep sc = wlm_step_from_lanes(stw);
    uint64_t* xs = xp + (t & 1) * P * (int64_t)batch;
    const uint32_t tag = (epoch << 16) | static_cast<uint32_t>(t + 1);
    const int j = wave * 64 + lane;  // B / poll row
    const bool prow = wave < nrb && j < B;
    // ---- B: partial p_j over the own words, published from the lane
    float pown = 0.f;
    if (wave < nrb) {
      if (j < B) {
        const uint32_t* row = Rb + j * rp;
        if (ow <= 4) {  // the usual 3 words per part: all row words, then all lookups (2 LDS round trips)
          uint32_t wv[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) wv[h] = row[h < ow ? h : 0];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const float x = nib8(T + ((h < ow ? h : 0) * 8) * kTabPitch, wv[h]);
            pown += h < ow ? x : 0.f;
          }
        } else {
          for (int kw = 0; kw < ow; kw += 2) {  // 16 lookups in flight (lgkmcnt limit 15)
            uint32_t wv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) wv[h] = row[kw + h < ow ? kw + h : kw];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float x = nib8(T + ((kw + h < ow ? kw + h : kw) * 8) * kTabPitch, wv[h]);
              pown += kw + h < ow ? x : 0.f;
            }
          }
        }
        const bool skip_pub = fault_part == part && f == 0 && t == 0;  // fault injection (tests only)
        if (!skip_pub) {
          const uint64_t gv = (static_cast<uint64_t>(tag) << 32) | __float_as_uint(pown);
          if (plain)
            __hip_atomic_store(xs + part * (int64_t)batch + j, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            st64_sc1(xs + part * (int64_t)batch + j, gv);
        }
      }
    }
    XPG_STAMP(0)
    // ---- stage: the next step's data and constants; the pre-step weights
    if (t + 1 < nsteps) {
      XPG_MC_LOAD(t + 1)
      stw = lane < kStepDw ? stp32[(t + 1) * kStepDw + lane] : 0u;
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int i = (wave + 16 * c) * cw + col_lo;
      if (sl == 0 && i < ncol) w_hist[t * cols + i] = w[c];
    }
    XPG_STAMP(1)
    // ---- poll: p_j over the parts in order, g_j, the G table entries
    if (wave < nrb) {
      float p = 0.f;
      if (prow) {
        // parts in rounds of kMcPollRound (all of a round's granule loads in flight, then the
        // bounded spins), summed in part order 0..P-1 either way
        for (int q0 = 0; q0 < P; q0 += kMcPollRound) {
          uint64_t gr[kMcPollRound];
#pragma unroll
          for (int qq = 0; qq < kMcPollRound; ++qq) {
            const int q = q0 + qq;
            gr[qq] = q < P && q != part ? ld64_sc1(xs + q * (int64_t)batch + j) : (static_cast<uint64_t>(tag) << 32);
          }
#pragma unroll
          for (int qq = 0; qq < kMcPollRound; ++qq) {
            const int q = q0 + qq;
            if (q < P) {
              uint32_t n = 0;
              while (static_cast<uint32_t>(gr[qq] >> 32) != tag) {
                __builtin_amdgcn_s_sleep(1);
                gr[qq] = ld64_sc1(xs + q * (int64_t)batch + j);
                ++n;
                // bounded: a partner that never publishes (grid not co-resident, or a partner
                // that already left after an error) ends the fit with the error word set, which
                // xpg_wlm_fit hands to the caller's status word
                if (n > spin_limit || ((n & 63u) == 0 &&
                                       __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                  __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  abort_s = 1;
                  break;
                }
              }
              p += q == part ? pown : __uint_as_float(static_cast<uint32_t>(gr[qq]));
            }
          }
        }
      }
      float g = 0.f;
      if (prow) {
        if (part == 0) p_hist[r0 + j] = p;
        g = static_cast<float>(kbuf[j] * sc.cg * (static_cast<double>(p) - sc.ybar));
      }
      // rows >= B of the last group hold g = 0; whole quads stay inside the batch
      if (j < ((B + 3) & ~3)) quad_table_entries(g, G + (j >> 2) * kTabPitch);
    }
    XPG_STAMP(2)
    lds_barrier();  // G complete; Rb(t), kbuf(t) free
    XPG_STAMP(3)
    if (abort_s) break;  // workgroup-uniform (read after the barrier): the fit is invalid, stop
    // ---- D + Adam + T on the own column chunks
    {
      const uint32_t* cbt = Cb + (t & 1) * cbuf;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int ch = wave + 16 * c;
        if (ch < nchunk) {  // wave-uniform
          const int i = ch * cw + col_lo;
          float s = 0.f;
          if (i < ncol) {
            const uint32_t* cb = cbt + i * cp;
            for (int kk = k0; kk < k1; kk += 2) {
              uint32_t wv[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) wv[h] = cb[kk + h < k1 ? kk + h : kk];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const float x = nib8(G + ((kk + h < k1 ? kk + h : kk) * 8) * kTabPitch, wv[h]);
                s += kk + h < k1 ? x : 0.f;
              }
            }
          }
          // xor reduction over the slices: distances 16 and 32 on the VALU (permlane swaps; the
          // sum is commutative, so bitwise the shuffle's), shorter ones by ds_bpermute
          for (int o = cw; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
          if (cw <= 16) {
            const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
            s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
          }
          if (cw <= 32) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
            s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
          }
          if (sl == 0) {
            if (i < ncol) {
              const float sg = w[c] > 0.f ? 1.f : (w[c] < 0.f ? -1.f : 0.f);
              float gi = fmaf(l1s, sg, s);
              gi = fmaf(Pm.weight_decay, w[c], gi);
              m[c] = fmaf(1.f - Pm.beta1, gi - m[c], m[c]);
              v[c] = fmaf(1.f - Pm.beta2, gi * gi, v[c] * Pm.beta2);
              // v_sqrt / v_rcp (1 ulp) instead of the correctly rounded sequences: the Adam update
              // is the step's dependent tail (torch: (sqrt(v) / bc2_sqrt + eps), addcdiv)
              const float denom = __builtin_amdgcn_sqrtf(v[c]) * sc.inv_bc2 + Pm.eps;
              w[c] = w[c] - sc.step_size * (m[c] * __builtin_amdgcn_rcpf(denom));
            }
            if (i < ow * 32) quad_table_entries(w[c], T + (i >> 2) * kTabPitch);
          }
        }
      }
    }
    XPG_STAMP(4)
    if (t + 1 < nsteps) XPG_MC_STORE(t + 1)
    XPG_STAMP(5)
    lds_barrier();  // T, Rb(t+1), kbuf(t+1), Cb(t+1) complete
    XPG_STAMP(6)
    XPG_STAMP(7)
  }
#ifdef XPG_WLM_STAMPS
  stamp_acc[7] = plain ? nsteps : 0;  // reported as 1 per step: the L2-resident publish path ran
  if (blockIdx.x == 0 && (tid == 0 || tid == 1023)) {
    for (int k = 0; k < 8; ++k) g_wlm_stamps[tid == 0 ? 0 : 1][k] = stamp_acc[k];
  }
#endif
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int i = (wave + 16 * c) * cw + col_lo;
    if (sl == 0 && i < ncol) {
      wg[i] = w[c];
      mg[i] = m[c];
      vg[i] = v[c];
    }
  }
  if (tid == 0) __hip_atomic_fetch_add(g_xcd_busy + my_xcc, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#undef XPG_MC_LOAD
#undef XPG_MC_STORE
}


// loss_t = sum_j k_j (p_j - ybar)^2 / (B sum k) + sum_i (y_i - ybar)^2 / B^2 + l1 * mean|w_t|
// One launch per fit chain for the losses and the best epoch: block (t, fit) computes loss_t
// (256 threads, the formula above), publishes it, and the fit's last block to finish (arrival
// counter, cleared by k_wlm_prep) takes the first argmin over the fit's steps in one wave
// (k_argmin_first's answer: the lowest step among equal minima, step 0 when none is below +inf).
// Also hands the multi-workgroup exchange's error word to the caller's status word.
__global__ __launch_bounds__(256) void k_wlm_loss_best(const float* __restrict__ p_hist,
                                                       const float* __restrict__ w_hist,
                                                       const double* __restrict__ kern,
                                                       const WlmStep* __restrict__ stp, int64_t rows,
                                                       int cols, int batch, float l1,
                                                       double* __restrict__ losses, int32_t* __restrict__ best,
                                                       uint32_t* __restrict__ arrive, const uint32_t* __restrict__ errw,
                                                       int32_t* __restrict__ status) {
  __shared__ double red[16];
  __shared__ int last_s;
  const int64_t t = blockIdx.x, f = blockIdx.y, steps = gridDim.x;
  // sticky: OR the exchange's error word into the caller's word (zeroed once by the caller), so
  // a timeout in any fit of a replayed chain stays visible after the last one (ABI v13)
  if (status && errw && f == 0 && t == 0 && threadIdx.x == 0 && *errw)
    *status = *status | static_cast<int32_t>(*errw);
  p_hist += f * rows;
  w_hist += f * steps * cols;
  kern += f * rows;
  stp += f * steps;
  losses += f * steps;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const WlmStep sc = stp[t];
  double tk = 0.0, sa = 0.0;
  for (int j = threadIdx.x; j < B; j += blockDim.x) {
    const double d = static_cast<double>(p_hist[r0 + j]) - sc.ybar;
    tk += kern[r0 + j] * d * d;
  }
  for (int i = threadIdx.x; i < cols; i += blockDim.x) sa += fabs(static_cast<double>(w_hist[t * cols + i]));
  const double Tk = block_sum_d(tk, red);
  const double Sa = block_sum_d(sa, red);
  if (threadIdx.x == 0) {
    const float reg = l1 * static_cast<float>(Sa / cols);
    const double loss = Tk / (static_cast<double>(B) * sc.ksum) + sc.vy / (static_cast<double>(B) * B) +
                        static_cast<double>(reg);
    __hip_atomic_store(losses + t, loss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t n = __hip_atomic_fetch_add(arrive + f, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last_s = n + 1 == static_cast<uint32_t>(steps);
  }
  __syncthreads();
  if (!last_s || threadIdx.x >= 64) return;
  // the fit's last block: every loss is published (acq_rel counter); one wave scans them
  const int lane = threadIdx.x;
  double bv = INFINITY;
  int64_t bi = -1;
  for (int64_t i = lane; i < steps; i += 64) {
    const double v = __hip_atomic_load(losses + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v < bv) {
      bv = v;
      bi = i;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int64_t oi = __shfl_xor(bi, off, 64);
    if (oi >= 0 && (bi < 0 || ov < bv || (ov == bv && oi < bi))) {
      bv = ov;
      bi = oi;
    }
  }
  if (lane == 0) best[f] = static_cast<int32_t>(bi < 0 ? 0 : bi);
}

// -------------------------------------------------------------- surrogate, many-column (grid) fit
// For S beyond the single-workgroup fit (graph_prediction on large graphs, regime (ii)) each
// Adam step is three grid launches over 2048-column chunks (64 mask words).  Both bit-streaming
// kernels read the step's B x S mask bits once, coalesced (lane = mask word, 32 rows per load
// round, 32 loads in flight per lane), so a step costs 2 * B * S / 8 bytes of HBM reads plus the
// Adam state:
//   k_gw_p     p_j = (M_b w)_j per chunk: nibble tables of w in LDS laid out [nibble pos][value]
//              [word] (lane = word: every lane its own bank), then a butterfly transpose-reduce
//              of the lane's 32 row partials over the wave; partial p per (chunk, row)
//   k_gw_g     p_j = sum of the partials, g_j = 2 k_j (p_j - ybar) / (B sum k), the loss term
//   k_gw_grad  (M_b^T g)_c per chunk: each lane transposes its 32 x 32 bit block in registers
//              (5 butterfly stages), then one lookup per nibble into 4-row tables of g; the four
//              waves' column sums meet in LDS; Adam update of the chunk's columns and sum |w|
constexpr int kGwWords = 64;    // mask words per chunk (2048 columns)
constexpr int kGpWaves = 8;     // k_gw_p: waves per workgroup (16: slower, r5_grid_fit_waves_ab.log)
constexpr int kGgWaves = 4;     // k_gw_grad: waves per workgroup (8: slower)

// Sum of v[0..31] over the wave's 64 lanes for every i: after the call lanes 2i and 2i + 1 hold
// sum_lanes v[i] in v[0] (5 halving exchange stages + a final pair add).
__device__ __forceinline__ float wave_transpose_reduce32(float (&v)[32], int lane) {
#pragma unroll
  for (int st = 0; st < 5; ++st) {
    const int half = 16 >> st;            // values kept after this stage
    const int xm = 32 >> st;              // partner lane distance
    const bool hi = (lane & xm) != 0;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      float lo_v = v[k], hi_v = v[k + half];
      asm volatile("" : "+v"(lo_v), "+v"(hi_v));  // opaque: keeps the selects on values, not indices
      const float keep = hi ? hi_v : lo_v;
      const float send = hi ? lo_v : hi_v;
      float r = keep + __shfl_xor(send, xm);
      asm volatile("" : "+v"(r));
      v[k] = r;
    }
  }
  return v[0] + __shfl_xor(v[0], 1);
}

// Sum of v[0..7] over the wave's 64 lanes for every i: after the call lanes 8i..8i+7 hold
// sum_lanes v[i] (k_gw_fused).  wave_transpose_reduce32's halving stages without LDS permutes:
// the 32- and 16-lane stages are v_permlane32_swap / v_permlane16_swap (swapping the two halves'
// values IS the stage's keep / send exchange), the 8-lane stage a DPP row rotation, then a DPP
// half-mirror and two quad permutes sum the 8 lanes that share a row.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_transpose_reduce8_pl(float (&v)[8], int lane) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // lanes 0-31 keep v[k], lanes 32-63 v[k + 4]
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 4]), false, false);
    v[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // even 16-lane rows keep v[k], odd rows v[k + 2]
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 2]), false, false);
    v[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool hi = (lane & 8) != 0;  // lanes l and l ^ 8 of a row: row_ror:8
  float lo_v = v[0], hi_v = v[1];
  asm volatile("" : "+v"(lo_v), "+v"(hi_v));
  const float keep = hi ? hi_v : lo_v, send = hi ? lo_v : hi_v;
  float r = keep + dpp_mov<0x128>(send);
  r += dpp_mov<0x141>(r);  // row_half_mirror: l <-> 7 - l
  r += dpp_mov<0x4E>(r);   // quad_perm [2,3,0,1]
  r += dpp_mov<0xB1>(r);   // quad_perm [1,0,3,2]
  return r;
}

// x[i] = word `wd` of row row0 + i for i < nr, else 0.  row0 / nr are wave-uniform, so the row
// test is a scalar branch and all loads are in flight together (no per-lane exec masking);
// callers mask lanes past the chunk.
__device__ __forceinline__ void gw_load32(const uint32_t* __restrict__ bits, int64_t words, int64_t row0, int nr,
                                          uint32_t wd, uint32_t (&x)[32]) {
  typedef const __attribute__((address_space(1))) uint32_t gu32;
  gu32* base = (gu32*)(bits + row0 * words);
#pragma unroll
  for (int i = 0; i < 32; ++i) x[i] = i < nr ? base[(int64_t)i * words + wd] : 0u;  // uniform branch
}

// grid (n_chunks, n_fits), kGpWaves * 64 threads; p_part [n_fits][n_chunks][batch]
__global__ __launch_bounds__(kGpWaves * 64) void k_gw_p(const uint32_t* __restrict__ bits, int64_t rows,
                                                       int64_t cols, int64_t words, int batch, int64_t t,
                                                       const float* __restrict__ wg, float* __restrict__ p_part) {
  __shared__ float T[8 * 16 * kGwWords];  // T[(q * 16 + v) * 64 + j]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t f = blockIdx.y;
  bits += f * rows * words;
  wg += f * cols;
  p_part += (f * gridDim.x + blockIdx.x) * (int64_t)batch;
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform row blocks
  uint32_t x[32];
  if (wv * 32 < B) gw_load32(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);  // in flight
  for (int task = tid; task < 8 * kGwWords; task += kGpWaves * 64) {  // during the table build:
    const int j = task & (kGwWords - 1), q = task >> 6;                // (word, nibble position)
    const int64_t c = (w0 + j) * 32 + 4 * q;
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = c + b < cols ? wg[c + b] : 0.f;
    float* Tq = T + q * 16 * kGwWords + j;  // entry v at Tq[v * 64]: lanes = words, no conflicts
#pragma unroll
    for (int v = 0; v < 16; ++v)
      Tq[v * kGwWords] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                         ((v & 8) ? a[3] : 0.f);
  }
  __syncthreads();
  const float* Tl = T + lane;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += kGpWaves) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];  // next block's words, in flight during this block's lookups
    const int rbn = rb + kGpWaves;
    if (rbn * 32 < B) gw_load32(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
    float c[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t xi = i < nr ? (x[i] & lmask) : 0u;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) s += Tl[(q * 16 + ((xi >> (4 * q)) & 15u)) * kGwWords];
      c[i] = s;
    }
    const float tot = wave_transpose_reduce32(c, lane);
    const int i = (lane >> 1) & 31;
    if (!(lane & 1) && i < nr) p_part[rb * 32 + i] = tot;
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
}

// grid (ceil(batch / 64), n_fits), 1024 threads: 16 waves split the partials of 64 rows
__global__ __launch_bounds__(1024) void k_gw_g(const float* __restrict__ p_part, int n_wg, int64_t rows,
                                               int batch, int64_t t, const double* __restrict__ kern,
                                               const WlmStep* __restrict__ stp, int64_t steps,
                                               float* __restrict__ g, float* __restrict__ p_hist,
                                               double* __restrict__ tk_part) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t f = blockIdx.y;
  p_part += f * n_wg * (int64_t)batch;
  kern += f * rows;
  g += f * batch;
  p_hist += f * rows;
  const WlmStep sc = stp[f * steps + t];
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int j = blockIdx.x * 64 + lane;
  float p = 0.f;
  if (j < B) {
#pragma unroll 8
    for (int w = wave; w < n_wg; w += 16) p += p_part[(int64_t)w * batch + j];
  }
  red[wave][lane] = p;
  __syncthreads();
  if (wave != 0) return;
  p = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) p += red[w][lane];
  double tk = 0.0;
  if (j < B) {
    const double kj = kern[r0 + j];
    const double d = static_cast<double>(p) - sc.ybar;
    g[j] = static_cast<float>(kj * (2.0 / (static_cast<double>(B) * sc.ksum)) * d);
    p_hist[r0 + j] = p;
    tk = kj * d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tk += __shfl_xor(tk, o);
  if (lane == 0) tk_part[(f * steps + t) * gridDim.x + blockIdx.x] = tk;
}

// grid (n_chunks, n_fits), kGgWaves * 64 threads, dynamic LDS 16 * (ceil(batch/32) * 8 | 1) + 2080
// floats (rounded to 4)
__global__ __launch_bounds__(kGgWaves * 64) void k_gw_grad(const uint32_t* __restrict__ bits, int64_t rows,
                                                          int64_t cols, int64_t words, int batch, int64_t t,
                                                          const float* __restrict__ g, const WlmStep* __restrict__ stp,
                                                          int64_t steps, xpg_wlm_params P, float* __restrict__ wg,
                                                          float* __restrict__ mg, float* __restrict__ vg,
                                                          double* __restrict__ aw_part) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  __shared__ double red[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t f = blockIdx.y;
  bits += f * rows * words;
  g += f * batch;
  wg += f * cols;
  mg += f * cols;
  vg += f * cols;
  const WlmStep sc = stp[f * steps + t];
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const int ngrp = ((B + 31) / 32) * 8;  // 4-row groups of whole 32-row blocks (tail groups 0)
  const int64_t w0 = (int64_t)blockIdx.x * kGwWords;
  const int nw = static_cast<int>((words - w0) < kGwWords ? (words - w0) : kGwWords);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform row blocks
  uint32_t x[32];
  if (wv * 32 < B) gw_load32(bits, words, r0 + wv * 32, min(32, B - wv * 32), wd, x);  // in flight
  const int gp = ngrp | 1;                     // odd pitch: the 16 entries of a group on 16 banks
  float* G = gsm;                              // G[v * gp + group]
  float* colsum = gsm + ((16 * gp + 3) & ~3);  // [32 bit][65]: column (word j, bit b) at b * 65 + j
  for (int grp = tid; grp < ngrp; grp += kGgWaves * 64) {  // thread = 4-row group: subset sums
    float a[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) a[b] = 4 * grp + b < B ? g[4 * grp + b] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      G[v * gp + grp] = ((v & 1) ? a[0] : 0.f) + ((v & 2) ? a[1] : 0.f) + ((v & 4) ? a[2] : 0.f) +
                        ((v & 8) ? a[3] : 0.f);
  }
  for (int e = tid; e < 32 * 65; e += kGgWaves * 64) colsum[e] = 0.f;
  __syncthreads();
  float acc[32];
#pragma unroll
  for (int b = 0; b < 32; ++b) acc[b] = 0.f;
#pragma unroll 1
  for (int rb = wv; rb * 32 < B; rb += kGgWaves) {
    const int nr = min(32, B - rb * 32);
    uint32_t xn[32];  // next block's words, in flight during this block's transpose + lookups
    const int rbn = rb + kGgWaves;
    if (rbn * 32 < B) gw_load32(bits, words, r0 + rbn * 32, min(32, B - rbn * 32), wd, xn);
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = i < nr ? (x[i] & lmask) : 0u;
    transpose32(x);  // x[b] = column 32 * word + b over the block's 32 rows
    const float* Gb = G + rb * 8;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < 8; ++n) s += Gb[((x[b] >> (4 * n)) & 15u) * gp + n];  // rows past B: bits 0
      acc[b] += s;
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = xn[k];
  }
  for (int w = 0; w < kGgWaves; ++w) {  // waves add in a fixed order: deterministic sums
    if (wave == w) {
#pragma unroll
      for (int b = 0; b < 32; ++b) colsum[b * 65 + lane] += acc[b];
    }
    __syncthreads();
  }
  const float l1s = P.l1_lambda / static_cast<float>(cols);
  double aw = 0.0;
  for (int e = tid; e < 32 * kGwWords; e += kGgWaves * 64) {
    const int64_t c = w0 * 32 + e;
    if (c < cols) {
      const float gsum = colsum[(e & 31) * 65 + (e >> 5)];
      float w = wg[c], m = mg[c], v = vg[c];
      aw += fabs(static_cast<double>(w));
      const float sgn = w > 0.f ? 1.f : (w < 0.f ? -1.f : 0.f);
      float gr = fmaf(l1s, sgn, gsum);
      gr = fmaf(P.weight_decay, w, gr);
      m = fmaf(1.f - P.beta1, gr - m, m);
      v = fmaf(1.f - P.beta2, gr * gr, v * P.beta2);
      const float denom = sqrtf(v) / sc.bc2_sqrt + P.eps;
      w = w - sc.step_size * (m / denom);
      wg[c] = w;
      mg[c] = m;
      vg[c] = v;
    }
  }
  const double A = block_sum_d(aw, red);
  if (tid == 0) aw_part[(f * steps + t) * gridDim.x + blockIdx.x] = A;
}

__global__ __launch_bounds__(64) void k_gw_loss(const double* __restrict__ tk_part, int n_tk,
                                                const double* __restrict__ aw_part, int n_aw,
                                                const WlmStep* __restrict__ stp, int64_t rows, int64_t cols,
                                                int batch, float l1, double* __restrict__ losses) {
  const int64_t t = blockIdx.x, steps = gridDim.x, f = blockIdx.y;
  const int lane = threadIdx.x;  // 64 lanes: lane-strided partial sums, then a fixed butterfly
  const int64_t k = f * steps + t;
  double Tk = 0.0, Sa = 0.0;
  for (int i = lane; i < n_tk; i += 64) Tk += tk_part[k * n_tk + i];
  for (int i = lane; i < n_aw; i += 64) Sa += aw_part[k * n_aw + i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Tk += __shfl_xor(Tk, o);
    Sa += __shfl_xor(Sa, o);
  }
  if (lane != 0) return;
  const WlmStep sc = stp[k];
  const int64_t r0 = t * batch;
  const int B = static_cast<int>((rows - r0) < batch ? (rows - r0) : batch);
  const float reg = l1 * static_cast<float>(Sa / cols);
  losses[k] = Tk / (static_cast<double>(B) * sc.ksum) + sc.vy / (static_cast<double>(B) * B) +
              static_cast<double>(reg);
}


// ------------------------------------------------------------ surrogate, fused many-column fit
// The three launches per Adam step above read the step's mask bits twice from HBM (p, then the
// gradient) and stream w / m / v (24 B per column) through HBM every step.  k_gw_fused is ONE
// persistent launch per fit: nwg co-resident 512-thread workgroups (one per CU, LDS-bound), each
// owning `ch` chunks of 64 mask words (2048 columns).  Per step:
//   phase 1  the step's bits of the own chunks are in registers (x[4][32]: a wave holds four
//            32-row blocks of one chunk, lane = word; 8 waves at up to 256 VGPRs); p partials by
//            the nibble tables of w (as k_gw_p), chunk partials added in chunk order, published
//            as tagged 8-B granules {step + 1, p} -> xp[row][wg]
//   reduce   row j belongs to workgroup j mod nwg: one wave polls its nwg granules, sums them
//            (lane-strided, then a fixed butterfly), g_j = k_j cg (p_j - ybar), p_hist, the loss
//            term; publishes {step + 1, g_j} -> xg[j]
//   phase 3  every workgroup polls the batch's g, builds 4-row G tables, and the SAME bit
//            registers (transposed in place) give the column sums (as k_gw_grad); the waves of a
//            chunk add their sums in a fixed tree through LDS; Adam on w / m / v held in LDS for
//            the whole fit; the next step's bits are loaded into the freed registers right after
//            the lookups, in flight during the tree, Adam and the w-table build
// so a step reads its bits once and w / m / v never leave the CU until the end.  Granule slots
// are cleared by k_wlm_stats before the launch (tags t + 1 never match a cleared slot); data
// flow makes one slot per row enough (a row's step-(t+1) granule is written only after every
// workgroup read the step-t g values, i.e. after every reducer finished step t).  Polls are
// bounded: a workgroup that never arrives sets the error word, every workgroup leaves, and the
// caller's status word reports it (k_argmin_first).  All arithmetic is deterministic.
constexpr int kGfMaxCh = 2;        // chunks per workgroup (LDS: w tables + w / m / v per chunk)
constexpr int kGfWaves = 8;        // waves per workgroup
constexpr int kGfTpw = 4;          // resident 32-row blocks per wave
constexpr int kGfThreads = kGfWaves * 64;
constexpr int kGfLook1 = 8;        // phase 1: rows whose 8 lookups issue together
constexpr int kGfLook3 = 4;        // phase 3: columns whose 8 lookups issue together (acc[32] live)
constexpr int kGfColPitch = 65;    // column-sum image [b][j] pitch: conflict-free both ways
constexpr int kGfSlot = 32 * kGfColPitch;  // one wave's column-sum slot (floats)
constexpr int kGfMaxWg = 512;      // workgroups per fit (a reducer lane polls nwg / 64 granules)

struct GfArgs {
  const uint32_t* bits;
  const double* kern;
  const WlmStep* stp;
  float *wg, *mg, *vg, *p_hist;
  double *tk_part, *aw_part;  // [steps][nwg]
  uint64_t* xp;               // [batch][nwg] p granules, then [batch] g granules
  uint32_t* err;
  xpg_wlm_params P;
  int rows, cols, words, steps, batch, ch, nrbp, nwg, fault_wg;
  uint32_t spin_limit;
#ifdef XPG_GF_STAMPS
  int dbg;  // diagnostics build: 1 = no next-step bit loads (compute alone), 2 = phase-1 / 3
            // lookups without LDS (the address as the value), 4 = lookups at a fixed address
#endif
};

// LDS image of k_gw_fused (floats): [R0: w tables | tree slots][cs][w][m][v][pp][gb][G] + doubles.
// nrbp = row blocks rounded up to kGfTpw; a chunk has nrbp / kGfTpw waves.
struct GfLds {
  int r0, w, m, v, pp, gb, G, total;  // float offsets; total in floats (doubles follow)
};
__host__ __device__ inline GfLds gf_lds(int ch, int nrbp) {
  GfLds L;
  const int nwc = nrbp / kGfTpw, r0 = ch * (nwc * kGfSlot > 8 * 16 * 64 ? nwc * kGfSlot : 8 * 16 * 64);
  int o = 0;
  L.r0 = o;  o += (r0 + 15) & ~15;  // the w tables | the waves' column-sum slots
  L.w = o;   o += ch * 2048;
  L.m = o;   o += ch * 2048;
  L.v = o;   o += ch * 2048;
  L.pp = o;  o += ch * nrbp * 32;
  L.gb = o;  o += nrbp * 32;
  L.G = o;   o += 16 * nrbp * 8;
  L.total = (o + 1) & ~1;
  return L;
}

// x >> sh for sh >= 0, x << -sh otherwise (sh a compile-time constant after unrolling)
__device__ __forceinline__ uint32_t shr_i(uint32_t x, int sh) { return sh >= 0 ? x >> sh : x << -sh; }
// (x & m) | b in one v_and_or_b32 (the compiler turns a disjoint or into an add and then adds
// the base separately)
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t b) {
  uint32_t r;
  asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(m), "v"(b));
  return r;
}
// LDS float at byte address a + imm (imm folded into the instruction's offset)
__device__ __forceinline__ float lds_f32(uint32_t a, int imm) {
  typedef __attribute__((address_space(3))) const float lf32;
  return *reinterpret_cast<lf32*>(static_cast<uintptr_t>(a + imm));
}

__device__ __forceinline__ float gf_poll(const uint64_t* p, uint32_t tag, uint32_t spin_limit, uint32_t* err,
                                         int* abort_s) {
  uint64_t v = ld64_sc1(p);
  uint32_t n = 0;
  while (static_cast<uint32_t>(v >> 32) != tag) {
    __builtin_amdgcn_s_sleep(1);
    v = ld64_sc1(p);
    ++n;
    if (n > spin_limit || ((n & 63u) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *abort_s = 1;
      return 0.f;
    }
  }
  return __uint_as_float(static_cast<uint32_t>(v));
}

#ifdef XPG_GF_STAMPS  // diagnostics build (tools/gf_probe): per-phase s_memtime cycles of thread 0
__device__ uint64_t g_gf_stamps[1024 * 8];
#define GF_STAMP(k)                                  \
  if (tid == 0) {                                    \
    __builtin_amdgcn_sched_barrier(0);               \
    const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
    gst[k] += now_ - glast;                          \
    glast = now_;                                    \
    __builtin_amdgcn_sched_barrier(0);               \
  }
#ifdef XPG_GF_ABL  // lookup ablations (dbg 2 / 4): a runtime select per lookup, slower as such
#define GF_LOOK(addr, imm, base)                                                             \
  ((a.dbg & 2) ? __uint_as_float(addr) : (a.dbg & 4) ? lds_f32((base) | (addr & 0u), imm) : lds_f32(addr, imm))
#else
#define GF_LOOK(addr, imm, base) lds_f32(addr, imm)
#endif
#else
#define GF_STAMP(k) {}
#define GF_LOOK(addr, imm, base) lds_f32(addr, imm)
#endif

__global__ __launch_bounds__(kGfThreads) void k_gw_fused(GfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];
#ifdef XPG_GF_STAMPS
  uint64_t gst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, glast = __builtin_amdgcn_s_memtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform roles and row blocks
  const int wg = blockIdx.x, CH = a.ch, nwc = a.nrbp / kGfTpw;
  const GfLds L = gf_lds(CH, a.nrbp);
  double* red = reinterpret_cast<double*>(gsm + L.total);  // [kGfWaves] aw, [kGfWaves] tk
  // abort flag after the doubles: no static LDS, so the image (and the w tables) start at LDS
  // address 0 and a table address is an and-or of the shifted nibble with the lane's base
  int& abort_s = *reinterpret_cast<int*>(red + 2 * kGfWaves);
  if (tid == 0) abort_s = 0;
  const int n_chunks = (a.words + kGwWords - 1) / kGwWords;
  const int chunk0 = wg * CH;
  const int nch = min(CH, n_chunks - chunk0);  // own chunks (>= 1)
  // this wave's role in phases 1 / 3: chunk h, row blocks kGfTpw * k ...
  const int h = wave / nwc, k = wave - h * nwc;
  const bool wvalid = h < nch;
  const int w0 = (chunk0 + (wvalid ? h : 0)) * kGwWords;
  const int nw = min(kGwWords, a.words - w0);
  const uint32_t lmask = lane < nw ? ~0u : 0u;
  const uint32_t wd = static_cast<uint32_t>(w0 + (lane < nw ? lane : 0));
  const int64_t c_lo = (int64_t)chunk0 * 2048;  // first own column
  float* Wt = gsm + L.r0;
  float* Wv = gsm + L.w;
  float* Mv = gsm + L.m;
  float* Vv = gsm + L.v;
  float* pp = gsm + L.pp;
  float* gb = gsm + L.gb;
  float* G = gsm + L.G;
  const int RB = a.nrbp * 32;
  const uint32_t pitch = static_cast<uint32_t>(a.words) * 4u;

  uint32_t x[kGfTpw][32];
  // the bits of step t's row block kGfTpw * k + u: buffer loads (descriptor at the block's first
  // row in SGPRs, lane word in voffset, row in soffset); rows past the batch re-read its last row
  // (masked at use)
  // rows i0 .. i0 + n - 1 of step t's block u (u, i0, n compile-time after unrolling)
  // No branch: a block past the batch or past the last step (or a wave without a chunk) gets a
  // descriptor of zero records, whose loads return 0 without touching memory (a conditional
  // load keeps the registers' old values alive beside the new ones)
  auto load_rows = [&](int64_t t, int u, int i0, int n) {
    const int64_t r0 = t * a.batch;
    const int B = t < a.steps ? static_cast<int>(min((int64_t)a.batch, (int64_t)a.rows - r0)) : 0;
    const int rb = kGfTpw * k + u;
    const int nr = wvalid ? max(0, min(32, B - rb * 32)) : 0, last = max(nr - 1, 0);
#ifdef XPG_GF_STAMPS
    const int64_t roff = (a.dbg & 8) ? 0 : (r0 + rb * 32) * (int64_t)a.words;  // dbg 8: always block 0
#else
    const int64_t roff = (r0 + rb * 32) * (int64_t)a.words;
#endif
    // the descriptor's inputs made provably wave-uniform (readfirstlane): otherwise the compiler
    // wraps every buffer load in a waterfall loop (cdna_hip_programming.md T20), which cost the
    // step ~16k cycles of its 128 loads per wave
    const uint64_t base = reinterpret_cast<uint64_t>(a.bits + (nr > 0 ? roff : 0));
    const uint32_t blo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base));
    const uint32_t bhi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane(static_cast<int>(pitch * static_cast<uint32_t>(nr)));
    const int lastu = __builtin_amdgcn_readfirstlane(last);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint32_t*>((static_cast<uint64_t>(bhi) << 32) | blo), 0, bytes, 0x00020000);
#pragma unroll
    for (int i = i0; i < i0 + n; ++i)
      x[u][i] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, wd * 4u, static_cast<uint32_t>(min(i, lastu)) * pitch, 0);
  };
#pragma unroll
  for (int u = 0; u < kGfTpw; ++u) load_rows(0, u, 0, 32);  // in flight during the set-up

  // w / m / v of the own columns into LDS (0 past cols), then the w tables
  for (int e = tid; e < CH * 2048; e += kGfThreads) {
    const int64_t c = c_lo + e;
    const bool ok = (e >> 11) < nch && c < a.cols;
    Wv[e] = ok ? a.wg[c] : 0.f;
    Mv[e] = ok ? a.mg[c] : 0.f;
    Vv[e] = ok ? a.vg[c] : 0.f;
  }
  // thread = (chunk hh, nibble q, word j); 512 threads = one chunk per pass, unrolled so both
  // chunks' w reads are in flight together
  static_assert(kGfThreads == 8 * 64, "one chunk's tables per pass");
  auto build_w_tables = [&]() {
    const int q = tid >> 6, j = tid & 63;
    float aq[kGfMaxCh][4];
#pragma unroll
    for (int hh = 0; hh < kGfMaxCh; ++hh)
      if (hh < CH) {
        const float* wq = Wv + hh * 2048 + 32 * j + 4 * q;
#pragma unroll
        for (int b = 0; b < 4; ++b) aq[hh][b] = wq[b];
      }
#pragma unroll
    for (int hh = 0; hh < kGfMaxCh; ++hh)
      if (hh < CH) {
        const float a0 = aq[hh][0], a1 = aq[hh][1], a2 = aq[hh][2], a3 = aq[hh][3];
        float* Tq = Wt + ((hh * 8 + q) * 16) * 64 + j;
#pragma unroll
        for (int v = 0; v < 16; ++v)
          Tq[v * 64] = ((v & 1) ? a0 : 0.f) + ((v & 2) ? a1 : 0.f) + ((v & 4) ? a2 : 0.f) + ((v & 8) ? a3 : 0.f);
      }
  };
  lds_barrier();
  build_w_tables();
  lds_barrier();

  const float l1s = a.P.l1_lambda / static_cast<float>(a.cols);
  bool aborted = false;
  // Rows split in two halves by row block (rb & 3 < 2: the waves' blocks u = 0, 1; else u = 2, 3)
  // so the exchanges overlap compute: half 0's partials travel while half 1's phase 1 runs, half
  // 1's g values while half 0's phase 3 runs
  auto half_of_row = [](int r) { return ((r >> 5) & 3) >> 1; };
  for (int t = 0; t < a.steps; ++t) {
    const WlmStep sc = a.stp[t];
    const int64_t r0 = (int64_t)t * a.batch;
    const int B = static_cast<int>(min((int64_t)a.batch, (int64_t)a.rows - r0));
    const uint32_t tag = static_cast<uint32_t>(t + 1);
    GF_STAMP(7)
    double tk = 0.0;
#pragma unroll
    for (int H = 0; H < 2; ++H) {
      // ---- phase 1 (this half's blocks): chunk partials of p over the own words, 8 rows at a time
      if (wvalid) {
        // table entry (q, v) of this lane's word: byte (h * 8 + q) * 4096 + v * 256 + lane * 4 of
        // the table image (at LDS offset 0), so the nibble lands in bits 8-11 with one shift and
        // one and-or
        const uint32_t tb = static_cast<uint32_t>(h * 8 * 16 * 64 + lane) * 4u;
#pragma unroll
        for (int u = 2 * H; u < 2 * H + 2; ++u) {
          const int rb = kGfTpw * k + u;
          const int nr = min(32, B - rb * 32);
          if (nr > 0) {
            // rows past the batch and words past the chunk read as 0 (here and in phase 3)
#pragma unroll
            for (int i = 0; i < 32; ++i) x[u][i] = i < nr ? (x[u][i] & lmask) : 0u;
#pragma unroll
            for (int i0 = 0; i0 < 32; i0 += 8) {
              // the lookups of kGfLook1 rows issued before their adds (a chained add per lookup
              // kept one LDS read in flight)
              float c[8];
#pragma unroll
              for (int i1 = 0; i1 < 8; i1 += kGfLook1) {
                float v[kGfLook1][8];
#pragma unroll
                for (int i = 0; i < kGfLook1; ++i)
#pragma unroll
                  for (int q = 0; q < 8; ++q)
                    v[i][q] = GF_LOOK(and_or(shr_i(x[u][i0 + i1 + i], 4 * q - 8), 0xf00u, tb), q * 4096, tb);
#pragma unroll
                for (int i = 0; i < kGfLook1; i += 2) {  // two rows per packed add
                  f32x2 s2 = {v[i][0], v[i + 1][0]};
#pragma unroll
                  for (int q = 1; q < 8; ++q) s2 += f32x2{v[i][q], v[i + 1][q]};
                  c[i1 + i] = s2.x;
                  c[i1 + i + 1] = s2.y;
                }
              }
              const float tot = wave_transpose_reduce8_pl(c, lane);  // row i0 + (lane >> 3)
              const int i = i0 + (lane >> 3);
              if (!(lane & 7) && i < nr) pp[h * RB + rb * 32 + i] = tot;
            }
          }
        }
      }
      lds_barrier();
      // ---- publish the workgroup's partial of every row of the half (chunks added in order)
      if (!(a.fault_wg == wg && t == 0)) {
        for (int r = tid; r < B; r += kGfThreads) {
          if (half_of_row(r) != H) continue;
          float v = 0.f;
          for (int hh = 0; hh < nch; ++hh) v += pp[hh * RB + r];
          st64_sc1(a.xp + (int64_t)r * a.nwg + wg, (static_cast<uint64_t>(tag) << 32) | __float_as_uint(v));
        }
      }
    }
    GF_STAMP(0)
#pragma unroll
    for (int H = 0; H < 2; ++H) {
      // ---- reduce the half's rows this workgroup owns: p_j, g_j, the loss term
      for (int j = wg + wave * a.nwg; j < B; j += kGfWaves * a.nwg) {
        if (half_of_row(j) != H) continue;  // wave-uniform
        const uint64_t* src = a.xp + (int64_t)j * a.nwg;
        // the lane's granules c = lane + 64 i: all loads in flight first, then any spins
        uint64_t gr[kGfMaxWg / 64];
#pragma unroll
        for (int i = 0; i < kGfMaxWg / 64; ++i)
          gr[i] = lane + 64 * i < a.nwg ? ld64_sc1(src + lane + 64 * i) : (static_cast<uint64_t>(tag) << 32);
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < kGfMaxWg / 64; ++i)
          part += static_cast<uint32_t>(gr[i] >> 32) == tag
                      ? __uint_as_float(static_cast<uint32_t>(gr[i]))
                      : gf_poll(src + lane + 64 * i, tag, a.spin_limit, a.err, &abort_s);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        const float p = __shfl(part, 0);
        if (lane == 0) {
          const double kj = a.kern[r0 + j];
          const double d = static_cast<double>(p) - sc.ybar;
          const float g = static_cast<float>(kj * sc.cg * d);
          a.p_hist[r0 + j] = p;
          tk += kj * d * d;
          st64_sc1(a.xp + (int64_t)a.batch * a.nwg + j, (static_cast<uint64_t>(tag) << 32) | __float_as_uint(g));
        }
      }
    }
    if (lane == 0) red[kGfWaves + wave] = tk;
    GF_STAMP(1)
    // ---- phase 3 per half: the half's g (rows past B: 0), its G tables, then column sums from
    // the same registers; each block's registers take the next step's bits once its lookups are
    // done
    float acc[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) acc[b] = 0.f;
#pragma unroll
    for (int H = 0; H < 2; ++H) {
      for (int r = tid; r < RB; r += kGfThreads)
        if (half_of_row(r) == H)
          gb[r] = r < B ? gf_poll(a.xp + (int64_t)a.batch * a.nwg + r, tag, a.spin_limit, a.err, &abort_s) : 0.f;
      lds_barrier();
      if (H == 0) { GF_STAMP(2) }
      if (abort_s) {
        aborted = true;
        break;
      }
      if (H == 1 && tid == 0) {
        double s = 0.0;
        for (int i = 0; i < kGfWaves; ++i) s += red[kGfWaves + i];
        a.tk_part[(int64_t)t * a.nwg + wg] = s;
      }
      for (int e = tid; e < 16 * (a.nrbp * 8); e += kGfThreads) {  // G[group * 16 + v]: a lookup's
        const int v = e & 15, grp = e >> 4;                          // 16 entries on 16 banks
        if (half_of_row(grp * 4) != H) continue;
        const float* gg = gb + 4 * grp;
        G[e] = ((v & 1) ? gg[0] : 0.f) + ((v & 2) ? gg[1] : 0.f) + ((v & 4) ? gg[2] : 0.f) + ((v & 8) ? gg[3] : 0.f);
      }
      lds_barrier();
      if (H == 0) { GF_STAMP(3) }
#pragma unroll
      for (int u = 2 * H; u < 2 * H + 2; ++u) {
        const int rb = kGfTpw * k + u;
        const int nr = min(32, B - rb * 32);
        if (wvalid && nr > 0) {
          transpose32_perm(x[u]);  // x[u][b] = column 32 * word + b over the block's rows (masked in phase 1)
          // G[group][v], group = 4 rows: the block's groups at byte gbase + n * 64 (gbase: a
          // multiple of 64, so the nibble's 4-B slot is an and-or)
          const uint32_t gbase = static_cast<uint32_t>(L.G + rb * 8 * 16) * 4u;
#pragma unroll
          for (int b0 = 0; b0 < 32; b0 += kGfLook3) {
            float v[kGfLook3][8];  // the lookups of kGfLook3 columns in flight, then the adds
#pragma unroll
            for (int b = 0; b < kGfLook3; ++b)
#pragma unroll
              for (int n = 0; n < 8; ++n)
                v[b][n] = GF_LOOK(and_or(shr_i(x[u][b0 + b], 4 * n - 2), 0x3cu, gbase), n * 64, gbase);
#pragma unroll
            for (int b = 0; b < kGfLook3; b += 2) {  // two columns per packed add
              f32x2 s2 = {v[b][0], v[b + 1][0]};
#pragma unroll
              for (int n = 1; n < 8; ++n) s2 += f32x2{v[b][n], v[b + 1][n]};
              f32x2 a2 = {acc[b0 + b], acc[b0 + b + 1]};
              a2 += s2;
              acc[b0 + b] = a2.x;
              acc[b0 + b + 1] = a2.y;
            }
            // the next step's rows into the registers of the columns consumed so far: half the
            // block half-way, the rest at the end (a wave stalls issuing its 64th vector memory
            // op in flight; 32 at a time per block kept it waiting on the fetch)
            if (b0 == 16 - kGfLook3) load_rows(t + 1, u, 0, 16);
          }
          load_rows(t + 1, u, 16, 16);
        } else {
          load_rows(t + 1, u, 0, 32);
        }
      }
    }
    if (aborted) break;
    GF_STAMP(4)
    // every wave's column sums to its own slot [b][j] (over the w tables, dead until rebuilt);
    // the Adam threads add a column's nwc slots in wave order
    if (wvalid) {
      float* sl = Wt + (h * nwc + k) * kGfSlot + lane;
#pragma unroll
      for (int b = 0; b < 32; ++b) sl[b * kGfColPitch] = acc[b];
    }
    lds_barrier();
    GF_STAMP(5)
    // ---- Adam on the own columns (w before the step counts in the loss's |w| sum).  A runtime
    // loop over the thread's columns (with the next step's bits live, 128 VGPRs, a fully unrolled
    // form had no registers to keep its reads in flight and spilled); the nwc slot reads and
    // w / m / v are issued together for the common slot counts (a runtime slot loop waited for
    // each read), then added in wave order
    // two columns (e, e + 512: the same chunk) per iteration, their reads issued together and
    // their Adam chains interleaved (one column's sqrt / division sequence is serial); computed
    // branch-free, stored (and counted in the |w| sum) for columns below cols
    auto slot_sum2 = [&](const float* sl0, const float* sl1, float& g0, float& g1, auto nwc_c) {
      constexpr int NW = decltype(nwc_c)::value;
      float s0[NW], s1[NW];
#pragma unroll
      for (int kk = 0; kk < NW; ++kk) {
        s0[kk] = sl0[kk * kGfSlot];
        s1[kk] = sl1[kk * kGfSlot];
      }
      g0 = s0[0];
      g1 = s1[0];
#pragma unroll
      for (int kk = 1; kk < NW; ++kk) {
        g0 += s0[kk];
        g1 += s1[kk];
      }
    };
    static_assert((2048 / kGfThreads) % 2 == 0, "column pairs within a chunk");
    double aw = 0.0;
    for (int e0 = tid; e0 < CH * 2048; e0 += 2 * kGfThreads) {
      const int hh = e0 >> 11;
      if (hh >= nch) break;  // wave-uniform; chunks ascend with e0
      float w[2], m[2], v[2], gs[2];
      const float* sl[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int e = e0 + j * kGfThreads, el = e & 2047;
        sl[j] = Wt + hh * nwc * kGfSlot + (el & 31) * kGfColPitch + (el >> 5);
        w[j] = Wv[e];
        m[j] = Mv[e];
        v[j] = Vv[e];
      }
      if (nwc == 4) slot_sum2(sl[0], sl[1], gs[0], gs[1], std::integral_constant<int, 4>{});
      else if (nwc == 2) slot_sum2(sl[0], sl[1], gs[0], gs[1], std::integral_constant<int, 2>{});
      else if (nwc == 8) slot_sum2(sl[0], sl[1], gs[0], gs[1], std::integral_constant<int, 8>{});
      else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          gs[j] = sl[j][0];
          for (int kk = 1; kk < nwc; ++kk) gs[j] += sl[j][kk * kGfSlot];
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = c_lo + e0 + j * kGfThreads < a.cols;
        aw += ok ? fabs(static_cast<double>(w[j])) : 0.0;
        const float sgn = w[j] > 0.f ? 1.f : (w[j] < 0.f ? -1.f : 0.f);
        float gr = fmaf(l1s, sgn, gs[j]);
        gr = fmaf(a.P.weight_decay, w[j], gr);
        m[j] = fmaf(1.f - a.P.beta1, gr - m[j], m[j]);
        v[j] = fmaf(1.f - a.P.beta2, gr * gr, v[j] * a.P.beta2);
        const float denom = sqrtf(v[j]) / sc.bc2_sqrt + a.P.eps;
        w[j] = w[j] - sc.step_size * (m[j] / denom);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int e = e0 + j * kGfThreads;
        if (c_lo + e < a.cols) {
          Wv[e] = w[j];
          Mv[e] = m[j];
          Vv[e] = v[j];
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) aw += __shfl_xor(aw, o);
    if (lane == 0) red[wave] = aw;
    lds_barrier();
    if (tid == 0) {
      double s = 0.0;
      for (int i = 0; i < kGfWaves; ++i) s += red[i];
      a.aw_part[(int64_t)t * a.nwg + wg] = s;
    }
    GF_STAMP(6)
    build_w_tables();
    lds_barrier();
  }
#ifdef XPG_GF_STAMPS
  if (tid == 0)
    for (int i = 0; i < 8; ++i) g_gf_stamps[wg * 8 + i] = gst[i];
#endif
  if (aborted) return;
  for (int e = tid; e < CH * 2048; e += kGfThreads) {
    const int64_t c = c_lo + e;
    if ((e >> 11) < nch && c < a.cols) {
      a.wg[c] = Wv[e];
      a.mg[c] = Mv[e];
      a.vg[c] = Vv[e];
    }
  }
}

// Also hands the fit's status word to the caller: the multi-workgroup exchange's error word, or 0.
__global__ void k_argmin_first(const double* __restrict__ v, int64_t n, int32_t* __restrict__ out,
                               const uint32_t* __restrict__ errw, int32_t* __restrict__ status) {
  if (threadIdx.x != 0) return;
  if (status && errw && blockIdx.x == 0 && *errw) *status = *status | static_cast<int32_t>(*errw);
  v += blockIdx.x * n;
  out += blockIdx.x;
  double best = INFINITY;
  int32_t bi = 0;
  for (int64_t i = 0; i < n; ++i)
    if (v[i] < best) {
      best = v[i];
      bi = static_cast<int32_t>(i);
    }
  *out = bi;
}

// ------------------------------------------------------------------------------------ helpers
size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// node-type-gated terms (multi-node-type HeteroConv) run on the multi-kernel path only
bool plan_multi_type(const xpg_forward_plan* p) {
  for (int l = 0; l < p->n_layers; ++l)
    if (p->layers[l].tgt_type) return true;
  return false;
}

// k_degree's kept prefix of F_0 (see k_degree): F_1 for plans without GCN terms or edge masks
int deg_pitch(const xpg_forward_plan* p) {
  if (p->edge_masks) return p->n0;
  for (int l = 0; l < p->n_layers; ++l)
    for (int k = 0; k < p->layers[l].n_terms; ++k)
      if (p->layers[l].terms[k].kind == XPG_TERM_GCN) return p->n0;
  return std::max(1, std::min(p->n0, p->layers[0].n_tgt));
}

struct WsLayout {
  size_t kin = 0, agg = 0, head0 = 0, head1 = 0, ctl = 0, total = 0;
  size_t h[64];
};

int layout_ws(const xpg_forward_plan* p, int64_t rows, WsLayout* L) {
  XPG_REQ(p && p->n_layers >= 1 && p->n_layers <= 64, "plan: 1..64 conv layers required");
  size_t off = 0;
  L->kin = off;
  off += align_up(sizeof(float) * (size_t)rows * p->n_rel * deg_pitch(p));
  size_t agg_max = 0;
  for (int l = 0; l < p->n_layers; ++l) {
    const xpg_layer_desc& ly = p->layers[l];
    L->h[l] = off;
    off += align_up(sizeof(float) * (size_t)rows * ly.n_tgt * ly.f_out_pad);
    if (l > 0) {
      size_t a = sizeof(float) * (size_t)rows * ly.n_tgt * ly.n_terms * ly.f_in_pad;
      agg_max = a > agg_max ? a : agg_max;
    }
  }
  L->agg = off;
  off += align_up(agg_max);
  size_t hmax = 0;
  const int64_t n_last = p->layers[p->n_layers - 1].n_tgt;
  for (int i = 0; i < p->n_head; ++i) {
    size_t hb = sizeof(float) * (size_t)rows * n_last * p->head[i].n_pad;
    hmax = hb > hmax ? hb : hmax;
  }
  L->head0 = off;
  off += align_up(hmax);
  L->head1 = off;
  off += align_up(hmax);
  L->ctl = off;  // the rows forward's block-scheduling counters (zeroed before each launch)
  off += align_up(sizeof(int) * 32);
  L->total = off;
  return XPG_OK;
}

// OutColumn: the output column of the network's last dense layer computed in this launch's
// epilogue (k_dense HEAD): y[m] = act(sum_c v[m][c] w[c] + b[0])
struct OutColumn {
  const float* w = nullptr;  // the output column's weight row (the layer's k_pad entries)
  const float* b = nullptr;  // its bias (one float)
  int act = 0;
  float* y = nullptr;
};

int launch_dense(const float* A, int64_t M, int64_t lda, const float* W, int64_t ldw, int64_t k_pad,
                 const float* bias, int64_t n_real, int64_t n_pad, int act, float* C, int64_t ldc,
                 hipStream_t st, const int32_t* row_type = nullptr, int64_t type_mod = 1, int bias_ld = 0,
                 const OutColumn* head = nullptr) {
  XPG_REQ(k_pad % 8 == 0 && n_pad % 32 == 0 && n_pad >= 32 && n_pad <= 256,
          "xpg_dense: k_pad % 8, n_pad in {32..256} step 32 required");
  XPG_REQ(lda % 4 == 0 && ldw % 4 == 0, "xpg_dense: lda/ldw must be multiples of 4");
  if (M <= 0) return XPG_OK;
  // 4+ column tiles: split them over column groups of one or two tiles per wave (a 128-wide layer
  // on one wave per 32 rows left a workgroup of 4 waves per CU, latency-bound)
  const int tiles = static_cast<int>(n_pad / 32);
  const int groups = tiles >= 4 && tiles % 4 == 0 ? 4 : 1;
  const int64_t waves = cdiv(M, 32) * groups;
  dim3 grid(static_cast<unsigned>(cdiv(waves, 4))), block(256);
  const int kp = static_cast<int>(k_pad), nr = static_cast<int>(n_real);
  switch (tiles / groups) {
#define XPG_DENSE_CASE(NT)                                                                                      \
    case NT:                                                                                                    \
      if (head)                                                                                                 \
        hipLaunchKernelGGL((k_dense<NT, true>), grid, block, 0, st, A, M, lda, W, ldw, kp, bias, nr, act, C,   \
                           ldc, row_type, type_mod, bias_ld, groups, head->w, head->b, head->act, head->y);     \
      else                                                                                                      \
        hipLaunchKernelGGL((k_dense<NT, false>), grid, block, 0, st, A, M, lda, W, ldw, kp, bias, nr, act, C,  \
                           ldc, row_type, type_mod, bias_ld, groups, nullptr, nullptr, 0, nullptr);             \
      break;
    XPG_DENSE_CASE(1) XPG_DENSE_CASE(2) XPG_DENSE_CASE(3) XPG_DENSE_CASE(4)
    XPG_DENSE_CASE(5) XPG_DENSE_CASE(6) XPG_DENSE_CASE(7) XPG_DENSE_CASE(8)
#undef XPG_DENSE_CASE
    default: return fail(XPG_EINVAL, "xpg_dense: unsupported n_pad");
  }
  XPG_LAUNCHED();
  return XPG_OK;
}

template <bool L1>
int launch_agg(const AggArgs& a, hipStream_t st) {
  XPG_REQ(a.width % 32 == 0 && a.width > 0, "agg: row width must be a positive multiple of 32");
  // layer 1, widths 32 / 64 / 128 / 256, no edge masks: lanes = mask rows (XPG_AGG_GENERIC=1, a diagnostics
  // switch: the generic k_agg, which the parity suite compares bitwise)
  int generic = 0;
  if (const int rc = diag_env("XPG_AGG_GENERIC", &generic)) return rc;
  if (L1 && !a.agg_eid && (a.width == 32 || a.width == 64 || a.width == 128 || a.width == 256) && !generic) {
    const int slice = a.width == 32 ? 32 : 64;  // features per wave
    const int64_t waves = cdiv(a.rows, 64) * a.n_tgt * (a.width / slice);
    if (waves == 0) return XPG_OK;
    const dim3 grid(static_cast<unsigned>(cdiv(waves, 4))), block(256);
    AggArgs b = a;
    if (const int rc = diag_env("XPG_L1_DBG", &b.rows_blk)) return rc;
    bool one = a.kind[0] != XPG_TERM_ROOT;
    for (int k = 1; k < a.n_terms; ++k) one = one && a.kind[k] == XPG_TERM_ROOT;
    if (slice == 64 && one) hipLaunchKernelGGL((k_agg_l1_rows<64, true>), grid, block, 0, st, b);
    else if (slice == 64) hipLaunchKernelGGL((k_agg_l1_rows<64, false>), grid, block, 0, st, b);
    else if (one) hipLaunchKernelGGL((k_agg_l1_rows<32, true>), grid, block, 0, st, b);
    else hipLaunchKernelGGL((k_agg_l1_rows<32, false>), grid, block, 0, st, b);
    XPG_LAUNCHED();
    return XPG_OK;
  }
  const int f4 = a.width / 4;  // float4 chunks per row (>= 8)
  const int lps = f4 >= 64 ? 64 : f4;
  const int nv = f4 / lps;
  XPG_REQ(f4 % lps == 0 && (nv == 1 || nv == 2 || nv == 4), "agg: unsupported row width");
  const int64_t threads = a.rows * a.n_tgt * lps;
  if (threads == 0) return XPG_OK;
  dim3 grid(static_cast<unsigned>(cdiv(threads, 256))), block(256);
#define XPG_AGG(LPS, NV) \
  if (lps == LPS && nv == NV) { hipLaunchKernelGGL((k_agg<L1, LPS, NV>), grid, block, 0, st, a); XPG_LAUNCHED(); return XPG_OK; }
  XPG_AGG(8, 1) XPG_AGG(16, 1) XPG_AGG(32, 1) XPG_AGG(64, 1) XPG_AGG(64, 2) XPG_AGG(64, 4)
  // widths that are odd multiples of 32 below 256 (e.g. 96) map to lps = f4 (non power of 2)
  XPG_AGG(24, 1) XPG_AGG(40, 1) XPG_AGG(48, 1) XPG_AGG(56, 1)
#undef XPG_AGG
  return fail(XPG_EINVAL, "agg: unsupported row width " + std::to_string(a.width));
}

// XPG_FORWARD=rows|fused|unfused|wide forces one xpg_masked_forward path (tests, A/B); unset or
// empty: the plan picks it
bool forward_is(const char* v) {
  const char* env = getenv("XPG_FORWARD");
  return v ? env && std::strcmp(env, v) == 0 : env && *env;
}

// Fused single-launch forward when the plan fits (returns 1 when it does not apply).
int try_fused_forward(const xpg_forward_plan* p, const uint32_t* bits, int64_t rows, float* y, hipStream_t st) {
  // opt-in (XPG_FORWARD=fused): per-row latency chains make it slower than k_rows_forward
  if (!forward_is("fused")) return 1;
  if (p->n_layers > kFusedMaxLayers || p->n_head > kFusedMaxHead || plan_multi_type(p)) return 1;
  if (p->edge_masks || p->edge_dot) return 1;  // edge problems: multi-kernel path only
  FusedArgs a;
  std::memset(&a, 0, sizeof(a));
  a.rows = rows;
  a.bits = bits;
  a.y = y;
  a.words = words_of(p->cols);
  a.n0 = p->n0;
  a.n_rel = p->n_rel;
  a.n_layers = p->n_layers;
  a.n_head = p->n_head;
  a.out_col = p->out_col;
  a.n_last = p->layers[p->n_layers - 1].n_tgt;
  a.f0_node = p->f0_node;
  a.deg_ptr = p->deg_ptr;
  a.deg_src = p->deg_src;
  auto up4 = [](int64_t x) { return (x + 3) & ~int64_t(3); };
  int64_t shared = 0, h_max = 0, a_max = 0;
  for (int l = 0; l < p->n_layers; ++l) {
    const xpg_layer_desc& ly = p->layers[l];
    FusedLayer& L = a.L[l];
    if (ly.f_out_pad > 256 || ly.f_out_pad % 32 || ly.n_terms < 1 || ly.n_terms > XPG_MAX_TERMS) return 1;
    L.n_tgt = ly.n_tgt;
    L.n_terms = ly.n_terms;
    L.act = ly.act;
    L.f_in_pad = ly.f_in_pad;
    L.f_out = ly.f_out;
    L.f_out_pad = ly.f_out_pad;
    L.tgt_prev = ly.tgt_prev;
    L.tgt_f0 = ly.tgt_f0;
    L.agg_ptr = ly.agg_ptr;
    L.agg_src = ly.agg_src;
    L.agg_f0 = ly.agg_f0;
    L.self_mult = ly.self_mult;
    L.weight = ly.weight;
    L.bias = ly.bias;
    for (int k = 0; k < ly.n_terms; ++k) {
      L.kind[k] = ly.terms[k].kind;
      L.rel[k] = ly.terms[k].rel;
      L.table[k] = ly.terms[k].table;
    }
    h_max = std::max<int64_t>(h_max, (int64_t)ly.n_tgt * ly.f_out_pad);
    if (l == 0) {
      for (int k = 0; k < ly.n_terms; ++k) {
        if (!ly.terms[k].table) return 1;
        L.lds_tab[k] = static_cast<int>(shared);
        shared += up4((int64_t)p->n0 * ly.f_out_pad);
      }
    } else {
      const xpg_layer_desc& prev = p->layers[l - 1];
      if (ly.f_in_pad != prev.f_out_pad || !ly.weight) return 1;
      L.K = ly.n_terms * ly.f_in_pad;
      L.w_ld = L.K + 4;  // 16-B rows, bank-shifted by 4 words per output row
      L.lds_w = static_cast<int>(shared);
      shared += (int64_t)ly.f_out_pad * L.w_ld;
      const int tpp = 64 / (ly.f_in_pad / 4);
      a_max = std::max<int64_t>(a_max, (int64_t)tpp * L.K);
    }
  }
  int cur_w = p->layers[p->n_layers - 1].f_out_pad;
  for (int i = 0; i < p->n_head; ++i) {
    const xpg_head_desc& hd = p->head[i];
    if (hd.k_pad != cur_w || hd.k_pad % 4) return 1;
    a.H[i].k_pad = hd.k_pad;
    a.H[i].n_real = hd.n_real;
    a.H[i].n_pad = hd.n_pad;
    a.H[i].act = hd.act;
    a.H[i].weight = hd.weight;
    a.H[i].bias = hd.bias;
    h_max = std::max<int64_t>(h_max, (int64_t)a.n_last * hd.n_pad);
    cur_w = hd.n_pad;
  }
  if (p->out_col < 0 || p->out_col >= cur_w) return 1;
  a.shared_floats = static_cast<int>(shared);
  a.o_kin = static_cast<int>(up4(a.words));
  a.o_h0 = a.o_kin + static_cast<int>(up4((int64_t)p->n_rel * p->n0));
  a.o_h1 = a.o_h0 + static_cast<int>(up4(h_max));
  a.o_a = a.o_h1 + static_cast<int>(up4(h_max));
  a.wave_floats = a.o_a + static_cast<int>(up4(a_max));
  const int64_t lds_cap = 160 * 1024 / 4 - 64;
  int wpb = 0;
  for (int c : {8, 4, 2}) {
    if (shared + (int64_t)c * a.wave_floats <= lds_cap) {
      wpb = c;
      break;
    }
  }
  if (!wpb) return 1;
  const size_t lds = sizeof(float) * (size_t)(shared + (int64_t)wpb * a.wave_floats);
  const int64_t per_cu = std::max<int64_t>(1, (160 * 1024) / (int64_t)lds);
  const int64_t grid = std::min<int64_t>(cdiv(rows, wpb), 256 * per_cu);
#define XPG_FUSED(W)                                                                                     \
  if (wpb == W) {                                                                                        \
    XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_fused_forward<W>)));       \
    hipLaunchKernelGGL(k_fused_forward<W>, dim3(static_cast<unsigned>(grid)), dim3(W * 64), lds, st, a); \
    XPG_LAUNCHED();                                                                                      \
    return XPG_OK;                                                                                       \
  }
  XPG_FUSED(8) XPG_FUSED(4) XPG_FUSED(2)
#undef XPG_FUSED
  return 1;
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 1;
  }
  return cus;
}

// XCDs of the current device (hipDeviceAttributeNumberOfXccs: 8 on an MI355X in SPX mode, 1 per
// device in CPX); 1 when the attribute is unavailable (the XCD-aware schedules then treat the
// device as one XCD: correct, only without the per-XCD balance)
int device_xcds() {
  static int xcds = 0;
  if (!xcds) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) == hipSuccess &&
        n > 0 && n <= 8)
      xcds = n;
    else
      xcds = 1;
  }
  return xcds;
}

// Optional per-kernel timing (xpg_profile_enable / xpg_profile_read): a pair of hipEvents on the
// launch stream around each profiled launch, read back (and released) by xpg_profile_read.  Off
// by default; never enable it around a graph capture.
bool g_prof_on = false;
struct ProfRec {
  hipEvent_t a, b;
  int slot;
};
std::vector<ProfRec> g_prof;
void prof_begin(hipStream_t st, int slot) {
  if (!g_prof_on || g_prof.size() >= 65536) return;
  ProfRec r{nullptr, nullptr, slot};
  if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return;
  (void)hipEventRecord(r.a, st);
  g_prof.push_back(r);
}
void prof_end(hipStream_t st, int slot) {
  if (!g_prof_on || g_prof.empty() || g_prof.back().slot != slot) return;
  (void)hipEventRecord(g_prof.back().b, st);
}

// Wide (full-graph) forward: 2-layer plans with large frontiers (returns 1 when it does not apply).
struct WideWs {
  size_t mT, mT0, kin, h1, ct, total;
  size_t set;  // bytes of one per-pass buffer set {mT, mT0, kin, h1, ct}
  int nset;    // 2: passes alternate buffer sets (layer 1 of pass p+1 beside layer 2 of pass p)
  int nfi, a_ld, h_ld, o_h0, o_h1, o_e, kw;
  int o_hw[kFusedMaxHead];
  size_t lds;
  bool gcn;
};

bool wide_overlap();

int wide_layout(const xpg_forward_plan* p, int64_t rows, WideWs* W) {
  if (p->n_layers != 2 || p->n_head > kFusedMaxHead || p->n_head < 0 || plan_multi_type(p)) return 1;
  const xpg_layer_desc& l1 = p->layers[0];
  const xpg_layer_desc& l2 = p->layers[1];
  if (l1.n_terms < 1 || l1.n_terms > XPG_MAX_TERMS || l2.n_terms < 1 || l2.n_terms > XPG_MAX_TERMS) return 1;
  for (int k = 0; k < l1.n_terms; ++k)
    if (!l1.terms[k].table) return 1;
  if (!l2.weight || l2.f_in_pad != l1.f_out_pad) return 1;
  const int f1 = l1.f_out_pad;
  W->nfi = f1 / 16;
  if (f1 % 16) return 1;
  if (W->nfi != 2 && W->nfi != 4 && W->nfi != 8 && W->nfi != 12 && W->nfi != 16) return 1;
  const int K = l2.n_terms * l2.f_in_pad;
  if (K % 32 || l2.f_out_pad % 32 || l2.f_out_pad > 256) return 1;
  int hw = l2.f_out_pad, cur = l2.f_out_pad;
  for (int i = 0; i < p->n_head; ++i) {
    if (p->head[i].k_pad != cur || p->head[i].n_pad > 256) return 1;
    hw = std::max(hw, p->head[i].n_pad);
    cur = p->head[i].n_pad;
  }
  if (p->out_col < 0 || p->out_col >= cur) return 1;
  W->gcn = false;  // kinT (kept in-degrees): GCN norms, layer-1 MEAN counts
  for (int l = 0; l < 2; ++l)
    for (int k = 0; k < p->layers[l].n_terms; ++k)
      W->gcn |= p->layers[l].terms[k].kind == XPG_TERM_GCN || (l == 0 && p->layers[l].terms[k].kind == XPG_TERM_MEAN);
  W->a_ld = K + 4;
  W->h_ld = hw + 4;
  W->o_h0 = 32 * W->a_ld;
  // a single-logit head is fused into the MFMA epilogue: H0 then holds one partial per
  // (column block, sample) only — the smaller LDS footprint lets more workgroups share a CU
  const bool head1 = p->n_head == 1 && p->head[0].n_real == 1 && p->out_col == 0;
  int off_f = W->o_h0 + (head1 ? ((l2.f_out_pad + 3) & ~3) : 32 * W->h_ld);
  if (head1 || W->h_ld <= W->a_ld) {
    W->o_h1 = 0;  // the second head tile reuses the A tile (dead after the MFMA)
  } else {
    W->o_h1 = off_f;
    off_f += 32 * W->h_ld;
  }
  W->o_e = off_f;
  off_f += 4 * kWideCap;
  for (int i = 0; i < p->n_head; ++i) {
    W->o_hw[i] = off_f;
    off_f += (p->head[i].n_real * p->head[i].k_pad + 3) & ~3;
  }
  W->lds = sizeof(float) * (size_t)off_f;
  if (W->lds > 150 * 1024) return 1;
  W->kw = 0;  // layer weights in registers (one 32-column block per wave) when they fit
  if (l2.f_out_pad <= 128 && (K == 32 || K == 64 || K == 128)) W->kw = K / 8;
  size_t off = 0;
  W->mT = off;
  off += align_up(sizeof(uint32_t) * (size_t)p->cols);
  W->mT0 = off;
  off += align_up(sizeof(uint32_t) * (size_t)p->n0);
  W->kin = off;
  off += align_up(W->gcn ? sizeof(float) * 32 * (size_t)p->n_rel * p->n0 : 0);
  W->h1 = off;
  off += align_up(sizeof(float) * 32 * (size_t)l1.n_tgt * f1);
  W->ct = off;  // inactive-row table of layer 1 (WideArgs::ctab)
  off += align_up(sizeof(float) * (size_t)l1.n_tgt * f1);
  W->set = off;
  W->nset = rows > kWideS && wide_overlap() ? 2 : 1;
  W->total = off * W->nset;
  return 0;
}

// More than one 32-row pass: layer 1 (and the pass's keep words) of pass p+1 run on a second
// stream beside layer 2 of pass p, on a second buffer set (XPG_WIDE_OVERLAP=0: one stream).
bool wide_overlap() {
  const char* e = getenv("XPG_WIDE_OVERLAP");
  return !(e && std::strcmp(e, "0") == 0);
}

// one non-blocking side stream and the pass hand-off events per device, created once (the only
// handles an entry point creates; no device memory).  `mu` is held across a call's whole enqueue
// sequence: callers on different streams then never interleave their records of / waits on the
// shared events (a wait binds to the record made before it, so a call's waits always see its own
// records), and their side-stream work runs in call order.
struct WideSide {
  std::mutex mu;
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, l1[2] = {nullptr, nullptr}, l2[2] = {nullptr, nullptr};
};
int wide_side(WideSide** out) {
  static std::mutex mu;
  static std::unordered_map<int, WideSide> sides;
  int dev = 0;
  XPG_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  WideSide& w = sides[dev];
  if (!w.s) {
    XPG_HIP(hipStreamCreateWithFlags(&w.s, hipStreamNonBlocking));
    XPG_HIP(hipEventCreateWithFlags(&w.fork, hipEventDisableTiming));
    for (int b = 0; b < 2; ++b) {
      XPG_HIP(hipEventCreateWithFlags(&w.l1[b], hipEventDisableTiming));
      XPG_HIP(hipEventCreateWithFlags(&w.l2[b], hipEventDisableTiming));
    }
  }
  *out = &w;
  return XPG_OK;
}

bool wide_wanted(const xpg_forward_plan* p) {
  if (p->edge_masks || p->edge_dot) return false;  // edge problems: multi-kernel path only
  if (forward_is("wide")) return true;
  if (forward_is(nullptr)) return false;  // another path forced
  return p->n_layers == 2 && p->layers[0].n_tgt >= 8192;
}

template <bool LAST>
void (*wide_kernel(int nfi, int kw))(WideArgs) {
#define XPG_WK(NFI, KW) \
  if (nfi == NFI && kw == KW) return k_wide_tgt<NFI, LAST, KW>;
  if constexpr (LAST) {
    XPG_WK(2, 4) XPG_WK(2, 8) XPG_WK(4, 8) XPG_WK(4, 16) XPG_WK(8, 16)
  }
  XPG_WK(2, 0) XPG_WK(4, 0) XPG_WK(8, 0) XPG_WK(12, 0) XPG_WK(16, 0)
#undef XPG_WK
  return nullptr;
}

int run_wide_forward(const xpg_forward_plan* p, const WideWs& W, const uint32_t* bits, int64_t rows, float* y,
                     char* ws, hipStream_t st) {
  const xpg_layer_desc& l1 = p->layers[0];
  const xpg_layer_desc& l2 = p->layers[1];
  const int words = words_of(p->cols);
  uint32_t* mT = reinterpret_cast<uint32_t*>(ws + W.mT);
  uint32_t* mT0 = reinterpret_cast<uint32_t*>(ws + W.mT0);
  float* kinT = reinterpret_cast<float*>(ws + W.kin);
  float* h1 = reinterpret_cast<float*>(ws + W.h1);
  float* ctab = reinterpret_cast<float*>(ws + W.ct);
  auto fill = [&](WideArgs& a, const xpg_layer_desc& ly) {
    std::memset(&a, 0, sizeof(a));
    a.n0 = p->n0;
    a.n_rel = p->n_rel;
    a.n_tgt = ly.n_tgt;
    a.n_terms = ly.n_terms;
    a.act = ly.act;
    a.mT0 = mT0;
    a.kinT = kinT;
    a.tgt_prev = ly.tgt_prev;
    a.tgt_f0 = ly.tgt_f0;
    a.agg_ptr = ly.agg_ptr;
    a.agg_src = ly.agg_src;
    a.agg_f0 = ly.agg_f0;
    a.self_mult = ly.self_mult;
    a.bias = ly.bias;
    int nagg = 0;
    a.agg1 = -1;
    for (int k = 0; k < ly.n_terms; ++k) {
      a.kind[k] = ly.terms[k].kind;
      a.rel[k] = ly.terms[k].rel;
      a.table[k] = ly.terms[k].table;
      if (a.kind[k] != XPG_TERM_ROOT) {
        ++nagg;
        a.agg1 = k;
      }
    }
    if (nagg != 1) a.agg1 = -1;
  };
  WideArgs a1{}, a2{};
  fill(a1, l1);
  if (const int rc = diag_env("XPG_WIDE_DBG", &a1.dbg)) return rc;
  a1.n_src = p->n0;
  a1.w_row = l1.f_out_pad;
  a1.rstride = l1.f_out_pad;
  a1.f_real = l1.f_out;
  a1.o_e = 0;
  a1.out = h1;
  fill(a2, l2);
  a2.dbg = a1.dbg;
  a2.n_src = l1.n_tgt;
  a2.w_row = l2.f_in_pad;
  a2.rstride = 32 * (int64_t)l2.f_in_pad;  // h1 is node-major: [n1][32 samples][w_row]
  a2.K = l2.n_terms * l2.f_in_pad;
  a2.a_ld = W.a_ld;
  a2.f_out = l2.f_out;
  a2.f_out_pad = l2.f_out_pad;
  a2.n_head = p->n_head;
  a2.out_col = p->out_col;
  a2.h_ld = W.h_ld;
  a2.o_h0 = W.o_h0;
  a2.o_h1 = W.o_h1;
  a2.o_e = W.o_e;
  for (int i = 0; i < p->n_head; ++i) {
    a2.o_hw[i] = W.o_hw[i];
    a2.H[i].k_pad = p->head[i].k_pad;
    a2.H[i].n_real = p->head[i].n_real;
    a2.H[i].n_pad = p->head[i].n_pad;
    a2.H[i].act = p->head[i].act;
    a2.H[i].weight = p->head[i].weight;
    a2.H[i].bias = p->head[i].bias;
  }
  a2.weight = l2.weight;
  a2.head1 = p->n_head == 1 && p->head[0].n_real == 1 && p->out_col == 0;
  a2.src = h1;
  a2.out = y;
  // layer 1: one wave per target for all 32 samples, each table row read once (k_wide_l1s,
  // widths 64 / 128 / 256) when term 0 aggregates and the others are ROOT, else the 16-lane-group
  // gather kernel (XPG_WIDE_L1_GATHER=1, a diagnostics switch, forces it: its parity suite)
  int l1_gather = 0;
  if (const int rc = diag_env("XPG_WIDE_L1_GATHER", &l1_gather)) return rc;
  void (*k1)(WideArgs) = wide_kernel<false>(l1.f_out_pad / 16, 0);
  bool l1s_ok = a1.n_terms >= 1 && a1.kind[0] != XPG_TERM_ROOT;  // term 0 aggregates, the rest ROOT
  for (int k = 1; k < a1.n_terms; ++k) l1s_ok &= a1.kind[k] == XPG_TERM_ROOT;
  if (!l1_gather && l1s_ok) {
    const bool g = a1.kind[0] == XPG_TERM_GCN;
    if (l1.f_out_pad == 64) k1 = g ? k_wide_l1s<1, true> : k_wide_l1s<1, false>;
    else if (l1.f_out_pad == 128) k1 = g ? k_wide_l1s<2, true> : k_wide_l1s<2, false>;
    else if (l1.f_out_pad == 256) k1 = g ? k_wide_l1s<4, true> : k_wide_l1s<4, false>;
  }
  void (*k2)(WideArgs) = wide_kernel<true>(l2.f_in_pad / 16, W.kw);
  if (!k1 || !k2) return fail(XPG_EINVAL, "wide forward: unsupported layer width");
  // warp-specialised layer 2 (8 gather waves || 4 MFMA waves) for single-logit heads over one
  // aggregating term; K = 256 (two 128-wide terms: SAGE): the MFMA waves hold their weight
  // columns in registers and run the products as three bf16 MFMAs (XPG_WIDE_B3=0: the exact f32
  // MFMA, the parity reference of the split products)
  const int nfi2 = l2.f_in_pad / 16;
  const bool ws2 = a2.head1 && W.kw == 0 && a2.agg1 >= 0 && l2.f_out_pad <= 128 && (nfi2 == 4 || nfi2 == 8) &&
                   !(a2.dbg & 15);
  const bool kw32 = a2.K == 256;
  const char* b3e = getenv("XPG_WIDE_B3");
  const bool b3 = kw32 && nfi2 == 8 && !(b3e && std::strcmp(b3e, "0") == 0);
  const size_t lds_ws = sizeof(float) * (size_t)(2 * (b3 ? 32 * (a2.K + 8) : 32 * W.a_ld) + 2 * l2.f_out_pad) +
                        (b3 ? sizeof(uint16_t) * (size_t)a2.K * l2.f_out_pad : 0);  // weight lo pieces (bf16)
  // SAGE-shaped plans ({MEAN, ROOT}) with the B3 products: the pipelined gather with shared
  // in-edge lists (the index chain once per workgroup), 8 prefetched kept rows per group, the
  // transposed product with the in-lane head epilogue, active samples first and the next
  // target's rows issued early
  const bool pipe = b3 && a2.n_terms == 2 && a2.agg1 >= 0 && a2.kind[a2.agg1] == XPG_TERM_MEAN &&
                    a2.kind[1 - a2.agg1] == XPG_TERM_ROOT;
  a2.sort_samples = pipe ? 1 : 0;
  a2.early_prefetch = pipe ? 1 : 0;
  if (ws2) {
    if (pipe) k2 = k_wide_last_ws<8, 32, 8, true, 1, true, 8, true, true>;
    else k2 = nfi2 == 8 ? (b3 ? k_wide_last_ws<8, 32, 8, true> : kw32 ? k_wide_last_ws<8, 32, 8> : k_wide_last_ws<8, 0, 8>)
                        : (kw32 ? k_wide_last_ws<4, 32, 8> : k_wide_last_ws<4, 0, 8>);
  }
  // inactive-row table for the default pair k_wide_l1s -> k_wide_last_ws; the other kernels
  // read / write h1 only
  const bool l1s_k = k1 == k_wide_l1s<1, true> || k1 == k_wide_l1s<1, false> || k1 == k_wide_l1s<2, true> ||
                     k1 == k_wide_l1s<2, false> || k1 == k_wide_l1s<4, true> || k1 == k_wide_l1s<4, false>;
  const bool use_ct = ws2 && l1s_k;
  // kept in-degrees (k_wide_degree) are read by GCN terms and by the gather layer 1's MEAN
  // counts; k_wide_l1s and the layer-2 kernels count a MEAN term's kept edges themselves (SAGE:
  // no degree pass, 0.37 ms per c3 pass)
  bool any_gcn = false;
  for (int l = 0; l < 2; ++l)
    for (int k = 0; k < p->layers[l].n_terms; ++k) any_gcn |= p->layers[l].terms[k].kind == XPG_TERM_GCN;
  const bool need_kin = W.gcn && (any_gcn || !l1s_k);
  const size_t lds2 = ws2 ? lds_ws + (pipe ? sizeof(int) * 3 * kIxInts + sizeof(float) * 2 * l2.f_out_pad : 0)
                          : W.lds;
  const int thr2 = ws2 ? 64 * (8 + 4) : 256;
  const size_t lds1 = sizeof(float) * 3 * kWideCap;
  const int thr1 = 256;
  XPG_HIP(lds_limit(reinterpret_cast<const void*>(k1)));
  XPG_HIP(lds_limit(reinterpret_cast<const void*>(k2)));
  const int cus = device_cus();
  // persistent grids sized to residency (static target striding: no late starters)
  int per_cu1 = 0, per_cu2 = 0;
  XPG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu1, reinterpret_cast<const void*>(k1), thr1, lds1));
  XPG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, reinterpret_cast<const void*>(k2), thr2, lds2));
  per_cu1 = std::max(1, per_cu1);
  per_cu2 = std::max(1, per_cu2);
  const unsigned g1 = static_cast<unsigned>(std::min<int64_t>(l1.n_tgt, per_cu1 * (int64_t)cus));
  const unsigned g2 = static_cast<unsigned>(std::min<int64_t>(l2.n_tgt, per_cu2 * (int64_t)cus));
  // two buffer sets (W.nset == 2, more than one pass): pass p's keep words, layer 1 and h1 on the
  // side stream into set p & 1, layer 2 on the caller's stream; set b is written again only after
  // layer 2 of pass p - 2 released it.  Not while the caller's stream is being captured.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  XPG_HIP(hipStreamIsCapturing(st, &cap));
  WideSide* side = nullptr;
  const bool two = W.nset == 2 && cap == hipStreamCaptureStatusNone;
  std::unique_lock<std::mutex> side_lock;
  if (two) {
    if (const int rc = wide_side(&side)) return rc;
    side_lock = std::unique_lock<std::mutex>(side->mu);
    XPG_HIP(hipEventRecord(side->fork, st));
    XPG_HIP(hipStreamWaitEvent(side->s, side->fork, 0));
  }
  int64_t pass = 0;
  for (int64_t r0 = 0; r0 < rows; r0 += kWideS, ++pass) {
    const int nr = static_cast<int>(std::min<int64_t>(kWideS, rows - r0));
    const int b = two ? static_cast<int>(pass & 1) : 0;
    const size_t sb = W.set * static_cast<size_t>(b);
    hipStream_t s1 = two ? side->s : st;
    if (two && pass >= 2) XPG_HIP(hipStreamWaitEvent(s1, side->l2[b], 0));
    uint32_t* mTb = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(mT) + sb);
    uint32_t* mT0b = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(mT0) + sb);
    float* kinb = reinterpret_cast<float*>(reinterpret_cast<char*>(kinT) + sb);
    float* h1b = reinterpret_cast<float*>(reinterpret_cast<char*>(h1) + sb);
    float* ctb = use_ct ? reinterpret_cast<float*>(reinterpret_cast<char*>(ctab) + sb) : nullptr;
    a1.mT0 = a2.mT0 = mT0b;
    a1.kinT = a2.kinT = kinb;
    a1.out = h1b;
    a2.src = h1b;
    a1.ctab = a2.ctab = ctb;
    prof_begin(s1, XPG_PROF_WIDE_BITS);
    hipLaunchKernelGGL(k_wide_bits, dim3(static_cast<unsigned>(cdiv(words, 256))), dim3(256), 0, s1, bits, r0, nr,
                       words, p->cols, mTb);
    XPG_LAUNCHED();
    prof_end(s1, XPG_PROF_WIDE_BITS);
    prof_begin(s1, XPG_PROF_WIDE_F0);
    hipLaunchKernelGGL(k_wide_f0, dim3(static_cast<unsigned>(cdiv(p->n0, 256))), dim3(256), 0, s1, mTb, p->f0_node,
                       p->n0, mT0b);
    XPG_LAUNCHED();
    prof_end(s1, XPG_PROF_WIDE_F0);
    if (need_kin) {
      const int64_t n = (int64_t)p->n_rel * p->n0 * 32;
      prof_begin(s1, XPG_PROF_WIDE_DEGREE);
      hipLaunchKernelGGL(k_wide_degree, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, s1, mTb, mT0b,
                         p->n0, p->n_rel, p->deg_ptr, p->deg_src, kinb);
      XPG_LAUNCHED();
      prof_end(s1, XPG_PROF_WIDE_DEGREE);
    }
    a1.nr = nr;
    a1.row0 = r0;
    prof_begin(s1, XPG_PROF_WIDE_L1);
    hipLaunchKernelGGL(k1, dim3(g1), dim3(thr1), lds1, s1, a1);
    XPG_LAUNCHED();
    prof_end(s1, XPG_PROF_WIDE_L1);
    if (two) {
      XPG_HIP(hipEventRecord(side->l1[b], s1));
      XPG_HIP(hipStreamWaitEvent(st, side->l1[b], 0));
    }
    a2.nr = nr;
    a2.row0 = r0;
    prof_begin(st, XPG_PROF_WIDE_L2);
    hipLaunchKernelGGL(k2, dim3(g2), dim3(thr2), lds2, st, a2);
    XPG_LAUNCHED();
    prof_end(st, XPG_PROF_WIDE_L2);
    if (two) XPG_HIP(hipEventRecord(side->l2[b], st));
  }
  return XPG_OK;
}

// Lanes-=-rows fused forward for 1- and 2-layer plans (returns 1 when it does not apply).
int try_rows_forward(const xpg_forward_plan* p, const uint32_t* bits, int64_t rows, float* y, hipStream_t st,
                     int* ctl) {
  if (p->n_layers < 1 || p->n_layers > 2 || p->n_head > kFusedMaxHead || plan_multi_type(p)) return 1;
  if (p->edge_masks || p->edge_dot) return 1;  // edge problems: multi-kernel path only
  RowsFwdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.rows = rows;
  a.bits = bits;
  a.y = y;
  a.words = words_of(p->cols);
  a.n0 = p->n0;
  a.n_rel = p->n_rel;
  a.n_layers = p->n_layers;
  a.out_col = p->out_col;
  a.f0_node = p->f0_node;
  a.deg_ptr = p->deg_ptr;
  a.deg_src = p->deg_src;
  a.n_deg_edges = static_cast<int>(p->n_deg_edges);
  const xpg_layer_desc& l1 = p->layers[0];
  if (l1.n_terms < 1 || l1.n_terms > XPG_MAX_TERMS || p->n_deg_edges < 0 || l1.n_edges < 0) return 1;
  a.n1 = l1.n_tgt;
  a.n1_edges = l1.n_edges;
  a.n_terms1 = l1.n_terms;
  a.act1 = l1.act;
  a.f1_out = l1.f_out;
  a.f1_pad = l1.f_out_pad;
  a.l1_ptr = l1.agg_ptr;
  a.l1_f0 = l1.agg_f0;
  a.l1_smul = l1.self_mult;
  a.l1_tgt_f0 = l1.tgt_f0;
  a.bias1 = l1.bias;
  for (int k = 0; k < l1.n_terms; ++k) {
    if (!l1.terms[k].table) return 1;
    a.kind1[k] = l1.terms[k].kind;
    a.rel1[k] = l1.terms[k].rel;
    a.tab1[k] = l1.terms[k].table;
  }
  const int fs = a.f1_pad / kRowsWaves;
  if (a.f1_pad % kRowsWaves || (fs != 2 && fs != 4 && fs != 8)) return 1;
  int cur_w = a.f1_pad;
  a.n_last = a.n1;
  int64_t k2 = 0;
  if (p->n_layers == 2) {
    const xpg_layer_desc& l2 = p->layers[1];
    if (l2.n_terms < 1 || l2.n_terms > XPG_MAX_TERMS || l2.f_in_pad != a.f1_pad || !l2.weight || l2.n_edges < 0)
      return 1;
    a.n2 = l2.n_tgt;
    a.n2_edges = l2.n_edges;
    a.n_terms2 = l2.n_terms;
    a.act2 = l2.act;
    a.f2_out = l2.f_out;
    a.f2_pad = l2.f_out_pad;
    a.l2_ptr = l2.agg_ptr;
    a.l2_src = l2.agg_src;
    a.l2_f0 = l2.agg_f0;
    a.l2_smul = l2.self_mult;
    a.l2_tgt_f0 = l2.tgt_f0;
    a.l2_tgt_prev = l2.tgt_prev;
    a.w2 = l2.weight;
    a.bias2 = l2.bias;
    for (int k = 0; k < l2.n_terms; ++k) {
      a.kind2[k] = l2.terms[k].kind;
      a.rel2[k] = l2.terms[k].rel;
    }
    a.n_last = a.n2;
    cur_w = a.f2_pad;
    k2 = (int64_t)l2.n_terms * a.f1_pad;
  }
  int h0w = cur_w, h1w = 0;
  a.n_head = p->n_head;
  for (int i = 0; i < p->n_head; ++i) {
    const xpg_head_desc& hd = p->head[i];
    if (hd.k_pad != cur_w || hd.k_pad % 4) return 1;
    a.H[i].k_pad = hd.k_pad;
    a.H[i].n_real = hd.n_real;
    a.H[i].n_pad = hd.n_pad;
    a.H[i].act = hd.act;
    a.H[i].weight = hd.weight;
    a.H[i].bias = hd.bias;
    if (i % 2 == 0) h1w = std::max(h1w, hd.n_pad);
    else h0w = std::max(h0w, hd.n_pad);
    cur_w = hd.n_pad;
  }
  if (p->out_col < 0 || p->out_col >= cur_w) return 1;
  int64_t off = 0;
  auto take = [&](int64_t n) {
    const int64_t o = off;
    off += (n + 3) & ~int64_t(3);
    return static_cast<int>(o);
  };
  a.o_tab = take((int64_t)a.n_terms1 * a.n0 * a.f1_pad);
  a.o_dv = take((int64_t)a.n_rel * a.n0 * 64);
  a.o_kt = take((int64_t)a.n_rel * a.n1 * 64);
  a.o_a2 = take(k2 * 64);
  a.o_h0 = take((int64_t)h0w * 64);
  a.o_h1 = take((int64_t)std::max(h1w, 1) * 64);
  a.o_dptr = take((int64_t)a.n_rel * (a.n0 + 1));
  a.o_f0n = take(a.n0);
  a.o_dsrc = take(std::max<int64_t>(1, p->n_deg_edges));
  a.o_l1ptr = take((int64_t)a.n_rel * (a.n1 + 1));
  a.o_l1f0 = take(std::max(1, a.n1_edges));
  a.o_l1smul = take((int64_t)a.n_rel * a.n1);
  a.o_l1tgt = take(a.n1);
  a.o_l2ptr = take((int64_t)a.n_rel * (a.n2 + 1));
  a.o_l2src = take(std::max(1, a.n2_edges));
  a.o_l2f0 = take(std::max(1, a.n2_edges));
  a.o_l2smul = take((int64_t)a.n_rel * a.n2);
  a.o_l2tgt = take(a.n2);
  a.o_l2prev = take(a.n2);
  const int64_t cap = 160 * 1024 / 4 - 256;
  if (off > cap) return 1;
  a.mb_pitch = a.words | 1;
  a.stage_bits = off + 64 * (int64_t)a.mb_pitch <= cap ? 1 : 0;
  if (a.stage_bits) a.o_mb = take(64 * (int64_t)a.mb_pitch);
  a.w2_lds = 0;
  if (p->n_layers == 2 && off + (int64_t)a.f2_pad * k2 <= cap) {
    a.w2_lds = 1;
    a.o_w2 = take((int64_t)a.f2_pad * k2);
  }
  for (int i = 0; i < kFusedMaxHead; ++i) a.o_hw[i] = -1;
  for (int i = 0; i < p->n_head; ++i) {
    const int64_t n = (int64_t)p->head[i].n_pad * p->head[i].k_pad;
    if (off + n <= cap) a.o_hw[i] = take(n);
  }
  const size_t lds = sizeof(float) * (size_t)off;
  a.n_blocks = static_cast<int>(cdiv(rows, 64));
  a.cus_per_xcd = std::max(1, device_cus() / device_xcds());
  a.ctl = ctl;
  unsigned nwg = static_cast<unsigned>(a.n_blocks);
  if (ctl) {  // one workgroup per CU at most (LDS-bound); extra ones leave at once
    XPG_HIP(hipMemsetAsync(ctl, 0, sizeof(int) * 32, st));
    nwg = static_cast<unsigned>(std::min<int64_t>((int64_t)device_xcds() * a.cus_per_xcd,
                                                  (int64_t)a.n_blocks + 4 * a.cus_per_xcd));
  }
  const dim3 grid(nwg);
#define XPG_ROWS(F)                                                                                     \
  if (fs == F) {                                                                                        \
    XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_rows_forward<F>)));      \
    hipLaunchKernelGGL(k_rows_forward<F>, grid, dim3(64 * kRowsWaves), lds, st, a);                      \
    XPG_LAUNCHED();                                                                                     \
    return XPG_OK;                                                                                      \
  }
  XPG_ROWS(2) XPG_ROWS(4) XPG_ROWS(8)
#undef XPG_ROWS
  return 1;
}

int launch_shapley(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols, uint32_t* bits, int32_t* counts,
                   hipStream_t st, const uint64_t* seed_dev = nullptr) {
  const int words = words_of(cols);
  const int quads = (words + 3) / 4;
  if (rows == 0) return XPG_OK;
  XPG_REQ(quads <= (1 << 30), "shapley: row too long");
  if (quads < 64) {  // short rows: lanes over (row, quad)
    const unsigned nb = static_cast<unsigned>(std::min<int64_t>(cdiv(rows * quads, 256), 65535 * 8));
    if (words % 4 == 0)
      hipLaunchKernelGGL(k_shapley_flat<4>, dim3(nb), dim3(256), 0, st, seed, row_offset, rows, cols, words, bits,
                         counts, seed_dev);
    else if (words % 2 == 0)
      hipLaunchKernelGGL(k_shapley_flat<2>, dim3(nb), dim3(256), 0, st, seed, row_offset, rows, cols, words, bits,
                         counts, seed_dev);
    else
      hipLaunchKernelGGL(k_shapley_flat<1>, dim3(nb), dim3(256), 0, st, seed, row_offset, rows, cols, words, bits,
                         counts, seed_dev);
    XPG_LAUNCHED();
    return XPG_OK;
  }
  // rows per block: each thread makes 16 B per row, so one row per block (25,600 x 31 blocks at
  // the c3 graph_prediction shape) left the kernel at the block-dispatch rate; the blocks now
  // stride over rows, ~64 per CU (XPG_SHAPLEY_BLOCKS, a diagnostics switch: total blocks, -1 =
  // one row per block; bits are the same either way: counter-based per (quad, row))
  const int64_t gx = cdiv(quads, 256);
  int env_blk = 0;
  if (const int rc = diag_env("XPG_SHAPLEY_BLOCKS", &env_blk)) return rc;
  const int64_t nblk = env_blk != 0 ? env_blk : 64 * (int64_t)device_cus();
  const int64_t gy = nblk > 0 ? std::max<int64_t>(1, std::min<int64_t>(rows, nblk / gx)) : std::min<int64_t>(rows, 65535);
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(std::min<int64_t>(gy, 65535)));
  if (words % 4 == 0)
    hipLaunchKernelGGL(k_shapley<4>, grid, dim3(256), 0, st, seed, row_offset, rows, cols, words, bits, counts, seed_dev);
  else if (words % 2 == 0)
    hipLaunchKernelGGL(k_shapley<2>, grid, dim3(256), 0, st, seed, row_offset, rows, cols, words, bits, counts, seed_dev);
  else
    hipLaunchKernelGGL(k_shapley<1>, grid, dim3(256), 0, st, seed, row_offset, rows, cols, words, bits, counts, seed_dev);
  XPG_LAUNCHED();
  return XPG_OK;
}

}  // namespace

// ==================================================================================== C-ABI
extern "C" {

int xpg_abi_version(void) { return XPG_ABI_VERSION; }

int xpg_mt19937_mask_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t rows, int64_t cols,
                          uint32_t* bits) {
  XPG_REQ(state && left && next && (bits || rows == 0) && rows >= 0 && cols > 0, "mt19937_mask_bits: bad arguments");
  const bool fresh = *left == 1 && *next == 0;  // seeded, not drawn from yet
  XPG_REQ(fresh || (*left >= 1 && *next >= 0 && *next + *left - 1 == hostrng::kN),
          "mt19937_mask_bits: generator position (left, next) is not an at::mt19937 state");
  if (rows > 0) hostrng::mask_bits(state, left, next, rows, cols, bits);
  return XPG_OK;
}

int xpg_mt19937_repeat_draws(uint32_t* state, int32_t* left, int32_t* next, int32_t times, int64_t S, float from,
                             float to, int32_t fma, int64_t* seeds, float* w0) {
  XPG_REQ(state && left && next && times >= 0 && S >= 0 && (seeds || times == 0) && (w0 || times == 0 || S == 0) &&
              from <= to,
          "mt19937_repeat_draws: bad arguments");
  const bool fresh = *left == 1 && *next == 0;
  XPG_REQ(fresh || (*left >= 1 && *next >= 0 && *next + *left - 1 == hostrng::kN),
          "mt19937_repeat_draws: generator position (left, next) is not an at::mt19937 state");
  hostrng::repeat_draws(state, left, next, times, S, from, to, fma, seeds, w0);
  return XPG_OK;
}

int xpg_mt19937_community_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t cols, int32_t n_comm,
                               const int32_t* comm_ptr, const int32_t* comm_cols, const int32_t* blocks,
                               int32_t n_blocks, int64_t rows, uint32_t* bits) {
  XPG_REQ(state && left && next && comm_ptr && blocks && bits && cols > 0 && n_comm > 0 && n_blocks > 0 &&
              n_blocks <= n_comm && rows > 0,
          "mt19937_community_bits: bad arguments");
  const bool fresh = *left == 1 && *next == 0;
  XPG_REQ(fresh || (*left >= 1 && *next >= 0 && *next + *left - 1 == hostrng::kN),
          "mt19937_community_bits: generator position (left, next) is not an at::mt19937 state");
  XPG_REQ(comm_ptr[0] == 0, "mt19937_community_bits: comm_ptr[0] != 0");
  for (int32_t c = 0; c < n_comm; ++c) {
    XPG_REQ(comm_ptr[c + 1] >= comm_ptr[c], "mt19937_community_bits: comm_ptr not monotone");
    for (int32_t k = comm_ptr[c]; k < comm_ptr[c + 1]; ++k) {
      XPG_REQ(comm_cols[k] >= 0 && comm_cols[k] < cols, "mt19937_community_bits: member column out of range");
      XPG_REQ(k == comm_ptr[c] || comm_cols[k] >= comm_cols[k - 1], "mt19937_community_bits: members not sorted");
    }
  }
  int64_t end = 0;
  for (int32_t b = 0; b < n_blocks; ++b) {
    const int32_t* q = blocks + 5 * b;
    XPG_REQ(q[0] == end && q[1] >= 1 && q[2] >= 1 && q[2] <= q[1] && q[3] >= 0 && q[3] < n_comm && q[4] == b,
            "mt19937_community_bits: blocks must be {row_start, size, size_internal, own, b} back to back");
    end += q[1];
  }
  XPG_REQ(end == rows, "mt19937_community_bits: rows != the blocks' total");
  std::memset(bits, 0, sizeof(uint32_t) * static_cast<size_t>(rows) * static_cast<size_t>(words_of(cols)));
  hostrng::community_rows(state, left, next, cols, n_comm, comm_ptr, comm_cols, blocks, n_blocks, bits);
  return XPG_OK;
}

int xpg_plan_arrays_build(int64_t S, int32_t n_rel, const int64_t* rel_ptr, const int64_t* src, const int64_t* dst,
                          const int64_t* eid, const int64_t* queries, int64_t nq, int32_t L, void** handle,
                          int64_t* sizes) {
  XPG_REQ(handle && sizes && rel_ptr && queries && S > 0 && n_rel >= 0 && nq > 0 && L >= 1 && L <= 64,
          "plan_arrays: bad arguments");
  *handle = nullptr;
  XPG_REQ(rel_ptr[0] == 0, "plan_arrays: rel_ptr[0] != 0");
  for (int32_t r = 0; r < n_rel; ++r) XPG_REQ(rel_ptr[r + 1] >= rel_ptr[r], "plan_arrays: rel_ptr not monotone");
  const int64_t E = rel_ptr[n_rel];
  XPG_REQ(E == 0 || (src && dst), "plan_arrays: missing edges");
  for (int64_t e = 0; e < E; ++e)
    XPG_REQ(src[e] >= 0 && src[e] < S && dst[e] >= 0 && dst[e] < S, "plan_arrays: edge endpoint out of range");
  {
    std::vector<uint8_t> seen(S);
    for (int64_t i = 0; i < nq; ++i) {
      XPG_REQ(queries[i] >= 0 && queries[i] < S, "plan_arrays: query positions out of range");
      XPG_REQ(!seen[queries[i]], "plan_arrays: duplicate query positions");
      seen[queries[i]] = 1;
    }
  }
  auto* A = new planhost::Arrays();
  planhost::build(S, n_rel, rel_ptr, src, dst, eid, queries, nq, L, *A);
  int64_t k = 0;
  for (int32_t l = 0; l <= L; ++l) sizes[k++] = static_cast<int64_t>(A->fr[l].size());
  auto put = [&](const planhost::Csr& c) {
    for (const std::vector<int64_t>* v : {&c.ptr, &c.src, &c.eid, &c.smul, &c.sptr, &c.seid})
      sizes[k++] = static_cast<int64_t>(v->size());
  };
  put(A->deg);
  for (const planhost::Csr& c : A->lay) put(c);
  *handle = A;
  return XPG_OK;
}

int xpg_plan_arrays_take(void* handle, int64_t* out) {
  XPG_REQ(handle && out, "plan_arrays_take: bad arguments");
  auto* A = static_cast<planhost::Arrays*>(handle);
  int64_t* o = out;
  auto cp = [&](const std::vector<int64_t>& v) {
    if (!v.empty()) std::memcpy(o, v.data(), sizeof(int64_t) * v.size());
    o += v.size();
  };
  auto cp_csr = [&](const planhost::Csr& c) {
    for (const std::vector<int64_t>* v : {&c.ptr, &c.src, &c.eid, &c.smul, &c.sptr, &c.seid}) cp(*v);
  };
  for (const auto& f : A->fr) cp(f);
  cp_csr(A->deg);
  for (const planhost::Csr& c : A->lay) cp_csr(c);
  delete A;
  return XPG_OK;
}

int xpg_plan_arrays_free(void* handle) {
  delete static_cast<planhost::Arrays*>(handle);
  return XPG_OK;
}

#ifdef XPG_WIDE_STAMPS  // diagnostic build only: layer-2 phase cycles [512 workgroups][16 waves][8]
int xpg_debug_wide_stamps(uint64_t* out) {
  XPG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wide_stamps), sizeof(uint64_t) * 512 * 16 * 8));
  return XPG_OK;
}
#endif

#ifdef XPG_WLM_STAMPS  // diagnostic build only: per-phase cycle stamps of the last stamped launch
int xpg_debug_stamps(uint64_t* out) {
  XPG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wlm_stamps), sizeof(uint64_t) * 16));
  return XPG_OK;
}
#endif

const char* xpg_last_error(void) { return g_err.c_str(); }

int xpg_pack_masks(const uint8_t* mask, int64_t rows, int64_t cols, uint32_t* bits, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0, "pack: bad shape");
  const int words = words_of(cols);
  const int64_t n = rows * words;
  if (n == 0) return XPG_OK;
  hipLaunchKernelGGL(k_pack, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, S(stream), mask, rows, cols, words, bits);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_unpack_masks(const uint32_t* bits, int64_t rows, int64_t cols, uint8_t* mask, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0, "unpack: bad shape");
  const int64_t n = rows * cols;
  if (n == 0) return XPG_OK;
  hipLaunchKernelGGL(k_unpack, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, S(stream), bits, rows, cols, words_of(cols), mask);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_sample_shapley(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols, uint32_t* bits, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0 && row_offset >= 0, "shapley: bad shape");
  return launch_shapley(seed, row_offset, rows, cols, bits, nullptr, S(stream));
}

int xpg_sample_shapley_dev(const uint64_t* seed, int64_t row_offset, int64_t rows, int64_t cols, uint32_t* bits,
                           xpg_stream_t stream) {
  XPG_REQ(seed && rows >= 0 && cols > 0 && row_offset >= 0, "shapley: bad shape");
  return launch_shapley(0, row_offset, rows, cols, bits, nullptr, S(stream), seed);
}

int xpg_sample_shapley_sets(const uint64_t* seeds, int32_t n_sets, int64_t rows, int64_t cols, uint32_t* bits,
                            xpg_stream_t stream) {
  XPG_REQ(seeds && n_sets >= 0 && rows >= 0 && cols > 0 && (bits || n_sets == 0 || rows == 0),
          "shapley sets: bad shape");
  const int64_t set_words = rows * ((cols + 31) / 32);
  for (int32_t k = 0; k < n_sets; ++k) {
    const int rc = launch_shapley(seeds[k], 0, rows, cols, bits + k * set_words, nullptr, S(stream));
    if (rc != XPG_OK) return rc;
  }
  return XPG_OK;
}

int xpg_sample_shapley_counts(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols, uint32_t* bits,
                              int32_t* counts, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0 && row_offset >= 0 && counts, "shapley: bad shape");
  if (rows == 0) return XPG_OK;
  XPG_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)rows, S(stream)));
  return launch_shapley(seed, row_offset, rows, cols, bits, counts, S(stream));
}

int xpg_sample_communities(uint64_t seed, int64_t rows, int64_t cols, int32_t n_comm, const int32_t* blocks,
                           int32_t n_blocks, int64_t src_rows, int32_t shuffle, const int32_t* col_ptr,
                           const int32_t* col_comm, uint32_t* bits, int32_t* prow, xpg_stream_t stream) {
  return xpg_sample_communities_rows(seed, 0, rows, cols, n_comm, blocks, n_blocks, src_rows, shuffle, col_ptr,
                                     col_comm, bits, prow, stream);
}

int xpg_sample_communities_rows(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols, int32_t n_comm,
                                const int32_t* blocks, int32_t n_blocks, int64_t src_rows, int32_t shuffle,
                                const int32_t* col_ptr, const int32_t* col_comm, uint32_t* bits, int32_t* prow,
                                xpg_stream_t stream) {
  XPG_REQ(cols > 0 && rows >= 0 && row_offset >= 0 && n_comm > 0 && n_comm <= 32 * kCommMaxWords &&
              n_blocks > 0 && n_blocks <= n_comm && src_rows >= row_offset + rows &&
              src_rows < (int64_t(1) << 31) && blocks && col_ptr && col_comm && bits,
          "communities: bad shape");
  if (rows == 0) return XPG_OK;
  int nb = 1;  // bit length of src_rows - 1
  while ((int64_t(1) << nb) < src_rows) ++nb;
  const int hb = (nb + 1) / 2;
  const bool small = n_comm <= 64;
  const size_t flag_bytes = small ? 0 : sizeof(uint32_t) * 4 * static_cast<size_t>((n_comm + 31) / 32);
  const size_t stage_bytes = sizeof(int32_t) * 5 * static_cast<size_t>(n_blocks) + sizeof(int16_t) * static_cast<size_t>(cols);
  const bool staged = cols <= kCommStageCols && flag_bytes + stage_bytes <= 64 * 1024;
  // XPG_COMM_PERCOL=1 (diagnostics): the per-column lookup, which the parity suite compares bitwise
  int percol = 0;
  if (const int rc = diag_env("XPG_COMM_PERCOL", &percol)) return rc;
  const bool cmode = small && cols <= kCommStageCols && sizeof(int32_t) * (5 * static_cast<size_t>(n_blocks) +
                     static_cast<size_t>(n_comm) * words_of(cols)) <= 48 * 1024 && !percol;
  const size_t lds = cmode ? sizeof(int32_t) * (5 * static_cast<size_t>(n_blocks) + static_cast<size_t>(n_comm) * words_of(cols))
                           : flag_bytes + (staged ? stage_bytes : 0);
  const int64_t cap = staged ? 2048 : 65536;
  const int64_t want = std::min<int64_t>(cdiv(rows, 4), cap);
  const dim3 g(static_cast<unsigned>(want));
#define XPG_COMM(SM, ST)                                                                                      \
  hipLaunchKernelGGL((k_communities<SM, ST>), g, dim3(256), lds, S(stream), seed, row_offset, rows, cols, words_of(cols), n_comm, \
                     blocks, n_blocks, static_cast<uint32_t>(src_rows), hb, shuffle ? 1 : 0, col_ptr, col_comm, bits, \
                     prow)
  if (cmode) {
    hipLaunchKernelGGL((k_communities<true, true, true>), g, dim3(256), lds, S(stream), seed, row_offset, rows, cols,
                       words_of(cols), n_comm, blocks, n_blocks, static_cast<uint32_t>(src_rows), hb, shuffle ? 1 : 0,
                       col_ptr, col_comm, bits, prow);
  } else if (small) {
    if (staged) XPG_COMM(true, true); else XPG_COMM(true, false);
  } else {
    if (staged) XPG_COMM(false, true); else XPG_COMM(false, false);
  }
#undef XPG_COMM
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_edge_keep(const uint32_t* bits, int64_t rows, int64_t cols, const int32_t* src, const int32_t* dst,
                  int64_t n_edges, uint8_t* keep, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0 && n_edges >= 0, "edge_keep: bad shape");
  const int64_t n = rows * n_edges;
  if (n == 0) return XPG_OK;
  hipLaunchKernelGGL(k_edge_keep, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, S(stream), bits, rows, words_of(cols), src, dst, n_edges, keep);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_rows_no_edge(const uint32_t* bits, int64_t rows, int64_t cols, const int32_t* src, const int32_t* dst,
                     int64_t n_edges, uint8_t* empty, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0 && n_edges >= 0, "rows_no_edge: bad shape");
  if (rows == 0) return XPG_OK;
  const int rpw = 4;  // rows per wave, one after another (8: no better)
  hipLaunchKernelGGL(k_rows_no_edge, dim3(static_cast<unsigned>(cdiv(cdiv(rows, rpw), 4))), dim3(256), 0, S(stream),
                     bits, rows, words_of(cols), src, dst, n_edges, empty, rpw);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_popcount_rows(const uint32_t* bits, int64_t rows, int64_t cols, int32_t* counts, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 0, "popcount: bad shape");
  if (rows == 0) return XPG_OK;
  hipLaunchKernelGGL(k_popcount, dim3(static_cast<unsigned>(cdiv(rows, 4))), dim3(256), 0, S(stream), bits, rows, words_of(cols), counts);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_shap_kernel(const int32_t* counts, int64_t rows, int64_t cols, double* kernel_out, xpg_stream_t stream) {
  XPG_REQ(rows >= 0 && cols > 1, "shap_kernel: need cols > 1");
  if (rows == 0) return XPG_OK;
  if (cols - 1 <= 1000)
    hipLaunchKernelGGL(k_shap_exact, dim3(static_cast<unsigned>(cdiv(rows, 256))), dim3(256), 0, S(stream), counts,
                       rows, cols, kernel_out);
  else {
    hipLaunchKernelGGL(k_shap_approx_rows, dim3(static_cast<unsigned>(cdiv(rows, 256))), dim3(256), 0, S(stream),
                       counts, rows, cols, kernel_out);
    XPG_LAUNCHED();
    hipLaunchKernelGGL(k_shap_approx_finish, dim3(1), dim3(1024), 0, S(stream), counts, rows, cols, kernel_out);
    XPG_LAUNCHED();
    hipLaunchKernelGGL(k_shap_clean, dim3(static_cast<unsigned>(cdiv(rows, 256))), dim3(256), 0, S(stream), rows,
                       kernel_out);
  }
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_dense(const float* A, int64_t M, int64_t lda, const float* W, int64_t ldw, int64_t k_pad, const float* bias,
              int64_t n_real, int64_t n_pad, int act, float* C, int64_t ldc, xpg_stream_t stream) {
  return launch_dense(A, M, lda, W, ldw, k_pad, bias, n_real, n_pad, act, C, ldc, S(stream));
}

int xpg_profile_enable(int on) {
  for (ProfRec& r : g_prof) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.clear();
  g_prof_on = on != 0;
  return XPG_OK;
}

int xpg_profile_read(double* ms, int64_t* launches, int32_t n_slots) {
  XPG_REQ(ms != nullptr && launches != nullptr && n_slots > 0, "profile_read: bad arguments");
  for (int i = 0; i < n_slots; ++i) {
    ms[i] = 0.0;
    launches[i] = 0;
  }
  int rc = XPG_OK;
  for (ProfRec& r : g_prof) {
    float t = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) rc = XPG_EHIP;
    if (r.slot >= 0 && r.slot < n_slots) {
      ms[r.slot] += t;
      ++launches[r.slot];
    }
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.clear();
  if (rc) return fail(rc, "profile_read: event timing failed");
  return XPG_OK;
}

int xpg_forward_workspace(const xpg_forward_plan* plan, int64_t rows, size_t* bytes) {
  WsLayout L;
  int rc = layout_ws(plan, rows, &L);
  if (rc) return rc;
  WideWs W;
  if (wide_wanted(plan) && wide_layout(plan, rows, &W) == 0) {
    *bytes = W.total;  // 32-row passes: one buffer set, or two when rows > 32
    return XPG_OK;
  }
  *bytes = L.total;
  return XPG_OK;
}

int xpg_masked_forward(const xpg_forward_plan* p, const uint32_t* bits, int64_t rows, float* y,
                       void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  WsLayout L;
  int rc = layout_ws(p, rows, &L);
  if (rc) return rc;
  XPG_REQ(p->n_rel >= 1 && p->n0 >= 1 && p->cols > 0, "masked_forward: bad plan sizes");
  hipStream_t st = S(stream);
  {
    WideWs W;
    if (wide_wanted(p) && wide_layout(p, rows, &W) == 0) {
      XPG_REQ(workspace_bytes >= W.total, "masked_forward: workspace too small");
      if (rows == 0) return XPG_OK;
      return run_wide_forward(p, W, bits, rows, y, static_cast<char*>(workspace), st);
    }
  }
  XPG_REQ(workspace_bytes >= L.total, "masked_forward: workspace too small");
  if (rows == 0) return XPG_OK;
  {
    // XPG_FORWARD_STRICT=1 (tests): a forced path that does not take the plan is an error
    // instead of a fall-back to the multi-kernel path
    const char* strict_env = getenv("XPG_FORWARD_STRICT");
    const bool multi = forward_is("unfused");
    const bool strict = forward_is(nullptr) && !multi && strict_env && std::strcmp(strict_env, "1") == 0;
    const bool wave_rows = forward_is("fused");
    if (wave_rows) {
      rc = try_fused_forward(p, bits, rows, y, st);
      if (rc != 1) return rc;
    } else if (!multi) {
      rc = try_rows_forward(p, bits, rows, y, st, reinterpret_cast<int*>(static_cast<char*>(workspace) + L.ctl));
      if (rc != 1) return rc;
    }
    if (strict) return fail(XPG_EINVAL, "masked_forward: the forced XPG_FORWARD path does not take this plan");
  }
  char* ws = static_cast<char*>(workspace);
  float* kin = reinterpret_cast<float*>(ws + L.kin);
  const int words = words_of(p->cols);
  const int kpitch = deg_pitch(p);
  // The picked output column is fused into the last dense layer's epilogue (k_dense HEAD) when the
  // network ends in a head layer that follows a dense layer (another head layer, or a conv layer
  // past the first) and no link decoder: no 32-wide padded head tile, no column pick.
  OutColumn fh;
  bool fuse_out = false;
  if (!p->edge_dot && p->n_head >= 1 && (p->n_head >= 2 || p->n_layers >= 2)) {
    const xpg_head_desc& hl = p->head[p->n_head - 1];
    const int64_t prev_pad = p->n_head >= 2 ? p->head[p->n_head - 2].n_pad : p->layers[p->n_layers - 1].f_out_pad;
    if (hl.k_pad == prev_pad && p->out_col >= 0 && p->out_col < hl.n_real) {
      fuse_out = true;
      fh.w = hl.weight + (int64_t)p->out_col * hl.k_pad;
      fh.b = hl.bias + p->out_col;
      fh.act = hl.act;
      fh.y = y;
    }
  }
  {
    const int64_t n = rows * (int64_t)p->n_rel * kpitch;
    XPG_REQ(!p->edge_masks || p->deg_eid || p->n_deg_edges == 0, "masked_forward: edge-mask plan without deg_eid");
    hipLaunchKernelGGL(k_degree, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, st, bits, rows, words, p->n0,
                       kpitch, p->n_rel, p->f0_node, p->deg_ptr, p->deg_src, p->edge_masks ? p->deg_eid : nullptr, kin);
    XPG_LAUNCHED();
  }
  for (int l = 0; l < p->n_layers; ++l) {
    const xpg_layer_desc& ly = p->layers[l];
    XPG_REQ(ly.n_terms >= 1 && ly.n_terms <= XPG_MAX_TERMS, "layer: 1..8 terms");
    AggArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rows = rows;
    a.n0 = p->n0;
    a.n_rel = p->n_rel;
    a.n_tgt = ly.n_tgt;
    a.n_prev = l == 0 ? p->n0 : p->layers[l - 1].n_tgt;
    a.kin = kin;
    a.kpitch = kpitch;
    if (kpitch < p->n0) {  // kin holds the targets only: MEAN sources test their own bit
      a.mbits = bits;
      a.words = words;
      a.f0_node = p->f0_node;
    }
    a.tgt_prev = ly.tgt_prev;
    a.tgt_f0 = ly.tgt_f0;
    a.agg_ptr = ly.agg_ptr;
    a.agg_src = ly.agg_src;
    a.agg_f0 = ly.agg_f0;
    a.self_mult = ly.self_mult;
    a.n_terms = ly.n_terms;
    a.tgt_type = ly.tgt_type;
    if (p->edge_masks) {
      XPG_REQ(ly.agg_eid && ly.self_ptr && ly.self_eid, "masked_forward: edge-mask layer without edge columns");
      a.bits = bits;
      a.words = words;
      a.agg_eid = ly.agg_eid;
      a.self_ptr = ly.self_ptr;
      a.self_eid = ly.self_eid;
    }
    for (int k = 0; k < ly.n_terms; ++k) {
      a.kind[k] = ly.terms[k].kind;
      a.rel[k] = ly.terms[k].rel;
      a.table[k] = ly.terms[k].table;
      a.dst_type[k] = ly.tgt_type ? ly.terms[k].dst_type : -1;
      XPG_REQ(a.kind[k] == XPG_TERM_ROOT || (a.rel[k] >= 0 && a.rel[k] < p->n_rel), "term: bad relation");
      XPG_REQ(!ly.tgt_type || a.dst_type[k] < ly.n_types, "term: destination type out of range");
    }
    float* hout = reinterpret_cast<float*>(ws + L.h[l]);
    if (l == 0) {
      a.width = ly.f_out_pad;
      a.out = hout;
      a.out_ld = ly.f_out_pad;
      a.bias = ly.bias;
      a.act = ly.act;
      a.f_real = ly.f_out;
      rc = launch_agg<true>(a, st);
      if (rc) return rc;
    } else {
      const xpg_layer_desc& prev = p->layers[l - 1];
      XPG_REQ(ly.f_in_pad == prev.f_out_pad, "layer: f_in_pad must equal previous f_out_pad");
      float* agg = reinterpret_cast<float*>(ws + L.agg);
      a.hprev = reinterpret_cast<const float*>(ws + L.h[l - 1]);
      a.width = ly.f_in_pad;
      a.out = agg;
      a.out_ld = (int64_t)ly.n_terms * ly.f_in_pad;
      rc = launch_agg<false>(a, st);
      if (rc) return rc;
      const bool fuse_here = fuse_out && p->n_head == 1 && l == p->n_layers - 1;
      rc = launch_dense(agg, rows * ly.n_tgt, a.out_ld, ly.weight, a.out_ld, a.out_ld, ly.bias, ly.f_out,
                        ly.f_out_pad, ly.act, hout, ly.f_out_pad, st, ly.tgt_type, ly.n_tgt, ly.f_out_pad,
                        fuse_here ? &fh : nullptr);
      if (rc) return rc;
    }
  }
  const xpg_layer_desc& last = p->layers[p->n_layers - 1];
  const int64_t M = rows * last.n_tgt;
  const float* cur = reinterpret_cast<const float*>(ws + L.h[p->n_layers - 1]);
  int64_t cur_ld = last.f_out_pad;
  const int n_head_launch = p->n_head - (fuse_out ? 1 : 0);  // the last head layer fused (fh)
  for (int i = 0; i < n_head_launch; ++i) {
    const xpg_head_desc& hd = p->head[i];
    XPG_REQ(hd.k_pad == cur_ld, "head: k_pad must equal the previous padded width");
    float* nxt = reinterpret_cast<float*>(ws + ((i & 1) ? L.head1 : L.head0));
    rc = launch_dense(cur, M, cur_ld, hd.weight, hd.k_pad, hd.k_pad, hd.bias, hd.n_real, hd.n_pad, hd.act, nxt,
                      hd.n_pad, st, nullptr, 1, 0, fuse_out && i == n_head_launch - 1 ? &fh : nullptr);
    if (rc) return rc;
    cur = nxt;
    cur_ld = hd.n_pad;
  }
  if (fuse_out) return XPG_OK;
  if (p->edge_dot) {
    const int n_real = p->n_head > 0 ? p->head[p->n_head - 1].n_real : last.f_out;
    XPG_REQ(p->dot_a >= 0 && p->dot_a < last.n_tgt && p->dot_b >= 0 && p->dot_b < last.n_tgt,
            "masked_forward: link decoder targets out of range");
    hipLaunchKernelGGL(k_edge_dot, dim3(static_cast<unsigned>(cdiv(rows, 256))), dim3(256), 0, st, cur, rows,
                       last.n_tgt, cur_ld, n_real, p->dot_a, p->dot_b, p->dot_act, y);
  } else {
    hipLaunchKernelGGL(k_take_col, dim3(static_cast<unsigned>(cdiv(M, 256))), dim3(256), 0, st, cur, M, cur_ld,
                       p->out_col, y);
  }
  XPG_LAUNCHED();
  return XPG_OK;
}

struct WlmWs {
  size_t steps_off, colbits_off, phist_off, whist_off, tglob_off, total;
  int bw, n_bs, n_ds;
  bool stage;
  size_t lds;
  // multi-workgroup fit
  bool mc, xcd;
  int P, wpp, mc_ds, mc_cpl, mc_stg;
  size_t xp_off, cnt_off, ep_off, lds_mc;
  // grid (many-column) fit
  bool grid;
  int n_wg, n_tk;
  size_t ppart_off, g_off, tk_off, aw_off, lds_p, lds_g;
  // fused grid fit (k_gw_fused): chunks per workgroup, padded row blocks, workgroups, LDS bytes
  bool gf;
  int gf_ch, gf_nrbp, gf_nwg;
  size_t gf_lds, gfx_off, gferr_off;
};

static bool wlm_env(const char* v) {
  const char* env = getenv("XPG_WLM");
  return env && std::strcmp(env, v) == 0;
}
static bool wlm_force_grid() { return wlm_env("grid") || wlm_env("grid3"); }


// Word slices per wave item: minimise (rounds of 16 waves) x (words per item + 1 for the item's
// fixed cost) over blocks x slices items.
static int wlm_slices(int64_t blocks, int words) {
  int best = 1;
  int64_t best_cost = INT64_MAX;
  for (int n = 1; n <= words; ++n) {
    const int64_t cost = cdiv(blocks * n, 16) * (cdiv(words, n) + 1);
    if (cost < best_cost) {
      best_cost = cost;
      best = n;
    }
  }
  return best;
}

// The fused grid fit takes a shape when a workgroup's waves can hold every 32-row block of its
// chunks in registers (two blocks per wave, 16 waves) and the chunks fit on the device's CUs one
// workgroup each; XPG_WLM=grid3 keeps the three-launch steps (A/B, tests).
static void wlm_plan_fused(int64_t rows, int64_t cols, int64_t batch, WlmWs* L) {
  L->gf = false;
  if (wlm_env("grid3")) return;
  const int64_t words = cdiv(cols, 32), n_chunks = cdiv(words, kGwWords);
  const int64_t nrb = cdiv(batch, 32);
  if (nrb > 32) return;
  const int nrbp = static_cast<int>(cdiv(nrb, kGfTpw) * kGfTpw), nwc = nrbp / kGfTpw;
  const int ch_max = std::min(kGfMaxCh, kGfWaves / nwc);
  if (ch_max < 1 || rows > INT32_MAX || cols > INT32_MAX) return;
  const int64_t cus = std::min(device_cus(), kGfMaxWg);
  const int64_t ch = cdiv(n_chunks, cus);
  if (ch > ch_max) return;
  const GfLds G = gf_lds(static_cast<int>(ch), nrbp);
  const size_t lds = sizeof(float) * (size_t)G.total + 2 * kGfWaves * sizeof(double) + sizeof(double);
  if (lds > 160 * 1024) return;
  L->gf = true;
  L->gf_ch = static_cast<int>(ch);
  L->gf_nrbp = nrbp;
  L->gf_nwg = static_cast<int>(cdiv(n_chunks, ch));
  L->gf_lds = std::max<size_t>(lds, 81 * 1024);  // > half the CU's LDS: one workgroup per CU
}

static int wlm_layout_grid(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, WlmWs* L) {
  const int64_t steps = cdiv(rows, batch);
  const int64_t words = cdiv(cols, 32);
  XPG_REQ(batch <= 8192, "wlm_fit: batch > 8192 rows is not supported by the many-column fit");
  L->grid = true;
  L->stage = false;
  L->n_wg = static_cast<int>(cdiv(words, kGwWords));
  L->n_tk = static_cast<int>(cdiv(batch, 64));
  L->lds_p = 0;  // static
  L->lds_g = sizeof(float) * (size_t)(((16 * ((((batch + 31) / 32) * 8) | 1) + 3) & ~3) + 32 * 65);
  wlm_plan_fused(rows, cols, batch, L);
  const int n_part = L->gf ? std::max(L->n_wg, L->gf_nwg) : L->n_wg;  // aw partials per step
  const int n_tkp = L->gf ? std::max(L->n_tk, L->gf_nwg) : L->n_tk;  // loss-term partials per step
  const size_t F = static_cast<size_t>(n_fits);
  size_t off = 0;
  L->steps_off = off;
  off += align_up(F * sizeof(WlmStep) * (size_t)steps);
  L->ppart_off = off;
  off += align_up(F * sizeof(float) * (size_t)L->n_wg * batch);
  L->g_off = off;
  off += align_up(F * sizeof(float) * (size_t)batch);
  L->phist_off = off;
  off += align_up(F * sizeof(float) * (size_t)rows);
  L->tk_off = off;
  off += align_up(F * sizeof(double) * (size_t)steps * n_tkp);
  L->aw_off = off;
  off += align_up(F * sizeof(double) * (size_t)steps * n_part);
  L->gfx_off = off;  // fused: per fit [batch][nwg] p granules + [batch] g granules
  off += align_up(L->gf ? F * sizeof(uint64_t) * (size_t)batch * (L->gf_nwg + 1) : 0);
  L->gferr_off = off;
  off += align_up(L->gf ? sizeof(uint32_t) : 0);
  L->total = off;
  return XPG_OK;
}

static int wlm_layout(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, WlmWs* L) {
  XPG_REQ(n_fits > 0 && rows > 0 && cols > 0 && batch > 0, "wlm_fit: bad arguments");
  XPG_REQ(batch <= 1 << 20, "wlm_fit: batch too large");
  L->grid = false;
  if (cols > 16 * 1024 || wlm_force_grid()) return wlm_layout_grid(n_fits, rows, cols, batch, L);
  const int64_t steps = cdiv(rows, batch);
  const int words = words_of(cols);
  L->bw = static_cast<int>(cdiv(batch, 32));
  L->n_bs = wlm_slices(cdiv(batch, 64), words);
  L->n_ds = wlm_slices(cdiv(cols, 64), L->bw);
  const int64_t cpad = (cols + 63) & ~int64_t(63);
  const size_t lds_cap = 150 * 1024;
  auto g_bytes = [&]() {  // G tables + partial sums, rounded to 8 B (the kernel's kb_off)
    return sizeof(float) * (size_t)((L->bw * 8 * kTabPitch + L->n_bs * batch + L->n_ds * cpad + 1) & ~int64_t(1));
  };
  while (g_bytes() > lds_cap && (L->n_bs > 1 || L->n_ds > 1)) {
    if (L->n_ds > 1) L->n_ds = 1;
    else L->n_bs = 1;
  }
  XPG_REQ(g_bytes() <= lds_cap, "wlm_fit: batch too large for the single-workgroup fit (LDS)");
  const size_t t_bytes = sizeof(float) * (size_t)words * 8 * kTabPitch;
  const size_t stage_bytes = sizeof(double) * (size_t)batch +
                             sizeof(uint32_t) * ((size_t)batch * (words | 1) + (size_t)cols * (L->bw | 1));
  L->stage = g_bytes() + t_bytes + stage_bytes <= lds_cap && (int64_t)batch * words <= kStage * 1024 &&
             cols * (int64_t)L->bw <= kStage * 1024;
  L->lds = g_bytes() + (L->stage ? t_bytes + stage_bytes : 0);
  // multi-workgroup fit: P workgroups (one per CU, all co-resident) per fit
  L->mc = false;
  if (!wlm_env("single") && (words >= 8 || wlm_env("mc")) && batch <= 1024) {
    L->xcd = true;
    // up to 16 parts (the exchange is one poll round); more only when the staging budget asks
    // for them (the loop below, at most kMcMaxP)
    int P = std::min(kMcPollRound, std::max(2, static_cast<int>(cdiv(words, 3))));
    // stagers: the waves past the B / poll waves when batch <= 512 (k_wlm_fit_mc's split_stage)
    const int64_t nrb = cdiv(batch, 64), ns = nrb <= 8 ? 1024 - 64 * nrb : 1024;
    // the staged rows / column vectors must fit kMcMaxStage words per stager: more parts if not
    while (P < kMcMaxP && std::max<int64_t>(batch, 32 * L->bw) * cdiv(words, P) > kMcMaxStage * ns) ++P;
    while (P > 1 && (L->xcd ? cdiv(n_fits, device_xcds()) * P > device_cus() / device_xcds() : n_fits * P > device_cus()))
      --P;
    if (P >= 2) {
      const int wpp = static_cast<int>(cdiv(words, P));
      P = static_cast<int>(cdiv(words, wpp));
      // slices of the column row words per D lane.  A SIMD issues the waves of ceil(chunks / 4)
      // chunks, each ~4 instructions per lookup plus ~100 for Adam, the T quad and the loop, plus
      // the xor reduction; each lane's lookups also wait one LDS round trip (~400 cycles) per 16
      // in flight (probe-measured on the c2 fit); at most 4 column chunks per wave
      int nd_best = 0, cpl_best = 0;
      int64_t cost_best = INT64_MAX;
      for (int nd = 1, lg = 0; nd <= 16; nd <<= 1, ++lg) {
        const int64_t chunks = cdiv((int64_t)wpp * 32, 64 / nd), cpl = cdiv(chunks, 16);
        if (cpl > 4) continue;
        const int64_t look = cdiv(L->bw, nd) * 8;
        const int64_t cost = cdiv(chunks, 4) * (look * 4 + 100 + 10 * lg) + cdiv(look, 16) * 400;
        if (cost < cost_best) {
          cost_best = cost;
          nd_best = nd;
          cpl_best = static_cast<int>(cpl == 3 ? 4 : cpl);
        }
      }
      const int64_t stage = std::max<int64_t>(batch * wpp, (int64_t)wpp * 32 * L->bw);
      int stg = static_cast<int>(cdiv(stage, ns));
      stg = stg <= 1 ? 1 : stg <= 2 ? 2 : 4;
      const size_t lds = sizeof(float) * (size_t)((L->bw * 8 * kTabPitch + 1) & ~int64_t(1)) +
                         sizeof(double) * (size_t)batch + sizeof(float) * (size_t)wpp * 8 * kTabPitch +
                         sizeof(uint32_t) * ((size_t)batch * (wpp | 1) + 2 * (size_t)wpp * 32 * (L->bw | 1));
      if (nd_best > 0 && lds <= lds_cap && stage <= kMcMaxStage * ns) {
        L->mc = true;
        L->P = P;
        L->wpp = wpp;
        L->mc_ds = nd_best;
        L->mc_cpl = cpl_best;
        L->mc_stg = stg;
        L->lds_mc = std::max<size_t>(lds, 81 * 1024);  // > half the CU's LDS: one workgroup per CU
      }
    }
  }
  const size_t F = static_cast<size_t>(n_fits);
  size_t off = 0;
  L->steps_off = off;
  off += align_up(F * sizeof(WlmStep) * (size_t)steps);
  L->colbits_off = off;
  off += align_up(F * sizeof(uint32_t) * (size_t)steps * cols * L->bw);
  L->phist_off = off;
  off += align_up(F * sizeof(float) * (size_t)rows);
  L->whist_off = off;
  off += align_up(F * sizeof(float) * (size_t)steps * cols);
  L->tglob_off = off;
  off += align_up(L->stage ? 0 : F * t_bytes);
  L->xp_off = off;
  off += align_up(L->mc ? F * sizeof(uint64_t) * (2 * L->P * (size_t)batch + L->P) : 0);
  L->cnt_off = off;  // [F] (unused) + error word + [F] loss arrival counters
  off += align_up(sizeof(uint32_t) * (2 * F + 1));
  L->ep_off = off;   // device epoch word (not cleared)
  off += align_up(sizeof(uint32_t));
  L->total = off;
  return XPG_OK;
}

static int wlm_fit_grid(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                        const float* y, const double* kernel, const xpg_wlm_params& P, int64_t step0, float* w,
                        float* adam_m, float* adam_v, double* losses, int32_t* best_epoch, int32_t* status, char* ws,
                        const WlmWs& L, hipStream_t st) {
  const int64_t steps = cdiv(rows, batch);
  const int64_t words = cdiv(cols, 32);
  const int ib = static_cast<int>(batch);
  const unsigned nf = static_cast<unsigned>(n_fits);
  WlmStep* stp = reinterpret_cast<WlmStep*>(ws + L.steps_off);
  float* p_part = reinterpret_cast<float*>(ws + L.ppart_off);
  float* g = reinterpret_cast<float*>(ws + L.g_off);
  float* p_hist = reinterpret_cast<float*>(ws + L.phist_off);
  double* tk_part = reinterpret_cast<double*>(ws + L.tk_off);
  double* aw_part = reinterpret_cast<double*>(ws + L.aw_off);
  if (L.gf) {
    uint64_t* gx = reinterpret_cast<uint64_t*>(ws + L.gfx_off);
    uint32_t* err = reinterpret_cast<uint32_t*>(ws + L.gferr_off);
    const int64_t n_gx = (int64_t)batch * (L.gf_nwg + 1);
    // per-step constants + granule / error-word clearing, one launch
    hipLaunchKernelGGL(k_wlm_stats, dim3(static_cast<unsigned>(steps), nf), dim3(256), 0, st, y, kernel, rows, ib,
                       P, step0, stp, gx, n_gx * n_fits, err, 1);
    XPG_LAUNCHED();
    // test hooks (diagnostics switches, as the multi-workgroup fit): XPG_MC_SPIN (poll bound),
    // XPG_MC_FAULT = k >= 1 (workgroup k - 1 of fit 0 skips its first publish)
    int spin_env = 0, fault_env = 0;
    if (const int rc = diag_env("XPG_MC_SPIN", &spin_env)) return rc;
    if (const int rc = diag_env("XPG_MC_FAULT", &fault_env)) return rc;
    XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_gw_fused)));
    for (int64_t f = 0; f < n_fits; ++f) {  // one persistent launch per fit, in stream order
      GfArgs a;
      a.bits = bits + f * rows * words;
      a.rows = static_cast<int>(rows);
      a.cols = static_cast<int>(cols);
      a.words = static_cast<int>(words);
      a.steps = static_cast<int>(steps);
      a.batch = ib;
      a.ch = L.gf_ch;
      a.nrbp = L.gf_nrbp;
      a.nwg = L.gf_nwg;
      a.fault_wg = (f == 0 && fault_env > 0) ? fault_env - 1 : -1;
      a.spin_limit = spin_env > 0 ? static_cast<uint32_t>(spin_env) : kMcSpinLimit;
      a.kern = kernel + f * rows;
      a.stp = stp + f * steps;
      a.P = P;
      a.wg = w + f * cols;
      a.mg = adam_m + f * cols;
      a.vg = adam_v + f * cols;
      a.p_hist = p_hist + f * rows;
      a.tk_part = tk_part + f * steps * L.gf_nwg;
      a.aw_part = aw_part + f * steps * L.gf_nwg;
      a.xp = gx + f * n_gx;
      a.err = err;
      hipLaunchKernelGGL(k_gw_fused, dim3(static_cast<unsigned>(L.gf_nwg)), dim3(kGfThreads), L.gf_lds, st, a);
      XPG_LAUNCHED();
    }
    hipLaunchKernelGGL(k_gw_loss, dim3(static_cast<unsigned>(steps), nf), dim3(64), 0, st, tk_part, L.gf_nwg,
                       aw_part, L.gf_nwg, stp, rows, cols, ib, P.l1_lambda, losses);
    XPG_LAUNCHED();
    hipLaunchKernelGGL(k_argmin_first, dim3(nf), dim3(64), 0, st, losses, steps, best_epoch, err, status);
    XPG_LAUNCHED();
    return XPG_OK;
  }
  hipLaunchKernelGGL(k_wlm_stats, dim3(static_cast<unsigned>(steps), nf), dim3(256), 0, st, y, kernel, rows, ib, P,
                     step0, stp, nullptr, int64_t(0), nullptr, 0);
  XPG_LAUNCHED();
  XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_gw_grad)));
  const dim3 gw(static_cast<unsigned>(L.n_wg), nf);
  for (int64_t t = 0; t < steps; ++t) {
    hipLaunchKernelGGL(k_gw_p, gw, dim3(kGpWaves * 64), 0, st, bits, rows, cols, words, ib, t, w, p_part);
    XPG_LAUNCHED();
    hipLaunchKernelGGL(k_gw_g, dim3(static_cast<unsigned>(L.n_tk), nf), dim3(1024), 0, st, p_part, L.n_wg, rows, ib,
                       t, kernel, stp, steps, g, p_hist, tk_part);
    XPG_LAUNCHED();
    hipLaunchKernelGGL(k_gw_grad, gw, dim3(kGgWaves * 64), L.lds_g, st, bits, rows, cols, words, ib, t, g, stp, steps,
                       P, w, adam_m, adam_v, aw_part);
    XPG_LAUNCHED();
  }
  hipLaunchKernelGGL(k_gw_loss, dim3(static_cast<unsigned>(steps), nf), dim3(64), 0, st, tk_part, L.n_tk, aw_part,
                     L.n_wg, stp, rows, cols, ib, P.l1_lambda, losses);
  XPG_LAUNCHED();
  hipLaunchKernelGGL(k_argmin_first, dim3(nf), dim3(64), 0, st, losses, steps, best_epoch, nullptr, status);
  XPG_LAUNCHED();
  return XPG_OK;
}

int xpg_wlm_workspace(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, size_t* bytes) {
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  *bytes = L.total;
  return XPG_OK;
}

int xpg_wlm_plan(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, int32_t* kind, int32_t* parts) {
  XPG_REQ(kind != nullptr && parts != nullptr, "wlm_plan: null output");
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  *kind = L.grid ? (L.gf ? XPG_WLM_GRID_FUSED : XPG_WLM_GRID) : (L.mc ? XPG_WLM_MULTI : XPG_WLM_SINGLE);
  *parts = L.grid ? (L.gf ? L.gf_nwg : 1) : (L.mc ? L.P : 1);
  return XPG_OK;
}

static int wlm_fit_impl(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                        const float* y, const double* kernel, const xpg_wlm_params* params, int64_t step0,
                        const float* w0, float* w, float* adam_m, float* adam_v, double* losses,
                        int32_t* best_epoch, int32_t* status, void* workspace, size_t workspace_bytes,
                        xpg_stream_t stream);
static int wlm_launch_prep(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                           const float* y, const double* kernel, const xpg_wlm_params* params, int64_t step0,
                           const float* w0, float* w, float* adam_m, float* adam_v, char* ws, const WlmWs& L,
                           hipStream_t st);
static int wlm_launch_fit(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                          const double* kernel, const xpg_wlm_params* params, float* w, float* adam_m, float* adam_v,
                          double* losses, int32_t* best_epoch, int32_t* status, char* ws, const WlmWs& L,
                          hipStream_t st, int which = 3);

int xpg_wlm_prepare(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                    const float* y, const double* kernel, const xpg_wlm_params* params, const float* w0,
                    float* w, float* adam_m, float* adam_v, void* workspace, size_t workspace_bytes,
                    xpg_stream_t stream) {
  XPG_REQ(params != nullptr && w0 != nullptr, "wlm_prepare: params and w0 required");
  XPG_REQ(n_fits <= 65535, "wlm_fit: at most 65535 fits per launch");
  XPG_REQ(rows / std::max<int64_t>(batch, 1) < 65535, "wlm_fit: at most 65534 steps per fit");
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  XPG_REQ(workspace_bytes >= L.total, "wlm_fit: workspace too small");
  XPG_REQ(!L.grid, "wlm_prepare: this shape takes the grid fit (no prologue kernel); use xpg_wlm_fit_from");
  return wlm_launch_prep(n_fits, bits, rows, cols, batch, y, kernel, params, 0, w0, w, adam_m, adam_v,
                         static_cast<char*>(workspace), L, S(stream));
}

int xpg_wlm_fit_prepared(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                         const double* kernel, const xpg_wlm_params* params, float* w, float* adam_m,
                         float* adam_v, double* losses, int32_t* best_epoch, int32_t* status, void* workspace,
                         size_t workspace_bytes, xpg_stream_t stream) {
  XPG_REQ(params != nullptr, "wlm_fit: params required");
  XPG_REQ(n_fits <= 65535, "wlm_fit: at most 65535 fits per launch");
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  XPG_REQ(workspace_bytes >= L.total, "wlm_fit: workspace too small");
  XPG_REQ(!L.grid, "wlm_fit_prepared: this shape takes the grid fit; use xpg_wlm_fit_from");
  return wlm_launch_fit(n_fits, bits, rows, cols, batch, kernel, params, w, adam_m, adam_v, losses, best_epoch,
                        status, static_cast<char*>(workspace), L, S(stream));
}

static int wlm_prepared_part(int which, int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols,
                             int64_t batch, const double* kernel, const xpg_wlm_params* params, float* w,
                             float* adam_m, float* adam_v, double* losses, int32_t* best_epoch, int32_t* status,
                             void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  XPG_REQ(params != nullptr, "wlm_fit: params required");
  XPG_REQ(n_fits <= 65535, "wlm_fit: at most 65535 fits per launch");
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  XPG_REQ(workspace_bytes >= L.total, "wlm_fit: workspace too small");
  XPG_REQ(!L.grid, "wlm_fit_steps / wlm_fit_losses: this shape takes the grid fit; use xpg_wlm_fit_from");
  return wlm_launch_fit(n_fits, bits, rows, cols, batch, kernel, params, w, adam_m, adam_v, losses, best_epoch,
                        status, static_cast<char*>(workspace), L, S(stream), which);
}

int xpg_wlm_fit_steps(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                      const double* kernel, const xpg_wlm_params* params, float* w, float* adam_m, float* adam_v,
                      void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  return wlm_prepared_part(1, n_fits, bits, rows, cols, batch, kernel, params, w, adam_m, adam_v, nullptr, nullptr,
                           nullptr, workspace, workspace_bytes, stream);
}

int xpg_wlm_fit_losses(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, const double* kernel,
                       const xpg_wlm_params* params, double* losses, int32_t* best_epoch, int32_t* status,
                       void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  XPG_REQ(losses && best_epoch, "wlm_fit_losses: losses and best_epoch required");
  return wlm_prepared_part(2, n_fits, nullptr, rows, cols, batch, kernel, params, nullptr, nullptr, nullptr, losses,
                           best_epoch, status, workspace, workspace_bytes, stream);
}

int xpg_wlm_fit(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                const float* y, const double* kernel, const xpg_wlm_params* params, int64_t step0,
                float* w, float* adam_m, float* adam_v, double* losses, int32_t* best_epoch,
                int32_t* status, void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  return wlm_fit_impl(n_fits, bits, rows, cols, batch, y, kernel, params, step0, nullptr, w, adam_m, adam_v,
                      losses, best_epoch, status, workspace, workspace_bytes, stream);
}

int xpg_wlm_fit_from(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                     const float* y, const double* kernel, const xpg_wlm_params* params, const float* w0,
                     float* w, float* adam_m, float* adam_v, double* losses, int32_t* best_epoch,
                     int32_t* status, void* workspace, size_t workspace_bytes, xpg_stream_t stream) {
  XPG_REQ(w0 != nullptr, "wlm_fit_from: w0 required");
  return wlm_fit_impl(n_fits, bits, rows, cols, batch, y, kernel, params, 0, w0, w, adam_m, adam_v, losses,
                      best_epoch, status, workspace, workspace_bytes, stream);
}

static int wlm_fit_impl(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                        const float* y, const double* kernel, const xpg_wlm_params* params, int64_t step0,
                        const float* w0, float* w, float* adam_m, float* adam_v, double* losses,
                        int32_t* best_epoch, int32_t* status, void* workspace, size_t workspace_bytes,
                        xpg_stream_t stream) {
  XPG_REQ(params != nullptr, "wlm_fit: params required");
  XPG_REQ(n_fits <= 65535, "wlm_fit: at most 65535 fits per launch");
  XPG_REQ(rows / std::max<int64_t>(batch, 1) < 65535, "wlm_fit: at most 65534 steps per fit");
  WlmWs L;
  int rc = wlm_layout(n_fits, rows, cols, batch, &L);
  if (rc) return rc;
  XPG_REQ(workspace_bytes >= L.total, "wlm_fit: workspace too small");
  hipStream_t st = S(stream);
  char* ws = static_cast<char*>(workspace);
  if (L.grid) {
    if (w0) {  // the grid fit has no prologue kernel: stream-ordered copy / clears
      const size_t nb = sizeof(float) * (size_t)n_fits * (size_t)cols;
      XPG_HIP(hipMemcpyAsync(w, w0, nb, hipMemcpyDeviceToDevice, st));
      XPG_HIP(hipMemsetAsync(adam_m, 0, nb, st));
      XPG_HIP(hipMemsetAsync(adam_v, 0, nb, st));
    }
    return wlm_fit_grid(n_fits, bits, rows, cols, batch, y, kernel, *params, step0, w, adam_m, adam_v,
                        losses, best_epoch, status, ws, L, st);
  }
  int rc2 = wlm_launch_prep(n_fits, bits, rows, cols, batch, y, kernel, params, step0, w0, w, adam_m, adam_v, ws, L,
                            st);
  if (rc2) return rc2;
  return wlm_launch_fit(n_fits, bits, rows, cols, batch, kernel, params, w, adam_m, adam_v, losses, best_epoch,
                        status, ws, L, st);
}

// k_wlm_prep: the per-step constants (+ exchange slot clearing, epoch advance, optional fresh
// start w = w0, m = v = 0) and the column bit vectors, one launch
static int wlm_launch_prep(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                           const float* y, const double* kernel, const xpg_wlm_params* params, int64_t step0,
                           const float* w0, float* w, float* adam_m, float* adam_v, char* ws, const WlmWs& L,
                           hipStream_t st) {
  WlmStep* stp = reinterpret_cast<WlmStep*>(ws + L.steps_off);
  uint32_t* colbits = reinterpret_cast<uint32_t*>(ws + L.colbits_off);
  const int64_t steps = cdiv(rows, batch);
  const int words = words_of(cols);
  const int ic = static_cast<int>(cols), ib = static_cast<int>(batch);
  const unsigned nf = static_cast<unsigned>(n_fits);
  // the multi-workgroup fit's exchange slots and error words are cleared by k_wlm_prep
  const int64_t n_xp = L.mc ? n_fits * (2 * L.P * batch + L.P) : 0;
  const int64_t lanes = steps * L.bw * words;
  hipLaunchKernelGGL(k_wlm_prep, dim3(static_cast<unsigned>(steps + cdiv(lanes, 256)), nf), dim3(256), 0, st, y,
                     kernel, bits, rows, ic, words, ib, L.bw, steps, *params, step0, stp, colbits,
                     L.mc ? reinterpret_cast<uint64_t*>(ws + L.xp_off) : nullptr, n_xp,
                     reinterpret_cast<uint32_t*>(ws + L.cnt_off), static_cast<int>(2 * n_fits + 1),
                     reinterpret_cast<uint32_t*>(ws + L.ep_off), w0, w, adam_m, adam_v, n_fits * cols);
  XPG_LAUNCHED();
  return XPG_OK;
}

// the fit proper (multi-workgroup or one-workgroup kernel) + losses / best epoch / status, on a
// workspace k_wlm_prep has prepared
// which: 1 = the Adam steps (fit kernel), 2 = losses / best epoch / status (k_wlm_loss_best),
// 3 = both in stream order
static int wlm_launch_fit(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                          const double* kernel, const xpg_wlm_params* params, float* w, float* adam_m, float* adam_v,
                          double* losses, int32_t* best_epoch, int32_t* status, char* ws, const WlmWs& L,
                          hipStream_t st, int which) {
  WlmStep* stp = reinterpret_cast<WlmStep*>(ws + L.steps_off);
  uint32_t* colbits = reinterpret_cast<uint32_t*>(ws + L.colbits_off);
  float* p_hist = reinterpret_cast<float*>(ws + L.phist_off);
  float* w_hist = reinterpret_cast<float*>(ws + L.whist_off);
  float* t_glob = reinterpret_cast<float*>(ws + L.tglob_off);
  const int64_t steps = cdiv(rows, batch);
  const int words = words_of(cols);
  const int ic = static_cast<int>(cols), ib = static_cast<int>(batch);
  const unsigned nf = static_cast<unsigned>(n_fits);
  bool launched = (which & 1) == 0;
  // the multi-workgroup exchange's error word (nonzero: a partner's poll timed out, the weights
  // are invalid) reaches the caller's status through k_wlm_loss_best
  const uint32_t* errw = L.mc ? reinterpret_cast<uint32_t*>(ws + L.cnt_off) + n_fits : nullptr;
  if (L.mc && (which & 1)) {
    uint32_t* cnt = reinterpret_cast<uint32_t*>(ws + L.cnt_off);
    uint64_t* xp = reinterpret_cast<uint64_t*>(ws + L.xp_off);
    // granule tags carry a per-call epoch (stale cache lines of earlier calls never match)
    static uint32_t epoch = 0;
    epoch = (epoch + 1) & 0xFFFFu;
    if (epoch == 0) epoch = 1;
    const int plain_ok = 1;
    // test hooks (diagnostics switches): XPG_MC_SPIN (poll bound), XPG_MC_FAULT = k >= 1 (part k
    // of fit 0 skips its first publish)
    int spin_env = 0, fault_env = 0;
    if (const int rc = diag_env("XPG_MC_SPIN", &spin_env)) return rc;
    if (const int rc = diag_env("XPG_MC_FAULT", &fault_env)) return rc;
    const uint32_t spin = spin_env > 0 ? static_cast<uint32_t>(spin_env) : kMcSpinLimit;
    const int fault = fault_env > 0 ? fault_env : -1;
    const dim3 grid(static_cast<unsigned>(L.xcd ? 8 * L.P * cdiv(n_fits, 8) : n_fits * L.P));
#define XPG_WLM_MC(C, G)                                                                                    \
    if (!launched && L.mc_cpl == C && L.mc_stg == G) {                                                      \
      XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_wlm_fit_mc<C, G>))); \
      hipLaunchKernelGGL((k_wlm_fit_mc<C, G>), grid, dim3(1024), L.lds_mc, st, bits, colbits, rows, ic, words, ib, \
                         L.bw, L.P, L.wpp, L.mc_ds, n_fits, L.xcd ? 1 : 0, kernel, stp, *params, w, adam_m,      \
                         adam_v, p_hist, w_hist, xp, cnt + n_fits, spin, fault, epoch, plain_ok,             \
                         reinterpret_cast<const uint32_t*>(ws + L.ep_off));                                  \
      XPG_LAUNCHED();                                                                                       \
      launched = true;                                                                                      \
    }
    XPG_WLM_MC(1, 1) XPG_WLM_MC(1, 2) XPG_WLM_MC(1, 4)
    XPG_WLM_MC(2, 1) XPG_WLM_MC(2, 2) XPG_WLM_MC(2, 4)
    XPG_WLM_MC(4, 1) XPG_WLM_MC(4, 2) XPG_WLM_MC(4, 4)
#undef XPG_WLM_MC
    if (!launched) return fail(XPG_EINVAL, "wlm_fit: unsupported slice width");
  }
  const int cpt = static_cast<int>(cdiv(cols, 1024));
#define XPG_WLM(C, TL)                                                                                     \
  if (!launched && cpt <= C && L.stage == TL) {                                                                      \
    XPG_HIP(lds_limit(reinterpret_cast<const void*>(&k_wlm_fit<C, TL>)));     \
    hipLaunchKernelGGL((k_wlm_fit<C, TL>), dim3(nf), dim3(1024), L.lds, st, bits, colbits, rows, ic, words, \
                       ib, L.bw, L.n_bs, L.n_ds, kernel, stp, *params, w, adam_m, adam_v, p_hist, w_hist,  \
                       t_glob);                                                                            \
    XPG_LAUNCHED();                                                                                        \
    launched = true;                                                                                       \
  }
  XPG_WLM(1, true) XPG_WLM(2, true) XPG_WLM(4, true) XPG_WLM(8, true) XPG_WLM(16, true)
  XPG_WLM(1, false) XPG_WLM(2, false) XPG_WLM(4, false) XPG_WLM(8, false) XPG_WLM(16, false)
#undef XPG_WLM
  if (!launched) return fail(XPG_EINVAL, "wlm_fit: unsupported column count");
  if (!(which & 2)) return XPG_OK;
  // one launch: every step's loss and the first best epoch (+ the exchange status word)
  hipLaunchKernelGGL(k_wlm_loss_best, dim3(static_cast<unsigned>(steps), nf), dim3(256), 0, st, p_hist, w_hist,
                     kernel, stp, rows, ic, ib, params->l1_lambda, losses, best_epoch,
                     reinterpret_cast<uint32_t*>(ws + L.cnt_off) + n_fits + 1, errw, status);
  XPG_LAUNCHED();
  return XPG_OK;
}

}  // extern "C"

#include "khop.hip"

