// host_rng.h — torch's CPU generator replayed natively for the compat mask sampler (host code).
//
// The reference draws Shapley masks as torch.randint(0, 2, (rows, cols), dtype=torch.bool) on the
// CPU (masks.py:231-260).  ATen's CPU generator is MT19937 (at::mt19937: state_[624], left_,
// next_; each element consumes one 32-bit output `operator()()` in row-major order, and the bool
// value is output % 2).  Replayed element by element through torch this costs ~5 ns per element
// plus a bool [rows, cols] tensor and its row gather; here the same outputs are produced from the
// generator's own state and written straight as bit-packed rows, then the state is handed back.
//
// The output's low bit is linear in the untempered state word y: tempering is
//   y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680; y ^= (y << 15) & 0xefc60000; y ^= y >> 18
// and following bit 0 through it gives bit0 = y0 ^ y3 ^ y14 ^ y18 ^ y22 ^ y29, the parity of
// y & 0x20444009 — no tempering per element, one AND + popcount.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <cmath>
#include <vector>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>  // SSE2 (x86-64 baseline) + AVX2 paths behind a CPU check: host code only
#endif

namespace hostrng {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
constexpr uint32_t kLsbTaps = 0x20444009u;

inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & kUpper) | (v & kLower)) >> 1) ^ ((0u - (v & 1u)) & kMatrixA);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// AVX2 (8 words per op) where the CPU has it: the regeneration and the low-bit extraction are
// ~60 % of the compat sampler's host time (c2: 15.3 M outputs per repeat)
// XPG_HOST_SIMD = sse2 | avx2 | avx512 caps the level (the CPU tests run every path); read once
inline int simd_cap() {
  static const int v = [] {
    const char* e = getenv("XPG_HOST_SIMD");
    if (!e) return 3;
    return std::strcmp(e, "sse2") == 0 ? 0 : std::strcmp(e, "avx2") == 0 ? 1 : std::strcmp(e, "avx512") == 0 ? 2 : 3;
  }();
  return v;
}

inline bool have_avx2() {
  static const int v = simd_cap() >= 1 && __builtin_cpu_supports("avx2") ? 1 : 0;
  return v != 0;
}

__attribute__((target("avx2"))) inline __m256i twist8(__m256i u, __m256i v) {
  const __m256i y = _mm256_or_si256(_mm256_and_si256(u, _mm256_set1_epi32(static_cast<int>(kUpper))),
                                    _mm256_and_si256(v, _mm256_set1_epi32(static_cast<int>(kLower))));
  const __m256i odd = _mm256_sub_epi32(_mm256_setzero_si256(), _mm256_and_si256(v, _mm256_set1_epi32(1)));
  return _mm256_xor_si256(_mm256_srli_epi32(y, 1),
                          _mm256_and_si256(odd, _mm256_set1_epi32(static_cast<int>(kMatrixA))));
}

// next_state below, 8 words at a time: a block reads s[i + 1 .. i + 8] before it writes s[i .. i + 7]
// (the originals the recurrence wants) and s[i - 227 ..] that earlier blocks wrote
__attribute__((target("avx2"))) inline void next_state_avx2(uint32_t* s) {
  int i = 0;
  for (; i + 8 <= kN - kM; i += 8) {
    const __m256i u = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 1));
    const __m256i m = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + kM));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(s + i), _mm256_xor_si256(m, twist8(u, v)));
  }
  for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ twist(s[i], s[i + 1]);
  for (; i + 8 <= kN - 1; i += 8) {
    const __m256i u = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 1));
    const __m256i m = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + kM - kN));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(s + i), _mm256_xor_si256(m, twist8(u, v)));
  }
  for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ twist(s[i], s[i + 1]);
  s[kN - 1] = s[kM - 1] ^ twist(s[kN - 1], s[0]);
}

// the low bits of 32 consecutive outputs s[0 .. 32) as one word (the parity trick of emit_lsb)
// nw words of 32 low bits each (out[k] = outputs s[32k .. 32k + 32)); one call per regeneration
// chunk (a target-specific function is not inlined into a baseline caller)
__attribute__((target("avx2"))) inline void lsb_words_avx2(const uint32_t* s, int nw, uint32_t* out) {
  for (int k = 0; k < nw; ++k, s += 32) {
  uint32_t w = 0u;
  for (int q = 0; q < 4; ++q) {
    const __m256i y = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 8 * q));
    __m256i v = _mm256_xor_si256(y, _mm256_srli_epi32(y, 3));
    v = _mm256_xor_si256(v, _mm256_srli_epi32(y, 14));
    v = _mm256_xor_si256(v, _mm256_srli_epi32(y, 18));
    v = _mm256_xor_si256(v, _mm256_srli_epi32(y, 22));
    v = _mm256_xor_si256(v, _mm256_srli_epi32(y, 29));
    w |= static_cast<uint32_t>(_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_slli_epi32(v, 31)))) << (8 * q);
  }
  out[k] = w;
  }
}

// AVX-512 (16 words per op: F + DQ for the sign-bit mask)
inline bool have_avx512() {
  static const int v = simd_cap() >= 2 && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") ? 1 : 0;
  return v != 0;
}

__attribute__((target("avx512f,avx512dq"))) inline __m512i twist16(__m512i u, __m512i v) {
  const __m512i y = _mm512_or_si512(_mm512_and_si512(u, _mm512_set1_epi32(static_cast<int>(kUpper))),
                                    _mm512_and_si512(v, _mm512_set1_epi32(static_cast<int>(kLower))));
  const __m512i odd = _mm512_sub_epi32(_mm512_setzero_si512(), _mm512_and_si512(v, _mm512_set1_epi32(1)));
  return _mm512_xor_si512(_mm512_srli_epi32(y, 1),
                          _mm512_and_si512(odd, _mm512_set1_epi32(static_cast<int>(kMatrixA))));
}

__attribute__((target("avx512f,avx512dq"))) inline void next_state_avx512(uint32_t* s) {
  int i = 0;
  for (; i + 16 <= kN - kM; i += 16) {
    const __m512i u = _mm512_loadu_si512(s + i);
    const __m512i v = _mm512_loadu_si512(s + i + 1);
    const __m512i m = _mm512_loadu_si512(s + i + kM);
    _mm512_storeu_si512(s + i, _mm512_xor_si512(m, twist16(u, v)));
  }
  for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ twist(s[i], s[i + 1]);
  for (; i + 16 <= kN - 1; i += 16) {
    const __m512i u = _mm512_loadu_si512(s + i);
    const __m512i v = _mm512_loadu_si512(s + i + 1);
    const __m512i m = _mm512_loadu_si512(s + i + kM - kN);
    _mm512_storeu_si512(s + i, _mm512_xor_si512(m, twist16(u, v)));
  }
  for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ twist(s[i], s[i + 1]);
  s[kN - 1] = s[kM - 1] ^ twist(s[kN - 1], s[0]);
}

inline bool have_vpopcnt() {
  static const int v = simd_cap() >= 3 && have_avx512() && __builtin_cpu_supports("avx512vpopcntdq") ? 1 : 0;
  return v != 0;
}

// with VPOPCNTDQ: the low bit is popcount(y & taps) & 1, one test per 16 outputs
__attribute__((target("avx512f,avx512dq,avx512vpopcntdq"))) inline void lsb_words_popcnt(const uint32_t* s, int nw,
                                                                                        uint32_t* out) {
  const __m512i taps = _mm512_set1_epi32(static_cast<int>(kLsbTaps)), one = _mm512_set1_epi32(1);
  for (int k = 0; k < nw; ++k, s += 32) {
    const __m512i a = _mm512_popcnt_epi32(_mm512_and_si512(_mm512_loadu_si512(s), taps));
    const __m512i b = _mm512_popcnt_epi32(_mm512_and_si512(_mm512_loadu_si512(s + 16), taps));
    out[k] = static_cast<uint32_t>(_mm512_test_epi32_mask(a, one)) |
             (static_cast<uint32_t>(_mm512_test_epi32_mask(b, one)) << 16);
  }
}

__attribute__((target("avx512f,avx512dq"))) inline void lsb_words_avx512(const uint32_t* s, int nw, uint32_t* out) {
  for (int k = 0; k < nw; ++k, s += 32) {
  uint32_t w = 0u;
  for (int q = 0; q < 2; ++q) {
    const __m512i y = _mm512_loadu_si512(s + 16 * q);
    __m512i v = _mm512_xor_si512(y, _mm512_srli_epi32(y, 3));
    v = _mm512_xor_si512(v, _mm512_srli_epi32(y, 14));
    v = _mm512_xor_si512(v, _mm512_srli_epi32(y, 18));
    v = _mm512_xor_si512(v, _mm512_srli_epi32(y, 22));
    v = _mm512_xor_si512(v, _mm512_srli_epi32(y, 29));
    w |= static_cast<uint32_t>(_mm512_movepi32_mask(_mm512_slli_epi32(v, 31))) << (16 * q);
  }
  out[k] = w;
  }
}
#endif

// at::mt19937::next_state (the standard MT19937 regeneration, in place)
inline void next_state(uint32_t* s) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (have_avx512()) {
    next_state_avx512(s);
    return;
  }
  if (have_avx2()) {
    next_state_avx2(s);
    return;
  }
#endif
  int i = 0;
  for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ twist(s[i], s[i + 1]);
  for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ twist(s[i], s[i + 1]);
  s[kN - 1] = s[kM - 1] ^ twist(s[kN - 1], s[0]);
}

// low bits of words s[i0 .. i0 + n) appended to the packed stream at bit position *pos
inline void emit_lsb(const uint32_t* s, int i0, int n, uint32_t* stream, int64_t* pos) {
  int64_t p = *pos;
  int j = 0;
  while (j < n && (p & 31)) {  // up to the next stream word
    stream[p >> 5] |= static_cast<uint32_t>(__builtin_parity(s[i0 + j] & kLsbTaps)) << (p & 31);
    ++j;
    ++p;
  }
#if !defined(__HIP_DEVICE_COMPILE__)
  // whole words, 4 outputs per SSE2 op (8 per AVX2 op): bit0 of y ^ y>>3 ^ y>>14 ^ y>>18 ^
  // y>>22 ^ y>>29 is the parity above; movemask collects the low bits (shifted to the sign bits)
  if ((have_avx512() || have_avx2()) && j + 32 <= n) {
    const int nw = (n - j) / 32;  // p is word-aligned here
    if (have_vpopcnt())
      lsb_words_popcnt(s + i0 + j, nw, stream + (p >> 5));
    else if (have_avx512())
      lsb_words_avx512(s + i0 + j, nw, stream + (p >> 5));
    else
      lsb_words_avx2(s + i0 + j, nw, stream + (p >> 5));
    j += 32 * nw;
    p += 32 * nw;
  }
  for (; j + 32 <= n; j += 32, p += 32) {
    uint32_t w = 0u;
    for (int q = 0; q < 8; ++q) {
      const __m128i y = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i0 + j + 4 * q));
      __m128i v = _mm_xor_si128(y, _mm_srli_epi32(y, 3));
      v = _mm_xor_si128(v, _mm_srli_epi32(y, 14));
      v = _mm_xor_si128(v, _mm_srli_epi32(y, 18));
      v = _mm_xor_si128(v, _mm_srli_epi32(y, 22));
      v = _mm_xor_si128(v, _mm_srli_epi32(y, 29));
      w |= static_cast<uint32_t>(_mm_movemask_ps(_mm_castsi128_ps(_mm_slli_epi32(v, 31)))) << (4 * q);
    }
    stream[p >> 5] = w;
  }
#endif
  for (; j < n; ++j, ++p)
    stream[p >> 5] |= static_cast<uint32_t>(__builtin_parity(s[i0 + j] & kLsbTaps)) << (p & 31);
  *pos = p;
}

// `count` outputs' low bits from the generator (state, left, next in at::mt19937's meaning: the
// next output regenerates the state when --left reaches 0), packed LSB-first into `stream`
// (zeroed, >= ceil(count / 32) words); the generator is advanced past them.
inline void lsb_stream(uint32_t* state, int32_t* left, int32_t* next, int64_t count, uint32_t* stream) {
  int64_t pos = 0;
  int32_t l = *left, nx = *next;
  while (pos < count) {
    int avail = l - 1;  // outputs before the next regeneration
    if (avail == 0) {
      next_state(state);
      l = kN + 1;  // the regenerating call reads state[0] and leaves left = N, next = 1
      nx = 0;
      avail = kN;
    }
    const int take = static_cast<int>(count - pos < avail ? count - pos : avail);
    emit_lsb(state, nx, take, stream, &pos);
    nx += take;
    l -= take;
  }
  *left = l;
  *next = nx;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// rows of `words` words cut from the packed stream (row r starts at stream bit r * cols): 16 words
// per op (a per-row funnel shift of two overlapping stream loads); the last word masked to `tail`
__attribute__((target("avx512f"))) inline void cut_rows_avx512(const uint32_t* stream, int64_t rows, int64_t cols,
                                                                int64_t words, uint32_t tail, uint32_t* out) {
  for (int64_t r = 0; r < rows; ++r) {
    const int64_t bit = r * cols;
    const uint32_t* src = stream + (bit >> 5);
    const int sh = static_cast<int>(bit & 31);
    const __m128i shr = _mm_cvtsi32_si128(sh), shl = _mm_cvtsi32_si128(32 - sh);
    uint32_t* o = out + r * words;
    int64_t w = 0;
    for (; w + 16 <= words; w += 16) {
      const __m512i lo = _mm512_loadu_si512(src + w), hi = _mm512_loadu_si512(src + w + 1);
      const __m512i v = sh ? _mm512_or_si512(_mm512_srl_epi32(lo, shr), _mm512_sll_epi32(hi, shl)) : lo;
      _mm512_storeu_si512(o + w, v);
    }
    for (; w < words; ++w) {
      const uint64_t two = static_cast<uint64_t>(src[w]) | (static_cast<uint64_t>(src[w + 1]) << 32);
      o[w] = static_cast<uint32_t>(two >> sh);
    }
    o[words - 1] &= tail;
  }
}
#endif

// torch.randint(0, 2, (rows, cols), dtype=torch.bool) as bit-packed rows out[rows][words]
// (words = ceil(cols / 32), bit c % 32 of word c / 32 = element c, tail bits 0).
inline void mask_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t rows, int64_t cols, uint32_t* out) {
  const int64_t n = rows * cols;
  const int64_t words = (cols + 31) / 32;
  std::vector<uint32_t> stream(static_cast<size_t>((n + 31) / 32 + 2), 0u);
  lsb_stream(state, left, next, n, stream.data());
  const uint32_t tail = (cols & 31) ? ((1u << (cols & 31)) - 1u) : 0xFFFFFFFFu;
#if !defined(__HIP_DEVICE_COMPILE__)
  if (have_avx512()) {
    cut_rows_avx512(stream.data(), rows, cols, words, tail, out);
    return;
  }
#endif
  for (int64_t r = 0; r < rows; ++r) {
    uint32_t* o = out + r * words;
    const int64_t base = r * cols;
    for (int64_t w = 0; w < words; ++w) {
      const int64_t off = base + 32 * w;
      const uint64_t two = static_cast<uint64_t>(stream[off >> 5]) | (static_cast<uint64_t>(stream[(off >> 5) + 1]) << 32);
      uint32_t v = static_cast<uint32_t>(two >> (off & 31));
      if (w == words - 1) v &= tail;
      o[w] = v;
    }
  }
}

// at::mt19937::operator(): one tempered 32-bit output (CPUGeneratorImpl::random())
inline uint32_t next_u32(uint32_t* s, int32_t* left, int32_t* next) {
  if (--*left == 0) {
    next_state(s);
    *left = kN;
    *next = 0;
  }
  uint32_t y = s[(*next)++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// CPUGeneratorImpl::random64(): two outputs, the first one the high word
inline uint64_t next_u64(uint32_t* s, int32_t* left, int32_t* next) {
  const uint64_t hi = next_u32(s, left, next);
  const uint64_t lo = next_u32(s, left, next);
  return (hi << 32) | lo;
}

// The per-repeat draws of Explainer.run with the device Shapley sampler, in the reference's
// order (explainer.py:490-519: mask_generator, LinearRegression init, DataLoader iterator), on
// the CPU generator:
//   seed  = torch.randint(0, 2**62, (1,))    uniform_int_from_to: random64() % 2^62
//   w0[S] = torch.empty(S).uniform_(from, to) per element: x = (random() & (2^24 - 1)) * 2^-24 (float),
//           x * (to - from) + from in float arithmetic (ATen uniform_real on dist_acctype<float>);
//           `fma` = 1 evaluates it as one fused multiply-add (how a -mfma build of the ATen
//           kernel may contract it; the CPU tests pin which form torch's build uses)
//   base  = torch.empty((), int64).random_()  uniform_int<int64>: random64() % 2^63
// seeds[times], w0[times][S]; the generator is left where torch would leave it.
inline void repeat_draws(uint32_t* s, int32_t* left, int32_t* next, int times, int64_t S, float from, float to,
                         int fma, int64_t* seeds, float* w0) {
  const float span = to - from;
  for (int t = 0; t < times; ++t) {
    seeds[t] = static_cast<int64_t>(next_u64(s, left, next) % (1ULL << 62));
    float* w = w0 + static_cast<int64_t>(t) * S;
    for (int64_t i = 0; i < S; ++i) {
      const float x = static_cast<float>(next_u32(s, left, next) & 0xFFFFFFu) * (1.0f / 16777216.0f);
      w[i] = fma ? std::fma(x, span, from) : x * span + from;
    }
    (void)next_u64(s, left, next);  // the DataLoader's base seed (value unused)
  }
}

// torch.randperm(n) on the CPU generator (ATen randperm_cpu, n < 2^32 / 20): Fisher-Yates with
// z = random() % (n - i), swapping positions i and i + z, for i = 0 .. n - 2.
inline void randperm(uint32_t* s, int32_t* left, int32_t* next, int64_t n, std::vector<int64_t>* out) {
  out->resize(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) (*out)[i] = i;
  for (int64_t i = 0; i + 1 < n; ++i) {
    const int64_t z = static_cast<int64_t>(next_u32(s, left, next)) % (n - i);
    std::swap((*out)[i], (*out)[i + z]);
  }
}

inline bool stream_bit(const std::vector<uint32_t>& st, int64_t i) { return (st[i >> 5] >> (i & 31)) & 1u; }

// `nb` (<= 32) stream bits from bit position i, LSB first (the stream has 2 words of slack)
inline uint32_t stream_bits(const uint32_t* st, int64_t i, int nb) {
  const uint64_t two = static_cast<uint64_t>(st[i >> 5]) | (static_cast<uint64_t>(st[(i >> 5) + 1]) << 32);
  const uint32_t v = static_cast<uint32_t>(two >> (i & 31));
  return nb >= 32 ? v : v & ((1u << nb) - 1u);
}

// The compat community mask rows of Mask.mask_generator (reference masks.py:299-348 with
// get_internal_mask masks.py:81-136, get_external_indices masks.py:138-194 and Pathways'
// mask_generator / activate_dead_mask / pathway_mask2node_mask, pathways.py:234-385), drawn from
// torch's CPU generator in the reference's call order, written UNSHUFFLED as bit-packed rows
// out[rows][words] (zeroed by the caller).  Per block {row_start, size, size_internal, own, e}
// in length-descending community order:
//   internal = randint(0, 2, (size, |own|), bool)                    masks.py:130
//   pm = randint(0, 2, (half, n), bool), then ~pm, then (if size - size_internal is odd) one
//        more randint(0, 2, (1, n), bool) row; half = (size - size_internal) // 2  pathways.py:260-281
//   pm[:, e] = False  (the reference switches off column e, the block's position in sorted
//        order, not the block's own community)                         masks.py:178
//   n > 1 and pm all False: order = randperm(n) without e, row r switches on order[r % (n-1)]
//                                                                      pathways.py:318-333
//   rows size_internal.. of the block: OR of the members of every community pm switches on
//   every row of the block: column own[j] := internal[r][j], j ascending (members sorted)
// comm_ptr / comm_cols: CSR of every community's member columns (ascending), n communities.
//
// The external OR runs over tables of the member masks of groups of g communities (all 2^g
// unions per group, g chosen so the tables stay <= 4 M words): a row ORs ceil(n / g) table rows
// instead of one member mask per switched-on community.  The internal assignment clears the
// own community's columns and sets the drawn ones (a community listing a column twice keeps
// the sequential last-write semantics instead).
inline void community_rows(uint32_t* s, int32_t* left, int32_t* next, int64_t cols, int32_t n,
                           const int32_t* comm_ptr, const int32_t* comm_cols, const int32_t* blocks,
                           int32_t n_blocks, uint32_t* out) {
  const int64_t words = (cols + 31) / 32;
  int g = 8;
  while (g > 1 && ((n + g - 1) / g) * (int64_t(1) << g) * words > (int64_t(4) << 20)) --g;
  const int groups = (n + g - 1) / g;
  // member masks per community (also the own-column clear masks of the internal assignment)
  std::vector<uint32_t> cmask(static_cast<size_t>(n) * words, 0u);
  std::vector<uint8_t> dup(n, 0);
  for (int c = 0; c < n; ++c)
    for (int64_t k = comm_ptr[c]; k < comm_ptr[c + 1]; ++k) {
      cmask[c * words + (comm_cols[k] >> 5)] |= 1u << (comm_cols[k] & 31);
      if (k > comm_ptr[c] && comm_cols[k] == comm_cols[k - 1]) dup[c] = 1;
    }
  const bool tables = (int64_t)groups * (int64_t(1) << g) * words <= (int64_t(4) << 20);
  std::vector<uint32_t> tab;
  if (tables) {
    tab.assign(static_cast<size_t>(groups) * (size_t(1) << g) * words, 0u);
    for (int G = 0; G < groups; ++G) {
      uint32_t* tg = tab.data() + static_cast<size_t>(G) * (size_t(1) << g) * words;
      for (uint32_t code = 1; code < (1u << g); ++code) {
        const int low = __builtin_ctz(code), c = G * g + low;
        const uint32_t* prev = tg + static_cast<size_t>(code & (code - 1)) * words;
        uint32_t* dst = tg + static_cast<size_t>(code) * words;
        if (c < n) {
          const uint32_t* m = cmask.data() + static_cast<size_t>(c) * words;
          for (int64_t w = 0; w < words; ++w) dst[w] = prev[w] | m[w];
        } else {
          for (int64_t w = 0; w < words; ++w) dst[w] = prev[w];
        }
      }
    }
  }
  const int pmw = (n + 31) / 32;  // words of one community-flag row
  std::vector<uint32_t> st_int, st_ext, st_extra, pm;
  std::vector<int64_t> perm;
  for (int b = 0; b < n_blocks; ++b) {
    const int64_t start = blocks[5 * b], size = blocks[5 * b + 1], si = blocks[5 * b + 2];
    const int own = blocks[5 * b + 3], e = blocks[5 * b + 4];
    const int64_t o0 = comm_ptr[own], len = comm_ptr[own + 1] - o0;
    auto draw = [&](int64_t count, std::vector<uint32_t>* st) {
      st->assign(static_cast<size_t>((count + 31) / 32 + 2), 0u);
      if (count > 0) lsb_stream(s, left, next, count, st->data());
    };
    draw(size * len, &st_int);
    const int64_t ext = size - si, half = ext / 2;
    draw(half * n, &st_ext);
    const bool extra = (ext % 2) != 0;
    if (extra) draw(n, &st_extra);
    // community flags per external row, packed: drawn rows, their complements, the extra row
    pm.assign(static_cast<size_t>(ext * pmw), 0u);
    const uint32_t emask = ~(1u << (e & 31));
    bool any = false;
    for (int64_t r = 0; r < ext; ++r) {
      uint32_t* f = pm.data() + r * pmw;
      const uint32_t* src = r < 2 * half ? st_ext.data() : st_extra.data();
      const int64_t base = r < half ? r * n : r < 2 * half ? (r - half) * n : 0;
      const bool flip = r >= half && r < 2 * half;
      for (int w = 0; w < pmw; ++w) {
        const int nb = std::min(32, n - 32 * w);
        uint32_t v = stream_bits(src, base + 32 * w, nb);
        if (flip) v = ~v & (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u));
        if (w == (e >> 5)) v &= emask;
        f[w] = v;
        any = any || v != 0u;
      }
    }
    if (n - 1 > 0 && !any) {
      randperm(s, left, next, n, &perm);
      std::vector<int64_t> order;
      for (int64_t v : perm)
        if (v != e) order.push_back(v);
      if (!order.empty())
        for (int64_t r = 0; r < ext; ++r) {
          const int64_t c = order[r % static_cast<int64_t>(order.size())];
          pm[r * pmw + (c >> 5)] |= 1u << (c & 31);
        }
    }
    for (int64_t r = 0; r < ext; ++r) {
      uint32_t* __restrict__ row = out + (start + si + r) * words;
      const uint32_t* f = pm.data() + r * pmw;
      if (tables) {
        for (int G = 0; G < groups; ++G) {
          const int bit = G * g;
          const uint64_t two = static_cast<uint64_t>(f[bit >> 5]) |
                               ((bit >> 5) + 1 < pmw ? static_cast<uint64_t>(f[(bit >> 5) + 1]) << 32 : 0ull);
          const uint32_t code = static_cast<uint32_t>(two >> (bit & 31)) & ((1u << g) - 1u);
          if (!code) continue;
          const uint32_t* __restrict__ t = tab.data() + (static_cast<size_t>(G) << g | code) * words;
          for (int64_t w = 0; w < words; ++w) row[w] |= t[w];
        }
      } else {
        for (int c = 0; c < n; ++c)
          if ((f[c >> 5] >> (c & 31)) & 1u)
            for (int64_t k = comm_ptr[c]; k < comm_ptr[c + 1]; ++k)
              row[comm_cols[k] >> 5] |= 1u << (comm_cols[k] & 31);
      }
    }
    const int32_t* oc = comm_cols + o0;
    if (!dup[own]) {
      const uint32_t* om = cmask.data() + static_cast<size_t>(own) * words;
      const int64_t wlo = len ? oc[0] >> 5 : 0, whi = len ? oc[len - 1] >> 5 : -1;
      for (int64_t r = 0; r < size; ++r) {
        uint32_t* __restrict__ row = out + (start + r) * words;
        for (int64_t w = wlo; w <= whi; ++w) row[w] &= ~om[w];
        for (int64_t j0 = 0; j0 < len; j0 += 32) {
          uint32_t v = stream_bits(st_int.data(), r * len + j0, static_cast<int>(std::min<int64_t>(32, len - j0)));
          while (v) {
            const int32_t col = oc[j0 + __builtin_ctz(v)];
            row[col >> 5] |= 1u << (col & 31);
            v &= v - 1u;
          }
        }
      }
    } else {
      for (int64_t r = 0; r < size; ++r) {
        uint32_t* row = out + (start + r) * words;
        for (int64_t j = 0; j < len; ++j) {
          const int32_t col = oc[j];
          const uint32_t bit = 1u << (col & 31);
          const uint32_t v = static_cast<uint32_t>(stream_bit(st_int, r * len + j));
          row[col >> 5] = (row[col >> 5] & ~bit) | (v << (col & 31));
        }
      }
    }
  }
}

}  // namespace hostrng
