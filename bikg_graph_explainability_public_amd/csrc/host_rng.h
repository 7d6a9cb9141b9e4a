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
#include <cstdint>
#include <cstring>
#include <vector>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <emmintrin.h>  // SSE2 (x86-64 baseline): host code only
#endif

namespace hostrng {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
constexpr uint32_t kLsbTaps = 0x20444009u;

inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & kUpper) | (v & kLower)) >> 1) ^ ((0u - (v & 1u)) & kMatrixA);
}

// at::mt19937::next_state (the standard MT19937 regeneration, in place)
inline void next_state(uint32_t* s) {
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
  // whole words, 4 outputs per SSE2 op: bit0 of y ^ y>>3 ^ y>>14 ^ y>>18 ^ y>>22 ^ y>>29 is the
  // parity above; movemask collects the four low bits (shifted to the sign bits)
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

// torch.randint(0, 2, (rows, cols), dtype=torch.bool) as bit-packed rows out[rows][words]
// (words = ceil(cols / 32), bit c % 32 of word c / 32 = element c, tail bits 0).
inline void mask_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t rows, int64_t cols, uint32_t* out) {
  const int64_t n = rows * cols;
  const int64_t words = (cols + 31) / 32;
  std::vector<uint32_t> stream(static_cast<size_t>((n + 31) / 32 + 2), 0u);
  lsb_stream(state, left, next, n, stream.data());
  const uint32_t tail = (cols & 31) ? ((1u << (cols & 31)) - 1u) : 0xFFFFFFFFu;
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

}  // namespace hostrng
