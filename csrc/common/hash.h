// Composable polynomial string hashing modulo the Mersenne prime 2^61-1.
//
// H(s) = sum_i (s_i + 1) * B^(|s|-1-i)  (mod 2^61-1), so H(xy) = H(x) * B^|y| + H(y).
// The repetition filters need exact string equality (reference src/utils/text.rs:184-259
// uses HashSet<String>); every hash hit is verified byte-for-byte by the callers, so the hash
// only has to make verification rare, never decide equality on its own.
#pragma once
#include "tb_common.h"

namespace tb {

constexpr uint64_t kM61 = (1ull << 61) - 1;
constexpr uint64_t kHashBase = 0x1F3A5C7D9B2E4F61ull % kM61;
constexpr uint64_t kHashBaseInv = 0x0BD8A5E56DEDF53Eull;  // kHashBase^(p-2) mod p: B * B^-1 = 1

TB_HD uint64_t mulmod61(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t lo = a * b;
  const uint64_t hi = __umul64hi(a, b);
#else
  const __uint128_t r = (__uint128_t)a * b;
  const uint64_t lo = (uint64_t)r, hi = (uint64_t)(r >> 64);
#endif
  uint64_t x = (lo & kM61) + (lo >> 61) + (hi << 3);
  x = (x & kM61) + (x >> 61);
  return x >= kM61 ? x - kM61 : x;
}

TB_HD uint64_t addmod61(uint64_t a, uint64_t b) {
  uint64_t x = a + b;
  return x >= kM61 ? x - kM61 : x;
}

TB_HD uint64_t powmod61(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mulmod61(r, b);
    b = mulmod61(b, b);
    e >>= 1;
  }
  return r;
}

TB_HD uint64_t hash_push(uint64_t h, uint8_t byte) { return addmod61(mulmod61(h, kHashBase), (uint64_t)byte + 1); }

TB_HD uint64_t hash_bytes(const uint8_t* s, uint32_t n) {
  uint64_t h = 0;
  for (uint32_t i = 0; i < n; ++i) h = hash_push(h, s[i]);
  return h;
}

// H(x || y) given H(x), H(y), |y|.
TB_HD uint64_t hash_concat(uint64_t hx, uint64_t hy, uint32_t ylen) {
  return addmod61(mulmod61(hx, powmod61(kHashBase, ylen)), hy);
}

// 64-bit finalizer used to spread keys over open-addressing tables.
TB_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

}  // namespace tb
