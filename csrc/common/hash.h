// Composable polynomial string hashing in the ring of integers modulo 2^64.
//
// H(s) = sum_i (s_i + 1) * B^(|s|-1-i)  (mod 2^64), B odd (so B is invertible), H(xy) = H(x) * B^|y| + H(y).
// The repetition filters need exact string equality (reference src/utils/text.rs:184-259
// uses HashSet<String>); every hash hit is verified byte-for-byte by the callers, so the hash
// only has to make verification rare, never decide equality on its own. Wrap-around arithmetic
// keeps a Horner step at one 64-bit multiply-add (a 2^61-1 reduction costs the high half of a
// 128-bit product on top: ~25 VALU instructions per step instead of ~6 on CDNA); the known
// structured collisions of power-of-two moduli (Thue-Morse strings) only cost a verification.
#pragma once
#include "tb_common.h"

namespace tb {

constexpr uint64_t kHashBase = 0x9E3779B97F4A7C15ull;  // odd
constexpr uint64_t hash_inverse(uint64_t b) {  // b^-1 mod 2^64 (Newton: each step doubles the bits)
  uint64_t x = b;
  for (int i = 0; i < 6; ++i) x *= 2 - b * x;
  return x;
}
constexpr uint64_t kHashBaseInv = hash_inverse(kHashBase);
static_assert(kHashBase * kHashBaseInv == 1ull, "hash base must be invertible");

TB_HD uint64_t hmul(uint64_t a, uint64_t b) { return a * b; }
TB_HD uint64_t hadd(uint64_t a, uint64_t b) { return a + b; }
TB_HD uint64_t hsub(uint64_t a, uint64_t b) { return a - b; }

TB_HD uint64_t hpow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}

TB_HD uint64_t hash_push(uint64_t h, uint8_t byte) { return h * kHashBase + ((uint64_t)byte + 1); }

TB_HD uint64_t hash_bytes(const uint8_t* s, uint32_t n) {
  uint64_t h = 0;
  for (uint32_t i = 0; i < n; ++i) h = hash_push(h, s[i]);
  return h;
}

// H(x || y) given H(x), H(y), |y|.
TB_HD uint64_t hash_concat(uint64_t hx, uint64_t hy, uint32_t ylen) { return hx * hpow(kHashBase, ylen) + hy; }

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
