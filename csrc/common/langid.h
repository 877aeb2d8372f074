// Character n-gram featurizer for the fastText-style language identifier that stands in for
// lingua (reference src/pipeline/filters/language_filter.rs:35-93; survey H5).
//
// Model: doc vector = mean over hashed char n-gram embeddings E[bucket] (bf16 table, summed in
// exact 2^-16 fixed point so the host and the device produce bit-identical doc vectors), rounded
// to bf16, then logits = doc . W + b (bf16 x bf16 -> f32, MFMA on the device), softmax over the
// 5 candidate languages; the confidence is the top probability.
//
// N-grams: the text is scanned as code points (first kLidMaxCps only); letters (Alphabetic) are
// lowercased, every maximal letter run is a word padded as "<w>"; n-grams of length 1..3 of the
// padded word are hashed (the lone boundary markers are not features).
#pragma once
#include "ucd.h"

namespace tb {

constexpr int kLidDim = 32;
constexpr int kLidLangs = 5;
constexpr int kLidLangsPad = 16;
constexpr int kLidBucketsLog2 = 16;
constexpr uint32_t kLidBuckets = 1u << kLidBucketsLog2;
constexpr int kLidMaxCps = 4096;
constexpr uint32_t kLidBoundary = 0x20;
constexpr float kLidFixedScale = 65536.0f;

TB_HD uint32_t lid_hash(uint32_t a, uint32_t b, uint32_t c, int n) {
  uint32_t h = 2166136261u ^ (uint32_t)n * 0x9E3779B1u;
  h = (h ^ a) * 16777619u;
  if (n >= 2) h = (h ^ b) * 16777619u;
  if (n >= 3) h = (h ^ c) * 16777619u;
  h ^= h >> 15;
  h *= 0x2c1b3c6dU;
  h ^= h >> 12;
  return h & (kLidBuckets - 1);
}

// Emits the buckets of every n-gram that ENDS at code point position i (0 <= i <= lim), given
// the lowercased letters L(i) (0 when position i is not a letter or is past lim-1).
// Position lim acts as a virtual non-letter so a word that reaches the cut still gets its ">" grams.
template <class F>
TB_HD int lid_grams_at(uint32_t lm2, uint32_t lm1, uint32_t l0, bool has_m1, bool has_m2, F&& emit) {
  // lm2 = L(i-2), lm1 = L(i-1), l0 = L(i); 0 = not a letter / out of range.
  int cnt = 0;
  (void)has_m1; (void)has_m2;
  if (l0) {
    emit(lid_hash(l0, 0, 0, 1)); ++cnt;
    uint32_t p1 = lm1 ? lm1 : kLidBoundary;
    emit(lid_hash(p1, l0, 0, 2)); ++cnt;
    if (lm1) {
      uint32_t p2 = lm2 ? lm2 : kLidBoundary;
      emit(lid_hash(p2, lm1, l0, 3)); ++cnt;
    }
  } else if (lm1) {
    emit(lid_hash(lm1, kLidBoundary, 0, 2)); ++cnt;
    uint32_t p2 = lm2 ? lm2 : kLidBoundary;
    emit(lid_hash(p2, lm1, kLidBoundary, 3)); ++cnt;
  }
  return cnt;
}

// bf16 helpers (round-to-nearest-even), identical on host and device.
TB_HD float bf16_to_f32(uint16_t h) {
  union { uint32_t u; float f; } v;
  v.u = (uint32_t)h << 16;
  return v.f;
}
TB_HD uint16_t f32_to_bf16(float f) {
  union { uint32_t u; float f; } v;
  v.f = f;
  uint32_t u = v.u;
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);  // inf / nan
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
// Fixed-point value of an embedding entry (exact for |e| >= 2^-9, deterministic otherwise).
TB_HD int32_t lid_fixed(uint16_t e) {
  float f = bf16_to_f32(e) * kLidFixedScale;
  return (int32_t)__builtin_rintf(f);
}

}  // namespace tb
