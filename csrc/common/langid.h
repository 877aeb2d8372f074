// Character n-gram language identifier that stands in for lingua (reference
// src/pipeline/filters/language_filter.rs:35-93; survey H5).
//
// Model: a linear classifier over hashed character n-grams. Every bucket holds the int16
// fixed-point logit contributions of its n-grams to the 5 candidate languages (P[bucket][8],
// 5 used, scale kLidScale); logits = (sum over the document's grams of P[g]) / #grams / kLidScale
// + b, softmax over the 5 languages, the confidence is the top probability. The sums are exact
// integers, so host and device agree bit for bit; the per-gram work is one 16-byte gather.
// (Equivalent to a mean-of-embeddings fastText model with its linear head folded into the
// table offline: (mean E) W = mean (E W). The folded table has more capacity than the rank-32
// factorisation and needs no doc-vector GEMM; tools/train_langid.py trains it directly.)
//
// N-grams: the text is scanned as code points (first kLidMaxCps only); letters (Alphabetic) are
// lowercased, every maximal letter run is a word padded as "<w>"; n-grams of length 1..4 of the
// padded word are hashed (the lone boundary markers are not features).
#pragma once
#include <cmath>

#include "ucd.h"

namespace tb {

constexpr int kLidLangs = 5;
constexpr int kLidRow = 8;  // int16 per bucket (languages 0..4, zero padding): one 16-byte load
constexpr int kLidBucketsLog2 = 16;
constexpr uint32_t kLidBuckets = 1u << kLidBucketsLog2;
constexpr int kLidMaxCps = 4096;
constexpr int kLidMaxGrams = 4;  // n-grams emitted per code point position, at most
constexpr uint32_t kLidBoundary = 0x20;
constexpr double kLidScale = 1024.0;  // P = int16 / 1024 (|P| < 32)

TB_HD uint32_t lid_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int n) {
  uint32_t h = 2166136261u ^ (uint32_t)n * 0x9E3779B1u;
  h = (h ^ a) * 16777619u;
  if (n >= 2) h = (h ^ b) * 16777619u;
  if (n >= 3) h = (h ^ c) * 16777619u;
  if (n >= 4) h = (h ^ d) * 16777619u;
  h ^= h >> 15;
  h *= 0x2c1b3c6dU;
  h ^= h >> 12;
  return h & (kLidBuckets - 1);
}

// Emits the buckets of every n-gram that ENDS at code point position i (0 <= i <= lim), given
// the lowercased letters L(i-3) .. L(i) (0 when a position is not a letter or is past lim-1).
// Position lim acts as a virtual non-letter so a word that reaches the cut still gets its ">"
// grams. Returns the number of grams (<= kLidMaxGrams).
template <class F>
TB_HD int lid_grams_at(uint32_t lm3, uint32_t lm2, uint32_t lm1, uint32_t l0, F&& emit) {
  const uint32_t B = kLidBoundary;
  if (l0) {
    emit(lid_hash(l0, 0, 0, 0, 1));
    emit(lid_hash(lm1 ? lm1 : B, l0, 0, 0, 2));
    if (!lm1) return 2;
    emit(lid_hash(lm2 ? lm2 : B, lm1, l0, 0, 3));
    if (!lm2) return 3;
    emit(lid_hash(lm3 ? lm3 : B, lm2, lm1, l0, 4));
    return 4;
  }
  if (!lm1) return 0;
  emit(lid_hash(lm1, B, 0, 0, 2));
  emit(lid_hash(lm2 ? lm2 : B, lm1, B, 0, 3));
  if (!lm2) return 2;
  emit(lid_hash(lm3 ? lm3 : B, lm2, lm1, B, 4));
  return 3;
}

// Adds the int16 row of bucket g to the 5 language sums.
TB_HD void lid_add_row(const int16_t* P, uint32_t g, int32_t* acc) {
  const int16_t* r = P + (size_t)g * kLidRow;
#pragma unroll
  for (int l = 0; l < kLidLangs; ++l) acc[l] += r[l];
}

// Decision from the exact sums: r[0] = language index (-1: no n-gram), r[1] = confidence bits
// (f64). Ties go to the lowest index. Same double arithmetic on host and device.
TB_HD void lid_decide(const int64_t* sums, int64_t cnt, const float* bias, int64_t* r) {
  if (cnt <= 0) {
    r[0] = -1;
    r[1] = 0;
    return;
  }
  double logit[kLidLangs];
  for (int l = 0; l < kLidLangs; ++l) logit[l] = (double)sums[l] / (double)cnt / kLidScale + (double)bias[l];
  int best = 0;
  for (int l = 1; l < kLidLangs; ++l) if (logit[l] > logit[best]) best = l;
  double den = 0;
  for (int l = 0; l < kLidLangs; ++l) den += exp(logit[l] - logit[best]);
  const double conf = 1.0 / den;
  r[0] = best;
  union { double d; int64_t i; } u;
  u.d = conf;
  r[1] = u.i;
}

// Lowercased letter of the code point starting at byte s (0: not a letter / out of range).
TB_HD uint32_t lid_letter(const UcdView& ucd, const uint8_t* b, uint32_t n, int64_t s) {
  if (s < 0) return 0;
  const uint32_t c0 = b[s];
  if (c0 < 0x80u) {  // ASCII: alphabetic = A-Z / a-z, lowercase = c | 0x20 (no table lookups)
    const uint32_t l = c0 | 0x20u;
    return (l >= 'a' && l <= 'z') ? l : 0u;
  }
  int len;
  const uint32_t c = utf8_decode(b, (uint32_t)s, n, &len);
  if (!(ucd.props(c) & P_ALPHA)) return 0;
  const uint32_t l = ucd.lower(c);
  return l ? l : c;
}

TB_HD int64_t prev_lead(const uint8_t* b, int64_t s) {
  int64_t k = s - 1;
  while (k >= 0 && !utf8_is_lead(b[k])) --k;
  return k;
}

// The model's tables as the kernels see them.
struct LidTables {
  const int16_t* P;    // [kLidBuckets * kLidRow]
  const float* bias;   // [kLidRow]
};

}  // namespace tb
