// Character n-gram language identifier that stands in for lingua (reference
// src/pipeline/filters/language_filter.rs:35-93; survey H5), "fastText + bf16 MFMA head":
// a document vector of kLidDim = 32 dims, the
// concatenation of two 16-dim bags over one int8 embedding table of kLidRowDim = 16 values per
// bucket (16 bytes per n-gram gather): the 1- and 2-grams are summed into the lower half, the 3-
// and 4-grams into the upper half. A document's rows are summed exactly (int32), the mean doc
// vector is
// quantised to integers |a| <= 255 with one exponent per document (block floating point, every
// value exact in bf16), and the 32 -> 5 linear head runs as one v_mfma_f32_16x16x32_bf16 tile per
// 16 documents with integer bf16 weights |W| <= 255. All products and partial sums are integers
// below 2^24, so the MFMA's fp32 result is exact in any summation order and the host computes the
// same integers: logits = C * w_scale * 2^-e + b, softmax, confidence = top probability.
//
// The decision uses lid_exp (a fixed polynomial with explicit fma), so host and device agree on the
// confidence bits, not only on the integer sums.
//
// N-grams: the text is scanned as code points (first kLidMaxCps only); letters (Alphabetic) are
// lowercased, every maximal letter run is a word padded as "<w>"; n-grams of length 1..4 of the
// padded word are hashed (the lone boundary markers are not features).
#pragma once
#include <cmath>

#include "ucd.h"

namespace tb {

constexpr int kLidLangs = 5;
constexpr int kLidRow = 8;  // bias floats (languages 0..4, zero padding)
constexpr int kLidBucketsLog2 = 16;
constexpr uint32_t kLidBuckets = 1u << kLidBucketsLog2;
constexpr int kLidMaxCps = 4096;
constexpr int kLidMaxGrams = 4;  // n-grams emitted per code point position, at most
constexpr uint32_t kLidBoundary = 0x20;
constexpr int kLidDim = 32;           // v3 doc-vector dims = the MFMA K
constexpr int kLidRowDim = 16;        // v3 stored dims per bucket (half of the doc vector)
constexpr int kLidHeadCols = 16;      // v3 head columns (5 languages, zero padded to the MFMA N)
constexpr int kLidQMax = 255;         // v3 doc-vector / head integers: |v| <= 255 (exact in bf16)

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
// the lowercased letters L(i-3) .. L(i) (0 when a position is not a letter or is past lim-1),
// as emit(bucket, n). Position lim acts as a virtual non-letter so a word that reaches the cut
// still gets its ">" grams. At most one gram per order n; returns the number of grams (<= 4).
template <class F>
TB_HD int lid_grams_n(uint32_t lm3, uint32_t lm2, uint32_t lm1, uint32_t l0, F&& emit) {
  const uint32_t B = kLidBoundary;
  if (l0) {
    emit(lid_hash(l0, 0, 0, 0, 1), 1);
    emit(lid_hash(lm1 ? lm1 : B, l0, 0, 0, 2), 2);
    if (!lm1) return 2;
    emit(lid_hash(lm2 ? lm2 : B, lm1, l0, 0, 3), 3);
    if (!lm2) return 3;
    emit(lid_hash(lm3 ? lm3 : B, lm2, lm1, l0, 4), 4);
    return 4;
  }
  if (!lm1) return 0;
  emit(lid_hash(lm1, B, 0, 0, 2), 2);
  emit(lid_hash(lm2 ? lm2 : B, lm1, B, 0, 3), 3);
  if (!lm2) return 2;
  emit(lid_hash(lm3 ? lm3 : B, lm2, lm1, B, 4), 4);
  return 3;
}

template <class F>
TB_HD int lid_grams_at(uint32_t lm3, uint32_t lm2, uint32_t lm1, uint32_t l0, F&& emit) {
  return lid_grams_n(lm3, lm2, lm1, l0, [&](uint32_t g, int) { emit(g); });
}

// exp(x) for x <= 0 with the same bits on host and device: range reduction by ln 2 and a
// degree-13 Taylor polynomial on |r| <= 0.35 (truncation error < 4e-18), every multiply-add an
// explicit fma (correctly rounded on both sides; no contraction choices left to the compiler).
TB_HD double lid_exp(double x) {
  if (!(x > -745.0)) return 0.0;
  const double k = floor(fma(x, 1.4426950408889634, 0.5));
  double r = fma(-k, 6.93147180369123816490e-01, x);  // ln2 hi
  r = fma(-k, 1.90821492927058770002e-10, r);         // ln2 lo
  double p = 1.0 / 6227020800.0;                      // 1/13!
  const double inv[13] = {1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0,
                          1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
#pragma unroll
  for (int i = 0; i < 13; ++i) p = fma(p, r, inv[i]);
  return ldexp(p, (int)k);
}

// Softmax decision over kLidLangs logits: r[0] = language index (ties: lowest), r[1] = the
// confidence (top probability) as f64 bits.
TB_HD void lid_softmax_decide(const double* logit, int64_t* r) {
  int best = 0;
  for (int l = 1; l < kLidLangs; ++l) if (logit[l] > logit[best]) best = l;
  double den = 0;
  for (int l = 0; l < kLidLangs; ++l) den += lid_exp(logit[l] - logit[best]);
  const double conf = 1.0 / den;
  r[0] = best;
  union { double d; int64_t i; } u;
  u.d = conf;
  r[1] = u.i;
}

// Block exponent of a document: the largest e in [0, 30] with max|S| * 2^e <= 255 * cnt, so every
// a[k] = round(S[k] * 2^e / cnt) satisfies |a[k]| <= 255.
TB_HD int lid_block_exp(int64_t smax, int64_t cnt) {
  int e = 0;
  while (e < 30 && (smax << (e + 1)) <= (int64_t)kLidQMax * cnt) ++e;
  return e;
}

// round(s * 2^e / cnt), ties to even, exact integer arithmetic (|s| * 2^e < 2^62).
TB_HD int32_t lid_quant(int64_t s, int e, int64_t cnt) {
  const bool neg = s < 0;
  const int64_t num = (neg ? -s : s) << e;
  int64_t q = num / cnt;
  const int64_t rem = num - q * cnt;
  if (2 * rem > cnt || (2 * rem == cnt && (q & 1))) ++q;
  return (int32_t)(neg ? -q : q);
}

// v3 decision from the head's integer outputs C[l] (exact: the MFMA fp32 values) and the block
// exponent e; cnt <= 0: no n-gram (no language).
TB_HD void lid_decide_v3(const double* C, int e, int64_t cnt, double w_scale, const float* bias, int64_t* r) {
  if (cnt <= 0) {
    r[0] = -1;
    r[1] = 0;
    return;
  }
  const double sc = ldexp(w_scale, -e);
  double logit[kLidLangs];
  for (int l = 0; l < kLidLangs; ++l) logit[l] = fma(C[l], sc, (double)bias[l]);
  lid_softmax_decide(logit, r);
}

// Float <-> bf16 bits for values that are exact in bf16 (the v3 operands are integers <= 256).
TB_HD uint16_t lid_bf16_bits(float v) {
  union { float f; uint32_t u; } x;
  x.f = v;
  return (uint16_t)(x.u >> 16);
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

// The model's tables as the kernels see them (E == nullptr: no model).
struct LidTables {
  const float* bias = nullptr;  // [kLidRow]
  const int8_t* E = nullptr;    // [kLidBuckets * kLidRowDim] int8 embedding rows
  const int16_t* W = nullptr;   // [kLidDim * kLidLangs] integer head (|W| <= 255)
  double w_scale = 0;           // logit units per head unit at e = 0
};

// Dims of the doc vector that an n-gram of order n feeds: [lid_half(n), lid_half(n) + 16).
TB_HD int lid_half(int n) { return n >= 3 ? kLidRowDim : 0; }

// Adds the int8 embedding row of bucket g (an n-gram of order n) to its half of the sums.
TB_HD void lid_add_emb(const int8_t* E, uint32_t g, int n, int32_t* acc) {
  const int8_t* r = E + (size_t)g * kLidRowDim;
  int32_t* a = acc + lid_half(n);
#pragma unroll
  for (int d = 0; d < kLidRowDim; ++d) a[d] += r[d];
}

// Record from the exact embedding sums S[kLidDim] and the n-gram count (host reference of the
// device's MFMA tile: the same integers).
TB_HD void lid_record_v3(const int64_t* S, int64_t cnt, const LidTables& lt, int64_t* r) {
  if (cnt <= 0) {
    r[0] = -1;
    r[1] = 0;
    return;
  }
  int64_t smax = 0;
  for (int d = 0; d < kLidDim; ++d) smax = (S[d] < 0 ? -S[d] : S[d]) > smax ? (S[d] < 0 ? -S[d] : S[d]) : smax;
  const int e = lid_block_exp(smax, cnt);
  int32_t a[kLidDim];
  for (int d = 0; d < kLidDim; ++d) a[d] = lid_quant(S[d], e, cnt);
  double C[kLidLangs];
  for (int l = 0; l < kLidLangs; ++l) {
    int64_t c = 0;
    for (int d = 0; d < kLidDim; ++d) c += (int64_t)a[d] * lt.W[d * kLidLangs + l];
    C[l] = (double)c;
  }
  lid_decide_v3(C, e, cnt, lt.w_scale, lt.bias, r);
}

}  // namespace tb
