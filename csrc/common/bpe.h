// Byte-level BPE token counting (TokenCounter, reference src/pipeline/token/token_counter.rs:31-42:
// ``tokenizer.encode(text, true).get_tokens().len()``) for GPT-2-style tokenizers: the ByteLevel
// pre-tokenizer regex, then BPE merges per pre-token, plus the tokens the post-processor adds.
// Shared by the HIP kernel (csrc/hip/bpe.hip: one lane per kept document, merge state in LDS)
// and its host emulation (csrc/host/module.cpp bpe_count), which CPU tests pin to the
// `tokenizers` library itself.
//
// Pre-tokenization. The regex ``'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|
// \s+(?!\S)|\s+`` is leftmost-first from each token start s, so the token is decided locally:
//   * an apostrophe followed by s/t/m/d (2 bytes) or re/ve/ll (3) is a contraction;
//   * a U+0020 followed by a letter / number / other code point joins the run of that class;
//   * a letter / number / other code point starts a maximal run of its class;
//   * a whitespace run [s, e) of k code points is one token when it ends the text or k == 1, else
//     it stops before its last code point (the lookahead of \s+(?!\S)).
// Character classes come from bpe_classes.inc, generated from the tokenizers library's own regex
// (its Unicode version differs from ICU's); ASCII is classified inline.
//
// Merges. HuggingFace's BPE (word.rs merge_all) pops (rank, position)-ordered candidates from a
// heap and skips stale ones; a stale candidate can never validate (symbols only grow, so the pair
// now at its position spells a longer string, i.e. a different token), so it equals: repeatedly
// merge the adjacent pair with the lowest rank, leftmost on ties. The lane keeps the word's
// symbol ids and pair ranks in two small arrays and deletes merged symbols in place.
//
// A pre-token longer than kBpeMaxWord bytes (the lane's merge arrays: long URLs, base64, runs of
// indentation or dashes) is merged by bpe_word_long over arrays of its own length (on the device:
// k_bpe_count marks the document kBpeLong and k_bpe_long recounts it with one wave per long
// pre-token, up to kBpeMaxLong bytes). A document goes back to the host tokenizer (count -2) when
// it contains the text of an added token (HF splits on those before pre-tokenizing), holds invalid
// UTF-8, or has a pre-token longer than kBpeMaxLong bytes.
#pragma once
#include "tb_common.h"

namespace tb {

constexpr int kBpeMaxWord = 64;
constexpr int kBpeMaxAdded = 8;
constexpr uint64_t kBpeEmpty = ~0ull;
constexpr uint32_t kBpeNoRank = 0xFFFFFFFFu;
constexpr int32_t kBpeHost = -2;  // count it on the host
// k_bpe_count: the document has a pre-token over kBpeMaxWord bytes; its count is kBpeLong - (the
// tokens of its other pre-tokens), which k_bpe_long completes
constexpr int32_t kBpeLong = -3;
constexpr int kBpeMaxLong = 2048;  // longest pre-token merged on the device

enum BpeCls : int { BPE_O = 0, BPE_L = 1, BPE_N = 2, BPE_W = 3 };

struct DevBpe {
  const uint32_t* byte_id;   // [256]: vocabulary id of each byte's byte-level character
  const uint64_t* keys;      // [mask + 1]: (left id << 32 | right id), kBpeEmpty = free slot
  const uint64_t* vals;      // [mask + 1]: (rank << 32 | merged id)
  const uint16_t* cls1;      // bpe_classes.inc two-stage class table
  const uint32_t* cls2;
  const uint8_t* added;      // contents of the added tokens, concatenated
  uint32_t mask;
  int32_t n_added;
  int32_t added_off[kBpeMaxAdded + 1];
  int32_t post_add;          // tokens the post-processor adds to every encoding
};

TB_HD uint64_t bpe_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// (rank << 32 | merged id) of the pair, or ~0 when it is not a merge
TB_HD uint64_t bpe_lookup(const DevBpe& T, uint32_t a, uint32_t b) {
  const uint64_t key = ((uint64_t)a << 32) | b;
  uint64_t h = bpe_hash(key) & T.mask;
  for (;;) {
    const uint64_t k = T.keys[h];
    if (k == key) return T.vals[h];
    if (k == kBpeEmpty) return ~0ull;
    h = (h + 1) & T.mask;
  }
}

TB_HD int bpe_cls(const DevBpe& T, uint32_t c) {
  if (c < 128) {
    const uint32_t l = c | 0x20;
    if (l >= 'a' && l <= 'z') return BPE_L;
    if (c >= '0' && c <= '9') return BPE_N;
    if (c == ' ' || (c >= 9 && c <= 13)) return BPE_W;
    return BPE_O;
  }
  const uint32_t w = T.cls2[(uint32_t)T.cls1[c >> 7] * 8 + ((c & 127) >> 4)];
  return (int)((w >> (2 * (c & 15))) & 3);
}

// Strict UTF-8 decode at b[i] (i < n): code point, *len bytes; -1 if invalid.
TB_HD int32_t bpe_decode(const uint8_t* b, int64_t i, int64_t n, int* len) {
  const uint32_t c0 = b[i];
  if (c0 < 0x80) {
    *len = 1;
    return (int32_t)c0;
  }
  int k;
  uint32_t c, lo;
  if (c0 >= 0xC2 && c0 <= 0xDF) { k = 1; c = c0 & 0x1F; lo = 0x80; }
  else if (c0 >= 0xE0 && c0 <= 0xEF) { k = 2; c = c0 & 0x0F; lo = 0x800; }
  else if (c0 >= 0xF0 && c0 <= 0xF4) { k = 3; c = c0 & 0x07; lo = 0x10000; }
  else return -1;
  if (i + k >= n) return -1;
  for (int j = 1; j <= k; ++j) {
    const uint32_t cc = b[i + j];
    if ((cc & 0xC0) != 0x80) return -1;
    c = (c << 6) | (cc & 0x3F);
  }
  if (c < lo || c > 0x10FFFF || (c >= 0xD800 && c <= 0xDFFF)) return -1;
  *len = k + 1;
  return (int32_t)c;
}

// Lane-local merge arrays: element i at p[i * stride] (stride = wave width in LDS, 1 on the host)
struct BpeArr {
  uint32_t* p;
  int stride;
  TB_HD uint32_t& operator[](int i) const { return p[i * stride]; }
};

// Tokens of one pre-token (its L <= kBpeMaxWord bytes) after the merges.
TB_HD int bpe_word(const DevBpe& T, const uint8_t* w, int L, BpeArr c, BpeArr r) {
  if (L <= 1) return L;
  for (int i = 0; i < L; ++i) c[i] = T.byte_id[w[i]];
  for (int i = 0; i + 1 < L; ++i) r[i] = (uint32_t)(bpe_lookup(T, c[i], c[i + 1]) >> 32);
  int m = L;
  while (m > 1) {
    uint32_t best = kBpeNoRank;
    int bi = -1;
    for (int i = 0; i + 1 < m; ++i) {
      const uint32_t v = r[i];
      if (v < best) { best = v; bi = i; }
    }
    if (bi < 0) break;
    c[bi] = (uint32_t)bpe_lookup(T, c[bi], c[bi + 1]);
    --m;  // symbol bi + 1 is gone: shift the tail down
    for (int j = bi + 1; j < m; ++j) c[j] = c[j + 1];
    for (int j = bi + 1; j + 1 < m; ++j) r[j] = r[j + 1];
    if (bi > 0) r[bi - 1] = (uint32_t)(bpe_lookup(T, c[bi - 1], c[bi]) >> 32);
    if (bi + 1 < m) r[bi] = (uint32_t)(bpe_lookup(T, c[bi], c[bi + 1]) >> 32);
  }
  return m;
}

// Tokens of a pre-token of L >= 2 bytes of any length: bpe_word's rule (the leftmost lowest-rank
// pair merges first) over a doubly linked list of symbols (nx / pv: next / previous live symbol,
// -1 / L at the ends), so a merge scans for the minimum but shifts nothing; v[i] holds the pair
// lookup of symbol i and its successor ((rank << 32 | merged id), ~0 = no merge), so a merge needs
// only the two lookups of its new neighbours. Sequential (host); k_bpe_long runs the same merges
// with the minimum search spread over a wave.
TB_HD int bpe_word_long(const DevBpe& T, const uint8_t* w, int L, uint32_t* c, uint64_t* v, int32_t* nx,
                        int32_t* pv) {
  if (L <= 1) return L;
  for (int i = 0; i < L; ++i) {
    c[i] = T.byte_id[w[i]];
    nx[i] = i + 1;
    pv[i] = i - 1;
  }
  for (int i = 0; i + 1 < L; ++i) v[i] = bpe_lookup(T, c[i], c[i + 1]);
  v[L - 1] = ~0ull;
  int m = L;
  while (m > 1) {
    uint64_t best = ~0ull;
    int bi = -1;
    for (int i = 0; i < L; i = nx[i]) {  // symbol 0 never dies: merges keep their left symbol
      const uint64_t r = v[i] | 0xFFFFFFFFull;  // rank only, ties to the leftmost
      if (r < best) { best = r; bi = i; }
    }
    if (bi < 0 || (best >> 32) == kBpeNoRank) break;
    const int j = nx[bi];
    c[bi] = (uint32_t)v[bi];
    nx[bi] = nx[j];
    if (nx[j] < L) pv[nx[j]] = bi;
    v[j] = ~0ull;
    --m;
    v[bi] = nx[bi] < L ? bpe_lookup(T, c[bi], c[nx[bi]]) : ~0ull;
    if (pv[bi] >= 0) v[pv[bi]] = bpe_lookup(T, c[pv[bi]], c[bi]);
  }
  return m;
}

// does the text of an added token start at a byte in [s0, s1)?
TB_HD bool bpe_has_added(const DevBpe& T, const uint8_t* b, int64_t n, int64_t s0 = 0, int64_t s1 = -1) {
  if (s1 < 0) s1 = n;
  for (int a = 0; a < T.n_added; ++a) {
    const uint8_t* t = T.added + T.added_off[a];
    const int64_t tl = T.added_off[a + 1] - T.added_off[a];
    if (tl <= 0 || tl > n) continue;
    for (int64_t i = s0; i < s1 && i + tl <= n; ++i) {
      if (b[i] != t[0]) continue;
      int64_t j = 1;
      while (j < tl && b[i + j] == t[j]) ++j;
      if (j == tl) return true;
    }
  }
  return false;
}

// End of the maximal run of class k starting at code point p (valid UTF-8 assumed up to e);
// -1 on invalid UTF-8.
TB_HD int64_t bpe_run_end(const DevBpe& T, const uint8_t* b, int64_t p, int64_t n, int k) {
  while (p < n) {
    int len;
    const int32_t c = bpe_decode(b, p, n, &len);
    if (c < 0) return -1;
    if (bpe_cls(T, (uint32_t)c) != k) break;
    p += len;
  }
  return p;
}

// End of the pre-token that starts at the code point start s (s < n); -1 on invalid UTF-8.
TB_HD int64_t bpe_next_token(const DevBpe& T, const uint8_t* b, int64_t n, int64_t s) {
  int len0;
  const int32_t c0 = bpe_decode(b, s, n, &len0);
  if (c0 < 0) return -1;
  if (c0 == '\'' && s + 1 < n) {
    const uint8_t x = b[s + 1];
    if (x == 's' || x == 't' || x == 'm' || x == 'd') return s + 2;
    if (s + 2 < n) {
      const uint8_t y = b[s + 2];
      if ((x == 'r' && y == 'e') || (x == 'v' && y == 'e') || (x == 'l' && y == 'l')) return s + 3;
    }
  }
  const int k0 = bpe_cls(T, (uint32_t)c0);
  if (k0 != BPE_W) return bpe_run_end(T, b, s + len0, n, k0);
  if (c0 == ' ' && s + 1 < n) {
    int len1;
    const int32_t c1 = bpe_decode(b, s + 1, n, &len1);
    if (c1 < 0) return -1;
    const int k1 = bpe_cls(T, (uint32_t)c1);
    if (k1 != BPE_W) return bpe_run_end(T, b, s + 1 + len1, n, k1);  // " ?\p{L}+" and friends
  }
  int64_t last = s, e = s + len0;
  int cnt = 1;
  while (e < n) {
    int l;
    const int32_t cc = bpe_decode(b, e, n, &l);
    if (cc < 0) return -1;
    if (bpe_cls(T, (uint32_t)cc) != BPE_W) break;
    last = e;
    e += l;
    ++cnt;
  }
  return (e < n && cnt >= 2) ? last : e;  // \s+(?!\S): the last whitespace starts the next token
}

// ---- local token boundaries (a wave splits a document into per-lane byte ranges) ----
// Pre-token starts are a local property of the text: i (a code point start, 0 < i < n) starts
// a token iff
//   R1  class(i) != class(i-1), unless cp(i-1) is U+0020 and class(i) is not whitespace (the
//       space joins the run after it), or
//   R2  i-1 and i are whitespace and the code point after i exists and is not (i is the last
//       whitespace of a run that \s+(?!\S) leaves for the next token),
// corrected for contractions: an apostrophe at a token start (R1/R2, or the text start) followed
// by s/t/m/d/re/ve/ll is a token of its own, so the letter after it is not a start, and the code
// point after the contraction is. So a lane can find the first start at or after any byte and
// tokenize sequentially from there; tests pin this against the sequential tokenizer.

TB_HD int64_t bpe_prev_start(const uint8_t* b, int64_t i) {
  int64_t p = i - 1;
  for (int k = 0; k < 3 && p > 0 && (b[p] & 0xC0) == 0x80; ++k) --p;
  return p;
}

// R1 || R2 at the code point start i (0 < i < n): 1 / 0, -1 on invalid UTF-8
TB_HD int bpe_b12(const DevBpe& T, const uint8_t* b, int64_t n, int64_t i) {
  int l1, l0;
  const int32_t c1 = bpe_decode(b, i, n, &l1);
  const int64_t p = bpe_prev_start(b, i);
  const int32_t c0 = bpe_decode(b, p, n, &l0);
  if (c1 < 0 || c0 < 0 || p + l0 != i) return -1;
  const int k1 = bpe_cls(T, (uint32_t)c1), k0 = bpe_cls(T, (uint32_t)c0);
  if (k1 != k0) return (c0 == ' ' && k1 != BPE_W) ? 0 : 1;
  if (k1 != BPE_W || i + l1 >= n) return 0;
  int l2;
  const int32_t c2 = bpe_decode(b, i + l1, n, &l2);
  if (c2 < 0) return -1;
  return bpe_cls(T, (uint32_t)c2) != BPE_W ? 1 : 0;
}

// length of the contraction token at p (an apostrophe at a token start), 0 if none, -1 invalid
TB_HD int bpe_contraction(const DevBpe& T, const uint8_t* b, int64_t n, int64_t p) {
  if (b[p] != '\'' || p + 1 >= n) return 0;
  const uint8_t x = b[p + 1];
  int L = 0;
  if (x == 's' || x == 't' || x == 'm' || x == 'd') L = 2;
  else if (p + 2 < n) {
    const uint8_t y = b[p + 2];
    if ((x == 'r' && y == 'e') || (x == 'v' && y == 'e') || (x == 'l' && y == 'l')) L = 3;
  }
  if (L == 0 || p == 0) return L;
  const int r = bpe_b12(T, b, n, p);
  return r < 0 ? -1 : (r ? L : 0);
}

// does a pre-token start at the code point start i (0 < i < n)? 1 / 0, -1 invalid
TB_HD int bpe_boundary(const DevBpe& T, const uint8_t* b, int64_t n, int64_t i) {
  for (int d = 1; d <= 3 && d <= i; ++d) {
    if (b[i - d] != '\'') continue;
    const int L = bpe_contraction(T, b, n, i - d);
    if (L < 0) return -1;
    if (L == d) return 1;                // right after a contraction
    if (d == 1 && L > 0) return 0;       // inside one
  }
  return bpe_b12(T, b, n, i);
}

// first pre-token start at or after byte s0 (n if none), -1 on invalid UTF-8
TB_HD int64_t bpe_first_start(const DevBpe& T, const uint8_t* b, int64_t n, int64_t s0) {
  int64_t i = s0;
  while (i < n && i > 0 && (b[i] & 0xC0) == 0x80) ++i;
  while (i < n && i > 0) {
    const int r = bpe_boundary(T, b, n, i);
    if (r < 0) return -1;
    if (r) return i;
    int l;
    if (bpe_decode(b, i, n, &l) < 0) return -1;
    i += l;
  }
  return i;
}

// Tokens (after merges) of the pre-tokens that start in [first_start(s0), first_start(s1)); a
// pre-token [s, e) over kBpeMaxWord bytes is handed to on_long(s, e) (its tokens, or < 0: fail).
// -1: count the document on the host (invalid UTF-8, or on_long failed).
struct BpeNoLong {
  TB_HD int64_t operator()(int64_t, int64_t) const { return -1; }
};
// (kMerge = false: short pre-tokens are only delimited, not merged; they count 0)
template <bool kMerge = true, class LongF = BpeNoLong>
TB_HD int64_t bpe_count_range(const DevBpe& T, const uint8_t* b, int64_t n, int64_t s0, int64_t s1, BpeArr c,
                              BpeArr r, LongF&& on_long = LongF{}) {
  int64_t s = s0 <= 0 ? 0 : bpe_first_start(T, b, n, s0);
  if (s < 0) return -1;
  int64_t total = 0;
  while (s < n && s < s1) {
    const int64_t e = bpe_next_token(T, b, n, s);
    if (e <= s) return -1;
    if (e - s > kBpeMaxWord) {
      const int64_t k = on_long(s, e);
      if (k < 0) return -1;
      total += k;
    } else if (kMerge) {
      total += bpe_word(T, b + s, (int)(e - s), c, r);
    }
    s = e;
  }
  return total;
}

// Token count of one document (kBpeHost: count it on the host), sequentially.
template <class LongF = BpeNoLong>
TB_HD int32_t bpe_count_doc(const DevBpe& T, const uint8_t* b, int64_t n, BpeArr c, BpeArr r,
                            LongF&& on_long = LongF{}) {
  if (T.n_added && bpe_has_added(T, b, n)) return kBpeHost;
  const int64_t k = bpe_count_range<true>(T, b, n, 0, n, c, r, on_long);
  if (k < 0 || k + T.post_add > 0x7FFFFFFF) return kBpeHost;
  return (int32_t)(k + T.post_add);
}

}  // namespace tb
