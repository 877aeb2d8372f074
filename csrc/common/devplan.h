// Device execution plan: the step parameters the document kernels need, as a flat POD that the
// host runtime builds from the validated pipeline config and uploads once per run.
#pragma once
#include "tb_common.h"

namespace tb {

constexpr int kMaxStageSteps = 8;
constexpr int kMaxNgramEntries = 16;
constexpr int kMaxStopChars = 16;
constexpr int kMaxStopWords = 512;
constexpr int kStopTableSize = 2048;  // power of two >= 2 * kMaxStopWords
constexpr int kStopBlobBytes = 16384;

enum DevStepKind : int32_t {
  DK_NONE = 0,
  DK_GOPHER_QUALITY = 1,
  DK_GOPHER_REP = 2,
  DK_FINEWEB = 3,
  DK_LANGID = 4,   // featurize only (the head runs in its own kernel)
};

// Max bytes a device C4 rewrite may add to one document (larger growth -> CPU path), so the host
// can size the next content version without reading the device scan back.
constexpr uint32_t kC4MaxGrowth = 16;

struct DevStep {
  int32_t kind;
  int32_t width;       // record width (int64 fields)
  int64_t rec_base;    // element offset of this step's records = rec_prefix * ndocs (set per batch)
  int32_t rec_prefix;  // sum of widths of earlier steps in the stage
  // GopherQuality: stop-word set id (index into DevPlan::stops)
  int32_t stop_set;
  // GopherRepetition
  int32_t n_top, n_dup;
  int32_t top_n[kMaxNgramEntries];
  int32_t dup_n[kMaxNgramEntries];
  // FineWeb
  int32_t n_stop_chars;
  uint32_t stop_chars[kMaxStopChars];
  int64_t short_line_length;
};

// Compact form of a small stop-word set for the LDS-resident kernel (copied into each wave's
// slice): open addressing on the FNV-1a hash of the word, lite_nslots (power of two) u32 entries
// (hash bits 16..31 << 16 | word index + 1, 0 = empty); the words are blob[off[w] .. off[w + 1]).
constexpr int kStopLiteMaxSlots = 256;
constexpr int kStopLiteMaxWords = 64;
constexpr int kStopLiteMaxBlob = 1024;

TB_HD uint32_t stop_lite_hash_push(uint32_t h, uint8_t v) { return (h ^ v) * 16777619u; }
constexpr uint32_t kStopLiteHash0 = 2166136261u;
TB_HD uint32_t stop_lite_slot(uint32_t h, uint32_t nslots) { return (h * 0x9E3779B1u) & (nslots - 1); }

struct DevStopSet {
  // open-addressing table of lowercase stop words: key (0 = empty) -> word index
  uint64_t keys[kStopTableSize];
  int32_t idx[kStopTableSize];
  int32_t off[kMaxStopWords + 1];  // byte offsets into blob
  int32_t n;
  int32_t max_len;  // longest entry in bytes: a word of more code points cannot match
  uint8_t blob[kStopBlobBytes];
  int32_t lite_nslots;  // 0: the set is too large for the compact form
  uint32_t lite_slots[kStopLiteMaxSlots];
  // ASCII words of <= 7 bytes: key = bytes (little endian) | length << 56, open addressing on
  // stop_fast_slot (lite_nslots entries, 0 = empty). An ASCII word of <= 7 bytes is a stop word
  // iff its lowercase key is here (no other entry can equal it), so those need no byte compare.
  uint64_t fast_keys[kStopLiteMaxSlots];
  // 1: every entry is ASCII of <= 7 bytes (all of them are in fast_keys). A word outside the fast
  // path then matches only if it lowercases to ASCII, which needs U+212A KELVIN SIGN (-> 'k', the
  // only non-ASCII code point with an ASCII lowercase; its UTF-8 starts with E2)
  int32_t all_ascii7;
};

TB_HD uint32_t stop_fast_slot(uint64_t key, uint32_t nslots) {
  uint64_t h = key * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(h >> 40) & (nslots - 1);
}

struct DevC4 {
  int32_t split_paragraph, remove_citations, filter_no_terminal_punct;
  int32_t filter_lorem_ipsum, filter_javascript, filter_curly_bracket, filter_policy;
  int64_t min_words_per_line, max_word_length;
  // sentences are counted only up to this (the decision and the reason string use smaller
  // counts only): the record's sentence field saturates here; 0 = not counted
  int64_t min_num_sentences;
};

struct DevStage {
  int32_t n_steps;
  int32_t width_total;  // sum of record widths
  DevStep steps[kMaxStageSteps];
};

constexpr int kMaxStopSets = 4;

struct DevPlan {
  int32_t n_stop_sets;
  DevStopSet stops[kMaxStopSets];
};

// Per-document HBM scratch of the generic (analyze_stage / c4_pass_a) kernels:
// rate * (len + 64) + 4096 bytes. The rates are the measured worst cases of the host port with
// no LDS slice (every working array in HBM; tools/scratch_need.py, profiles/r8_scratch) plus
// ~6%: 74.7 B/byte in one pass (one-letter words, 1 MB), 166.0 B/byte for a document whose
// n-gram orders are split over workgroups (k_gr_dup_split / k_gr_split_wave: the stage export,
// then one equal slice per task, each as large as the largest task needs). A document that still
// runs out is flagged DOC_OVERFLOW and re-run on the CPU path, so the rates size memory, not
// correctness.
constexpr uint64_t kScratchPerByte = 80;
constexpr uint64_t kScratchPerByteSplit = 176;
TB_HD uint64_t scratch_bytes_for_dev(uint32_t doc_len, bool split = false) {
  return (split ? kScratchPerByteSplit : kScratchPerByte) * ((uint64_t)doc_len + 64) + 4096;
}

TB_HD uint64_t dev_key(uint64_t h, uint32_t len) {
  uint64_t x = h ^ ((uint64_t)len * 0xD6E8FEB86659FD93ull);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x | 1ull;
}

// Dictionary-script documents (ICU segments their words by dictionary) of a stage's content
// version: the host's word-break bitmaps of the original text (version 0: moff[d] = word offset of
// document d's bitmap in `bits`, -1 none; text.h dict_word_marks), or per document the word count
// of the C4 rewrite (later versions: the kept lines' words from C4 pass A's export path, kNoWords
// when unknown). Read only for documents that hold such a script; without either they go to the
// CPU path as before.
constexpr uint32_t kNoWords = 0xFFFFFFFFu;
// C4 pass A's per-line word statistics of dictionary-script documents (text.h dict_c4_lines)
struct DictLines {
  const int64_t* off = nullptr;
  const uint32_t* data = nullptr;
  TB_HD const uint32_t* at(uint32_t d) const { return (off && off[d] >= 0) ? data + off[d] : nullptr; }
};
struct DictIn {
  const int64_t* moff = nullptr;
  const uint32_t* bits = nullptr;
  const uint32_t* words = nullptr;
  TB_HD const uint32_t* marks(uint32_t d) const { return (moff && moff[d] >= 0) ? bits + moff[d] : nullptr; }
  TB_HD uint32_t nwords(uint32_t d) const { return words ? words[d] : kNoWords; }
};

}  // namespace tb
