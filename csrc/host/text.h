// Host-side text primitives with the exact semantics of the reference's Rust helpers
// (reference src/utils/text.rs; Rust str::trim / lines / to_lowercase / chars().count()).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "../common/ucd.h"

namespace tb {

const UcdView& host_ucd();

enum class SegBackend : int { Rules = 0, Icu = 1 };

inline uint32_t props_of(uint32_t cp) { return host_ucd().props(cp); }

// Code-point view of a UTF-8 string: cps[i], byte offsets off[i] (off[n] == size), props[i].
struct CpView {
  std::vector<uint32_t> cp;
  std::vector<uint32_t> off;
  std::vector<uint32_t> prop;
  void build(std::string_view s);
  int n() const { return (int)cp.size(); }
  uint32_t p(int i) const { return prop[i]; }
};

size_t count_chars(std::string_view s);
std::string_view trim(std::string_view s);
std::string_view trim_start(std::string_view s);
std::string_view trim_end(std::string_view s);
bool is_ws_cp(uint32_t cp);
// Rust str::lines(): split on '\n', strip one trailing '\r' from lines that ended in "\r\n".
std::vector<std::string_view> rust_lines(std::string_view s);
// Rust str::to_lowercase (full mapping incl. U+0130 and the Final_Sigma rule).
std::string rust_lowercase(std::string_view s);
// Last code point of s (or 0xFFFFFFFF if empty).
uint32_t last_cp(std::string_view s);
uint32_t first_cp(std::string_view s);
bool ends_with(std::string_view s, std::string_view suf);
bool starts_with(std::string_view s, std::string_view pre);
size_t count_nonoverlap(std::string_view s, std::string_view pat);
bool has_dict_script(std::string_view s);

// Word-break marks of the documents that hold a dictionary-script code point (ICU4C word
// segmentation, dictionary breaking included: the CPU oracle's words), for the device kernels,
// which segment everything else themselves. ICU runs over the lines that hold such a code point
// only. moff[d] = word offset of document d's record in `bits`, or -1 (no dictionary script,
// mostly dictionary-script text, or not strictly valid UTF-8: then the device keeps sending the
// document to the CPU path). A record is two bitmaps of mw = ((C + 1 + 63) / 64) * 2 words over
// the code points [0, C] (UTF-8 lead bytes): ICU's marks (bit i = a boundary before code point i)
// and the positions that take them (the rest keep the device's UAX#29 rules).
// Documents are scanned in parallel on the native pool.
void dict_word_marks(const uint8_t* data, const int64_t* off, int64_t ndocs, int nthreads,
                     std::vector<int64_t>& moff, std::vector<uint32_t>& bits);
// C4QualityFilter's per-line word statistics of the dictionary-script documents (moff[d] >= 0)
// that hold a '[' (a possible citation): per Rust line of the text its processed form
// remove_citations(trim(line)) (c4_filters.rs; `citations` false: trim(line)), its ICU word count
// and its longest word in code points — what C4 pass A would segment on the device. loff[d] =
// offset of [NL, nw_0, mx_0, nw_1, mx_1, ...] in `data`, or -1.
void dict_c4_lines(const uint8_t* text, const int64_t* off, int64_t ndocs, const int64_t* moff, bool citations,
                   int nthreads, std::vector<int64_t>& loff, std::vector<uint32_t>& data);

// Segment boundaries as byte offsets, always including 0 and s.size() (for non-empty s).
std::vector<uint32_t> word_breaks(std::string_view s, SegBackend be);
std::vector<uint32_t> sentence_breaks(std::string_view s, SegBackend be);

// reference utils/text.rs split_into_words / split_into_sentences
std::vector<std::string_view> split_into_words(std::string_view s, SegBackend be);
std::vector<std::string_view> split_into_sentences(std::string_view s, SegBackend be);

// reference utils/text.rs find_duplicates: (#repeat elements, sum of repeat byte lengths)
std::pair<size_t, size_t> find_duplicates(const std::vector<std::string_view>& items);
// find_top_duplicate over space-joined n-grams of `words`
size_t find_top_duplicate_ngrams(const std::vector<std::string_view>& words, size_t n);
// find_all_duplicate: greedy walk over concatenated n-grams
size_t find_all_duplicate(const std::vector<std::string_view>& words, size_t n);
// Both statistics for several orders over one word list (GopherRepetition's n-gram fields):
// out_top[i] = find_top_duplicate_ngrams(words, top[i]), out_dup[i] = find_all_duplicate(words,
// dup[i]), without building n-gram strings (word hashes + exact verification).
void ngram_stats(const std::vector<std::string_view>& words, const std::vector<size_t>& top,
                 const std::vector<size_t>& dup, size_t* out_top, size_t* out_dup);

// Citation removal `\[\d+(?:,\s*\d+)*\]` (Unicode \d and \s), reference c4_filters.rs:33,201
std::string remove_citations(std::string_view s);

}  // namespace tb
