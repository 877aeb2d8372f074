// Pipeline step configuration, per-document statistic records, and the decision functions that
// turn a record into pass/filter + reason + metadata exactly as the reference filters do.
//
// Both execution paths produce the same records: the CPU path computes them with
// compute_record() below; the HIP kernels (csrc/hip) write them from device analysis. The
// decision/formatting code (decide()) is shared, so reason strings and metadata are identical.
#pragma once
#include <cstdint>
#include <optional>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "rustfmt.h"
#include "text.h"

namespace tb {

enum class StepKind : int {
  C4Quality = 0,
  GopherRepetition = 1,
  GopherQuality = 2,
  C4BadWords = 3,
  LanguageDetection = 4,
  FineWebQuality = 5,
  TokenCounter = 6,
};

struct StepCfg {
  StepKind kind;
  std::string name;
  // C4QualityFilter (reference config/pipeline.rs:67-80)
  bool split_paragraph = true, remove_citations = true, filter_no_terminal_punct = true;
  int64_t min_num_sentences = 0, min_words_per_line = 0, max_word_length = 0;
  bool filter_lorem_ipsum = false, filter_javascript = false, filter_curly_bracket = false,
       filter_policy = false;
  // GopherRepetitionFilter (pipeline.rs:103-117)
  std::optional<double> dup_line_frac, dup_para_frac, dup_line_char_frac, dup_para_char_frac;
  std::vector<std::pair<int64_t, double>> top_n_grams, dup_n_grams;
  // GopherQualityFilter (pipeline.rs:162-175)
  std::optional<int64_t> min_doc_words, max_doc_words, min_stop_words;
  std::optional<double> min_avg_word_length, max_avg_word_length, max_symbol_word_ratio,
      max_bullet_lines_ratio, max_ellipsis_lines_ratio, max_non_alpha_words_ratio;
  std::vector<std::string> stop_words;  // lowercase; default list filled by the Python side
  // FineWebQualityFilter (pipeline.rs:312-322)
  double line_punct_thr = 0, short_line_thr = 0, char_duplicates_ratio = 0, new_line_ratio = 0;
  bool line_punct_exclude_zero = false;
  int64_t short_line_length = 0;
  std::vector<uint32_t> stop_chars;
  // LanguageDetectionFilter (pipeline.rs:288-292)
  double min_confidence = 0;
  std::vector<int> allowed_langs;         // indices into kLangNames (candidates only)
  std::vector<std::string> allowed_codes; // every valid ISO 639-3 code, in config order
  // C4BadWordsFilter (pipeline.rs:260-267)
  double keep_fraction = 0;
  bool fail_on_missing_language = false;
  std::optional<uint64_t> seed;
  std::string default_language;
  // TokenCounter
  std::string tokenizer_name;
};

// Candidate languages of the reference detector (language_filter.rs:39-45), in model order.
extern const char* const kLangNames[5];   // lingua Display names
extern const char* const kLangCodes[5];   // ISO 639-3

// Record widths (int64 fields) per step kind.
int record_width(const StepCfg& c);

// Field indices
namespace rec {
// GopherQuality
enum { GQ_WORDS, GQ_SUM_CHARS, GQ_HASH, GQ_ELLIPSIS, GQ_LINES, GQ_BULLET, GQ_ELL_LINES, GQ_ALPHA,
       GQ_STOP, GQ_WIDTH };
// GopherRepetition: fixed part then |top_n_grams| then |dup_n_grams| results
enum { GR_CHARS, GR_PARA, GR_PARA_DUP, GR_PARA_DUP_BYTES, GR_LINES, GR_LINE_DUP, GR_LINE_DUP_BYTES,
       GR_FIXED };
// C4Quality
enum { C4_LOREM, C4_CURLY, C4_TOO_LONG, C4_NO_PUNCT, C4_TOO_FEW, C4_SENTENCES, C4_NEW_LEN,
       C4_WIDTH };
// FineWeb
enum { FW_LINES, FW_STOP_END, FW_SHORT, FW_DUP_BYTES, FW_CHARS_NO_NL, FW_NL, FW_WORDS, FW_WIDTH };
// LanguageDetection: lang index (-1 = undetected), confidence bits (f64)
enum { LD_LANG, LD_CONF_BITS, LD_WIDTH };
// TokenCounter: token count (-1 = tokenizer error)
enum { TC_COUNT, TC_WIDTH };
// C4BadWords: status code (see BwStatus), unused
enum { BW_STATUS, BW_WIDTH };
}  // namespace rec

enum BwStatus : int64_t {
  BW_PASSED = 0,
  BW_NO_REGEX = 1,
  BW_KEPT_BY_FRACTION = 2,
  BW_FILTERED = 3,
  BW_MISSING_LANG_FAIL = 4,
};

// Outcome of one step on one document.
// Metadata keys are string literals (static storage), values are formatted per document.
struct Decision {
  bool pass = true;
  bool error = false;  // unrecoverable step error (no outcome, like the reference's None path)
  std::string reason;
  std::vector<std::pair<std::string_view, std::string>> meta;  // in insertion order
};

// Full decision: pass/filtered/error + reason + metadata (formatting).
void decide(const StepCfg& c, const int64_t* r, Decision& d);
// Same branches without building any string: 0 pass, 1 filtered, 2 error.
uint8_t decide_status(const StepCfg& c, const int64_t* r);
// Same branches; appends the step's metadata as JSON object members ("k":"v", comma-separated,
// `first` tracks the leading comma) to `out` without per-call allocations (output assembly).
void decide_meta_json(const StepCfg& c, const int64_t* r, CharBuf& out, bool& first);

// CPU computation of a step record on `text` (the step's input content version).
// For C4Quality, `new_content` receives the rewritten content.
void compute_record(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r,
                    std::string* new_content);

// Rewritten content for a C4 step (needed even when decision is filtered with
// too_few_sentences; the doc carries the rewritten content then).
std::string c4_rewrite(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r);

}  // namespace tb
