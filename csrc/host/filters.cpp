#include "filters.h"

#include <algorithm>
#include <cstring>
#include <unordered_set>

#include "json.h"
#include "rustfmt.h"

namespace tb {

const char* const kLangNames[5] = {"English", "Danish", "Swedish", "Nynorsk", "Bokmal"};
const char* const kLangCodes[5] = {"eng", "dan", "swe", "nno", "nob"};

int record_width(const StepCfg& c) {
  switch (c.kind) {
    case StepKind::GopherQuality: return rec::GQ_WIDTH;
    case StepKind::GopherRepetition:
      return rec::GR_FIXED + (int)c.top_n_grams.size() + (int)c.dup_n_grams.size();
    case StepKind::C4Quality: return rec::C4_WIDTH;
    case StepKind::FineWebQuality: return rec::FW_WIDTH;
    case StepKind::LanguageDetection: return rec::LD_WIDTH;
    case StepKind::TokenCounter: return rec::TC_WIDTH;
    case StepKind::C4BadWords: return rec::BW_WIDTH;
  }
  return 1;
}

// reference c4_filters.rs:20 / fineweb_quality.rs:26
static const uint32_t kEndPunct[6] = {'.', '!', '?', '"', '\'', 0x201D};
static const char* const kPolicy[6] = {"terms of use", "privacy policy", "cookie policy",
                                       "uses cookies", "use of cookies", "use cookies"};

static bool is_end_punct(uint32_t c) {
  for (uint32_t e : kEndPunct) if (e == c) return true;
  return false;
}

static std::string join(const std::vector<std::string>& v, const char* sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

static bool word_has_alpha(std::string_view w) {
  const uint8_t* b = (const uint8_t*)w.data();
  uint32_t n = (uint32_t)w.size();
  for (uint32_t i = 0; i < n;) {
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    if (props_of(c) & P_ALPHA) return true;
    i += len;
  }
  return false;
}

// Split on a run of >= k newlines (regex \n{k,}); text is trimmed (no leading/trailing \n).
static std::vector<std::string_view> split_newline_runs(std::string_view t, int k) {
  std::vector<std::string_view> out;
  size_t start = 0, i = 0;
  while (i < t.size()) {
    if (t[i] != '\n') { ++i; continue; }
    size_t j = i;
    while (j < t.size() && t[j] == '\n') ++j;
    if ((int)(j - i) >= k) {
      out.push_back(t.substr(start, i - start));
      start = j;
    }
    i = j;
  }
  out.push_back(t.substr(start));
  return out;
}

// ------------------------------------------------------------------------------------------
static void compute_gq(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r) {
  auto words = split_into_words(text, be);
  int64_t sum = 0, alpha = 0, stop = 0;
  std::unordered_set<std::string> sw(c.stop_words.begin(), c.stop_words.end());
  for (auto w : words) {
    sum += (int64_t)count_chars(w);
    if (word_has_alpha(w)) ++alpha;
    if (!sw.empty() && sw.count(rust_lowercase(w))) ++stop;
  }
  int64_t nhash = 0;
  for (char ch : text) nhash += ch == '#';
  auto lines = rust_lines(text);
  int64_t bullet = 0, ell = 0;
  for (auto l : lines) {
    auto ls = trim_start(l);
    if (starts_with(ls, "\xE2\x80\xA2") || starts_with(ls, "-")) ++bullet;
    auto le = trim_end(l);
    if (ends_with(le, "...") || ends_with(le, "\xE2\x80\xA6")) ++ell;
  }
  r[rec::GQ_WORDS] = (int64_t)words.size();
  r[rec::GQ_SUM_CHARS] = sum;
  r[rec::GQ_HASH] = nhash;
  r[rec::GQ_ELLIPSIS] = (int64_t)(count_nonoverlap(text, "...") + count_nonoverlap(text, "\xE2\x80\xA6"));
  r[rec::GQ_LINES] = (int64_t)lines.size();
  r[rec::GQ_BULLET] = bullet;
  r[rec::GQ_ELL_LINES] = ell;
  r[rec::GQ_ALPHA] = alpha;
  r[rec::GQ_STOP] = stop;
}

static void compute_gr(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r) {
  std::string_view t = trim(text);
  for (int i = 0; i < record_width(c); ++i) r[i] = 0;
  if (t.empty()) { r[rec::GR_CHARS] = -1; return; }
  r[rec::GR_CHARS] = (int64_t)count_chars(t);
  auto paras = split_newline_runs(t, 2);
  auto pd = find_duplicates(paras);
  r[rec::GR_PARA] = (int64_t)paras.size();
  r[rec::GR_PARA_DUP] = (int64_t)pd.first;
  r[rec::GR_PARA_DUP_BYTES] = (int64_t)pd.second;
  auto lines = split_newline_runs(t, 1);
  auto ld = find_duplicates(lines);
  r[rec::GR_LINES] = (int64_t)lines.size();
  r[rec::GR_LINE_DUP] = (int64_t)ld.first;
  r[rec::GR_LINE_DUP_BYTES] = (int64_t)ld.second;
  auto words = split_into_words(t, be);
  std::vector<size_t> top, dup;
  for (auto& e : c.top_n_grams) top.push_back((size_t)std::max<int64_t>(0, e.first));
  for (auto& e : c.dup_n_grams) dup.push_back((size_t)std::max<int64_t>(0, e.first));
  std::vector<size_t> vt(top.size()), vd(dup.size());
  ngram_stats(words, top, dup, vt.data(), vd.data());
  int k = rec::GR_FIXED;
  for (size_t v : vt) r[k++] = (int64_t)v;
  for (size_t v : vd) r[k++] = (int64_t)v;
}

std::string c4_rewrite(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r) {
  for (int i = 0; i < rec::C4_WIDTH; ++i) r[i] = 0;
  if (c.filter_lorem_ipsum) {
    std::string low = rust_lowercase(text);
    r[rec::C4_LOREM] = low.find("lorem ipsum") != std::string::npos;
  }
  if (c.filter_curly_bracket)
    r[rec::C4_CURLY] = text.find('{') != std::string_view::npos || text.find('}') != std::string_view::npos;
  if (r[rec::C4_LOREM] || r[rec::C4_CURLY]) {
    r[rec::C4_NEW_LEN] = (int64_t)text.size();
    return std::string(text);
  }
  std::vector<std::string_view> lines =
      c.split_paragraph ? rust_lines(text) : split_into_sentences(text, be);
  std::vector<std::string> kept;
  for (auto line : lines) {
    std::string_view cur = trim(line);
    std::string proc = c.remove_citations ? remove_citations(cur) : std::string(cur);
    auto words = split_into_words(proc, be);
    if (c.max_word_length > 0) {
      bool too_long = false;
      for (auto w : words)
        if ((int64_t)count_chars(w) > c.max_word_length) { too_long = true; break; }
      if (too_long) { ++r[rec::C4_TOO_LONG]; continue; }
    }
    if (c.filter_no_terminal_punct) {
      uint32_t last = last_cp(proc);
      bool term = last != 0xFFFFFFFFu && is_end_punct(last);
      if (!term || ends_with(proc, "...")) { ++r[rec::C4_NO_PUNCT]; continue; }
    }
    if (c.min_words_per_line > 0 && (int64_t)words.size() < c.min_words_per_line) {
      ++r[rec::C4_TOO_FEW];
      continue;
    }
    if (c.filter_javascript || c.filter_policy) {
      std::string low = rust_lowercase(proc);
      if (c.filter_javascript && low.find("javascript") != std::string::npos) continue;
      if (c.filter_policy) {
        bool hit = false;
        for (auto p : kPolicy) if (low.find(p) != std::string::npos) { hit = true; break; }
        if (hit) continue;
      }
    }
    kept.push_back(std::move(proc));
  }
  std::string joined = join(kept, "\n");
  std::string out(trim(joined));
  r[rec::C4_SENTENCES] = (int64_t)split_into_sentences(out, be).size();
  r[rec::C4_NEW_LEN] = (int64_t)out.size();
  return out;
}

static void compute_fw(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r) {
  std::vector<std::string_view> lines;
  for (auto l : rust_lines(text))
    if (!trim(l).empty()) lines.push_back(l);
  int64_t stop_end = 0, shrt = 0;
  for (auto l : lines) {
    uint32_t last = last_cp(trim_end(l));
    if (last != 0xFFFFFFFFu &&
        std::find(c.stop_chars.begin(), c.stop_chars.end(), last) != c.stop_chars.end())
      ++stop_end;
    if ((int64_t)count_chars(l) <= c.short_line_length) ++shrt;
  }
  int64_t nl = 0;
  for (char ch : text) nl += ch == '\n';
  r[rec::FW_LINES] = (int64_t)lines.size();
  r[rec::FW_STOP_END] = stop_end;
  r[rec::FW_SHORT] = shrt;
  r[rec::FW_DUP_BYTES] = (int64_t)find_duplicates(lines).second;
  r[rec::FW_CHARS_NO_NL] = (int64_t)count_chars(text) - nl;
  r[rec::FW_NL] = nl;
  r[rec::FW_WORDS] = (int64_t)split_into_words(text, be).size();
}

void compute_record(const StepCfg& c, std::string_view text, SegBackend be, int64_t* r,
                    std::string* new_content) {
  switch (c.kind) {
    case StepKind::GopherQuality: compute_gq(c, text, be, r); break;
    case StepKind::GopherRepetition: compute_gr(c, text, be, r); break;
    case StepKind::C4Quality: {
      std::string s = c4_rewrite(c, text, be, r);
      if (new_content) *new_content = std::move(s);
      break;
    }
    case StepKind::FineWebQuality: compute_fw(c, text, be, r); break;
    default: break;  // language / token / badwords records are produced elsewhere
  }
}

// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// Decisions. One implementation of every step's decision logic (decide_t), instantiated with
// three sinks:
//   StatusSink    pass / filtered / error only (the per-batch resolve hot path: no text at all)
//   DecisionSink  + reason string and metadata pairs (per-document API, host steps)
//   JsonSink      + the step's metadata appended as JSON members straight into the output
//                 column buffer (output assembly: no per-document allocations)
// Reasons and values are built by appending into reusable buffers with the allocation-free
// Rust formatters of rustfmt.h; the sinks decide what is kept. Every instance takes exactly the
// same branches, so status, reasons and metadata cannot disagree.

namespace {

struct Arg {  // one piece of a formatted message
  enum K { S, I, F2, F4, F64 } k;
  std::string_view s;
  int64_t i = 0;
  double d = 0;
};
inline Arg A(std::string_view s) { return Arg{Arg::S, s}; }
inline Arg A(const char* s) { return Arg{Arg::S, std::string_view(s)}; }
inline Arg A(int64_t v) { Arg a{Arg::I, {}}; a.i = v; return a; }
inline Arg F2(double v) { Arg a{Arg::F2, {}}; a.d = v; return a; }
inline Arg F4(double v) { Arg a{Arg::F4, {}}; a.d = v; return a; }
inline Arg F64(double v) { Arg a{Arg::F64, {}}; a.d = v; return a; }

inline void put(CharBuf& out, const Arg& a) {
  switch (a.k) {
    case Arg::S: out.append(a.s.data(), a.s.size()); break;
    case Arg::I: append_i64(out, a.i); break;
    case Arg::F2: append_fixed(out, a.d, 2); break;
    case Arg::F4: append_fixed(out, a.d, 4); break;
    case Arg::F64: append_f64(out, a.d); break;
  }
}
inline void cat(CharBuf& out, std::initializer_list<Arg> args) {
  for (const Arg& a : args) put(out, a);
}

struct StatusSink {
  static constexpr bool kFmt = false;
  bool pass = true, error = false;
  void fail() { pass = false; }
  void fail_error() { pass = false; error = true; }
  void reason(std::initializer_list<Arg>) {}
  void set_reason(std::initializer_list<Arg>) {}
  void meta(std::string_view, std::initializer_list<Arg>) {}
  void meta_reasons(std::string_view) {}
};

// Shared by the formatting sinks: reasons joined with "; ".
struct ReasonBuf {
  CharBuf r;
  bool any = false;
  void add(std::initializer_list<Arg> args) {
    if (any) r.append("; ", 2);
    any = true;
    cat(r, args);
  }
  void set(std::initializer_list<Arg> args) {
    r.clear();
    any = true;
    cat(r, args);
  }
};

struct DecisionSink {
  static constexpr bool kFmt = true;
  Decision& d;
  ReasonBuf rb;
  CharBuf tmp;
  explicit DecisionSink(Decision& dd) : d(dd) {}
  void fail() { d.pass = false; }
  void fail_error() { d.pass = false; d.error = true; }
  void reason(std::initializer_list<Arg> args) { rb.add(args); }
  void set_reason(std::initializer_list<Arg> args) { rb.set(args); }
  void meta(std::string_view k, std::initializer_list<Arg> args) {
    tmp.clear();
    cat(tmp, args);
    d.meta.emplace_back(k, std::string(tmp.view()));
  }
  void meta_reasons(std::string_view k) { d.meta.emplace_back(k, std::string(rb.r.view())); }
  void finish() { d.reason = std::string(rb.r.view()); }
};

struct JsonSink {
  static constexpr bool kFmt = true;
  CharBuf& out;
  bool& first;
  ReasonBuf& rb;
  CharBuf& tmp;
  bool pass = true, error = false;
  void fail() { pass = false; }
  void fail_error() { pass = false; error = true; }
  void reason(std::initializer_list<Arg> args) { rb.add(args); }
  void set_reason(std::initializer_list<Arg> args) { rb.set(args); }
  void member(std::string_view k, std::string_view v) {
    // keys are literals of this file (plain ASCII, nothing to escape)
    out.reserve(k.size() + 5);
    if (!first) out.p[out.n++] = ',';
    first = false;
    out.p[out.n++] = '"';
    std::memcpy(out.p + out.n, k.data(), k.size());
    out.n += k.size();
    out.p[out.n++] = '"';
    out.p[out.n++] = ':';
    json_escape_append(out, v);
  }
  void meta(std::string_view k, std::initializer_list<Arg> args) {
    tmp.clear();
    cat(tmp, args);
    member(k, tmp.view());
  }
  void meta_reasons(std::string_view k) { member(k, rb.r.view()); }
};

}  // namespace

template <class Sink>
static void decide_t(const StepCfg& c, const int64_t* r, Sink& k) {
  bool any = false;  // at least one reason
  auto add = [&](std::initializer_list<Arg> args) {
    any = true;
    k.reason(args);
  };
  auto finish_multi = [&](std::string_view status_key, std::string_view reasons_key) {
    if (any) {
      k.fail();
      k.meta(status_key, {A("filtered")});
      k.meta_reasons(reasons_key);
    } else {
      k.meta(status_key, {A("passed")});
    }
  };
  switch (c.kind) {
    case StepKind::GopherQuality: {  // reference gopher_quality.rs:198-317
      const int64_t n = r[rec::GQ_WORDS];
      const double ncalc = (double)std::max<int64_t>(1, n);
      const double avg = n > 0 ? (double)r[rec::GQ_SUM_CHARS] / (double)n : 0.0;
      const double hash_ratio = (double)r[rec::GQ_HASH] / ncalc;
      const double ell_ratio = (double)r[rec::GQ_ELLIPSIS] / ncalc;
      const double lcalc = (double)std::max<int64_t>(1, r[rec::GQ_LINES]);
      const double bullet = (double)r[rec::GQ_BULLET] / lcalc;
      const double ell_lines = (double)r[rec::GQ_ELL_LINES] / lcalc;
      const double alpha = (double)r[rec::GQ_ALPHA] / ncalc;
      if (c.min_doc_words && n < *c.min_doc_words)
        add({A("gopher_short_doc ("), A(n), A(" non-symbol words, required "), A(*c.min_doc_words), A(")")});
      if (c.max_doc_words && n > *c.max_doc_words)
        add({A("gopher_long_doc ("), A(n), A(" non-symbol words, max "), A(*c.max_doc_words), A(")")});
      if (c.min_avg_word_length && avg < *c.min_avg_word_length)
        add({A("gopher_below_avg_threshold (avg len "), F2(avg), A(", required "), F2(*c.min_avg_word_length),
             A((n == 0 && *c.min_avg_word_length > 0.0) ? " - 0 non-symbol words" : ""), A(")")});
      if (c.max_avg_word_length && n > 0 && avg > *c.max_avg_word_length)
        add({A("gopher_above_avg_threshold (avg len "), F2(avg), A(", max "), F2(*c.max_avg_word_length), A(")")});
      if (c.max_symbol_word_ratio) {
        if (hash_ratio > *c.max_symbol_word_ratio)
          add({A("gopher_too_many_hashes (ratio "), F2(hash_ratio), A(", max "), F2(*c.max_symbol_word_ratio), A(")")});
        if (ell_ratio > *c.max_symbol_word_ratio)
          add({A("gopher_too_many_ellipsis_units (ratio "), F2(ell_ratio), A(", max "), F2(*c.max_symbol_word_ratio),
               A(")")});
      }
      if (c.max_bullet_lines_ratio && bullet > *c.max_bullet_lines_ratio)
        add({A("gopher_too_many_bullets (ratio "), F2(bullet), A(", max "), F2(*c.max_bullet_lines_ratio), A(")")});
      if (c.max_ellipsis_lines_ratio && ell_lines > *c.max_ellipsis_lines_ratio)
        add({A("gopher_too_many_end_ellipsis_lines (ratio "), F2(ell_lines), A(", max "),
             F2(*c.max_ellipsis_lines_ratio), A(")")});
      if (c.max_non_alpha_words_ratio && alpha < *c.max_non_alpha_words_ratio)
        add({A("gopher_below_alpha_threshold (alpha ratio "), F2(alpha), A(", required min "),
             F2(*c.max_non_alpha_words_ratio), A(")")});
      if (c.min_stop_words && *c.min_stop_words > 0 && r[rec::GQ_STOP] < *c.min_stop_words)
        add({A("gopher_too_few_stop_words (found "), A(r[rec::GQ_STOP]), A(", required "), A(*c.min_stop_words),
             A(")")});
      finish_multi("gopher_quality_filter_status", "gopher_quality_filter_reasons");
      return;
    }
    case StepKind::GopherRepetition: {  // reference gopher_rep.rs:52-220
      if (r[rec::GR_CHARS] < 0) {
        k.fail();
        k.set_reason({A("skipping empty content")});
        k.meta("gopher_repetition_filter_status", {A("filtered")});
        k.meta("gopher_repetition_filter_reason", {A("skipping empty content")});
        return;
      }
      const double C = (double)std::max<int64_t>(1, r[rec::GR_CHARS]);
      const double para_len = (double)std::max<int64_t>(1, r[rec::GR_PARA]);
      const double line_len = (double)std::max<int64_t>(1, r[rec::GR_LINES]);
      double v;
      v = (double)r[rec::GR_PARA_DUP] / para_len;
      if (c.dup_para_frac && v > *c.dup_para_frac)
        add({A("dup_para_frac (ratio "), F2(v), A(", max "), F2(*c.dup_para_frac), A(")")});
      v = (double)r[rec::GR_PARA_DUP_BYTES] / C;
      if (c.dup_para_char_frac && v > *c.dup_para_char_frac)
        add({A("dup_para_char_frac (ratio "), F2(v), A(", max "), F2(*c.dup_para_char_frac), A(")")});
      v = (double)r[rec::GR_LINE_DUP] / line_len;
      if (c.dup_line_frac && v > *c.dup_line_frac)
        add({A("dup_line_frac (ratio "), F2(v), A(", max "), F2(*c.dup_line_frac), A(")")});
      v = (double)r[rec::GR_LINE_DUP_BYTES] / C;
      if (c.dup_line_char_frac && v > *c.dup_line_char_frac)
        add({A("dup_line_char_frac (ratio "), F2(v), A(", max "), F2(*c.dup_line_char_frac), A(")")});
      int kk = rec::GR_FIXED;
      for (auto& e : c.top_n_grams) {
        v = (double)r[kk++] / C;
        if (e.first > 0 && v > e.second)
          add({A("top_"), A(e.first), A("_gram (ratio "), F2(v), A(", max "), F2(e.second), A(")")});
      }
      for (auto& e : c.dup_n_grams) {
        v = (double)r[kk++] / C;
        if (e.first > 0 && v > e.second)
          add({A("duplicated_"), A(e.first), A("_n_grams (ratio "), F2(v), A(", max "), F2(e.second), A(")")});
      }
      finish_multi("gopher_repetition_filter_status", "gopher_repetition_filter_reasons");
      return;
    }
    case StepKind::C4Quality: {  // reference c4_filters.rs:147-295
      if (r[rec::C4_LOREM]) add({A("lorem_ipsum")});
      if (r[rec::C4_CURLY]) add({A("curly_bracket")});
      if (any) {
        finish_multi("c4_filter_status", "c4_filter_reasons");
        return;
      }
      if (c.min_num_sentences > 0 && r[rec::C4_SENTENCES] < c.min_num_sentences) {
        k.fail();
        k.set_reason({A("too_few_sentences (found "), A(r[rec::C4_SENTENCES]), A(", required "),
                      A(c.min_num_sentences), A(")")});
        k.meta("c4_filter_status", {A("filtered")});
        k.meta_reasons("c4_filter_reasons");
        if (r[rec::C4_TOO_LONG]) k.meta("line-filter-too_long_word", {A(r[rec::C4_TOO_LONG])});
        if (r[rec::C4_NO_PUNCT]) k.meta("line-filter-no_terminal_punc", {A(r[rec::C4_NO_PUNCT])});
        if (r[rec::C4_TOO_FEW]) k.meta("line-filter-too_few_words", {A(r[rec::C4_TOO_FEW])});
        return;
      }
      k.meta("c4_filter_status", {A("passed")});
      return;
    }
    case StepKind::FineWebQuality: {  // reference fineweb_quality.rs:71-226
      auto fail = [&](std::initializer_list<Arg> reason, std::initializer_list<Arg> meta_value) {
        k.fail();
        k.set_reason(reason);
        k.meta("fineweb_filter_status", {A("filtered")});
        k.meta("fineweb_filter_reason", meta_value);
      };
      const int64_t nl = r[rec::FW_LINES];
      if (nl == 0) { fail({A("empty")}, {A("empty document")}); return; }
      double ratio = (double)r[rec::FW_STOP_END] / (double)nl;
      if (ratio < c.line_punct_thr && !(ratio == 0.0 && c.line_punct_exclude_zero)) {
        const std::initializer_list<Arg> m = {A("line_punct_ratio: "), F4(ratio), A(" < threshold "),
                                              F4(c.line_punct_thr), A(" (exclude_zero: "),
                                              A(c.line_punct_exclude_zero ? "true" : "false"), A(")")};
        fail(m, m);
        return;
      }
      ratio = (double)r[rec::FW_SHORT] / (double)nl;
      if (ratio > c.short_line_thr) {
        const std::initializer_list<Arg> m = {A("short_line_ratio: "), F4(ratio), A(" > threshold "),
                                              F4(c.short_line_thr)};
        fail(m, m);
        return;
      }
      const int64_t tot = r[rec::FW_CHARS_NO_NL];
      ratio = tot > 0 ? (double)r[rec::FW_DUP_BYTES] / (double)tot : 0.0;
      if (ratio > c.char_duplicates_ratio) {
        const std::initializer_list<Arg> m = {A("char_dup_ratio: "), F4(ratio), A(" > threshold "),
                                              F4(c.char_duplicates_ratio)};
        fail(m, m);
        return;
      }
      const int64_t w = r[rec::FW_WORDS], nls = r[rec::FW_NL];
      if (w == 0) {
        if (nls > 0) {
          const std::initializer_list<Arg> m = {A("list_ratio_no_words (newlines present but no words)")};
          fail(m, m);
        }
        return;
      }
      ratio = (double)nls / (double)w;
      if (ratio > c.new_line_ratio) {
        const std::initializer_list<Arg> m = {A("list_ratio: "), F4(ratio), A(" > threshold "), F4(c.new_line_ratio)};
        fail(m, m);
      }
      return;
    }
    case StepKind::LanguageDetection: {  // reference language_filter.rs:35-93
      const int64_t lang = r[rec::LD_LANG];
      if (lang < 0) {
        k.fail();
        k.set_reason({A("Language could not be confidently detected")});
        return;
      }
      double conf;
      std::memcpy(&conf, &r[rec::LD_CONF_BITS], sizeof(double));
      k.meta("Detected language", {A(kLangNames[lang])});
      k.meta("Detected language confidence", {F64(conf)});
      bool allowed = std::find(c.allowed_langs.begin(), c.allowed_langs.end(), (int)lang) != c.allowed_langs.end();
      if (!allowed) {
        k.fail();
        if constexpr (Sink::kFmt) {
          std::string joined;
          for (size_t i = 0; i < c.allowed_codes.size(); ++i) {
            if (i) joined += "; ";
            joined += c.allowed_codes[i];
          }
          const std::string dbg = fmt_debug_str(joined);
          k.set_reason({A("Document is not any of the following languages: "), A(std::string_view(dbg))});
        }
      } else if (conf < c.min_confidence) {
        k.fail();
        k.set_reason({A("Language detection confidence is not satified: "), F64(conf), A(" < "),
                      F64(c.min_confidence)});
      }
      return;
    }
    case StepKind::TokenCounter: {  // reference token_counter.rs:31-42
      if (r[rec::TC_COUNT] < 0) {
        k.fail_error();
        k.set_reason({A("TokenCounter failed")});
        return;
      }
      k.meta("token_count", {A(r[rec::TC_COUNT])});
      return;
    }
    case StepKind::C4BadWords:
      return;  // decided by the badwords module (needs per-document language strings)
  }
}

void decide(const StepCfg& c, const int64_t* r, Decision& d) {
  d.pass = true;
  d.error = false;
  d.reason.clear();
  d.meta.clear();
  DecisionSink k(d);
  decide_t(c, r, k);
  k.finish();
}

uint8_t decide_status(const StepCfg& c, const int64_t* r) {
  StatusSink k;
  decide_t(c, r, k);
  return k.pass ? 0 : (k.error ? 2 : 1);
}

void decide_meta_json(const StepCfg& c, const int64_t* r, CharBuf& out, bool& first) {
  thread_local ReasonBuf rb;
  thread_local CharBuf tmp;
  rb.r.clear();
  rb.any = false;
  JsonSink k{out, first, rb, tmp};
  decide_t(c, r, k);
}

}  // namespace tb
