#include "filters.h"

#include <algorithm>
#include <cstring>
#include <unordered_set>

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
  int k = rec::GR_FIXED;
  for (auto& e : c.top_n_grams) r[k++] = (int64_t)find_top_duplicate_ngrams(words, (size_t)e.first);
  for (auto& e : c.dup_n_grams) r[k++] = (int64_t)find_all_duplicate(words, (size_t)e.first);
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
static std::string f2(double x) { return fmt_fixed(x, 2); }
static std::string f4(double x) { return fmt_fixed(x, 4); }

// One implementation of every step's decision logic, instantiated twice: kFmt=false only
// derives pass/filtered/error (the per-batch resolve hot path: no strings are built),
// kFmt=true also formats the reason and the step's metadata (output assembly, per-document
// API). String-building expressions are wrapped in lambdas that the kFmt=false instance never
// calls, so both instances take exactly the same branches.
template <bool kFmt>
static void decide_t(const StepCfg& c, const int64_t* r, Decision& d) {
  d.pass = true;
  d.error = false;
  if constexpr (kFmt) {
    d.reason.clear();
    d.meta.clear();
  }
  std::vector<std::string> reasons;
  int nreasons = 0;
  auto add = [&](auto&& mk) {
    ++nreasons;
    if constexpr (kFmt) reasons.push_back(mk());
  };
  auto meta = [&](std::string_view k, auto&& mk) {
    if constexpr (kFmt) d.meta.emplace_back(k, mk());
  };
  auto lit = [](const char* s) { return [s]() { return std::string(s); }; };
  auto finish_multi = [&](std::string_view status_key, std::string_view reasons_key) {
    if (nreasons) {
      d.pass = false;
      if constexpr (kFmt) {
        d.reason = join(reasons, "; ");
        d.meta.emplace_back(status_key, "filtered");
        d.meta.emplace_back(reasons_key, d.reason);
      }
    } else {
      meta(status_key, lit("passed"));
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
        add([&] { return "gopher_short_doc (" + std::to_string(n) + " non-symbol words, required " +
                         std::to_string(*c.min_doc_words) + ")"; });
      if (c.max_doc_words && n > *c.max_doc_words)
        add([&] { return "gopher_long_doc (" + std::to_string(n) + " non-symbol words, max " +
                         std::to_string(*c.max_doc_words) + ")"; });
      if (c.min_avg_word_length && avg < *c.min_avg_word_length)
        add([&] { return "gopher_below_avg_threshold (avg len " + f2(avg) + ", required " +
                         f2(*c.min_avg_word_length) +
                         ((n == 0 && *c.min_avg_word_length > 0.0) ? " - 0 non-symbol words" : "") + ")"; });
      if (c.max_avg_word_length && n > 0 && avg > *c.max_avg_word_length)
        add([&] { return "gopher_above_avg_threshold (avg len " + f2(avg) + ", max " +
                         f2(*c.max_avg_word_length) + ")"; });
      if (c.max_symbol_word_ratio) {
        if (hash_ratio > *c.max_symbol_word_ratio)
          add([&] { return "gopher_too_many_hashes (ratio " + f2(hash_ratio) + ", max " +
                           f2(*c.max_symbol_word_ratio) + ")"; });
        if (ell_ratio > *c.max_symbol_word_ratio)
          add([&] { return "gopher_too_many_ellipsis_units (ratio " + f2(ell_ratio) + ", max " +
                           f2(*c.max_symbol_word_ratio) + ")"; });
      }
      if (c.max_bullet_lines_ratio && bullet > *c.max_bullet_lines_ratio)
        add([&] { return "gopher_too_many_bullets (ratio " + f2(bullet) + ", max " +
                         f2(*c.max_bullet_lines_ratio) + ")"; });
      if (c.max_ellipsis_lines_ratio && ell_lines > *c.max_ellipsis_lines_ratio)
        add([&] { return "gopher_too_many_end_ellipsis_lines (ratio " + f2(ell_lines) + ", max " +
                         f2(*c.max_ellipsis_lines_ratio) + ")"; });
      if (c.max_non_alpha_words_ratio && alpha < *c.max_non_alpha_words_ratio)
        add([&] { return "gopher_below_alpha_threshold (alpha ratio " + f2(alpha) + ", required min " +
                         f2(*c.max_non_alpha_words_ratio) + ")"; });
      if (c.min_stop_words && *c.min_stop_words > 0 && r[rec::GQ_STOP] < *c.min_stop_words)
        add([&] { return "gopher_too_few_stop_words (found " + std::to_string(r[rec::GQ_STOP]) + ", required " +
                         std::to_string(*c.min_stop_words) + ")"; });
      finish_multi("gopher_quality_filter_status", "gopher_quality_filter_reasons");
      return;
    }
    case StepKind::GopherRepetition: {  // reference gopher_rep.rs:52-220
      if (r[rec::GR_CHARS] < 0) {
        d.pass = false;
        if constexpr (kFmt) {
          d.reason = "skipping empty content";
          d.meta.emplace_back("gopher_repetition_filter_status", "filtered");
          d.meta.emplace_back("gopher_repetition_filter_reason", "skipping empty content");
        }
        return;
      }
      const double C = (double)std::max<int64_t>(1, r[rec::GR_CHARS]);
      const double para_len = (double)std::max<int64_t>(1, r[rec::GR_PARA]);
      const double line_len = (double)std::max<int64_t>(1, r[rec::GR_LINES]);
      double v;
      v = (double)r[rec::GR_PARA_DUP] / para_len;
      if (c.dup_para_frac && v > *c.dup_para_frac)
        add([&] { return "dup_para_frac (ratio " + f2(v) + ", max " + f2(*c.dup_para_frac) + ")"; });
      v = (double)r[rec::GR_PARA_DUP_BYTES] / C;
      if (c.dup_para_char_frac && v > *c.dup_para_char_frac)
        add([&] { return "dup_para_char_frac (ratio " + f2(v) + ", max " + f2(*c.dup_para_char_frac) + ")"; });
      v = (double)r[rec::GR_LINE_DUP] / line_len;
      if (c.dup_line_frac && v > *c.dup_line_frac)
        add([&] { return "dup_line_frac (ratio " + f2(v) + ", max " + f2(*c.dup_line_frac) + ")"; });
      v = (double)r[rec::GR_LINE_DUP_BYTES] / C;
      if (c.dup_line_char_frac && v > *c.dup_line_char_frac)
        add([&] { return "dup_line_char_frac (ratio " + f2(v) + ", max " + f2(*c.dup_line_char_frac) + ")"; });
      int k = rec::GR_FIXED;
      for (auto& e : c.top_n_grams) {
        v = (double)r[k++] / C;
        if (e.first > 0 && v > e.second)
          add([&] { return "top_" + std::to_string(e.first) + "_gram (ratio " + f2(v) + ", max " + f2(e.second) + ")"; });
      }
      for (auto& e : c.dup_n_grams) {
        v = (double)r[k++] / C;
        if (e.first > 0 && v > e.second)
          add([&] { return "duplicated_" + std::to_string(e.first) + "_n_grams (ratio " + f2(v) + ", max " +
                           f2(e.second) + ")"; });
      }
      finish_multi("gopher_repetition_filter_status", "gopher_repetition_filter_reasons");
      return;
    }
    case StepKind::C4Quality: {  // reference c4_filters.rs:147-295
      if (r[rec::C4_LOREM]) add(lit("lorem_ipsum"));
      if (r[rec::C4_CURLY]) add(lit("curly_bracket"));
      if (nreasons) {
        finish_multi("c4_filter_status", "c4_filter_reasons");
        return;
      }
      if (c.min_num_sentences > 0 && r[rec::C4_SENTENCES] < c.min_num_sentences) {
        d.pass = false;
        if constexpr (kFmt) {
          d.reason = "too_few_sentences (found " + std::to_string(r[rec::C4_SENTENCES]) + ", required " +
                     std::to_string(c.min_num_sentences) + ")";
          d.meta.emplace_back("c4_filter_status", "filtered");
          d.meta.emplace_back("c4_filter_reasons", d.reason);
          if (r[rec::C4_TOO_LONG]) d.meta.emplace_back("line-filter-too_long_word", std::to_string(r[rec::C4_TOO_LONG]));
          if (r[rec::C4_NO_PUNCT]) d.meta.emplace_back("line-filter-no_terminal_punc", std::to_string(r[rec::C4_NO_PUNCT]));
          if (r[rec::C4_TOO_FEW]) d.meta.emplace_back("line-filter-too_few_words", std::to_string(r[rec::C4_TOO_FEW]));
        }
        return;
      }
      meta("c4_filter_status", lit("passed"));
      return;
    }
    case StepKind::FineWebQuality: {  // reference fineweb_quality.rs:71-226
      auto fail = [&](auto&& mk_reason, auto&& mk_meta) {
        d.pass = false;
        if constexpr (kFmt) {
          d.reason = mk_reason();
          d.meta.emplace_back("fineweb_filter_status", "filtered");
          d.meta.emplace_back("fineweb_filter_reason", mk_meta());
        }
      };
      const int64_t nl = r[rec::FW_LINES];
      if (nl == 0) { fail(lit("empty"), lit("empty document")); return; }
      double ratio = (double)r[rec::FW_STOP_END] / (double)nl;
      if (ratio < c.line_punct_thr && !(ratio == 0.0 && c.line_punct_exclude_zero)) {
        auto mk = [&] {
          return "line_punct_ratio: " + f4(ratio) + " < threshold " + f4(c.line_punct_thr) + " (exclude_zero: " +
                 (c.line_punct_exclude_zero ? "true" : "false") + ")";
        };
        fail(mk, mk);
        return;
      }
      ratio = (double)r[rec::FW_SHORT] / (double)nl;
      if (ratio > c.short_line_thr) {
        auto mk = [&] { return "short_line_ratio: " + f4(ratio) + " > threshold " + f4(c.short_line_thr); };
        fail(mk, mk);
        return;
      }
      const int64_t tot = r[rec::FW_CHARS_NO_NL];
      ratio = tot > 0 ? (double)r[rec::FW_DUP_BYTES] / (double)tot : 0.0;
      if (ratio > c.char_duplicates_ratio) {
        auto mk = [&] { return "char_dup_ratio: " + f4(ratio) + " > threshold " + f4(c.char_duplicates_ratio); };
        fail(mk, mk);
        return;
      }
      const int64_t w = r[rec::FW_WORDS], nls = r[rec::FW_NL];
      if (w == 0) {
        if (nls > 0) {
          auto mk = lit("list_ratio_no_words (newlines present but no words)");
          fail(mk, mk);
        }
        return;
      }
      ratio = (double)nls / (double)w;
      if (ratio > c.new_line_ratio) {
        auto mk = [&] { return "list_ratio: " + f4(ratio) + " > threshold " + f4(c.new_line_ratio); };
        fail(mk, mk);
      }
      return;
    }
    case StepKind::LanguageDetection: {  // reference language_filter.rs:35-93
      const int64_t lang = r[rec::LD_LANG];
      if (lang < 0) {
        d.pass = false;
        if constexpr (kFmt) d.reason = "Language could not be confidently detected";
        return;
      }
      double conf;
      std::memcpy(&conf, &r[rec::LD_CONF_BITS], sizeof(double));
      meta("Detected language", [&] { return std::string(kLangNames[lang]); });
      meta("Detected language confidence", [&] { return fmt_f64(conf); });
      bool allowed = std::find(c.allowed_langs.begin(), c.allowed_langs.end(), (int)lang) != c.allowed_langs.end();
      if (!allowed) {
        d.pass = false;
        if constexpr (kFmt) {
          std::string joined;
          for (size_t i = 0; i < c.allowed_codes.size(); ++i) {
            if (i) joined += "; ";
            joined += c.allowed_codes[i];
          }
          d.reason = "Document is not any of the following languages: " + fmt_debug_str(joined);
        }
      } else if (conf < c.min_confidence) {
        d.pass = false;
        if constexpr (kFmt)
          d.reason = "Language detection confidence is not satified: " + fmt_f64(conf) + " < " +
                     fmt_f64(c.min_confidence);
      }
      return;
    }
    case StepKind::TokenCounter: {  // reference token_counter.rs:31-42
      if (r[rec::TC_COUNT] < 0) {
        d.pass = false;
        d.error = true;
        if constexpr (kFmt) d.reason = "TokenCounter failed";
        return;
      }
      meta("token_count", [&] { return std::to_string(r[rec::TC_COUNT]); });
      return;
    }
    case StepKind::C4BadWords:
      return;  // decided by the badwords module (needs per-document language strings)
  }
}

void decide(const StepCfg& c, const int64_t* r, Decision& d) { decide_t<true>(c, r, d); }

uint8_t decide_status(const StepCfg& c, const int64_t* r) {
  Decision d;
  decide_t<false>(c, r, d);
  return d.pass ? 0 : (d.error ? 2 : 1);
}

}  // namespace tb
