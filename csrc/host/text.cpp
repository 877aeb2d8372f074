#include "text.h"

#include <unicode/ubrk.h>
#include <unicode/utext.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "../common/ucd_tables.inc"
#include "../common/uax29.h"

namespace tb {

const UcdView& host_ucd() {
  static const UcdView v{TB_UCD_PROPS_STAGE1, (const uint32_t*)TB_UCD_PROPS_STAGE2,
                         TB_UCD_LOWER_STAGE1, TB_UCD_LOWER_STAGE2};
  return v;
}

void CpView::build(std::string_view s) {
  cp.clear(); off.clear(); prop.clear();
  cp.reserve(s.size()); off.reserve(s.size() + 1); prop.reserve(s.size());
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t n = (uint32_t)s.size();
  const UcdView& u = host_ucd();
  for (uint32_t i = 0; i < n;) {
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    cp.push_back(c);
    off.push_back(i);
    prop.push_back(u.props(c));
    i += len;
  }
  off.push_back(n);
}

size_t count_chars(std::string_view s) {
  size_t c = 0;
  for (unsigned char ch : s) c += (ch & 0xC0) != 0x80;
  return c;
}

bool is_ws_cp(uint32_t cp) { return (props_of(cp) & P_WS) != 0; }

std::string_view trim_start(std::string_view s) {
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t n = (uint32_t)s.size(), i = 0;
  while (i < n) {
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    if (!is_ws_cp(c)) break;
    i += len;
  }
  return s.substr(i);
}

std::string_view trim_end(std::string_view s) {
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t e = (uint32_t)s.size();
  while (e > 0) {
    uint32_t st = e - 1;
    while (st > 0 && (b[st] & 0xC0) == 0x80) --st;
    int len;
    uint32_t c = utf8_decode(b, st, e, &len);
    if (!is_ws_cp(c)) break;
    e = st;
  }
  return s.substr(0, e);
}

std::string_view trim(std::string_view s) { return trim_end(trim_start(s)); }

std::vector<std::string_view> rust_lines(std::string_view s) {
  std::vector<std::string_view> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find('\n', i);
    if (j == std::string_view::npos) {
      out.push_back(s.substr(i));
      break;
    }
    std::string_view line = s.substr(i, j - i);
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    out.push_back(line);
    i = j + 1;
  }
  return out;
}

static bool case_ignorable_then_cased_back(const CpView& v, int i) {
  // scan code points i-1, i-2, ... skipping case-ignorable; true if the first other one is cased
  for (int k = i - 1; k >= 0; --k) {
    uint32_t p = v.prop[k];
    if (p & P_CASE_IGN) continue;
    return (p & P_CASED) != 0;
  }
  return false;
}
static bool case_ignorable_then_cased_fwd(const CpView& v, int i) {
  for (int k = i + 1; k < v.n(); ++k) {
    uint32_t p = v.prop[k];
    if (p & P_CASE_IGN) continue;
    return (p & P_CASED) != 0;
  }
  return false;
}

std::string rust_lowercase(std::string_view s) {
  std::string out;
  out.reserve(s.size());
  bool ascii = true;
  for (unsigned char c : s) if (c >= 0x80) { ascii = false; break; }
  if (ascii) {
    for (unsigned char c : s) out.push_back((c >= 'A' && c <= 'Z') ? c + 32 : c);
    return out;
  }
  CpView v;
  v.build(s);
  const UcdView& u = host_ucd();
  uint8_t buf[4];
  for (int i = 0; i < v.n(); ++i) {
    uint32_t c = v.cp[i];
    uint32_t lc;
    if (c == 0x3A3) {
      bool fin = case_ignorable_then_cased_back(v, i) && !case_ignorable_then_cased_fwd(v, i);
      lc = fin ? 0x3C2 : 0x3C3;
    } else {
      lc = u.lower(c);
    }
    int k = utf8_encode(lc, buf);
    out.append((const char*)buf, k);
    if (c == 0x130) out.append("\xCC\x87");  // U+0307 COMBINING DOT ABOVE
  }
  return out;
}

uint32_t last_cp(std::string_view s) {
  if (s.empty()) return 0xFFFFFFFFu;
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t st = (uint32_t)s.size() - 1;
  while (st > 0 && (b[st] & 0xC0) == 0x80) --st;
  int len;
  return utf8_decode(b, st, (uint32_t)s.size(), &len);
}

uint32_t first_cp(std::string_view s) {
  if (s.empty()) return 0xFFFFFFFFu;
  int len;
  return utf8_decode((const uint8_t*)s.data(), 0, (uint32_t)s.size(), &len);
}

bool ends_with(std::string_view s, std::string_view suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}
bool starts_with(std::string_view s, std::string_view pre) {
  return s.size() >= pre.size() && s.compare(0, pre.size(), pre) == 0;
}

size_t count_nonoverlap(std::string_view s, std::string_view pat) {
  size_t c = 0, i = 0;
  while (true) {
    size_t j = s.find(pat, i);
    if (j == std::string_view::npos) break;
    ++c;
    i = j + pat.size();
  }
  return c;
}

bool has_dict_script(std::string_view s) {
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t n = (uint32_t)s.size();
  for (uint32_t i = 0; i < n;) {
    if (b[i] < 0xE0) { i += b[i] < 0x80 ? 1 : 2; continue; }  // dictionary scripts are >= U+0E00
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    if (props_of(c) & P_DICT) return true;
    i += len;
  }
  return false;
}

// ------------------------------------------------------------------------------------------
// ICU4C backend (the oracle). Break iterators are cached per thread.
namespace {
struct IcuIters {
  UBreakIterator* word = nullptr;
  UBreakIterator* sent = nullptr;
  UText* ut = nullptr;
  IcuIters() {
    UErrorCode ec = U_ZERO_ERROR;
    word = ubrk_open(UBRK_WORD, "", nullptr, 0, &ec);
    if (U_FAILURE(ec)) throw std::runtime_error("ubrk_open(word) failed");
    ec = U_ZERO_ERROR;
    sent = ubrk_open(UBRK_SENTENCE, "", nullptr, 0, &ec);
    if (U_FAILURE(ec)) throw std::runtime_error("ubrk_open(sentence) failed");
  }
  ~IcuIters() {
    if (word) ubrk_close(word);
    if (sent) ubrk_close(sent);
    if (ut) utext_close(ut);
  }
};
thread_local IcuIters tl_icu;

std::vector<uint32_t> icu_breaks(UBreakIterator* bi, std::string_view s) {
  std::vector<uint32_t> out;
  UErrorCode ec = U_ZERO_ERROR;
  tl_icu.ut = utext_openUTF8(tl_icu.ut, s.data(), (int64_t)s.size(), &ec);
  ec = U_ZERO_ERROR;
  ubrk_setUText(bi, tl_icu.ut, &ec);
  for (int32_t p = ubrk_first(bi); p != UBRK_DONE; p = ubrk_next(bi)) out.push_back((uint32_t)p);
  return out;
}

struct VecAcc {
  const CpView* v;
  uint32_t p(int i) const { return v->prop[i]; }
};

std::vector<uint32_t> rule_breaks(std::string_view s, bool word) {
  std::vector<uint32_t> out;
  if (s.empty()) return {0};
  CpView v;
  v.build(s);
  VecAcc a{&v};
  int n = v.n();
  out.push_back(0);
  for (int i = 1; i < n; ++i)
    if (word ? wb_break(a, n, i) : sb_break(a, n, i)) out.push_back(v.off[i]);
  out.push_back((uint32_t)s.size());
  return out;
}
}  // namespace

std::vector<uint32_t> word_breaks(std::string_view s, SegBackend be) {
  if (be == SegBackend::Icu || has_dict_script(s)) return icu_breaks(tl_icu.word, s);
  return rule_breaks(s, true);
}

std::vector<uint32_t> sentence_breaks(std::string_view s, SegBackend be) {
  if (be == SegBackend::Icu) return icu_breaks(tl_icu.sent, s);
  return rule_breaks(s, false);
}

static bool has_word_char(std::string_view t) {
  const uint8_t* b = (const uint8_t*)t.data();
  uint32_t n = (uint32_t)t.size();
  for (uint32_t i = 0; i < n;) {
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    uint32_t p = props_of(c);
    if (!(p & P_PUNCT) && !(p & P_WS)) return true;
    i += len;
  }
  return false;
}

std::vector<std::string_view> split_into_words(std::string_view s, SegBackend be) {
  std::vector<std::string_view> words;
  if (s.empty()) return words;
  std::vector<uint32_t> br = word_breaks(s, be);
  uint32_t prev = 0;
  auto consider = [&](uint32_t a, uint32_t b) {
    std::string_view seg = trim(s.substr(a, b - a));
    if (!seg.empty() && has_word_char(seg)) words.push_back(seg);
  };
  for (uint32_t cur : br) {
    if (cur > prev) consider(prev, cur);
    prev = cur;
  }
  if (s.size() > prev) consider(prev, (uint32_t)s.size());
  return words;
}

std::vector<std::string_view> split_into_sentences(std::string_view s, SegBackend be) {
  std::vector<std::string_view> out;
  std::string_view t = trim(s);
  if (t.empty()) return out;
  std::vector<uint32_t> br = sentence_breaks(t, be);
  // Starts are every break except the final end offset.
  for (size_t i = 0; i + 1 < br.size(); ++i) {
    uint32_t a = br[i], b = br[i + 1];
    if (a > b) continue;
    std::string_view seg = trim(t.substr(a, b - a));
    if (!seg.empty()) out.push_back(seg);
  }
  if (br.size() <= 1) out.push_back(t);
  return out;
}

std::pair<size_t, size_t> find_duplicates(const std::vector<std::string_view>& items) {
  std::unordered_set<std::string_view> seen;
  seen.reserve(items.size() * 2);
  size_t elems = 0, bytes = 0;
  for (auto& it : items) {
    if (!seen.insert(it).second) {
      ++elems;
      bytes += it.size();
    }
  }
  return {elems, bytes};
}

size_t find_top_duplicate_ngrams(const std::vector<std::string_view>& words, size_t n) {
  if (n == 0 || words.size() < n) return 0;
  std::unordered_map<std::string, size_t> cnt;
  cnt.reserve(words.size() * 2);
  std::string g;
  for (size_t i = 0; i + n <= words.size(); ++i) {
    g.clear();
    for (size_t k = 0; k < n; ++k) {
      if (k) g.push_back(' ');
      g.append(words[i + k].data(), words[i + k].size());
    }
    ++cnt[g];
  }
  size_t maxc = 0;
  for (auto& kv : cnt) maxc = std::max(maxc, kv.second);
  if (maxc <= 1) return 0;
  size_t best = 0;
  for (auto& kv : cnt)
    if (kv.second == maxc) best = std::max(best, kv.first.size() * maxc);
  return best;
}

size_t find_all_duplicate(const std::vector<std::string_view>& words, size_t n) {
  if (n == 0 || words.size() < n) return 0;
  std::unordered_set<std::string> uniq;
  uniq.reserve(words.size() * 2);
  size_t rep = 0, idx = 0, W = words.size();
  std::string g;
  while (idx + n <= W) {
    g.clear();
    for (size_t k = 0; k < n; ++k) g.append(words[idx + k].data(), words[idx + k].size());
    if (!uniq.insert(g).second) {
      rep += g.size();
      idx += n;
    } else {
      idx += 1;
    }
  }
  return rep;
}

std::string remove_citations(std::string_view s) {
  const uint8_t* b = (const uint8_t*)s.data();
  const uint32_t n = (uint32_t)s.size();
  std::string out;
  out.reserve(n);
  uint32_t i = 0, copied = 0;
  auto is_digit_at = [&](uint32_t pos, int* len) -> bool {
    if (pos >= n) return false;
    uint32_t c = utf8_decode(b, pos, n, len);
    return (props_of(c) & P_DIGIT) != 0;
  };
  auto is_space_at = [&](uint32_t pos, int* len) -> bool {
    if (pos >= n) return false;
    uint32_t c = utf8_decode(b, pos, n, len);
    return (props_of(c) & P_WS) != 0;
  };
  while (i < n) {
    if (b[i] != '[') { ++i; continue; }
    // try to match at i
    uint32_t p = i + 1;
    int len;
    bool ok = false;
    if (is_digit_at(p, &len)) {
      while (is_digit_at(p, &len)) p += len;
      while (true) {
        if (p < n && b[p] == ',') {
          uint32_t q = p + 1;
          while (is_space_at(q, &len)) q += len;
          if (is_digit_at(q, &len)) {
            while (is_digit_at(q, &len)) q += len;
            p = q;
            continue;
          }
        }
        break;
      }
      if (p < n && b[p] == ']') ok = true;
    }
    if (ok) {
      out.append(s.data() + copied, i - copied);
      i = p + 1;
      copied = i;
    } else {
      ++i;
    }
  }
  out.append(s.data() + copied, n - copied);
  return out;
}

}  // namespace tb
