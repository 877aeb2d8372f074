#include "text.h"

#include <unicode/ubrk.h>
#include <unicode/utext.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "../common/ucd_tables.inc"
#include "../common/uax29.h"
#include "../common/hash.h"
#include "pipeline.h"

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
  // dictionary scripts start at U+0E00: only 3- and 4-byte sequences (lead bytes >= 0xE0) can hold
  // one; eight bytes at a time are skipped while none of them is such a lead byte
  const uint8_t* b = (const uint8_t*)s.data();
  const uint32_t n = (uint32_t)s.size();
  uint32_t i = 0;
  while (i < n) {
    if (i + 8 <= n) {
      uint64_t v;
      std::memcpy(&v, b + i, 8);
      if (!(v & (v << 1) & (v << 2) & 0x8080808080808080ull)) {
        i += 8;
        continue;
      }
    }
    if (b[i] < 0xE0) { ++i; continue; }
    int len;
    const uint32_t c = utf8_decode(b, i, n, &len);
    if (props_of(c) & P_DICT) return true;
    i += (uint32_t)len;
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

namespace {
// any byte >= 0xE0 in [b, b + n): the lead bytes of the 3- and 4-byte sequences (dictionary
// scripts start at U+0E00); eight bytes per step (bit 7 of a byte & its bits 6 and 5)
bool any_e0(const uint8_t* b, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    std::memcpy(&v, b + i, 8);
    if (v & (v << 1) & (v << 2) & 0x8080808080808080ull) return true;
  }
  for (; i < n; ++i)
    if (b[i] >= 0xE0) return true;
  return false;
}
bool valid_utf8(const uint8_t* b, size_t n) {
  for (size_t i = 0; i < n;) {
    const uint8_t c = b[i];
    size_t len;
    uint32_t cp;
    if (c < 0x80) { ++i; continue; }
    if (c >= 0xC2 && c <= 0xDF) { len = 2; cp = c & 0x1F; }
    else if (c >= 0xE0 && c <= 0xEF) { len = 3; cp = c & 0x0F; }
    else if (c >= 0xF0 && c <= 0xF4) { len = 4; cp = c & 0x07; }
    else return false;
    if (i + len > n) return false;
    for (size_t k = 1; k < len; ++k) {
      if ((b[i + k] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (b[i + k] & 0x3F);
    }
    if ((len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    i += len;
  }
  return true;
}
}  // namespace

void dict_word_marks(const uint8_t* data, const int64_t* off, int64_t ndocs, int nthreads,
                     std::vector<int64_t>& moff, std::vector<uint32_t>& bits) {
  moff.assign(ndocs, -1);
  std::vector<std::vector<uint32_t>> per(ndocs);
  parallel_for(ndocs, nthreads, [&](int64_t a, int64_t e) {
    for (int64_t d = a; d < e; ++d) {
      const uint8_t* b = data + off[d];
      const size_t n = (size_t)(off[d + 1] - off[d]);
      if (!any_e0(b, n)) continue;
      const std::string_view s((const char*)b, n);
      if (!has_dict_script(s) || !valid_utf8(b, n)) continue;
      uint32_t C = 0, Cdict = 0;
      for (size_t i = 0; i < n;) {
        int len;
        const uint32_t c = utf8_decode(b, (uint32_t)i, (uint32_t)n, &len);
        ++C;
        Cdict += (props_of(c) & P_DICT) ? 1u : 0u;
        i += (size_t)len;
      }
      // mostly dictionary-script text (a CJK or Thai document): no marks — in a pipeline for other
      // languages the language gate filters it before any segmentation, and segmenting all of it
      // by dictionary costs the host more than the rare survivor's CPU path
      if (2 * Cdict > C) continue;
      const uint32_t mw = ((C + 1 + 63) / 64) * 2;
      std::vector<uint32_t>& m = per[d];
      m.assign(2 * (size_t)mw, 0u);
      uint32_t* hb = m.data();       // ICU's marks
      uint32_t* hm = m.data() + mw;  // which positions take them
      // lines ('\n'-separated) that hold a dictionary-script code point: ICU over that line alone
      // (word breaks never look across a line feed: WB3a / WB3b), marks for its code points
      // [line start, its '\n') — the '\n' itself and every other line keep the device's rules
      uint32_t cp0 = 0;
      size_t l0 = 0;
      bool ok = true;
      while (l0 <= n && ok) {
        size_t l1 = l0;
        while (l1 < n && b[l1] != '\n') ++l1;
        uint32_t ncp = 0;
        bool dict = false;
        for (size_t i = l0; i < l1;) {
          int len;
          const uint32_t c = utf8_decode(b, (uint32_t)i, (uint32_t)n, &len);
          dict |= (props_of(c) & P_DICT) != 0;
          ++ncp;
          i += (size_t)len;
        }
        if (dict) {
          const std::string_view line((const char*)b + l0, l1 - l0);
          const std::vector<uint32_t> br = icu_breaks(tl_icu.word, line);
          uint32_t cp = 0;
          size_t at = 0;
          for (uint32_t o : br) {
            if (o > line.size() || (o < line.size() && (line[o] & 0xC0) == 0x80)) { ok = false; break; }
            for (; at < o; ++at) cp += (line[at] & 0xC0) != 0x80;
            if (cp < ncp) hb[(cp0 + cp) >> 5] |= 1u << ((cp0 + cp) & 31);
          }
          for (uint32_t q = cp0; q < cp0 + ncp; ++q) hm[q >> 5] |= 1u << (q & 31);
        }
        cp0 += ncp + (l1 < n ? 1u : 0u);  // the line's code points and its '\n'
        l0 = l1 + 1;
      }
      if (!ok || cp0 != C) m.clear();
    }
  });
  size_t tot = 0;
  for (int64_t d = 0; d < ndocs; ++d)
    if (!per[d].empty()) { moff[d] = (int64_t)tot; tot += per[d].size(); }
  bits.assign(tot, 0u);
  for (int64_t d = 0; d < ndocs; ++d)
    if (moff[d] >= 0) std::memcpy(bits.data() + moff[d], per[d].data(), per[d].size() * 4);
}

void dict_c4_lines(const uint8_t* text, const int64_t* off, int64_t ndocs, const int64_t* moff, bool citations,
                   int nthreads, std::vector<int64_t>& loff, std::vector<uint32_t>& data) {
  loff.assign(ndocs, -1);
  std::vector<std::vector<uint32_t>> per(ndocs);
  parallel_for(ndocs, nthreads, [&](int64_t a, int64_t e) {
    for (int64_t d = a; d < e; ++d) {
      if (moff[d] < 0) continue;
      const std::string_view s((const char*)text + off[d], (size_t)(off[d + 1] - off[d]));
      if (s.find('[') == std::string_view::npos) continue;
      std::vector<uint32_t>& v = per[d];
      const std::vector<std::string_view> lines = rust_lines(s);
      v.reserve(1 + 2 * lines.size());
      v.push_back((uint32_t)lines.size());
      for (auto line : lines) {
        const std::string_view cur = trim(line);
        const std::string proc = citations ? remove_citations(cur) : std::string(cur);
        uint32_t nw = 0, mx = 0;
        // (Rules: word_breaks takes ICU for a line with a dictionary script, the UAX#29 rules for
        // the others, which match ICU there — the device's own segmentation)
        for (auto w : split_into_words(proc, SegBackend::Rules)) {
          ++nw;
          mx = std::max(mx, (uint32_t)count_chars(w));
        }
        v.push_back(nw);
        v.push_back(mx);
      }
    }
  });
  size_t tot = 0;
  for (int64_t d = 0; d < ndocs; ++d)
    if (!per[d].empty()) { loff[d] = (int64_t)tot; tot += per[d].size(); }
  data.assign(tot, 0u);
  for (int64_t d = 0; d < ndocs; ++d)
    if (loff[d] >= 0) std::memcpy(data.data() + loff[d], per[d].data(), per[d].size() * 4);
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

namespace {
// Open-addressing set of (64-bit key, element) pairs; equality of elements is decided by the
// caller's exact comparison, the key only groups candidates.
struct KeyTable {
  std::vector<uint64_t> key;
  std::vector<uint32_t> val;  // element + 1 (0 = empty)
  uint64_t mask = 0;
  explicit KeyTable(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 2) cap <<= 1;
    key.assign(cap, 0);
    val.assign(cap, 0);
    mask = cap - 1;
  }
  // slot of an element equal to `e` (eq(stored, e)), or the empty slot where it goes
  template <class Eq>
  size_t find(uint64_t k, Eq&& eq) const {
    size_t s = (size_t)((k ^ (k >> 29)) * 0x9E3779B97F4A7C15ull >> 20) & mask;
    while (val[s] != 0 && !(key[s] == k && eq(val[s] - 1))) s = (s + 1) & mask;
    return s;
  }
};

inline uint64_t mix64h(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
}  // namespace

void ngram_stats(const std::vector<std::string_view>& words, const std::vector<size_t>& top,
                 const std::vector<size_t>& dup, size_t* out_top, size_t* out_dup) {
  const size_t W = words.size();
  // word hashes (polynomial over the bytes), B^len, and canonical ids (smallest equal index)
  std::vector<uint64_t> wh(W), wp(W);
  std::vector<uint32_t> id(W);
  for (size_t j = 0; j < W; ++j) {
    uint64_t h = 0, p = 1;
    for (unsigned char c : words[j]) {
      h = hash_push(h, c);
      p *= kHashBase;
    }
    wh[j] = h;
    wp[j] = p;
  }
  bool need_ids = false;
  for (size_t n : top) need_ids |= n > 0 && W >= n;
  if (need_ids) {
    KeyTable t(W);
    for (size_t j = 0; j < W; ++j) {
      const uint64_t k = mix64h(wh[j] ^ ((uint64_t)words[j].size() << 48));
      const size_t s = t.find(k, [&](uint32_t e) { return words[e] == words[j]; });
      if (t.val[s] == 0) {
        t.key[s] = k;
        t.val[s] = (uint32_t)j + 1;
      }
      id[j] = t.val[s] - 1;
    }
  }
  for (size_t q = 0; q < top.size(); ++q) {
    const size_t n = top[q];
    out_top[q] = 0;
    if (n == 0 || W < n) continue;
    const size_t G = W - n + 1;
    KeyTable t(G);
    std::vector<uint32_t> cnt(G, 0);
    for (size_t p = 0; p < G; ++p) {
      uint64_t k = (uint64_t)n << 56;
      for (size_t i = 0; i < n; ++i) k = (k ^ id[p + i]) * 0x9E3779B97F4A7C15ull + i;
      k = mix64h(k);
      const size_t s = t.find(k, [&](uint32_t e) {
        for (size_t i = 0; i < n; ++i)
          if (id[e + i] != id[p + i]) return false;
        return true;
      });
      if (t.val[s] == 0) {
        t.key[s] = k;
        t.val[s] = (uint32_t)p + 1;
      }
      ++cnt[t.val[s] - 1];
    }
    size_t maxc = 0;
    for (size_t p = 0; p < G; ++p) maxc = std::max<size_t>(maxc, cnt[p]);
    if (maxc <= 1) continue;
    size_t best = 0;
    for (size_t p = 0; p < G; ++p) {
      if (cnt[p] != maxc) continue;
      size_t len = n - 1;  // the joining spaces
      for (size_t i = 0; i < n; ++i) len += words[p + i].size();
      best = std::max(best, len * maxc);
    }
    out_top[q] = best;
  }
  for (size_t q = 0; q < dup.size(); ++q) {
    const size_t n = dup[q];
    out_dup[q] = 0;
    if (n == 0 || W < n) continue;
    // concatenation (no separator) of words p .. p + n - 1: hash, byte length, byte equality
    auto concat = [&](size_t p, size_t* len) {
      uint64_t h = 0;
      size_t l = 0;
      for (size_t i = 0; i < n; ++i) {
        h = h * wp[p + i] + wh[p + i];
        l += words[p + i].size();
      }
      *len = l;
      return h;
    };
    auto concat_eq = [&](size_t a, size_t b) {
      size_t ia = a, ib = b, oa = 0, ob = 0;
      while (ia < a + n && ib < b + n) {
        const std::string_view x = words[ia], y = words[ib];
        const size_t m = std::min(x.size() - oa, y.size() - ob);
        if (std::memcmp(x.data() + oa, y.data() + ob, m) != 0) return false;
        oa += m;
        ob += m;
        if (oa == x.size()) { ++ia; oa = 0; }
        if (ob == y.size()) { ++ib; ob = 0; }
      }
      // (equal total lengths are checked by the caller; skip trailing empty words)
      while (ia < a + n && words[ia].empty()) ++ia;
      while (ib < b + n && words[ib].empty()) ++ib;
      return ia == a + n && ib == b + n;
    };
    KeyTable t(W - n + 1);
    std::vector<size_t> glen(W - n + 1, 0);
    size_t rep = 0, idx = 0;
    while (idx + n <= W) {
      size_t len;
      const uint64_t h = concat(idx, &len);
      const uint64_t k = mix64h(h ^ ((uint64_t)len << 40));
      const size_t s = t.find(k, [&](uint32_t e) { return glen[e] == len && concat_eq(e, idx); });
      if (t.val[s] != 0) {
        rep += len;
        idx += n;
      } else {
        t.key[s] = k;
        t.val[s] = (uint32_t)idx + 1;
        glen[idx] = len;
        idx += 1;
      }
    }
    out_dup[q] = rep;
  }
}

size_t find_top_duplicate_ngrams(const std::vector<std::string_view>& words, size_t n) {
  size_t out = 0;
  ngram_stats(words, {n}, {}, &out, nullptr);
  return out;
}

size_t find_all_duplicate(const std::vector<std::string_view>& words, size_t n) {
  size_t out = 0;
  ngram_stats(words, {}, {n}, nullptr, &out);
  return out;
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
