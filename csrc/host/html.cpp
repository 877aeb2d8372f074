// HTML entity decoding of input text, as the reference reader does with
// html_escape::decode_html_entities (reference parquet_reader.rs:177-179).
//
// Semantics implemented: `&name;` for the HTML5 named references, `&#DDD;` and `&#xHHH;`
// numeric references that denote a Unicode scalar value; anything else is copied verbatim.
// (Legacy references without the terminating ';' are left as-is: parity unpinned, the crate
// source is not available offline.)
#include "html.h"

#include <cstring>

#include "html_entities.inc"

namespace tb {

static const HtmlEntity* find_entity(const char* name, size_t len) {
  int lo = 0, hi = kHtmlEntityCount - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    int c = strncmp(kHtmlEntities[mid].name, name, len);
    if (c == 0 && kHtmlEntities[mid].name[len] != 0) c = 1;
    if (c == 0) return &kHtmlEntities[mid];
    if (c < 0) lo = mid + 1; else hi = mid - 1;
  }
  return nullptr;
}

static inline bool is_alnum(char c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}

static void put_utf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) o.push_back((char)cp);
  else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

bool html_decode(std::string_view s, std::string& out) {
  const void* amp = memchr(s.data(), '&', s.size());
  if (!amp) return false;
  out.clear();
  out.reserve(s.size());
  size_t i = 0, n = s.size();
  while (i < n) {
    const char* a = (const char*)memchr(s.data() + i, '&', n - i);
    if (!a) { out.append(s.data() + i, n - i); break; }
    size_t p = (size_t)(a - s.data());
    out.append(s.data() + i, p - i);
    size_t q = p + 1;
    bool done = false;
    if (q < n && s[q] == '#') {
      ++q;
      bool hex = false;
      if (q < n && (s[q] == 'x' || s[q] == 'X')) { hex = true; ++q; }
      size_t ds = q;
      uint64_t v = 0;
      bool overflow = false;
      while (q < n && (hex ? isxdigit((unsigned char)s[q]) : isdigit((unsigned char)s[q]))) {
        int d = isdigit((unsigned char)s[q]) ? s[q] - '0' : (tolower(s[q]) - 'a' + 10);
        v = v * (hex ? 16 : 10) + d;
        if (v > 0x10FFFF) overflow = true;
        ++q;
      }
      if (q > ds && q < n && s[q] == ';' && !overflow && !(v >= 0xD800 && v < 0xE000)) {
        put_utf8(out, (uint32_t)v);
        i = q + 1;
        done = true;
      }
    } else {
      size_t ns = q;
      while (q < n && is_alnum(s[q]) && q - ns < 40) ++q;
      if (q > ns && q < n && s[q] == ';') {
        const HtmlEntity* e = find_entity(s.data() + ns, q - ns);
        if (e) {
          out += e->utf8;
          i = q + 1;
          done = true;
        }
      }
    }
    if (!done) {
      out.push_back('&');
      i = p + 1;
    }
  }
  return true;
}

}  // namespace tb
