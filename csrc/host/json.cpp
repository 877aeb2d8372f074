#include "json.h"

#include <cstdint>
#include <cstring>

namespace tb {

namespace {
struct Parser {
  std::string_view s;
  size_t i = 0;
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  bool hex4(uint32_t& v) {
    if (i + 4 > s.size()) return false;
    v = 0;
    for (int k = 0; k < 4; ++k) {
      int h = hexv(s[i + k]);
      if (h < 0) return false;
      v = (v << 4) | (uint32_t)h;
    }
    i += 4;
    return true;
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
  bool str(std::string& o) {
    if (i >= s.size() || s[i] != '"') return false;
    ++i;
    while (i < s.size()) {
      char c = s[i++];
      if (c == '"') return true;
      if ((unsigned char)c < 0x20) return false;  // serde_json rejects raw control characters
      if (c != '\\') { o.push_back(c); continue; }
      if (i >= s.size()) return false;
      char e = s[i++];
      switch (e) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t v;
          if (!hex4(v)) return false;
          if (v >= 0xD800 && v < 0xDC00) {
            if (i + 2 > s.size() || s[i] != '\\' || s[i + 1] != 'u') return false;
            i += 2;
            uint32_t lo;
            if (!hex4(lo) || lo < 0xDC00 || lo >= 0xE000) return false;
            v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
          } else if (v >= 0xDC00 && v < 0xE000) {
            return false;
          }
          put_utf8(o, v);
          break;
        }
        default: return false;
      }
    }
    return false;
  }
};
}  // namespace

void meta_set(MetaMap& m, const std::string& k, const std::string& v) {
  for (auto& kv : m)
    if (kv.first == k) { kv.second = v; return; }
  m.emplace_back(k, v);
}

template <class Map>
static bool parse_into(std::string_view s, Map& out, std::string& k, std::string& v) {
  out.clear();
  Parser p{s};
  p.ws();
  if (p.i >= s.size() || s[p.i] != '{') return false;
  ++p.i;
  p.ws();
  if (p.i < s.size() && s[p.i] == '}') {
    ++p.i;
    p.ws();
    return p.i == s.size();
  }
  while (true) {
    k.clear();
    v.clear();
    p.ws();
    if (!p.str(k)) { out.clear(); return false; }
    p.ws();
    if (p.i >= s.size() || s[p.i] != ':') { out.clear(); return false; }
    ++p.i;
    p.ws();
    if (!p.str(v)) { out.clear(); return false; }
    out.set(k, v);
    p.ws();
    if (p.i < s.size() && s[p.i] == ',') { ++p.i; continue; }
    if (p.i < s.size() && s[p.i] == '}') { ++p.i; break; }
    out.clear();
    return false;
  }
  p.ws();
  if (p.i != s.size()) { out.clear(); return false; }
  return true;
}

namespace {
struct MetaMapSink {
  MetaMap& m;
  void clear() { m.clear(); }
  void set(const std::string& k, const std::string& v) { meta_set(m, k, v); }
};
}  // namespace

bool parse_meta_json(std::string_view s, MetaMap& out) {
  MetaMapSink sink{out};
  std::string k, v;
  return parse_into(s, sink, k, v);
}

bool parse_meta_json(std::string_view s, FlatMeta& out) {
  thread_local std::string k, v;
  return parse_into(s, out, k, v);
}

void FlatMeta::set(std::string_view k, std::string_view v) {
  for (auto& x : e)
    if (key(x) == k) {
      x.vo = (uint32_t)arena.size();
      x.vl = (uint32_t)v.size();
      arena.append(v.data(), v.size());
      return;
    }
  E x;
  x.ko = (uint32_t)arena.size();
  x.kl = (uint32_t)k.size();
  arena.append(k.data(), k.size());
  x.vo = (uint32_t)arena.size();
  x.vl = (uint32_t)v.size();
  arena.append(v.data(), v.size());
  e.push_back(x);
}

void FlatMeta::append_json(std::string& out) const {
  out.push_back('{');
  for (size_t i = 0; i < e.size(); ++i) {
    if (i) out.push_back(',');
    json_escape_append(out, key(e[i]));
    out.push_back(':');
    json_escape_append(out, value(e[i]));
  }
  out.push_back('}');
}

std::string_view FlatMeta::get(std::string_view k) const {
  for (auto& x : e)
    if (key(x) == k) return value(x);
  return std::string_view();
}

bool FlatMeta::has(std::string_view k) const {
  for (auto& x : e)
    if (key(x) == k) return true;
  return false;
}

void serialize_meta_json(const MetaMap& m, std::string& out) {
  out.push_back('{');
  bool first = true;
  for (auto& kv : m) {
    if (!first) out.push_back(',');
    first = false;
    json_escape_append(out, kv.first);
    out.push_back(':');
    json_escape_append(out, kv.second);
  }
  out.push_back('}');
}

}  // namespace tb
