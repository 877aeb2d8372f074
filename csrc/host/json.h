// Minimal JSON for document metadata: an object of string -> string, matching
// serde_json::from_str::<HashMap<String, String>> (reference parquet_reader.rs:225) on input
// and serde_json::to_string(&HashMap<String,String>) (parquet_writer.rs:107) on output.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace tb {

using MetaMap = std::vector<std::pair<std::string, std::string>>;  // insertion-ordered

// Allocation-free (after warm-up) insertion-ordered string map for the per-document hot
// path: keys and values live in one arena; set() has HashMap insert semantics.
struct FlatMeta {
  struct E { uint32_t ko, kl, vo, vl; };
  std::string arena;
  std::vector<E> e;
  void clear() { arena.clear(); e.clear(); }
  bool empty() const { return e.empty(); }
  std::string_view key(const E& x) const { return std::string_view(arena.data() + x.ko, x.kl); }
  std::string_view value(const E& x) const { return std::string_view(arena.data() + x.vo, x.vl); }
  void set(std::string_view k, std::string_view v);
  bool has(std::string_view k) const;
  std::string_view get(std::string_view k) const;  // empty view when absent
  void append_json(std::string& out) const;
};

// Returns false (and leaves `out` empty) unless `s` is a JSON object whose values are strings.
bool parse_meta_json(std::string_view s, MetaMap& out);
bool parse_meta_json(std::string_view s, FlatMeta& out);

// True if any of the 8 bytes is < 0x20, '"' or '\\' (SWAR: "has a zero byte" tests).
inline bool json_word_needs_escape(uint64_t x) {
  constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull;
  const uint64_t lt20 = (x - 0x2020202020202020ull) & ~x & kHigh;
  const uint64_t q = x ^ 0x2222222222222222ull, bs = x ^ 0x5C5C5C5C5C5C5C5Cull;
  const uint64_t zq = (q - kOnes) & ~q & kHigh, zb = (bs - kOnes) & ~bs & kHigh;
  return (lt20 | zq | zb) != 0;
}

template <class Out>
inline void json_escape_append(Out& out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  size_t run = 0;  // start of the pending run of bytes that need no escaping
  size_t i = 0;
  const size_t n = s.size();
  while (i < n) {
    // skip clean 8-byte words in bulk (the common case: generated ASCII values)
    while (i + 8 <= n) {
      uint64_t w;
      std::memcpy(&w, s.data() + i, 8);
      if (json_word_needs_escape(w)) break;
      i += 8;
    }
    if (i >= n) break;
    const unsigned char c = (unsigned char)s[i];
    if (c >= 0x20 && c != '"' && c != '\\') { ++i; continue; }
    out.append(s.data() + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        out += "\\u00";
        out.push_back(hex[c >> 4]);
        out.push_back(hex[c & 15]);
    }
    ++i;
  }
  out.append(s.data() + run, n - run);
  out.push_back('"');
}

void serialize_meta_json(const MetaMap& m, std::string& out);

// Insert-or-overwrite with HashMap semantics (position of an existing key is kept).
void meta_set(MetaMap& m, const std::string& k, const std::string& v);

}  // namespace tb
