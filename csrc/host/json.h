// Minimal JSON for document metadata: an object of string -> string, matching
// serde_json::from_str::<HashMap<String, String>> (reference parquet_reader.rs:225) on input
// and serde_json::to_string(&HashMap<String,String>) (parquet_writer.rs:107) on output.
#pragma once
#include <cstdint>
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

void json_escape_append(std::string& out, std::string_view s);
void serialize_meta_json(const MetaMap& m, std::string& out);

// Insert-or-overwrite with HashMap semantics (position of an existing key is kept).
void meta_set(MetaMap& m, const std::string& k, const std::string& v);

}  // namespace tb
