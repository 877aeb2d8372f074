// Minimal JSON for document metadata: an object of string -> string, matching
// serde_json::from_str::<HashMap<String, String>> (reference parquet_reader.rs:225) on input
// and serde_json::to_string(&HashMap<String,String>) (parquet_writer.rs:107) on output.
#pragma once
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace tb {

using MetaMap = std::vector<std::pair<std::string, std::string>>;  // insertion-ordered

// Returns false (and leaves `out` empty) unless `s` is a JSON object whose values are strings.
bool parse_meta_json(std::string_view s, MetaMap& out);

void json_escape_append(std::string& out, std::string_view s);
void serialize_meta_json(const MetaMap& m, std::string& out);

// Insert-or-overwrite with HashMap semantics (position of an existing key is kept).
void meta_set(MetaMap& m, const std::string& k, const std::string& v);

}  // namespace tb
