#pragma once
#include <string>
#include <string_view>

namespace tb {
// Decodes HTML character references in `s` into `out`. Returns false (out untouched) when `s`
// contains no '&' so callers can keep the original buffer.
bool html_decode(std::string_view s, std::string& out);
}  // namespace tb
