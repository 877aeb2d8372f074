// Formatting helpers that reproduce Rust's std::fmt output for the values that appear in
// reason strings and metadata (reference: format!("{:.2}"), format!("{:.4}"), f64::to_string).
#pragma once
#include <charconv>
#include <cmath>
#include <cstdio>
#include <string>

namespace tb {

// format!("{:.N}", x): exact decimal expansion, round-half-to-even (glibc printf is exact).
inline std::string fmt_fixed(double x, int prec) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%.*f", prec, x);
  return buf;
}

// f64 Display (`{}` / to_string): shortest digits that round-trip, never exponent notation.
inline std::string fmt_f64(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
  if (x == 0) return std::signbit(x) ? "-0" : "0";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  bool neg = s[0] == '-';
  if (neg) s.erase(0, 1);
  size_t epos = s.find('e');
  int exp10 = std::stoi(s.substr(epos + 1));
  std::string mant = s.substr(0, epos);
  std::string digits;
  for (char c : mant) if (c != '.') digits.push_back(c);
  // value = 0.d1d2d3... * 10^(exp10+1)
  int point = exp10 + 1;  // position of decimal point relative to digits start
  std::string out;
  if (point <= 0) {
    out = "0." + std::string(-point, '0') + digits;
  } else if ((size_t)point >= digits.size()) {
    out = digits + std::string(point - digits.size(), '0');
  } else {
    out = digits.substr(0, point) + "." + digits.substr(point);
  }
  return neg ? "-" + out : out;
}

// {:?} of a String: quotes + Rust escape_debug (enough for ISO codes and "; " separators).
inline std::string fmt_debug_str(const std::string& s) {
  std::string out = "\"";
  for (char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default: out.push_back(c);
    }
  }
  out += "\"";
  return out;
}

}  // namespace tb
