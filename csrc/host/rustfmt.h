// Formatting helpers that reproduce Rust's std::fmt output for the values that appear in
// reason strings and metadata (reference: format!("{:.2}"), format!("{:.4}"), f64::to_string).
//
// The append_* forms write into a caller-owned buffer without allocating (output assembly
// formats ~10^6 values per second per thread); the fmt_* forms wrap them.
#pragma once
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace tb {

// Growable byte buffer for hot formatting loops: appends check capacity with one compare and
// never zero-fill (std::string::append costs a call and bookkeeping per piece).
struct CharBuf {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  CharBuf() = default;
  CharBuf(const CharBuf&) = delete;
  CharBuf& operator=(const CharBuf&) = delete;
  ~CharBuf() { std::free(p); }
  void grow(size_t need) {
    size_t c = cap ? cap * 2 : 256;
    while (c < need) c *= 2;
    p = (char*)std::realloc(p, c);
    cap = c;
  }
  void reserve(size_t k) { if (n + k > cap) grow(n + k); }
  void append(const char* s, size_t k) {
    reserve(k);
    std::memcpy(p + n, s, k);
    n += k;
  }
  void append(size_t k, char c) {
    reserve(k);
    std::memset(p + n, c, k);
    n += k;
  }
  void push_back(char c) {
    if (n == cap) grow(n + 1);
    p[n++] = c;
  }
  CharBuf& operator+=(const char* s) { append(s, std::strlen(s)); return *this; }
  void clear() { n = 0; }
  size_t size() const { return n; }
  void resize(size_t k) { n = k; }  // shrink only
  const char* data() const { return p; }
  std::string_view view() const { return std::string_view(p, n); }
};

template <class Out>
inline void append_u64(Out& out, uint64_t v) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, (size_t)(r.ptr - buf));
}

template <class Out>
inline void append_i64(Out& out, int64_t v) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, (size_t)(r.ptr - buf));
}

// format!("{:.N}", x) for N <= 4: the exact binary value rounded half-to-even to N decimals
// (what Rust and glibc printf do). Finite |x| < 10^14 takes an integer path: x = m * 2^e, the
// scaled value m * 10^N * 2^e is split into quotient and remainder in 128-bit arithmetic, so the
// rounding decision is exact. Anything else goes through printf, which is exact too.
template <class Out>
inline void append_fixed(Out& out, double x, int prec) {
  static const uint64_t kPow10[5] = {1, 10, 100, 1000, 10000};
  if (prec < 0 || prec > 4 || !std::isfinite(x) || std::fabs(x) >= 1e14) {
    char buf[512];
    const int n = snprintf(buf, sizeof(buf), "%.*f", prec, x);
    out.append(buf, (size_t)n);
    return;
  }
  const bool neg = std::signbit(x);
  int e2;
  const double fr = std::frexp(std::fabs(x), &e2);          // |x| = fr * 2^e2, fr in [0.5, 1)
  const uint64_t m = (uint64_t)std::ldexp(fr, 53);          // exact 53-bit mantissa
  const int sh = 53 - e2;                                   // |x| = m * 2^-sh
  const unsigned __int128 scaled = (unsigned __int128)m * kPow10[prec];
  unsigned __int128 q;
  if (x == 0.0) {
    q = 0;
  } else if (sh <= 0) {
    q = scaled << (-sh);
  } else if (sh >= 120) {
    q = 0;  // |x| * 10^prec < 2^-50: rounds to zero
  } else {
    q = scaled >> sh;
    const unsigned __int128 rem = scaled - (q << sh);
    const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
    if (rem > half || (rem == half && (q & 1))) ++q;
  }
  const uint64_t qi = (uint64_t)q;
  const uint64_t ip = qi / kPow10[prec], fp = qi % kPow10[prec];
  if (neg) out.push_back('-');
  append_u64(out, ip);
  if (prec > 0) {
    char fb[8];
    for (int k = prec - 1, v = (int)fp; k >= 0; --k, v /= 10) fb[k] = (char)('0' + v % 10);
    out.push_back('.');
    out.append(fb, (size_t)prec);
  }
}

inline std::string fmt_fixed(double x, int prec) {
  std::string s;
  append_fixed(s, x, prec);
  return s;
}

// f64 Display (`{}` / to_string): shortest digits that round-trip, never exponent notation.
template <class Out>
inline void append_f64(Out& out, double x) {
  if (std::isnan(x)) { out += "NaN"; return; }
  if (std::isinf(x)) { out += x > 0 ? "inf" : "-inf"; return; }
  if (x == 0) { out += std::signbit(x) ? "-0" : "0"; return; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  const char* p = buf;
  const char* end = r.ptr;
  if (*p == '-') { out.push_back('-'); ++p; }
  const char* epos = (const char*)std::memchr(p, 'e', (size_t)(end - p));
  int exp10 = 0;
  std::from_chars(epos[1] == '+' ? epos + 2 : epos + 1, end, exp10);
  char digits[32];
  int nd = 0;
  for (const char* q = p; q < epos; ++q) if (*q != '.') digits[nd++] = *q;
  // value = 0.d1d2d3... * 10^(exp10+1)
  const int point = exp10 + 1;
  if (point <= 0) {
    out += "0.";
    out.append((size_t)(-point), '0');
    out.append(digits, (size_t)nd);
  } else if (point >= nd) {
    out.append(digits, (size_t)nd);
    out.append((size_t)(point - nd), '0');
  } else {
    out.append(digits, (size_t)point);
    out.push_back('.');
    out.append(digits + point, (size_t)(nd - point));
  }
}

inline std::string fmt_f64(double x) {
  std::string s;
  append_f64(s, x);
  return s;
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
