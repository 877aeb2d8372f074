// Unicode character database view: per-code-point properties for segmentation and the
// TextBlaster character predicates (reference src/utils/text.rs:28-57 PUNCTUATION,
// Rust char::is_whitespace / is_alphabetic / to_lowercase semantics).
//
// The tables are generated from ICU4C by tools/gen_unicode_tables.cpp. The host path reads
// the static arrays; the device path reads a copy uploaded to HBM (same layout).
#pragma once
#include "tb_common.h"

namespace tb {

enum : uint32_t {
  P_WB_MASK = 0x1F,
  P_SB_SHIFT = 5,
  P_SB_MASK = 0xF << 5,
  P_WS = 1u << 9,
  P_ALPHA = 1u << 10,
  P_PUNCT = 1u << 11,
  P_EXTPICT = 1u << 12,
  P_DIGIT = 1u << 13,
  P_DICT = 1u << 14,
  P_CASED = 1u << 15,
  P_CASE_IGN = 1u << 16,
  P_HAS_LOWER = 1u << 17,
  P_WORDCHAR = 1u << 18,
};

enum WB : int {
  WB_Other, WB_CR, WB_LF, WB_Newline, WB_Extend, WB_ZWJ, WB_RI, WB_Format, WB_Katakana,
  WB_Hebrew, WB_ALetter, WB_SQ, WB_DQ, WB_MidNumLet, WB_MidLetter, WB_MidNum, WB_Numeric,
  WB_ExtendNumLet, WB_WSegSpace
};
enum SB : int {
  SB_Other, SB_ATerm, SB_Close, SB_Format, SB_Lower, SB_Numeric, SB_OLetter, SB_Sep, SB_Sp,
  SB_STerm, SB_Upper, SB_CR, SB_LF, SB_Extend, SB_SContinue
};

struct UcdView {
  const uint16_t* props_s1;
  const uint32_t* props_s2;
  const uint16_t* lower_s1;
  const int32_t* lower_s2;

  TB_HD uint32_t props(uint32_t cp) const {
    if (cp > 0x10FFFF) cp = 0xFFFD;
    return props_s2[((uint32_t)props_s1[cp >> 7] << 7) | (cp & 127)];
  }
  // Simple (1:1) lowercase mapping; U+0130 additionally emits U+0307 (see lower_utf8).
  TB_HD uint32_t lower(uint32_t cp) const {
    if (cp < 128) return (cp - 'A' < 26u) ? cp + 32 : cp;  // ASCII: no table round trip
    if (cp > 0x10FFFF) return cp;
    return (uint32_t)((int32_t)cp + lower_s2[((uint32_t)lower_s1[cp >> 7] << 7) | (cp & 127)]);
  }
};

constexpr TB_HD int wb_of(uint32_t p) { return (int)(p & P_WB_MASK); }
TB_HD int sb_of(uint32_t p) { return (int)((p >> P_SB_SHIFT) & 0xF); }

// Decode one UTF-8 code point starting at s[i] (input is valid UTF-8: Arrow Utf8 guarantees it).
// Returns the code point and writes its byte length to *len.
TB_HD uint32_t utf8_decode(const uint8_t* s, uint32_t i, uint32_t n, int* len) {
  uint32_t c = s[i];
  if (c < 0x80) { *len = 1; return c; }
  if ((c >> 5) == 6 && i + 1 < n) { *len = 2; return ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); }
  if ((c >> 4) == 14 && i + 2 < n) {
    *len = 3;
    return ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
  }
  if (i + 3 < n) {
    *len = 4;
    return ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) |
           (s[i + 3] & 0x3F);
  }
  *len = 1;
  return 0xFFFD;
}

TB_HD bool utf8_is_lead(uint8_t b) { return (b & 0xC0) != 0x80; }

TB_HD int utf8_encode(uint32_t cp, uint8_t* out) {
  if (cp < 0x80) { out[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { out[0] = 0xC0 | (cp >> 6); out[1] = 0x80 | (cp & 0x3F); return 2; }
  if (cp < 0x10000) {
    out[0] = 0xE0 | (cp >> 12); out[1] = 0x80 | ((cp >> 6) & 0x3F); out[2] = 0x80 | (cp & 0x3F);
    return 3;
  }
  out[0] = 0xF0 | (cp >> 18); out[1] = 0x80 | ((cp >> 12) & 0x3F);
  out[2] = 0x80 | ((cp >> 6) & 0x3F); out[3] = 0x80 | (cp & 0x3F);
  return 4;
}

TB_HD int utf8_len(uint32_t cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

}  // namespace tb
