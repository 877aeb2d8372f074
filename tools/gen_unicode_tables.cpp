// Generates csrc/common/ucd_tables.inc from ICU4C (the segmentation oracle on this box).
//
// Every per-code-point property the filters need is packed into one u32 ("props") looked up
// through a two-stage table (stage1[cp >> 7] -> block, stage2[block * 128 + (cp & 127)]).
// The same table is used by the host C++ path and copied to HBM for the HIP kernels, so the
// CPU and GPU paths classify characters identically.
//
// Build: g++ -O2 tools/gen_unicode_tables.cpp -licuuc -o /tmp/gen && /tmp/gen > csrc/common/ucd_tables.inc
#include <unicode/uchar.h>
#include <unicode/ustring.h>
#include <unicode/uscript.h>
#include <cstdio>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

// Must match csrc/common/ucd.h
enum {
  P_WB_SHIFT = 0,   // 5 bits
  P_SB_SHIFT = 5,   // 4 bits
  P_WS = 1u << 9,
  P_ALPHA = 1u << 10,
  P_PUNCT = 1u << 11,
  P_EXTPICT = 1u << 12,
  P_DIGIT = 1u << 13,
  P_DICT = 1u << 14,
  P_CASED = 1u << 15,
  P_CASE_IGN = 1u << 16,
  P_HAS_LOWER = 1u << 17,
  P_WORDCHAR = 1u << 18,  // regex \w (Unicode): Alphabetic | M | Nd | Pc | Join_Control
};

// Our compact WB enum (csrc/common/ucd.h)
enum WB { WB_Other, WB_CR, WB_LF, WB_Newline, WB_Extend, WB_ZWJ, WB_RI, WB_Format, WB_Katakana,
          WB_Hebrew, WB_ALetter, WB_SQ, WB_DQ, WB_MidNumLet, WB_MidLetter, WB_MidNum, WB_Numeric,
          WB_ExtendNumLet, WB_WSegSpace };
enum SB { SB_Other, SB_ATerm, SB_Close, SB_Format, SB_Lower, SB_Numeric, SB_OLetter, SB_Sep, SB_Sp,
          SB_STerm, SB_Upper, SB_CR, SB_LF, SB_Extend, SB_SContinue };

static int map_wb(int v) {
  switch (v) {
    case U_WB_CR: return WB_CR;
    case U_WB_LF: return WB_LF;
    case U_WB_NEWLINE: return WB_Newline;
    case U_WB_EXTEND: return WB_Extend;
    case U_WB_ZWJ: return WB_ZWJ;
    case U_WB_REGIONAL_INDICATOR: return WB_RI;
    case U_WB_FORMAT: return WB_Format;
    case U_WB_KATAKANA: return WB_Katakana;
    case U_WB_HEBREW_LETTER: return WB_Hebrew;
    case U_WB_ALETTER: return WB_ALetter;
    case U_WB_SINGLE_QUOTE: return WB_SQ;
    case U_WB_DOUBLE_QUOTE: return WB_DQ;
    case U_WB_MIDNUMLET: return WB_MidNumLet;
    case U_WB_MIDLETTER: return WB_MidLetter;
    case U_WB_MIDNUM: return WB_MidNum;
    case U_WB_NUMERIC: return WB_Numeric;
    case U_WB_EXTENDNUMLET: return WB_ExtendNumLet;
    case U_WB_WSEGSPACE: return WB_WSegSpace;
    default: return WB_Other;
  }
}
static int map_sb(int v) {
  switch (v) {
    case U_SB_ATERM: return SB_ATerm;
    case U_SB_CLOSE: return SB_Close;
    case U_SB_FORMAT: return SB_Format;
    case U_SB_LOWER: return SB_Lower;
    case U_SB_NUMERIC: return SB_Numeric;
    case U_SB_OLETTER: return SB_OLetter;
    case U_SB_SEP: return SB_Sep;
    case U_SB_SP: return SB_Sp;
    case U_SB_STERM: return SB_STerm;
    case U_SB_UPPER: return SB_Upper;
    case U_SB_CR: return SB_CR;
    case U_SB_LF: return SB_LF;
    case U_SB_EXTEND: return SB_Extend;
    case U_SB_SCONTINUE: return SB_SContinue;
    default: return SB_Other;
  }
}

// TextBlaster's PUNCTUATION set: a literal list plus four C0/C1 control ranges
// (reference src/utils/text.rs:28-57). TAB (9) and LF (10) are NOT members.
static const char* kPunctLit =
    "!/\xE2\x80\x94\xE2\x80\x9D:\xEF\xBC\x85\xEF\xBC\x91\xE3\x80\x88&(\xE3\x80\x81\xE2\x94\x81\\"
    "\xE3\x80\x90#%\xE3\x80\x8C\xE3\x80\x8D\xEF\xBC\x8C\xE3\x80\x91\xEF\xBC\x9B+^]~\xE2\x80\x9C"
    "\xE3\x80\x8A\xE2\x80\x9E';\xE2\x80\x99{|\xE2\x88\xB6\xC2\xB4[=-`*\xEF\xBC\x8E\xEF\xBC\x88"
    "\xE2\x80\x93\xEF\xBC\x9F\xEF\xBC\x81\xEF\xBC\x9A$\xEF\xBD\x9E\xC2\xAB\xE3\x80\x89,><"
    "\xE3\x80\x8B)?\xEF\xBC\x89\xE3\x80\x82\xE2\x80\xA6@_.\"}\xE2\x96\xBA\xC2\xBB";

static std::vector<uint32_t> decode_utf8(const char* s) {
  std::vector<uint32_t> out;
  const unsigned char* p = (const unsigned char*)s;
  while (*p) {
    uint32_t c = *p;
    int n = 0;
    if (c < 0x80) n = 0;
    else if ((c >> 5) == 6) { c &= 0x1F; n = 1; }
    else if ((c >> 4) == 14) { c &= 0x0F; n = 2; }
    else { c &= 0x07; n = 3; }
    ++p;
    for (int i = 0; i < n; ++i) c = (c << 6) | (*p++ & 0x3F);
    out.push_back(c);
  }
  return out;
}

int main() {
  const uint32_t N = 0x110000;
  std::vector<uint8_t> punct(N, 0);
  for (uint32_t c : decode_utf8(kPunctLit)) punct[c] = 1;
  for (uint32_t c = 0; c < 9; ++c) punct[c] = 1;
  for (uint32_t c = 11; c < 13; ++c) punct[c] = 1;
  for (uint32_t c = 13; c < 32; ++c) punct[c] = 1;
  for (uint32_t c = 127; c < 160; ++c) punct[c] = 1;

  std::vector<uint32_t> props(N);
  std::vector<int32_t> lower(N);
  std::vector<int32_t> fold(N);  // simple case folding (u_foldCase, default): C4 bad-words matching
  for (uint32_t c = 0; c < N; ++c) {
    fold[c] = (int32_t)u_foldCase((UChar32)c, U_FOLD_CASE_DEFAULT) - (int32_t)c;
    uint32_t p = 0;
    p |= (uint32_t)map_wb(u_getIntPropertyValue(c, UCHAR_WORD_BREAK)) << P_WB_SHIFT;
    p |= (uint32_t)map_sb(u_getIntPropertyValue(c, UCHAR_SENTENCE_BREAK)) << P_SB_SHIFT;
    if (u_hasBinaryProperty(c, UCHAR_WHITE_SPACE)) p |= P_WS;
    if (u_hasBinaryProperty(c, UCHAR_ALPHABETIC)) p |= P_ALPHA;
    if (punct[c]) p |= P_PUNCT;
    if (u_hasBinaryProperty(c, UCHAR_EXTENDED_PICTOGRAPHIC)) p |= P_EXTPICT;
    if (u_charType(c) == U_DECIMAL_DIGIT_NUMBER) p |= P_DIGIT;
    UErrorCode ec = U_ZERO_ERROR;
    int sc = uscript_getScript(c, &ec);
    int lb = u_getIntPropertyValue(c, UCHAR_LINE_BREAK);
    if (lb == U_LB_COMPLEX_CONTEXT || sc == USCRIPT_HAN || sc == USCRIPT_HIRAGANA ||
        sc == USCRIPT_KATAKANA || sc == USCRIPT_THAI || sc == USCRIPT_LAO ||
        sc == USCRIPT_KHMER || sc == USCRIPT_MYANMAR)
      p |= P_DICT;
    if (u_hasBinaryProperty(c, UCHAR_CASED)) p |= P_CASED;
    if (u_hasBinaryProperty(c, UCHAR_CASE_IGNORABLE)) p |= P_CASE_IGN;
    int8_t gc = u_charType(c);
    if (u_hasBinaryProperty(c, UCHAR_ALPHABETIC) || gc == U_NON_SPACING_MARK ||
        gc == U_ENCLOSING_MARK || gc == U_COMBINING_SPACING_MARK || gc == U_DECIMAL_DIGIT_NUMBER ||
        gc == U_CONNECTOR_PUNCTUATION || u_hasBinaryProperty(c, UCHAR_JOIN_CONTROL))
      p |= P_WORDCHAR;
    // Full lowercase of a single code point (Rust char::to_lowercase is the full mapping;
    // only U+0130 expands, handled explicitly in ucd.h).
    int32_t lc = u_tolower(c);
    if (c == 0x130) lc = 0x69;
    if ((uint32_t)lc != c) p |= P_HAS_LOWER;
    lower[c] = lc - (int32_t)c;
    props[c] = p;
  }

  const int BS = 128;
  auto emit_two_stage = [&](const char* name, const std::vector<uint32_t>& vals, const char* ty) {
    std::map<std::vector<uint32_t>, int> blocks;
    std::vector<std::vector<uint32_t>> order;
    std::vector<int> stage1;
    for (uint32_t b = 0; b < N / BS; ++b) {
      std::vector<uint32_t> blk(vals.begin() + b * BS, vals.begin() + (b + 1) * BS);
      auto it = blocks.find(blk);
      int id;
      if (it == blocks.end()) { id = (int)order.size(); blocks[blk] = id; order.push_back(blk); }
      else id = it->second;
      stage1.push_back(id);
    }
    printf("static const uint16_t %s_STAGE1[%zu] = {", name, stage1.size());
    for (size_t i = 0; i < stage1.size(); ++i) printf("%s%d", i == 0 ? "\n" : ((i % 32) ? "," : ",\n"), stage1[i]);
    printf("};\n");
    printf("#define %s_NBLOCKS %zu\n", name, order.size());
    printf("static const %s %s_STAGE2[%zu] = {", ty, name, order.size() * BS);
    size_t k = 0;
    for (auto& blk : order)
      for (uint32_t v : blk) { printf("%s%d", k == 0 ? "\n" : ((k % 16) ? "," : ",\n"), (int32_t)v); ++k; }
    printf("};\n");
  };
  printf("// GENERATED by tools/gen_unicode_tables.cpp from ICU4C %s (Unicode %s). Do not edit.\n",
         U_ICU_VERSION, U_UNICODE_VERSION);
  printf("#pragma once\n#include <cstdint>\n");
  printf("#define TB_UCD_BLOCK_SHIFT 7\n");
  emit_two_stage("TB_UCD_PROPS", props, "uint32_t");
  std::vector<uint32_t> lv(lower.begin(), lower.end());
  emit_two_stage("TB_UCD_LOWER", lv, "int32_t");
  std::vector<uint32_t> fv(fold.begin(), fold.end());
  emit_two_stage("TB_UCD_FOLD", fv, "int32_t");
  return 0;
}
