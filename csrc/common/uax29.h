// UAX #29 word and sentence boundary rules (Unicode 14, as tailored by ICU's default rules for
// scripts that do not need a dictionary), written once for the host and the device.
//
// The reference segments with ICU4X (`WordSegmenter::new_auto`, `SentenceSegmenter::new`,
// reference src/utils/text.rs:59-181). Documents that contain dictionary/LSTM scripts (Han,
// Hiragana, Katakana, Thai, Lao, Khmer, Myanmar: P_DICT) are routed to the ICU4C path instead.
//
// The rule functions take an accessor `A` exposing `uint32_t p(int i)`: the packed property word of
// code point i of the text being segmented, with 0 <= i < n. `wb_break(a, n, i)` answers "is there a
// word boundary between code point i-1 and code point i" for 0 < i < n (sot/eot are boundaries).
#pragma once
#include "ucd.h"

namespace tb {

constexpr TB_HD bool wb_ign(int c) { return c == WB_Extend || c == WB_Format || c == WB_ZWJ; }
constexpr TB_HD bool wb_nl(int c) { return c == WB_CR || c == WB_LF || c == WB_Newline; }
constexpr TB_HD bool wb_ah(int c) { return c == WB_ALetter || c == WB_Hebrew; }
constexpr TB_HD bool wb_midletq(int c) { return c == WB_MidLetter || c == WB_MidNumLet || c == WB_SQ; }
constexpr TB_HD bool wb_midnumq(int c) { return c == WB_MidNum || c == WB_MidNumLet || c == WB_SQ; }

// Effective previous code point index for WB4: the nearest index < i that is not
// Extend/Format/ZWJ. Returns -1 if the run of ignorables reaches sot.
template <class A>
TB_HD int wb_prev_eff(const A& a, int i) {
  int k = i - 1;
  while (k >= 0 && wb_ign(wb_of(a.p(k)))) --k;
  return k;
}
template <class A>
TB_HD int wb_next_eff(const A& a, int n, int i) {
  int k = i + 1;
  while (k < n && wb_ign(wb_of(a.p(k)))) ++k;
  return k;
}

template <class A>
TB_HD bool wb_break(const A& a, int n, int i) {
  const uint32_t pp = a.p(i - 1), pc = a.p(i);
  const int cp = wb_of(pp), cc = wb_of(pc);
  // The common pairs of running text, decided without look-around: neither side is a newline,
  // ZWJ or ignorable, so the effective left context is cp itself; ALetter x ALetter is WB5,
  // ALetter / WSegSpace in either order matches no rule before WB999 (break).
  if (cp == WB_ALetter) {
    if (cc == WB_ALetter) return false;
    if (cc == WB_WSegSpace) return true;
  } else if (cp == WB_WSegSpace && cc == WB_ALetter) {
    return true;
  }
  if (cp == WB_CR && cc == WB_LF) return false;            // WB3
  if (wb_nl(cp)) return true;                              // WB3a
  if (wb_nl(cc)) return true;                              // WB3b
  if (cp == WB_ZWJ && (pc & P_EXTPICT)) return false;      // WB3c
  if (cp == WB_WSegSpace && cc == WB_WSegSpace) return false;  // WB3d
  if (wb_ign(cc)) return false;                            // WB4
  // Effective left context (ignorables attach to the preceding non-ignorable, unless the run
  // started at sot or right after a newline, in which case it stands alone as "Other").
  int k = wb_prev_eff(a, i);
  int L = WB_Other;
  if (k >= 0) {
    const int ck = wb_of(a.p(k));
    if (!wb_nl(ck)) L = ck;
  }
  const int R = cc;
  int LL = -1;
  auto left2 = [&]() -> int {
    if (k < 0 || L == WB_Other) return (int)WB_Other;
    int k2 = wb_prev_eff(a, k);
    return k2 >= 0 ? wb_of(a.p(k2)) : (int)WB_Other;
  };
  auto right2 = [&]() -> int {
    int m = wb_next_eff(a, n, i);
    return m < n ? wb_of(a.p(m)) : -1;
  };
  if (wb_ah(L) && wb_ah(R)) return false;                                   // WB5
  if (wb_ah(L) && wb_midletq(R) && wb_ah(right2())) return false;           // WB6
  if (wb_midletq(L) && wb_ah(R)) { LL = left2(); if (wb_ah(LL)) return false; }  // WB7
  if (L == WB_Hebrew && R == WB_SQ) return false;                          // WB7a
  if (L == WB_Hebrew && R == WB_DQ && right2() == WB_Hebrew) return false;  // WB7b
  if (L == WB_DQ && R == WB_Hebrew) { if (LL < 0) LL = left2(); if (LL == WB_Hebrew) return false; }  // WB7c
  if (L == WB_Numeric && R == WB_Numeric) return false;                    // WB8
  if (wb_ah(L) && R == WB_Numeric) return false;                           // WB9
  if (L == WB_Numeric && wb_ah(R)) return false;                           // WB10
  if (wb_midnumq(L) && R == WB_Numeric) { if (LL < 0) LL = left2(); if (LL == WB_Numeric) return false; }  // WB11
  if (L == WB_Numeric && wb_midnumq(R) && right2() == WB_Numeric) return false;  // WB12
  if (L == WB_Katakana && R == WB_Katakana) return false;                  // WB13
  if ((wb_ah(L) || L == WB_Numeric || L == WB_Katakana || L == WB_ExtendNumLet) &&
      R == WB_ExtendNumLet)
    return false;                                                          // WB13a
  if (L == WB_ExtendNumLet && (wb_ah(R) || R == WB_Numeric || R == WB_Katakana)) return false;  // WB13b
  if (L == WB_RI && R == WB_RI) {                                          // WB15/16
    int cnt = 0;
    int j = k;
    while (j >= 0 && wb_of(a.p(j)) == WB_RI) { ++cnt; j = wb_prev_eff(a, j); }
    return (cnt & 1) == 0;
  }
  return true;                                                             // WB999
}

// wb_break from the properties of code points i-2, i-1, i, i+1 alone (pm2 / pp1 = 0xFFFFFFFF when
// out of range), for positions whose window holds no Extend/Format/ZWJ/RI: then the effective
// left contexts are i-1 and i-2 and the effective right context is i+1, so every rule is decided
// from registers. Returns 0 / 1, or 2 when the window needs the general look-around.
constexpr TB_HD int wb_break_ctx(uint32_t pm2, uint32_t pm1, uint32_t p0, uint32_t pp1) {
  const int L0 = wb_of(pm1), R = wb_of(p0);
  if (L0 == WB_ALetter) {  // the common pairs first (as wb_break)
    if (R == WB_ALetter) return 0;
    if (R == WB_WSegSpace) return 1;
  } else if (L0 == WB_WSegSpace && R == WB_ALetter) {
    return 1;
  }
  const int LL0 = pm2 == 0xFFFFFFFFu ? -1 : wb_of(pm2);
  const int RR = pp1 == 0xFFFFFFFFu ? -1 : wb_of(pp1);
  auto special = [](int c) { return c == WB_Extend || c == WB_Format || c == WB_ZWJ || c == WB_RI; };
  if (special(L0) || special(R) || (LL0 >= 0 && special(LL0)) || (RR >= 0 && special(RR))) return 2;
  if (L0 == WB_CR && R == WB_LF) return 0;      // WB3
  if (wb_nl(L0)) return 1;                      // WB3a
  if (wb_nl(R)) return 1;                       // WB3b
  if (L0 == WB_WSegSpace && R == WB_WSegSpace) return 0;  // WB3d
  const int L = L0;                             // not a newline here
  // left2(): Other when there is no i-2 or L is Other (wb_break's definition)
  const int LL = (LL0 < 0 || L == WB_Other) ? (int)WB_Other : LL0;
  if (wb_ah(L) && wb_ah(R)) return 0;                                   // WB5
  if (wb_ah(L) && wb_midletq(R) && wb_ah(RR)) return 0;                 // WB6
  if (wb_midletq(L) && wb_ah(R) && wb_ah(LL)) return 0;                 // WB7
  if (L == WB_Hebrew && R == WB_SQ) return 0;                           // WB7a
  if (L == WB_Hebrew && R == WB_DQ && RR == WB_Hebrew) return 0;        // WB7b
  if (L == WB_DQ && R == WB_Hebrew && LL == WB_Hebrew) return 0;        // WB7c
  if (L == WB_Numeric && R == WB_Numeric) return 0;                     // WB8
  if (wb_ah(L) && R == WB_Numeric) return 0;                            // WB9
  if (L == WB_Numeric && wb_ah(R)) return 0;                            // WB10
  if (wb_midnumq(L) && R == WB_Numeric && LL == WB_Numeric) return 0;   // WB11
  if (L == WB_Numeric && wb_midnumq(R) && RR == WB_Numeric) return 0;   // WB12
  if (L == WB_Katakana && R == WB_Katakana) return 0;                   // WB13
  if ((wb_ah(L) || L == WB_Numeric || L == WB_Katakana || L == WB_ExtendNumLet) && R == WB_ExtendNumLet)
    return 0;                                                           // WB13a
  if (L == WB_ExtendNumLet && (wb_ah(R) || R == WB_Numeric || R == WB_Katakana)) return 0;  // WB13b
  return 1;                                                             // WB999
}

// The same decision from a table of the class pairs (L, R) = (i-1, i): once no Extend / Format /
// ZWJ / RI is in the window, every rule of wb_break_ctx either decides a pair outright or asks
// whether one context class (RR = i+1 for WB6 / 7b / 12, LL = i-2 for WB7 / 7c / 11) lies in a
// set (AHLetter, Hebrew or Numeric). The table holds that per pair as a 4-bit code, 8 pairs per
// dword; it is generated at compile time from wb_break_ctx itself (wb_pair_code), so the two agree
// by construction, and tools/host_selftest.cpp checks them against each other on every window.
// On the device one wave keeps the 46 table dwords in one register (lane k: dword k) and looks a
// pair up with one lane read (ds_bpermute): a handful of VALU instructions instead of the rule
// chain, which every lane of a wave runs through when its lanes hold different classes.
enum : uint32_t {
  WBC_NB = 0, WBC_BR = 1, WBC_RR_AH = 2, WBC_RR_HEB = 3, WBC_RR_NUM = 4, WBC_LL_AH = 5, WBC_LL_HEB = 6,
  WBC_LL_NUM = 7, WBC_BAD = 15
};
constexpr int kWbClasses = 19;
constexpr int kWbTabWords = (kWbClasses * kWbClasses + 7) / 8;  // 46
constexpr uint32_t kWbSpecial = (1u << WB_Extend) | (1u << WB_Format) | (1u << WB_ZWJ) | (1u << WB_RI);
constexpr uint32_t kWbSetAH = (1u << WB_ALetter) | (1u << WB_Hebrew);
constexpr uint32_t kWbSetHeb = 1u << WB_Hebrew;
constexpr uint32_t kWbSetNum = 1u << WB_Numeric;

// (the decision of every window against the rule chain and the general walk is checked by
// tools/host_selftest.cpp; here only which side, if any, a pair depends on)
constexpr uint32_t wb_pair_code(int L, int R) {
  if ((kWbSpecial >> L) & 1u || (kWbSpecial >> R) & 1u) return WBC_BR;  // (never looked up)
  auto r = [&](int ll, int rr) {
    return wb_break_ctx(ll < 0 ? 0xFFFFFFFFu : (uint32_t)ll, (uint32_t)L, (uint32_t)R, rr < 0 ? 0xFFFFFFFFu : (uint32_t)rr);
  };
  const int r0 = r(-1, -1);
  uint32_t set_ll = 0, set_rr = 0;  // context classes that change the decision
  for (int c = 0; c < kWbClasses; ++c) {
    if ((kWbSpecial >> c) & 1u) continue;
    if (r(c, -1) != r0) set_ll |= 1u << c;
    if (r(-1, c) != r0) set_rr |= 1u << c;
  }
  if (!set_ll && !set_rr) return r0 == 0 ? WBC_NB : (r0 == 1 ? WBC_BR : WBC_BAD);
  if ((set_ll && set_rr) || r0 != 1) return WBC_BAD;
  const uint32_t set = set_ll | set_rr;
  const uint32_t base = set_rr ? WBC_RR_AH : WBC_LL_AH;
  if (set == kWbSetAH) return base;
  if (set == kWbSetHeb) return base + 1;
  if (set == kWbSetNum) return base + 2;
  return WBC_BAD;
}
struct WbPairTab {
  uint32_t w[kWbTabWords];
};
constexpr WbPairTab make_wb_pair_tab() {
  WbPairTab t{};
  for (int L = 0; L < kWbClasses; ++L)
    for (int R = 0; R < kWbClasses; ++R) {
      const int i = L * kWbClasses + R;
      t.w[i >> 3] |= wb_pair_code(L, R) << ((i & 7) * 4);
    }
  return t;
}
constexpr bool wb_pair_tab_ok(const WbPairTab& t) {
  for (int i = 0; i < kWbClasses * kWbClasses; ++i)
    if (((t.w[i >> 3] >> ((i & 7) * 4)) & 0xFu) == WBC_BAD) return false;
  return true;
}
inline constexpr WbPairTab kWbPairTab = make_wb_pair_tab();
static_assert(wb_pair_tab_ok(kWbPairTab), "a word-break pair needs a context the table cannot encode");

// wb_break_ctx by the pair table; lookup(i) returns dword i >> 3 of kWbPairTab (any source).
template <class Lookup>
TB_HD int wb_break_ctx_tab(uint32_t pm2, uint32_t pm1, uint32_t p0, uint32_t pp1, Lookup&& lookup) {
  const uint32_t L = pm1 & P_WB_MASK, R = p0 & P_WB_MASK;
  if (((1u << L) | (1u << R)) & kWbSpecial) return 2;
  const uint32_t i = L * kWbClasses + R;
  const uint32_t code = (lookup(i >> 3) >> ((i & 7u) * 4u)) & 0xFu;
  // a pair decided outright does not look past i-1 and i (an ignorable at i-2 or i+1 only changes
  // the effective contexts further out); a context rule reads the effective i-2 / i+1, which the
  // window holds unless it is ignorable or RI (then the general walk)
  if (code <= WBC_BR) return (int)code;
  const uint32_t bLL = pm2 == 0xFFFFFFFFu ? 0u : 1u << (pm2 & P_WB_MASK);
  const uint32_t bRR = pp1 == 0xFFFFFFFFu ? 0u : 1u << (pp1 & P_WB_MASK);
  const uint32_t ctx = code <= WBC_RR_NUM ? bRR : bLL;
  if (ctx & kWbSpecial) return 2;
  const uint32_t set = (code == WBC_RR_AH || code == WBC_LL_AH) ? kWbSetAH
                       : (code == WBC_RR_HEB || code == WBC_LL_HEB) ? kWbSetHeb : kWbSetNum;
  return (ctx & set) ? 0 : 1;
}
TB_HD int wb_break_ctx_tab(uint32_t pm2, uint32_t pm1, uint32_t p0, uint32_t pp1) {
  return wb_break_ctx_tab(pm2, pm1, p0, pp1, [](uint32_t k) { return kWbPairTab.w[k]; });
}

// ---------------------------------------------------------------------------------------------
// Sentence boundaries.
TB_HD bool sb_ign(int c) { return c == SB_Extend || c == SB_Format; }
TB_HD bool sb_para(int c) { return c == SB_Sep || c == SB_CR || c == SB_LF; }
TB_HD bool sb_sterm_or_aterm(int c) { return c == SB_ATerm || c == SB_STerm; }

template <class A>
TB_HD int sb_prev_eff(const A& a, int i) {
  int k = i - 1;
  while (k >= 0 && sb_ign(sb_of(a.p(k)))) --k;
  return k;
}

template <class A>
TB_HD bool sb_break(const A& a, int n, int i) {
  const int cp = sb_of(a.p(i - 1)), cc = sb_of(a.p(i));
  if (cp == SB_CR && cc == SB_LF) return false;   // SB3
  if (sb_para(cp)) return true;                   // SB4
  if (sb_ign(cc)) return false;                   // SB5
  int k = sb_prev_eff(a, i);
  int L = SB_Other;
  if (k >= 0) {
    const int ck = sb_of(a.p(k));
    if (!sb_para(ck)) L = ck;
  }
  const int R = cc;
  if (L == SB_ATerm && R == SB_Numeric) return false;  // SB6
  if (L == SB_ATerm && R == SB_Upper) {               // SB7
    int k2 = sb_prev_eff(a, k);
    if (k2 >= 0) {
      int c2 = sb_of(a.p(k2));
      if (c2 == SB_Upper || c2 == SB_Lower) return false;
    }
  }
  // Match  SATerm Close* Sp*  ending at the effective left context.
  if (k < 0 || L == SB_Other) return false;  // SB998 (no terminator to the left)
  int j = k;
  bool saw_sp = false;
  while (j >= 0 && sb_of(a.p(j)) == SB_Sp) { saw_sp = true; j = sb_prev_eff(a, j); }
  while (j >= 0 && sb_of(a.p(j)) == SB_Close) { j = sb_prev_eff(a, j); }
  if (j < 0) return false;
  const int term = sb_of(a.p(j));
  if (!sb_sterm_or_aterm(term)) return false;  // SB998
  if (term == SB_ATerm) {                      // SB8
    int m = i;
    while (m < n) {
      int c = sb_of(a.p(m));
      if (c == SB_OLetter || c == SB_Upper || c == SB_Lower || sb_para(c) || sb_sterm_or_aterm(c)) break;
      ++m;
    }
    if (m < n && sb_of(a.p(m)) == SB_Lower) return false;
  }
  if (R == SB_SContinue || sb_sterm_or_aterm(R)) return false;              // SB8a
  if (!saw_sp && (R == SB_Close || R == SB_Sp || sb_para(R))) return false;  // SB9
  if (R == SB_Sp || sb_para(R)) return false;                                // SB10
  return true;                                                               // SB11
}

}  // namespace tb
