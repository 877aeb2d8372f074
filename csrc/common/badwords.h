// C4 bad-words matching over the flattened word-list tries (reference c4_filters.rs:431-441,516:
// `(?i)(?:\W|^)(w1|w2|...)(?:\W|$)`, no boundary requirement for the CJK lists). Shared by the
// device kernel (k_badwords_match: one wave per document, four start positions per lane) and the
// host emulation (bw_match_doc), so the CPU tests pin the exact walk the GPU runs.
//
// Transitions are one open-addressing hash table over (node, folded code point) instead of a
// per-node sorted edge list: a step is one 16-byte load (two when the probe collides) rather than
// a dependent binary search of ~log2(fan-out) loads; the root alone has ~30-60 edges per list.
// Entry = {node + 1 (0: empty), code point, child, child is terminal}.
#pragma once
#include "tb_common.h"
#include "ucd.h"

#if !defined(__HIP_DEVICE_COMPILE__)
#include <stdexcept>
#include <vector>
#endif

namespace tb {

struct BwTable {
  const uint32_t* e;  // 4 words per slot
  uint32_t mask;      // slots - 1 (power of two)
};

struct BwFold {  // simple case folding (ICU u_foldCase default): cp + f2[f1[cp >> 7] << 7 | cp & 127]
  const uint16_t* f1;
  const int32_t* f2;
  TB_HD uint32_t operator()(uint32_t c) const {
    if (c > 0x10FFFF) return c;
    return (uint32_t)((int32_t)c + f2[((uint32_t)f1[c >> 7] << 7) | (c & 127)]);
  }
};

TB_HD uint32_t bw_hash(uint32_t node, uint32_t cp) {
  uint32_t h = node * 0x9E3779B1u ^ cp * 0x85EBCA6Bu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return h ^ (h >> 13);
}

// Child of `node` on code point `cp` (-1: none); *term = the child ends a list entry.
TB_HD int32_t bw_step(const BwTable& t, int32_t node, uint32_t cp, bool* term) {
  uint32_t s = bw_hash((uint32_t)node, cp) & t.mask;
  for (;;) {
    const uint32_t* e = t.e + 4 * s;
    const uint32_t k = e[0];
    if (k == 0) return -1;
    if (k == (uint32_t)node + 1 && e[1] == cp) {
      *term = e[3] != 0;
      return (int32_t)e[2];
    }
    s = (s + 1) & t.mask;
  }
}

// ASCII code points resolved from a 128-entry table (word-character bit 7 | simple fold, from
// the same property / fold tables): the kernel keeps it in LDS, so the common case needs no
// dependent global lookups.
template <class A>
TB_HD bool bw_wordchar(const UcdView& ucd, const A& asc, uint32_t cp) {
  if (cp < 128) return (asc[cp] & 0x80u) != 0;
  return (ucd.props(cp) & P_WORDCHAR) != 0;
}
template <class A>
TB_HD uint32_t bw_fold(const BwFold& fold, const A& asc, uint32_t cp) {
  return cp < 128 ? (uint32_t)(asc[cp] & 0x7Fu) : fold(cp);
}
TB_HD uint8_t bw_ascii_entry(const UcdView& ucd, const BwFold& fold, uint32_t c) {
  return (uint8_t)(((ucd.props(c) & P_WORDCHAR) ? 0x80u : 0u) | (fold(c) & 0x7Fu));
}

// (?:\W|^) before byte s (a code point boundary): the previous code point is not a word character.
template <class A>
TB_HD bool bw_left_ok(const uint8_t* b, uint32_t n, uint32_t s, const UcdView& ucd, const A& asc) {
  if (s == 0) return true;
  const uint8_t pb = b[s - 1];
  if (pb < 0x80) return (asc[pb] & 0x80u) == 0;
  uint32_t p = s - 1;
  while (p > 0 && !utf8_is_lead(b[p])) --p;
  int len;
  return !bw_wordchar(ucd, asc, utf8_decode(b, p, n, &len));
}

// Does a list entry start at byte s (a code point boundary whose left side is already checked)?
template <class A>
TB_HD bool bw_walk_from(const uint8_t* b, uint32_t n, uint32_t s, int32_t root, bool cjk, const BwTable& t,
                        const UcdView& ucd, const BwFold& fold, const A& asc) {
  int32_t node = root;
  uint32_t j = s;
  while (j < n) {
    int len = 1;
    const uint32_t c = b[j] < 0x80 ? b[j] : utf8_decode(b, j, n, &len);
    bool term = false;
    node = bw_step(t, node, bw_fold(fold, asc, c), &term);
    if (node < 0) return false;
    j += (uint32_t)len;
    if (term) {
      if (cjk || j >= n) return true;
      int l2;
      const uint32_t d = b[j] < 0x80 ? b[j] : utf8_decode(b, j, n, &l2);
      if (!bw_wordchar(ucd, asc, d)) return true;  // (?:\W|$)
    }
  }
  return false;
}

// Host twin of k_badwords_match for one document.
template <class A>
TB_HD bool bw_match_doc(const uint8_t* b, uint32_t n, int32_t root, bool cjk, const BwTable& t, const UcdView& ucd,
                        const BwFold& fold, const A& asc) {
  for (uint32_t s = 0; s < n; ++s)
    if (utf8_is_lead(b[s]) && (cjk || bw_left_ok(b, n, s, ucd, asc)) && bw_walk_from(b, n, s, root, cjk, t, ucd, fold, asc))
      return true;
  return false;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Hash table of the flattened tries (BadWordsModule::flatten: CSR edges per node, sorted by code
// point): load factor <= 1/2, power-of-two slots.
inline std::vector<uint32_t> bw_build_table(const int32_t* first_edge, int64_t nodes, const uint32_t* edge_cp,
                                            const int32_t* edge_to, int64_t nedges, const uint8_t* term) {
  uint64_t slots = 16;
  while (slots < 2 * (uint64_t)nedges) slots <<= 1;
  if (slots > (1ull << 31)) throw std::length_error("bad-words automaton too large");
  std::vector<uint32_t> tab(4 * slots, 0);
  const uint32_t mask = (uint32_t)(slots - 1);
  for (int64_t v = 0; v < nodes; ++v) {
    for (int32_t k = first_edge[v]; k < first_edge[v + 1]; ++k) {
      if (k < 0 || k >= nedges || edge_to[k] < 0 || edge_to[k] >= nodes)
        throw std::invalid_argument("bad-words automaton edge out of range");
      uint32_t s = bw_hash((uint32_t)v, edge_cp[k]) & mask;
      while (tab[4 * s] != 0) s = (s + 1) & mask;
      tab[4 * s] = (uint32_t)v + 1;
      tab[4 * s + 1] = edge_cp[k];
      tab[4 * s + 2] = (uint32_t)edge_to[k];
      tab[4 * s + 3] = term[edge_to[k]] ? 1u : 0u;
    }
  }
  return tab;
}
#endif

}  // namespace tb
