// Per-document analysis algorithms shared by the HIP kernels (WavePar) and the host emulation
// (SeqPar). Everything a filter needs is derived from one decode + segmentation per content
// version, with exact (byte-verified) duplicate detection:
//
//   decode          UTF-8 -> code point byte offsets + 16-bit properties  (reference: chars())
//   prefix_hash8    PH8[k] = H(bytes[0..8k)): any substring hash is <= 14 Horner steps + 1 power
//   words           UAX#29 word segments, trimmed, kept iff they contain a non-PUNCTUATION,
//                   non-whitespace char; break bitmask + one fused scan/compaction pass
//                                                       (reference utils/text.rs:103-181)
//   canonicalize    smallest index with an equal element (hash table + byte verification)
//   gopher_quality / gopher_repetition / fineweb / c4 / langid features  (reference filters)
//
// A 64-bit hash collision between unequal elements is never trusted: it raises DOC_NEEDS_CPU and
// the host recomputes that document with the CPU oracle.
#pragma once
#include <type_traits>

#include "devplan.h"
#include "hash.h"
#include "langid.h"
#include "par.h"
#include "uax29.h"
#include "ucd.h"

namespace tb {

// Phase ids for DocCtx::stamp (profiling only).
enum : int {
  PH_START = 0, PH_DECODE, PH_DICT, PH_PREFIX_HASH, PH_WORDS, PH_LINES, PH_GQ, PH_GR_LINES, PH_GR_WORDS,
  PH_GR_TOP, PH_GR_DUP, PH_FW, PH_LID, PH_GR_DUP_WALK, PH_GR_DUP_CANON, PH_GR_TOP_CANON,
  PH_C4_LOREM = 16, PH_C4_DECODE, PH_C4_LINES, PH_C4_CITE, PH_C4_WORDS, PH_C4_CODES, PH_C4_JOIN, PH_C4_SENT,
  // sub-phases of the stage kernel's GopherRepetition / GopherQuality work
  PH_GR_NL = 24, PH_GR_LINE_DUP, PH_GR_WH, PH_GR_WCANON, PH_GQ_WORDS, PH_GQ_BYTES, PH_RUST_LINES,
  kPhaseSlots = 32
};

enum : uint32_t {
  DOC_OK = 0,
  DOC_NEEDS_CPU = 1,    // dictionary script / hash collision / scratch overflow
  DOC_OVERFLOW = 2,
};

// Code points of a text: byte offsets and compact properties. The code point values themselves
// are not stored: ASCII tests read the lead byte (b[off[i]], equal to the code point below 0x80
// and >= 0xC0 otherwise), the rest re-decode from the bytes.
//
// Compact property layout (16 bits): the UCD word bits 0..13 and 15 (WB class, SB class, WS,
// ALPHA, PUNCT, EXTPICT, DIGIT, CASED) unchanged; bit 14 carries CASE_IGN (bit 16 of the full
// word). P_DICT is consumed while decoding (decode() reports it) and not kept.
constexpr uint32_t P16_CASE_IGN = 1u << 14;
TB_HD uint16_t compact_prop(uint32_t p) {
  return (uint16_t)((p & 0xBFFFu) | ((p & P_CASE_IGN) ? P16_CASE_IGN : 0u));
}

// Per-code-point arrays. Texts under 64 KiB keep one packed u32 per code point (byte offset in
// the low half, compact properties in the high half: 4 bytes, one load); longer ones (workgroup
// path) keep a u32 offset array and a u16 property array. The accessors below hide the layout
// (the choice is uniform per document, so the branch is a scalar one).
struct PropArr {
  const uint32_t* ent = nullptr;
  const uint16_t* p16 = nullptr;
  TB_HD uint32_t operator[](uint32_t i) const { return ent ? (ent[i] >> 16) : (uint32_t)p16[i]; }
  TB_HD PropArr operator+(uint32_t s) const { return PropArr{ent ? ent + s : nullptr, ent ? nullptr : p16 + s}; }
};
struct OffArr {
  const uint32_t* ent = nullptr;
  const uint32_t* o32 = nullptr;
  TB_HD uint32_t operator[](uint32_t i) const { return ent ? (ent[i] & 0xFFFFu) : o32[i]; }
};

struct Cps {
  uint32_t n = 0;
  uint32_t* ent = nullptr;    // packed [n+1] (texts < 64 KiB) ...
  uint32_t* off = nullptr;    // ... or [n+1] byte offsets (off[n] = byte length)
  uint16_t* prop = nullptr;   //     and [n+1] compact properties
  const uint8_t* b = nullptr; // the text
  uint32_t nb = 0;            // its byte length
  TB_HD PropArr props() const { return PropArr{ent, prop}; }
  TB_HD OffArr offs() const { return OffArr{ent, off}; }
  TB_HD uint32_t o(uint32_t i) const { return ent ? (ent[i] & 0xFFFFu) : off[i]; }
  TB_HD uint32_t p(uint32_t i) const { return ent ? (ent[i] >> 16) : (uint32_t)prop[i]; }
  TB_HD uint8_t lead(uint32_t i) const { return b[o(i)]; }
  // lead(i) == '\n' from the properties alone (U+000A is the only code point of word-break
  // class LF): one read of the per-code-point array (LDS on the wave path) instead of the
  // offset read followed by a dependent read of the text
  TB_HD bool is_lf(uint32_t i) const { return (p(i) & P_WB_MASK) == (uint32_t)WB_LF; }
  TB_HD uint32_t cp(uint32_t i) const {
    int len;
    return utf8_decode(b, o(i), nb, &len);
  }
};

struct CpsAcc {  // accessor for the UAX#29 rule templates over a sub-range
  PropArr prop;
  TB_HD uint32_t p(int i) const { return prop[(uint32_t)i]; }
};

// Prefix hashes of a text kept at every 8th byte only (PH8[k] = H(b[0..8k)), PHn = H(b)): a
// prefix at any position is at most 7 Horner steps away, so the table costs 1 byte per text byte
// (LDS-resident for typical documents) instead of 8.
struct PHView {
  const uint64_t* ph8 = nullptr;
  uint64_t phn = 0;
  const uint8_t* b = nullptr;
  uint32_t n = 0;
  TB_HD uint64_t at(uint32_t x) const {
    if (x >= n) return phn;
    uint64_t h = ph8[x >> 3];
    for (uint32_t j = x & ~7u; j < x; ++j) h = hash_push(h, b[j]);
    return h;
  }
};

// a very long document's code points and UAX#29 word-break marks, computed before
// its stage workgroup runs by many workgroups at once (kernels.hip k_pre_count / k_pre_decode /
// k_pre_wb): the non-packed Cps layout (documents of 64 KiB and more) plus the marks words()
// would compute.
struct PreDoc {
  uint32_t* off;     // [n + 1] byte offset of every code point (off[C] = n)
  uint16_t* prop;    // [n + 1] compact properties
  uint32_t* wbm;     // [mask_words(n + 1)] bit i: word boundary before code point i
  uint32_t* nl_pos;  // [n / 2 + 2] code point index of every run of '\n' (GopherRepetition lines)
  uint32_t* nl_len;  //   and its length
  uint32_t n;        // bytes
  uint32_t C;        // code points
  uint32_t dict;     // a dictionary-script code point occurs (the document goes to the CPU path)
  uint32_t NL;       // runs of '\n'
  uint32_t tcs;      // first non-whitespace code point (host: 0xFFFFFFFF)
  uint32_t tce;      // one past the last one (host: 0)
  uint32_t nl_a;     // the runs of '\n' inside [tcs, tce): nl_pos[nl_a, nl_e)
  uint32_t nl_e;
  // the words (words() of the same code points): W entries of cs / ce / bs / be / alpha, and the
  // per-64-code-point chunk scratch of their segmented scan (aggregate, carry-in: 3 words each;
  // word count, first word index)
  uint32_t* wtmp;
  uint32_t* wcs;
  uint32_t* wce;
  uint32_t* wbs;
  uint32_t* wbe;
  uint8_t* wal;
  uint32_t W;
  uint32_t pad;
  // GopherRepetition's word arrays (gopher_rep_record) built by many workgroups
  // (kernels.hip k_pre_wcanon): word hashes, the canonicalisation table (1.5 W + 2 64-bit slots)
  // and each word's slot, per-2048-word chunk sums and bases, and the results wid / WL / K / PB
  // (W + 1 entries each); wready = 1 once they are filled.
  uint64_t* wh;
  uint64_t* wtab;
  uint64_t* wk;
  uint64_t* wpb;
  uint64_t* wcsum;
  uint32_t* wslot;
  uint32_t* wid;
  uint32_t* wl;
  uint32_t wready;
  uint32_t pad2;
};

struct Words {
  uint32_t n = 0;
  uint32_t* cs = nullptr;  // first code point
  uint32_t* ce = nullptr;  // one past last code point
  uint32_t* bs = nullptr;  // byte start
  uint32_t* be = nullptr;  // byte end
  uint8_t* alpha = nullptr;
};

struct Lines {  // Rust str::lines() in code point space
  uint32_t n = 0;
  uint32_t* ls = nullptr;  // start cp
  uint32_t* le = nullptr;  // end cp (excludes '\n' and a '\r' right before it)
};

struct HL {
  uint64_t h;
  uint32_t len;
  uint32_t pad;
};

template <class P>
struct DocCtx {
  P par;
  UcdView ucd;
  const uint64_t* pw = nullptr;  // pw[k] = B^k, k <= pw_n; followed by ipw
  const uint64_t* ipw = nullptr; // ipw[k] = B^-k, k <= pw_n
  uint32_t pw_n = 0;
  const uint16_t* asc = nullptr; // compact UCD properties of code points < 256 (LDS copy), or null
  char* scr = nullptr;       // global (HBM) scratch arena of this document
  uint64_t cap = 0;
  uint64_t used = 0;
  uint64_t peak = 0;         // high-water mark of `used`, host emulation (sizes devplan.h kScratchPerByte)
  char* lds = nullptr;      // optional fast arena (the wave's LDS slice on the device)
  uint32_t lcap = 0;
  uint32_t lused = 0;        // bytes allocated from the bottom of the LDS slice
  uint32_t lhi = 0;          // bytes allocated from the top (temporaries, releasable props)
  uint32_t* flag = nullptr;  // per-document status word
  bool weak_keys = false;     // test hook: canonicalize() sees keys cut to 2 bits (forced collisions)
  bool overflow = false;
  uint64_t* prof = nullptr;  // optional per-document phase cycle counters (kPhaseSlots)
  uint64_t t_last = 0;

  // Phase timing (profiling builds of a run): cycles since the previous stamp go to `id`.
  TB_HD void stamp(int id) {
    if (!prof) return;
    const uint64_t t = P::clock();
    if (t_last && par.leader()) prof[id] += t - t_last;
    t_last = t;
  }

  struct Mark { uint64_t g; uint32_t l, h; };
  TB_HD Mark mark() const { return Mark{used, lused, lhi}; }
  TB_HD void reset(Mark m) { used = m.g; lused = m.l; lhi = m.h; }

  // Placement: big streaming per-code-point arrays live in the HBM scratch arena (alloc);
  // small randomly-accessed ones (hash tables, per-word / per-n-gram arrays, reduction
  // buffers) go to the wave's LDS slice while it has room (alloc_hot), then to HBM. Both are
  // addressed through generic pointers, so algorithm code is the same for either arena.
  template <class T>
  TB_HD T* alloc(uint64_t count) { return alloc_global<T>(count); }
  template <class T>
  TB_HD T* alloc_hot(uint64_t count) {
    if (lds) {
      const uint64_t a = (lused + 15u) & ~15u;
      const uint64_t e = a + count * sizeof(T);
      if (e + lhi <= lcap) {
        lused = (uint32_t)e;
        return (T*)(lds + a);
      }
    }
    return alloc_global<T>(count);
  }
  // Same, from the top of the LDS slice: short-lived tables (released by reset()) and the
  // property array, which the n-gram statistics no longer need (release_hi()), so the space
  // they held goes back to the hash tables of the later phases.
  template <class T>
  TB_HD T* alloc_hot_hi(uint64_t count) {
    if (lds) {
      const uint64_t bytes = (count * sizeof(T) + 15u) & ~15ull;
      const uint64_t lo = (lused + 15u) & ~15u;
      if (lo + lhi + bytes <= lcap) {
        lhi += (uint32_t)bytes;
        return (T*)(lds + (lcap - lhi));
      }
    }
    return alloc_global<T>(count);
  }
  TB_HD void release_hi() { lhi = 0; }
  TB_HD bool in_lds(const void* p) const {
    return lds && (const char*)p >= lds && (const char*)p < lds + lcap;
  }
  // bytes of the LDS slice still free between the bottom and top allocations
  TB_HD uint32_t lds_free() const {
    if (!lds) return 0;
    const uint32_t lo = (lused + 15u) & ~15u;
    return lo + lhi >= lcap ? 0u : lcap - lo - lhi;
  }
  // alloc_hot, but only while `keep` bytes of the slice stay free afterwards (for the hash
  // tables of a later phase, whose random accesses gain far more from the LDS than the
  // sequential scans of this array do); otherwise HBM
  template <class T>
  TB_HD T* alloc_hot_keep(uint64_t count, uint64_t keep) {
    if (lds && (uint64_t)lds_free() >= count * sizeof(T) + 16 + keep) return alloc_hot<T>(count);
    return alloc_global<T>(count);
  }
  template <class T>
  TB_HD T* alloc_global(uint64_t count) {
    uint64_t a = (used + 15) & ~15ull;
    uint64_t e = a + count * sizeof(T) + 16;
    if (e > cap) {
      overflow = true;
      return (T*)scr;  // callers check `overflow` before using results
    }
    used = a + count * sizeof(T);
    // host emulation only: one more live 64-bit value triples the long-document kernels' spills
    if constexpr (P::kWaves == 0) {
      if (used > peak) peak = used;
    }
    return (T*)(scr + a);
  }
  TB_HD void set_flag(uint32_t f) {
    if (flag) P::or32(flag, f);  // atomic: kernels of different steps may run concurrently
  }
  TB_HD uint64_t powb(uint32_t k) const { return k <= pw_n ? pw[k] : hpow(kHashBase, k); }
  TB_HD uint64_t ipowb(uint32_t k) const { return (ipw && k <= pw_n) ? ipw[k] : hpow(kHashBaseInv, k); }
  // `count` elements from the bottom of the LDS slice, or nullptr when they do not fit
  template <class T>
  TB_HD T* try_lds(uint64_t count) {
    if (!lds) return nullptr;
    const uint64_t a = (lused + 15u) & ~15u;
    const uint64_t e = a + count * sizeof(T);
    if (e + lhi > lcap) return nullptr;
    lused = (uint32_t)e;
    return (T*)(lds + a);
  }
};

TB_HD bool is_ws(uint32_t p) { return (p & P_WS) != 0; }

// [tcs, tce): the code points of [0, C) without leading / trailing whitespace (tcs >= tce: all
// whitespace). One wave searches chunk by chunk from each end and stops at the first chunk with a
// non-whitespace code point (usually the first and the last chunk) instead of reducing over all
// code points.
template <class P, class PA>
TB_HD void trim_span(DocCtx<P>& x, const PA& prop, uint32_t C, uint32_t& tcs, uint32_t& tce) {
#if defined(__HIPCC__)
  if constexpr (P::kWaves == 1) {
    const uint32_t lane = x.par.lane;
    tcs = C;
    for (uint32_t base = 0; base < C; base += 64) {
      const uint32_t j = base + lane;
      const uint64_t m = __ballot(j < C && !is_ws(prop[j]));
      if (m) { tcs = base + (uint32_t)__builtin_ctzll(m); break; }
    }
    tce = 0;
    if (tcs < C) {
      for (uint32_t base = (C - 1) & ~63u;; base -= 64) {
        const uint32_t j = base + lane;
        const uint64_t m = __ballot(j < C && !is_ws(prop[j]));
        if (m) { tce = base + (uint32_t)(64 - __clzll((long long)m)); break; }
        if (base == 0) break;
      }
    }
    return;
  }
#endif
  tcs = x.par.template min<uint32_t>(C, C, [&](uint32_t i) { return is_ws(prop[i]) ? C : i; });
  tce = x.par.template max<uint32_t>(C, 0u, [&](uint32_t i) { return is_ws(prop[i]) ? 0u : i + 1; });
}
// Wave documents with fewer words than this keep n-gram canonical ids in 16 bits (every
// canonicalisation slot index < 1.5 n + 2 fits); more words send the document to the CPU path.
constexpr uint32_t kWave16 = 43000;
TB_HD constexpr int rec_gr_fixed() { return 7; }

// ---------------------------------------------------------------------------------------------
template <class P>
TB_HD Cps decode(DocCtx<P>& x, const uint8_t* b, uint32_t n, bool hot = false, uint32_t* dict = nullptr) {
  Cps c;
  c.b = b;
  c.nb = n;
  // read by every later pass (rule look-around, trims, spans): with `hot` they go to the top of
  // the LDS slice when the document is small enough (released before the n-gram statistics)
  const bool packed = n < 65536u;
  if (packed) {
    c.ent = hot ? x.template alloc_hot_hi<uint32_t>(n + 1) : x.template alloc<uint32_t>(n + 1);
  } else {
    c.prop = hot ? x.template alloc_hot_hi<uint16_t>(n + 1) : x.template alloc<uint16_t>(n + 1);
    c.off = hot ? x.template alloc_hot_hi<uint32_t>(n + 1) : x.template alloc<uint32_t>(n + 1);
  }
  if (x.overflow) return c;
  const UcdView ucd = x.ucd;
  const uint16_t* asc = x.asc;
  uint32_t* ent = c.ent;
  uint32_t* off = c.off;
  uint16_t* pra = c.prop;
  uint32_t dl = 0;
  c.n = x.par.template compact<int>(
      n, [&](uint32_t i, int&) { return utf8_is_lead(b[i]); },
      [&](uint32_t i, uint32_t k, int&) {
        uint16_t cpk;
        const uint32_t c0 = b[i];
        // U+0000..U+00FF (ASCII, and C2 / C3 leads: Latin-1, e.g. æ ø å ä ö é) from the LDS table,
        // decoded inline; none of them is a dictionary script
        if (asc && (c0 < 0x80 || (c0 & 0xFEu) == 0xC2u)) {
          cpk = asc[c0 < 0x80 ? c0 : (((c0 & 0x1Fu) << 6) | (b[i + 1] & 0x3Fu))];
        } else {
          int len;
          const uint32_t p = ucd.props(utf8_decode(b, i, n, &len));
          cpk = compact_prop(p);
          dl |= (p & P_DICT) ? 1u : 0u;
        }
        if (packed) {
          ent[k] = i | ((uint32_t)cpk << 16);
        } else {
          off[k] = i;
          pra[k] = cpk;
        }
      });
  const uint32_t cn = c.n;
  x.par.single([&]() {
    if (packed) ent[cn] = n;
    else { off[cn] = n; pra[cn] = 0; }
  });
  if (dict) *dict = x.par.reduce_or(dl);
  x.par.sync();
  return c;
}

template <class P>
TB_HD uint64_t span_hash8(const DocCtx<P>& x, const PHView& v, uint32_t s, uint32_t e) {
  const uint64_t hs = v.at(s), he = v.at(e);
  return he - hs * x.powb(e - s);
}

template <class P>
TB_HD PHView prefix_hash8(DocCtx<P>& x, const uint8_t* b, uint32_t n) {
  PHView v;
  v.b = b;
  v.n = n;
  const uint32_t nblk = (n + 7) >> 3;
  // top of the slice: released with the code point arrays before the n-gram statistics
  uint64_t* ph8 = x.template alloc_hot_hi<uint64_t>(nblk + 1);
  if (x.overflow) return v;
  const uint64_t* pw = x.pw;
  const uint32_t pwn = x.pw_n;
  HL tot = x.par.template scan<HL>(
      nblk, HL{0, 0, 0},
      [&](const HL& a, const HL& c) {
        uint64_t m = c.len <= pwn ? pw[c.len] : hpow(kHashBase, c.len);
        return HL{a.h * m + c.h, a.len + c.len, 0};
      },
      [&](uint32_t k) {
        const uint32_t s0 = k << 3, e0 = s0 + 8 < n ? s0 + 8 : n;
        uint64_t h = 0;
        // (a sum of independent (v_j + 1) * B^(L-1-j) terms measured slower: 23.1 K -> 31.5 K
        // prefix_hash cycles/doc, the power loads)
        for (uint32_t j = s0; j < e0; ++j) h = hash_push(h, b[j]);
        return HL{h, e0 - s0, 0};
      },
      [&](uint32_t k, const HL& e) { ph8[k] = e.h; });
  x.par.single([&]() { ph8[nblk] = tot.h; });
  x.par.sync();
  v.ph8 = ph8;
  v.phn = tot.h;
  return v;
}

// UAX#29 word segments of code points [0, C) -> words (trimmed, with a word character).
// Segments are aggregated with one segmented scan over the code points (no per-lane walk over a
// segment): a segment's first code point carries the reset flag, the running element ORs the
// word-character / alphabetic bits and tracks the first and last non-whitespace code point.
struct WSeg {
  uint32_t bits;   // bit0: segment start (reset), bit1: has a word char, bit2: alphabetic
  uint32_t first;  // first non-whitespace cp (0xFFFFFFFF if none)
  uint32_t last;   // one past the last non-whitespace cp
};
TB_HD WSeg wseg_op(const WSeg& a, const WSeg& b) {
  if (b.bits & 1u) return b;
  return WSeg{a.bits | (b.bits & 6u), a.first < b.first ? a.first : b.first, a.last > b.last ? a.last : b.last};
}

// Word-boundary mark before code point i of [0, C) (sot and eot included). The rules are first
// decided from the properties of i-2 .. i+1 (wb_break_ctx: straight-line compares, no look-around
// loops); only windows holding Extend / Format / ZWJ / RI take the general rule walk, so a chunk
// with punctuation or digits does not serialise the wave on it.
#ifndef TB_WB_CTX
#define TB_WB_CTX 1
#endif
#if defined(__HIPCC__)
// the word-break pair table (uax29.h kWbPairTab) in constant memory: the one-wave words() loads it
// into one register (lane k holds dword k) and reads a pair's dword from the lane that holds it;
// word_mark() on the device reads it directly
static __constant__ WbPairTab g_wb_pair_tab = kWbPairTab;
#endif
TB_HD bool word_mark(const PropArr& prop, uint32_t C, uint32_t i) {
  if (i == 0 || i == C) return true;
  if (TB_WB_CTX) {
    const uint32_t pm2 = i >= 2 ? prop[i - 2] : 0xFFFFFFFFu;
    const uint32_t pp1 = i + 1 < C ? prop[i + 1] : 0xFFFFFFFFu;
#if defined(__HIP_DEVICE_COMPILE__)
    const int r = wb_break_ctx_tab(pm2, prop[i - 1], prop[i], pp1, [](uint32_t k) { return g_wb_pair_tab.w[k]; });
#else
    const int r = wb_break_ctx_tab(pm2, prop[i - 1], prop[i], pp1);
#endif
    if (r != 2) return r != 0;
  }
  return wb_break(CpsAcc{prop}, (int)C, (int)i);
}

#if defined(__HIPCC__)
// words() for one wave (WavePar), in one pass over the code points instead of a mark pass and a
// scan pass: each chunk's packed entries are loaded once (the next chunk's while this one is
// processed, so the load is off the critical path), the neighbours the break rules look at come
// from DPP lane moves (wave_shr / wave_shl) plus a two-entry carry, and each word's extent comes
// from bit operations on the chunk's ballots (no segmented scan). Same words as the generic
// version (word_mark + the WSeg scan).
struct WSeg5 {  // the segment still open at a chunk's end
  uint32_t bits, first, last, fo, lo;  // WSeg bits + byte offsets of `first` / `last`
};
__device__ __forceinline__ uint32_t lane_prev(uint32_t v) {  // lane l gets lane l-1 (lane 0: v)
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {  // lane l gets lane l+1 (lane 63: v)
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xF, 0xF, false);
}
// The pair table dword of the pair (pm1, p0): read from the lane that holds it, by every lane of
// the wave at once (a lane read from a lane outside EXEC returns nothing useful, so this is never
// done under divergent control flow).
__device__ __forceinline__ uint32_t wb_pair_dword(uint32_t wbt, uint32_t pm1, uint32_t p0) {
  const uint32_t i = (pm1 & P_WB_MASK) * kWbClasses + (p0 & P_WB_MASK);
  return (uint32_t)__shfl((int)wbt, (int)(i >> 3));
}
// word_mark from the four properties around position i (sentinel 0xFFFFFFFF outside [0, C));
// tw: the pair table dword of (pm1, p0) (wb_pair_dword)
__device__ __forceinline__ bool word_mark4(const PropArr& prop, uint32_t C, uint32_t i, uint32_t pm2, uint32_t pm1,
                                           uint32_t p0, uint32_t pp1, uint32_t tw) {
  if (i == 0 || i >= C) return true;
  const int r = wb_break_ctx_tab(pm2, pm1, p0, pp1, [&](uint32_t) { return tw; });
  if (r != 2) return r != 0;
  return wb_break(CpsAcc{prop}, (int)C, (int)i);
}
template <class P>
__device__ Words words_wave(DocCtx<P>& x, const Cps& c, const uint32_t* marks) {
  Words w;
  const uint32_t C = c.n;
  w.cs = x.template alloc<uint32_t>(C + 1);
  w.ce = x.template alloc<uint32_t>(C + 1);
  w.bs = x.template alloc<uint32_t>(C + 1);
  w.be = x.template alloc<uint32_t>(C + 1);
  w.alpha = x.template alloc<uint8_t>(C + 1);
  if (x.overflow) return w;
  const PropArr prop = c.props();
  const uint32_t lane = x.par.lane;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // The word arrays are in the HBM arena (alloc): typed as global, their stores are global_store
  // (vmcnt only) instead of flat stores, which the next chunk's flat loads would have to wait for.
  typedef __attribute__((address_space(1))) uint32_t g32;
  typedef __attribute__((address_space(1))) uint8_t g8;
  g32 *cs = (g32*)w.cs, *ce = (g32*)w.ce, *bs = (g32*)w.bs, *be = (g32*)w.be;
  g8* al = (g8*)w.alpha;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  // entry i <= C: property (entry C: 0) and byte offset (entry C: the byte length)
  uint32_t cp = 0, co = 0, np = 0, no = 0;
  if (lane <= C) { cp = c.p(lane); co = c.o(lane); }
  const uint32_t wbt = lane < (uint32_t)kWbTabWords ? g_wb_pair_tab.w[lane] : 0u;
  uint32_t c1 = kNone, c2 = kNone;  // properties of the two code points before the chunk
  WSeg5 carry{0u, kNone, 0u, kNone, 0u};
  uint32_t k = 0;
  for (uint32_t base = 0; base < C; base += 64) {
    const uint32_t j = base + lane;
    const uint32_t jn = j + 64;
    if (jn <= C) { np = c.p(jn); no = c.o(jn); }  // prefetch of the next chunk
    // neighbours: i-1, i-2 (carry for the first lanes), i+1 (the next chunk's first for lane 63)
    const uint32_t n0p = (uint32_t)__builtin_amdgcn_readfirstlane((int)np);
    const uint32_t n1p = (uint32_t)__builtin_amdgcn_readlane((int)np, 1);
    const uint32_t n0o = (uint32_t)__builtin_amdgcn_readfirstlane((int)no);
    uint32_t pm1 = lane_prev(cp);
    if (lane == 0) pm1 = c1;
    uint32_t pm2 = lane_prev(pm1);
    if (lane == 0) pm2 = c2;
    uint32_t pp1 = lane_next(cp), on = lane_next(co);
    if (lane == 63) { pp1 = base + 64 <= C ? n0p : kNone; on = n0o; }
    // positions past C-1 do not exist for the rules (word_mark's sentinels)
    const uint32_t pm2s = j >= 2 ? pm2 : kNone;
    const uint32_t pp1s = j + 1 < C ? pp1 : kNone;
    // the mark at base + 64 (lane 63's successor): from the last two code points and the next
    // chunk's first two (uniform); with host marks (dictionary scripts, ICU) both from the bitmap
    const uint32_t l62 = (uint32_t)__builtin_amdgcn_readlane((int)cp, 62);
    const uint32_t l63 = (uint32_t)__builtin_amdgcn_readlane((int)cp, 63);
    const uint32_t i64 = base + 64;
    const uint32_t tw = wb_pair_dword(wbt, pm1, cp), tw64 = wb_pair_dword(wbt, l63, n0p);  // (all lanes)
    bool mk = j < C && word_mark4(prop, C, j, pm2s, pm1, cp, pp1s, tw);
    bool mk64 = i64 >= C || word_mark4(prop, C, i64, l62, l63, n0p, i64 + 1 < C ? n1p : kNone, tw64);
    if (marks) {  // host record: ICU marks (first bitmap) where its mask (second bitmap) is set
      const uint32_t* hm = marks + mask_words(C + 1);
      if (j < C && ((hm[j >> 5] >> (j & 31)) & 1u)) mk = ((marks[j >> 5] >> (j & 31)) & 1u) != 0;
      if (i64 < C && ((hm[i64 >> 5] >> (i64 & 31)) & 1u)) mk64 = ((marks[i64 >> 5] >> (i64 & 31)) & 1u) != 0;
    }
    // Segment aggregates from ballots instead of a scan: a lane's segment runs from the last mark
    // at or below it (or, with none, from an earlier chunk: the carry); its first / last
    // non-whitespace code point and its word-character / alphabetic bits are bit operations on
    // the chunk's masks, the byte offsets two lane reads (ds_bpermute).
    const bool valid = j < C;
    const bool ws = is_ws(cp);
    const uint64_t M = __ballot(mk);  // (mk implies j < C)
    const uint64_t NW = __ballot(valid && !ws);
    const uint64_t WC = __ballot(valid && !ws && !(cp & P_PUNCT));
    const uint64_t AL = __ballot(valid && (cp & P_ALPHA));
    const bool mnext = lane == 63 ? mk64 : (((M >> (lane + 1)) & 1ull) != 0 || j + 1 >= C);
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes 0 .. lane
    const uint64_t mb = M & le;
    const bool fc = mb == 0;  // the segment began in an earlier chunk
    const uint64_t seg = fc ? le : (le & (~0ull << (63 - __clzll((long long)mb))));
    const uint64_t nws = NW & seg;
    const bool hasw = (WC & seg) != 0 || (fc && (carry.bits & 2u));
    const int f = nws ? __builtin_ctzll(nws) : 0;
    const int l = nws ? 63 - __clzll((long long)nws) : 0;
    const uint32_t fo_l = (uint32_t)__shfl((int)co, f);
    const uint32_t lo_l = (uint32_t)__shfl((int)on, l);
    const bool sel = valid && mnext && hasw;
    const uint64_t sm = __ballot(sel);
    if (sel) {
      const uint32_t q = k + (uint32_t)__popcll(sm & lt);
      const bool cf = fc && carry.first != kNone;
      const uint32_t w0 = cf ? carry.first : base + (uint32_t)f, w1 = nws ? base + (uint32_t)l + 1u : carry.last;
      const uint32_t b0 = cf ? carry.fo : fo_l, b1 = nws ? lo_l : carry.lo;
      const bool alpha = (AL & seg) != 0 || (fc && (carry.bits & 4u));
      cs[q] = w0;
      bs[q] = b0;
      ce[q] = w1;
      be[q] = b1;
      al[q] = alpha ? 1 : 0;
    }
    k += (uint32_t)__popcll(sm);
    {  // carry: the segment open at the chunk's end (uniform)
      const bool rs = M != 0;
      const uint64_t sg = rs ? (~0ull << (63 - __clzll((long long)M))) : ~0ull;
      const uint64_t nwc = NW & sg;
      const uint32_t keep = rs ? 0u : carry.bits;
      carry.bits = (keep & 6u) | ((WC & sg) ? 2u : 0u) | ((AL & sg) ? 4u : 0u);
      if (rs || carry.first == kNone) {
        if (nwc) {
          const int f2 = __builtin_ctzll(nwc);
          carry.first = base + (uint32_t)f2;
          carry.fo = (uint32_t)__builtin_amdgcn_readlane((int)co, f2);
        } else {
          carry.first = kNone;
        }
      }
      if (nwc) {
        const int l2 = 63 - __clzll((long long)nwc);
        carry.last = base + (uint32_t)l2 + 1u;
        carry.lo = (uint32_t)__builtin_amdgcn_readlane((int)on, l2);
      } else if (rs) {
        carry.last = 0u;
        carry.lo = 0u;
      }
    }
    c2 = l62;
    c1 = l63;
    cp = np;
    co = no;
  }
  w.n = k;
  x.par.sync();
  return w;
}
#endif

template <class P>
// `marks`: a host record of the code points [0, C] (dictionary scripts: ICU's dictionary
// segmentation of their lines, text.h dict_word_marks): its marks replace word_mark where its mask
// is set.
TB_HD Words words(DocCtx<P>& x, const Cps& c, const PreDoc* pre = nullptr, const uint32_t* marks = nullptr) {
  Words w;
  if (pre) {  // the pre-pass segmented this document already (k_pre_words)
    w.n = pre->W;
    w.cs = pre->wcs;
    w.ce = pre->wce;
    w.bs = pre->wbs;
    w.be = pre->wbe;
    w.alpha = pre->wal;
    return w;
  }
#if defined(__HIPCC__) && !defined(TB_WORDS_GENERIC)
  if constexpr (P::kWaves == 1) return words_wave(x, c, marks);
#endif
  const uint32_t C = c.n;
  w.cs = x.template alloc<uint32_t>(C + 1);
  w.ce = x.template alloc<uint32_t>(C + 1);
  w.bs = x.template alloc<uint32_t>(C + 1);
  w.be = x.template alloc<uint32_t>(C + 1);
  w.alpha = x.template alloc<uint8_t>(C + 1);
  const auto mark = x.mark();
  // word-break positions as a bitmask (C/8 bytes, LDS): one rule evaluation per position, no
  // per-code-point arrays; the segment scan and the word compaction run in one fused pass
  uint32_t* wbm = x.template alloc_hot_hi<uint32_t>(mask_words(C + 1));
  if (x.overflow) return w;
  const PropArr prop = c.props();
  const OffArr off = c.offs();
  if (marks) {  // host record: ICU marks where its mask says so, the rules elsewhere
    const uint32_t* hm = marks + mask_words(C + 1);
    x.par.mask_bits(C + 1, [&](uint32_t i) {
      return ((hm[i >> 5] >> (i & 31)) & 1u) ? ((marks[i >> 5] >> (i & 31)) & 1u) != 0 : word_mark(prop, C, i);
    }, wbm);
  } else {
    x.par.mask_bits(C + 1, [&](uint32_t i) { return word_mark(prop, C, i); }, wbm);
  }
  x.par.sync();
  auto bit = [&](uint32_t i) { return (wbm[i >> 5] >> (i & 31)) & 1u; };
  uint32_t *cs = w.cs, *ce = w.ce, *bs = w.bs, *be = w.be;
  uint8_t* al = w.alpha;
  w.n = x.par.template scan_compact<WSeg>(
      C, WSeg{0u, 0xFFFFFFFFu, 0u} /* two-sided identity */, wseg_op,
      [&](uint32_t j) {
        const uint32_t p = prop[j];
        const bool ws = is_ws(p);
        WSeg e;
        e.bits = bit(j) | ((!(p & P_PUNCT) && !ws) ? 2u : 0u) | ((p & P_ALPHA) ? 4u : 0u);
        e.first = ws ? 0xFFFFFFFFu : j;
        e.last = ws ? 0u : j + 1;
        return e;
      },
      [&](uint32_t j, const WSeg& in) { return bit(j + 1) && (in.bits & 2u); },
      [&](uint32_t, uint32_t k, const WSeg& in) {
        cs[k] = in.first;
        ce[k] = in.last;
        bs[k] = off[in.first];
        be[k] = off[in.last];
        al[k] = (in.bits & 4u) ? 1 : 0;
      });
  x.par.sync();
  x.reset(mark);
  return w;
}

// Rust str::lines() of the whole text, in code point space.
template <class P>
TB_HD Lines rust_lines(DocCtx<P>& x, const Cps& c) {
  Lines L;
  const uint32_t C = c.n;
  L.ls = x.template alloc<uint32_t>(C + 1);
  L.le = x.template alloc<uint32_t>(C + 1);
  if (x.overflow) return L;
  uint32_t* ls = L.ls;
  uint32_t* le = L.le;
  L.n = x.par.template compact<int>(
      C, [&](uint32_t i, int&) { return i == 0 || c.is_lf(i - 1); },
      [&](uint32_t i, uint32_t k, int&) { ls[k] = i; });
  x.par.sync();
  const uint32_t NL = L.n;
  x.par.for_n(NL, [&](uint32_t k) {
    uint32_t e = (k + 1 < NL) ? ls[k + 1] - 1 : (c.is_lf(C - 1) ? C - 1 : C);
    uint32_t ce = e;
    if (e < C && ce > ls[k] && c.lead(ce - 1) == '\r') --ce;
    le[k] = ce;
  });
  x.par.sync();
  return L;
}

// canon[i] = smallest j with element j == element i (key() groups candidates, eq() verifies).
//
// Up to 65534 elements (every wave-path document): open addressing over ~1.5 n packed 32-bit
// slots (16-bit fingerprint from the key's high bits | smallest index + 1; 0 = empty), half the
// LDS of 64-bit slots, so the table stays on chip. An element joins a slot whose fingerprint
// matches only after eq() against the slot's member says they are equal (a fingerprint
// collision keeps probing), so the grouping is exact and no document is sent to the CPU for it;
// a 32-bit atomic min keeps the smallest index. Larger inputs (workgroup path) use 64-bit slots
// with a 32-bit fingerprint and a verification pass, where a collision between unequal elements
// sends the document to the CPU oracle.
#ifndef TB_ZERO4
#define TB_ZERO4 1
#endif
// Zeroes the u32 table t[0, count rounded up to 4) (allocated that large): 16-byte stores.
struct alignas(16) Zero4 { uint32_t v[4]; };
template <class P>
TB_HD void zero_table(DocCtx<P>& x, uint32_t* t, uint32_t count) {
  const uint32_t q = (count + 3u) >> 2;
  // (not in the one-wave kernel: the 16-byte stores cost it registers, measured slower there)
  if (TB_ZERO4 && P::kWaves != 1 && (((uintptr_t)t) & 15u) == 0) {
    Zero4* t4 = (Zero4*)t;
    x.par.for_n(q, [&](uint32_t i) { t4[i] = Zero4{{0u, 0u, 0u, 0u}}; });
  } else {
    x.par.for_n(count, [&](uint32_t i) { t[i] = 0; });
  }
}

struct NoResolve {
  TB_HD void operator()(uint32_t, uint32_t) const {}
};


template <class P, class KeyF, class EqF, class CT>
TB_HD void canonicalize(DocCtx<P>& x, uint32_t n, KeyF&& key, EqF&& eq, CT* canon);

// Same, and res(i, canon[i]) for every element once its canonical index is final (fused into
// the last pass, so callers need no extra pass over canon[]).
// canon may be 16-bit (wave documents: n < 43000, so every slot index fits) or 32-bit.
template <class P, class KeyF, class EqF, class CT, class ResF>
TB_HD void canonicalize_res(DocCtx<P>& x, uint32_t n, KeyF&& key, EqF&& eq, CT* canon, ResF&& res) {
  const uint32_t capn = n + (n >> 1) + 2;
  // allocated slots: whole 16-byte groups for zero_table's wide stores (exact in the one-wave kernel)
  const uint32_t capa = P::kWaves == 1 ? capn : (capn + 3u) & ~3u;
  const auto mark = x.mark();
  if (n < 65535u) {
    // The table's random probes want the LDS. When the whole table does not fit the free part
    // of the slice (long documents), the slot range is cut into parts that do: part q holds
    // the elements whose home slot falls in [q*capp, (q+1)*capp), and the parts are built one
    // after another in the same LDS table, from keys computed once into HBM. Equal elements
    // share a home slot, hence a part, so the grouping stays exact.
    const uint32_t fit = x.lds_free() >= 64u ? (x.lds_free() - 32u) / 4u : 0u;
    uint32_t parts = 1;
    if (P::kPartTables && x.lds && capn > fit && fit >= 2048u) parts = (capn + fit - 1) / fit;
    if (P::kPartTables && parts > 1) {
      const uint32_t capp = (capn + parts - 1) / parts;
      uint32_t* tab = x.template alloc_hot_hi<uint32_t>(P::kWaves == 1 ? capp : (capp + 3u) & ~3u);
      uint64_t* keys = x.template alloc<uint64_t>(n);
      if (x.overflow) return;
      x.par.for_n(n, [&](uint32_t i) { keys[i] = x.weak_keys ? (key(i) & 3ull) : key(i); });
      x.par.sync();
      bool full = false;
      for (uint32_t q = 0; q < parts; ++q) {
        zero_table(x, tab, capp);
        x.par.sync();
        x.par.for_n(n, [&](uint32_t i) {
          const uint64_t k = keys[i];
          const uint32_t home = (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
          if (home / capp != q) return;
          const uint32_t fp = (uint32_t)(k >> 48);
          const uint32_t mine = (fp << 16) | (i + 1);
          uint32_t slot = home - q * capp;
          for (uint32_t probes = 0;; ++probes) {
            if (probes >= capp) {  // a part ran full (never for hashed keys): exact CPU path
              full = true;
              slot = 0;
              break;
            }
            uint32_t cur = tab[slot];
            if (cur == 0) {
              cur = P::cas32(&tab[slot], 0u, mine);
              if (cur == 0) break;
            }
            if ((cur >> 16) == fp && eq(i, (cur & 0xFFFFu) - 1u)) {
              // the slot's index only decreases: no atomic when it is already below mine
              if ((cur & 0xFFFFu) > i + 1u) P::min32(&tab[slot], mine);
              break;
            }
            if (++slot == capp) slot = 0;
          }
          canon[i] = slot;
        });
        x.par.sync();
        x.par.for_n(n, [&](uint32_t i) {
          const uint32_t home = (uint32_t)(((keys[i] & 0xFFFFFFFFull) * capn) >> 32);
          if (home / capp == q) {
            const uint32_t c = (tab[canon[i]] & 0xFFFFu) - 1u;
            canon[i] = c;
            res(i, c);
          }
        });
        x.par.sync();
      }
      if (x.par.reduce_or(full ? 1u : 0u)) {  // uniform: every lane takes the branch together
        // (the document goes to the CPU oracle: res() results are discarded with it)
        x.set_flag(DOC_NEEDS_CPU);
        x.par.for_n(n, [&](uint32_t i) { canon[i] = i; });
        x.par.sync();
      }
      x.reset(mark);
      return;
    }
    uint32_t* tab = x.template alloc_hot_hi<uint32_t>(capa);
    if (x.overflow) return;
    zero_table(x, tab, capn);
    x.par.sync();
    x.par.for_n(n, [&](uint32_t i) {
      const uint64_t k = x.weak_keys ? (key(i) & 3ull) : key(i);
      const uint32_t fp = (uint32_t)(k >> 48);
      const uint32_t mine = (fp << 16) | (i + 1);
      uint32_t slot = (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
      while (true) {
        uint32_t cur = tab[slot];
        if (cur == 0) {
          cur = P::cas32(&tab[slot], 0u, mine);
          if (cur == 0) break;
        }
        if ((cur >> 16) == fp && eq(i, (cur & 0xFFFFu) - 1u)) {
          if ((cur & 0xFFFFu) > i + 1u) P::min32(&tab[slot], mine);
          break;
        }
        if (++slot == capn) slot = 0;
      }
      canon[i] = slot;
    });
    x.par.sync();
    x.par.for_n(n, [&](uint32_t i) {
      const uint32_t c = (tab[canon[i]] & 0xFFFFu) - 1u;
      canon[i] = c;
      res(i, c);
    });
    x.par.sync();
    x.reset(mark);
    return;
  }
  uint64_t* tab = x.template alloc_hot_hi<uint64_t>(capa);
  if (x.overflow) return;
  zero_table(x, (uint32_t*)tab, 2u * capn);
  x.par.sync();
  x.par.for_n(n, [&](uint32_t i) {
    const uint64_t k = x.weak_keys ? (key(i) & 3ull) : key(i);
    const uint64_t fp = (k >> 32) | 1ull;
    const uint64_t mine = (fp << 32) | (uint64_t)(i + 1);
    uint32_t slot = (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
    while (true) {
      uint64_t cur = tab[slot];
      if (cur == 0) {
        cur = P::cas64(&tab[slot], 0, mine);
        if (cur == 0) break;
      }
      if ((cur >> 32) == fp) {
        if ((cur & 0xFFFFFFFFull) > (uint64_t)i + 1u) P::min64(&tab[slot], mine);
        break;
      }
      if (++slot == capn) slot = 0;
    }
    canon[i] = slot;
  });
  x.par.sync();
  bool collided = false;
  x.par.for_n(n, [&](uint32_t i) {
    uint32_t c = (uint32_t)(tab[canon[i]] & 0xFFFFFFFFull) - 1u;
    if (c != i && !eq(i, c)) { collided = true; c = i; }
    canon[i] = c;
    res(i, c);
  });
  if (collided) x.set_flag(DOC_NEEDS_CPU);
  x.par.sync();
  x.reset(mark);  // the table is scratch; canon[] lives in the caller's allocation
}

template <class P, class KeyF, class EqF, class CT>
TB_HD void canonicalize(DocCtx<P>& x, uint32_t n, KeyF&& key, EqF&& eq, CT* canon) {
  canonicalize_res(x, n, key, eq, canon, NoResolve{});
}

template <class P>
TB_HD bool bytes_eq(const uint8_t* b, uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
  if (a1 - a0 != b1 - b0) return false;
  const uint32_t n = a1 - a0;
  // 16 independent byte loads per side before any compare: one memory round trip per 16 bytes
  // instead of one per byte (the equal case — a verified duplicate — reads everything anyway)
  uint32_t i = 0;
  for (; i + 16 <= n; i += 16) {
    uint32_t diff = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) diff |= (uint32_t)(b[a0 + i + k] ^ b[b0 + i + k]);
    if (diff) return false;
  }
  uint32_t diff = 0;
  for (; i < n; ++i) diff |= (uint32_t)(b[a0 + i] ^ b[b0 + i]);
  return diff == 0;
}

// find_duplicates over byte spans [s[i], e[i]): (#repeats, sum of repeat byte lengths).
template <class P, class SpanF>
TB_HD void dup_spans(DocCtx<P>& x, const uint8_t* b, const PHView& ph, uint32_t n, SpanF&& span,
                     int64_t* out_elems, int64_t* out_bytes) {
  if (n <= 1) {  // one span (a single line / paragraph) repeats nothing: no table, no scans
    *out_elems = 0;
    *out_bytes = 0;
    return;
  }
  const auto mark = x.mark();
  uint32_t* canon = x.template alloc_hot<uint32_t>(n + 1);
  if (x.overflow) return;
  canonicalize(
      x, n,
      [&](uint32_t i) {
        uint32_t s, e;
        span(i, s, e);
        return dev_key(span_hash8(x, ph, s, e), e - s);
      },
      [&](uint32_t i, uint32_t j) {
        uint32_t s0, e0, s1, e1;
        span(i, s0, e0);
        span(j, s1, e1);
        return bytes_eq<P>(b, s0, e0, s1, e1);
      },
      canon);
  *out_elems = x.par.template sum<int64_t>(n, [&](uint32_t i) { return canon[i] != i ? (int64_t)1 : (int64_t)0; });
  *out_bytes = x.par.template sum<int64_t>(n, [&](uint32_t i) {
    if (canon[i] == i) return (int64_t)0;
    uint32_t s, e;
    span(i, s, e);
    return (int64_t)(e - s);
  });
  x.reset(mark);
}

// Lowercase (Rust str::to_lowercase on the word) hashed on the fly; optionally compared to `ref`.
template <class F>
TB_HD void lower_bytes(const UcdView& ucd, const Cps& cv, uint32_t s, uint32_t e, F&& push) {
  uint8_t buf[4];
  const PropArr prop = cv.props();
  for (uint32_t k = s; k < e; ++k) {
    uint32_t c = cv.cp(k);
    uint32_t lc;
    if (c == 0x3A3) {
      bool before = false, after = false;
      for (uint32_t j = k; j > s; --j) {
        uint32_t p = prop[j - 1];
        if (p & P16_CASE_IGN) continue;
        before = (p & P_CASED) != 0;
        break;
      }
      for (uint32_t j = k + 1; j < e; ++j) {
        uint32_t p = prop[j];
        if (p & P16_CASE_IGN) continue;
        after = (p & P_CASED) != 0;
        break;
      }
      lc = (before && !after) ? 0x3C2 : 0x3C3;
    } else {
      lc = ucd.lower(c);
    }
    int nb = utf8_encode(lc, buf);
    for (int q = 0; q < nb; ++q) push(buf[q]);
    if (c == 0x130) { push(0xCC); push(0x87); }
  }
}

// [s, e): the word's code points, [b0, b1): its bytes (Words::bs / be: no offset loads)
TB_HD bool is_stop_word(const UcdView& ucd, const DevStopSet& ss, const Cps& cv, uint32_t s, uint32_t e,
                        uint32_t b0, uint32_t b1) {
  // every code point lowercases to at least one byte
  if (ss.n == 0 || (int32_t)(e - s) > ss.max_len) return false;
  if (ss.lite_nslots > 0) {
    // ASCII word of <= 7 bytes (as many bytes as code points): its lowercase bytes are the key
    // of the set's fast table, which holds every ASCII entry of <= 7 bytes (devplan.h)
    const uint32_t nb = b1 - b0;
    if (nb <= 7u && nb == e - s) {
      uint64_t key = (uint64_t)nb << 56;
      for (uint32_t k = 0; k < nb; ++k) {
        uint32_t c = cv.b[b0 + k];
        if (c >= 'A' && c <= 'Z') c += 32;
        key |= (uint64_t)c << (8 * k);
      }
      const uint32_t ns = (uint32_t)ss.lite_nslots;
      uint32_t slot = stop_fast_slot(key, ns);
      while (true) {
        const uint64_t f = ss.fast_keys[slot];
        if (f == 0) return false;
        if (f == key) return true;
        slot = (slot + 1) & (ns - 1);
      }
    }
    if (ss.all_ascii7) {  // (devplan.h) no lowercase of this word is in the set without a Kelvin sign
      bool e2 = false;
      for (uint32_t k = b0; k < b1; ++k) e2 |= cv.b[k] == 0xE2;
      if (!e2) return false;
    }
  }
  uint64_t h = 0;
  uint32_t len = 0;
  lower_bytes(ucd, cv, s, e, [&](uint8_t v) { h = hash_push(h, v); ++len; });
  const uint64_t key = dev_key(h, len);
  uint32_t slot = (uint32_t)(key >> 17) & (kStopTableSize - 1);
  while (true) {
    const uint64_t k = ss.keys[slot];
    if (k == 0) return false;
    if (k == key) {
      const int32_t w = ss.idx[slot];
      const int32_t o0 = ss.off[w], o1 = ss.off[w + 1];
      if ((uint32_t)(o1 - o0) != len) return false;
      int32_t pos = o0;
      bool ok = true;
      lower_bytes(ucd, cv, s, e, [&](uint8_t v) { ok = ok && ss.blob[pos++] == v; });
      return ok;
    }
    slot = (slot + 1) & (kStopTableSize - 1);
  }
}

// ---------------------------------------------------------------------------------------------
// Case-insensitive substring test as Rust `to_lowercase().contains(pat)` for an ASCII lowercase
// pattern: ASCII letters fold, U+212A KELVIN SIGN lowercases to 'k'; no other code point
// lowercases to a sequence that can match an ASCII-letter/space pattern.
TB_HD bool ci_contains(const uint8_t* b, uint32_t n, const char* pat, int plen) {
  for (uint32_t s = 0; s < n; ++s) {
    uint32_t i = s;
    int j = 0;
    for (; j < plen; ++j) {
      if (i >= n) break;
      const char pc = pat[j];
      uint8_t c = b[i];
      if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
      if (c == (uint8_t)pc) { ++i; continue; }
      if (pc == 'k' && i + 2 < n && b[i] == 0xE2 && b[i + 1] == 0x84 && b[i + 2] == 0xAA) { i += 3; continue; }
      break;
    }
    if (j == plen) return true;
  }
  return false;
}

// SURVEY 5.7 intra-document split (documents over TB_SPLIT_DOC_BYTES): the stage workgroup
// computes everything except the duplicated n-gram orders and exports the per-word arrays those
// need (all in the document's HBM scratch slice); then one workgroup per (document, order) —
// k_gr_dup_split — canonicalises its order, marks repeats and runs its greedy walk, in parallel.
struct GrExport {
  const uint32_t* wid;   // canonical word ids
  const uint32_t* WL;    // byte prefix of word lengths
  const uint64_t* K;     // concatenation hash prefixes (see gopher_rep_record)
  const uint64_t* PB;    // B^WL
  const uint32_t* bs;    // word byte starts / ends
  const uint32_t* be;
  const uint8_t* b;      // document bytes
  char* free_base;       // unused rest of the document's scratch slice
  uint64_t free_cap;
  uint32_t W;
  uint32_t valid;        // 1: exported (0: the document returned early / was skipped)
  // duplicated lines / paragraphs (lines_valid: their arrays are in HBM and the stage left the
  // four fields to the split kernel): line break runs rs/rl [NR], paragraph breaks prs [NPR]
  // (indices into rs), trimmed code point span [tcs, tce), byte offsets, prefix hashes
  const uint32_t* rs;
  const uint32_t* rl;
  const uint32_t* prs;
  OffArr off;
  PHView ph;
  uint32_t NR, NPR, tcs, tce;
  uint32_t lines_valid;
};

// Line / paragraph spans of gopher_rep_record (byte ranges of the trimmed text between runs of
// '\n'): line k of NR + 1, paragraph q of NPR + 1.
TB_HD void gr_line_span(const uint32_t* rs, const uint32_t* rl, const OffArr& off, uint32_t tcs, uint32_t tce,
                        uint32_t NR, uint32_t k, uint32_t& s0, uint32_t& e0) {
  const uint32_t cs = k == 0 ? tcs : rs[k - 1] + rl[k - 1];
  const uint32_t ce = k == NR ? tce : rs[k];
  s0 = off[cs];
  e0 = off[ce];
}
TB_HD void gr_para_span(const uint32_t* rs, const uint32_t* rl, const uint32_t* prs, const OffArr& off,
                        uint32_t tcs, uint32_t tce, uint32_t NPR, uint32_t q, uint32_t& s0, uint32_t& e0) {
  const uint32_t cs = q == 0 ? tcs : rs[prs[q - 1]] + rl[prs[q - 1]];
  const uint32_t ce = q == NPR ? tce : rs[prs[q]];
  s0 = off[cs];
  e0 = off[ce];
}

struct StageOut {
  int64_t* rec;     // record buffer (all steps of the stage)
  uint32_t ndocs;
  uint32_t doc;
  GrExport* gr_export = nullptr;  // non-null: split mode for this document (see GrExport)
  // non-null: this document's C4 line export (LineStat region, see export_line_stats), for the C4
  // pass of the same content version
  uint32_t* line_stats = nullptr;
  const PreDoc* pre = nullptr;  // non-null: decode and word-break marks were precomputed
  // the document's bytes in HBM (split mode exports them: the stage may read an LDS copy)
  const uint8_t* b_global = nullptr;
  // dictionary-script documents: where their words come from (DictIn)
  DictIn dict;
};

// The C4 line export of one document: a header (line count, or kLineStatsNone while / when the
// stage did not export) and per Rust line its trimmed byte span, word count and longest word in
// code points. Region of document d at u32 index line_stats_base(off[d], d) of the batch buffer
// (4 * (total bytes / 8 + 16 * documents) + 16 u32): room for line_stats_cap(n) lines.
constexpr uint32_t kLineStatsNone = 0xFFFFFFFFu;
struct alignas(16) LineStat { uint32_t bs, be, nw, mx; };
TB_HD uint64_t line_stats_base(int64_t off_d, int64_t d) { return 4ull * ((uint64_t)off_d / 8u + 16ull * (uint64_t)d); }
TB_HD uint32_t line_stats_cap(uint32_t n) { return n / 8u + 15u; }
TB_HD uint64_t line_stats_words(const int64_t* off, int64_t ndocs) {  // buffer size in u32
  return line_stats_base(off[ndocs], ndocs) + 16u;
}

// C4 line export from the stage's words and lines (StageOut::line_stats): per Rust line its span
// trimmed of whitespace (in bytes), its word count and its longest word in code points. Words are
// assigned to the last line starting at or before their first code point (words never cross a
// line feed), word-parallel with LDS atomics on per-line counters. The header is written last;
// documents with more lines than the region holds, or whose counters do not fit the scratch,
// keep kLineStatsNone (the export never changes the stage's own results).
template <class P>
TB_HD void export_line_stats(DocCtx<P>& x, const Cps& c, const Words& w, const Lines& L, uint32_t n, uint32_t* out) {
  const uint32_t NL = L.n;
  if (NL > line_stats_cap(n) || x.overflow) return;
  const auto mark = x.mark();
  uint32_t* ls = x.template alloc_hot<uint32_t>(NL + 1);
  uint32_t* nw = x.template alloc_hot<uint32_t>(NL + 1);
  uint32_t* mx = x.template alloc_hot<uint32_t>(NL + 1);
  if (x.overflow) {
    x.overflow = false;
    x.reset(mark);
    return;
  }
  const PropArr prop = c.props();
  const OffArr off = c.offs();
  x.par.for_n(NL, [&](uint32_t k) { ls[k] = L.ls[k]; nw[k] = 0; mx[k] = 0; });
  x.par.sync();
  x.par.for_n(w.n, [&](uint32_t q) {
    const uint32_t cs = w.cs[q];
    uint32_t lo = 0, hi = NL;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ls[mid] <= cs) lo = mid; else hi = mid;
    }
    P::add32(&nw[lo], 1u);
    P::max32(&mx[lo], w.ce[q] - cs);
  });
  x.par.sync();
  LineStat* st = (LineStat*)(out + 4);
  x.par.for_n(NL, [&](uint32_t k) {
    uint32_t s0 = ls[k], e0 = L.le[k];
    while (s0 < e0 && is_ws(prop[s0])) ++s0;
    while (e0 > s0 && is_ws(prop[e0 - 1])) --e0;
    st[k] = LineStat{off[s0], off[e0], nw[k], mx[k]};
  });
  x.par.sync();
  x.par.single([&]() { out[0] = NL; });
  x.reset(mark);
}

// The duplicated n-gram key / equality of order n over the exported word arrays (one definition
// for the in-stage path and the split kernel): grams are equal iff their concatenations are.
struct DupGrams {
  const uint32_t* wid;
  const uint32_t* WL;
  const uint64_t* K;
  const uint64_t* PB;
  const uint32_t* bs;
  const uint32_t* be;
  const uint8_t* b;
  TB_HD uint64_t run_hash(uint32_t p, uint32_t n) const {
    return PB[p + n] * (K[p + n] - K[p]);
  }
  TB_HD uint64_t key(uint32_t p, uint32_t n) const { return dev_key(run_hash(p, n), WL[p + n] - WL[p]); }
  TB_HD bool eq(uint32_t p, uint32_t q, uint32_t n) const {
    if (WL[p + n] - WL[p] != WL[q + n] - WL[q]) return false;
    // same canonical word sequence => same concatenation (the common case); only different word
    // splits of equal-hash text need the byte comparison. All n id pairs are loaded before the
    // compare (no early exit), so the loads overlap instead of forming a dependent chain.
    uint32_t dw = 0;
#pragma unroll 5
    for (uint32_t k = 0; k < n; ++k) dw |= wid[p + k] ^ wid[q + k];
    if (dw == 0) return true;
    uint32_t wp = p, wq = q, bp = bs[p], bq = bs[q];
    const uint32_t L = WL[p + n] - WL[p];
    for (uint32_t i = 0; i < L; ++i) {
      while (bp == be[wp]) { ++wp; bp = bs[wp]; }
      while (bq == be[wq]) { ++wq; bq = bs[wq]; }
      if (b[bp] != b[bq]) return false;
      ++bp;
      ++bq;
    }
    return true;
  }
};

// Greedy duplicated-n-gram walk of one order (reference find_all_duplicate, utils/text.rs:
// 241-259) over canonical gram ids gc[0, G), repeat bitmap R (bit p: gram p occurs more than
// once) and the seen-bitmap sn (zeroed): bytes of the repeated grams the walk counts. A walk only
// stops at repeated grams; at a gram that occurs once it would mark an id nobody else has and
// advance by one, so it jumps from one set bit of R to the next.
template <class GcT>
TB_HD int64_t dup_walk(uint32_t G, uint32_t n, const GcT* gc, const uint32_t* R, uint32_t* sn,
                       const uint32_t* WL) {
  const uint32_t nw = (G + 31) >> 5;
  auto next_rep = [&](uint32_t from) -> uint32_t {  // first repeated position >= from, or G
    if (from >= G) return G;
    uint32_t wi = from >> 5;
    uint32_t bw = R[wi] & (~0u << (from & 31));
    while (!bw) {
      if (++wi >= nw) return G;
      bw = R[wi];
    }
    const uint32_t q = (wi << 5) + (uint32_t)__builtin_ctz(bw);
    return q < G ? q : G;
  };
  int64_t rep = 0;
  uint32_t idx = next_rep(0);
  while (idx < G) {
    const uint32_t g = gc[idx];
    if ((sn[g >> 5] >> (g & 31)) & 1u) {
      rep += (int64_t)(WL[idx + n] - WL[idx]);
      idx = next_rep(idx + n);
    } else {
      sn[g >> 5] |= 1u << (g & 31);
      idx = next_rep(idx + 1);
    }
  }
  return rep;
}

// dup_walk by one whole wave (every lane calls it with the same arguments; the result is
// uniform). The chain of the scalar walk pays a memory round trip per step (gc[idx], seen bit);
// here the wave takes a window of 64 positions starting at the next repeated one, its lanes load
// the window's canonical ids, seen bits and gram lengths together (one round trip per window),
// and the walk steps through the window's repeated positions in scalar registers: a first visit
// marks every lane holding the same id seen (one ballot), a repeat drops the lanes it jumps over.
// The window's first visits then set their seen bits and the counted lanes' lengths are summed.
// Same visits, same result as dup_walk.
template <class P, class GcT>
TB_HD int64_t dup_walk_wave(const P& par, uint32_t G, uint32_t n, const GcT* gc, const uint32_t* R,
                            uint32_t* sn, const uint32_t* WL) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lane = par.lane;
  const uint32_t nw = (G + 31) >> 5;
  int64_t rep = 0;
  uint32_t idx = 0;
  while (idx < G) {
    uint32_t p0 = G;  // next repeated position >= idx: 64 bitmap words per ballot
    for (uint32_t base = idx >> 5; base < nw; base += 64) {
      const uint32_t w = base + lane;
      uint32_t bw = w < nw ? R[w] : 0u;
      if (w == (idx >> 5)) bw &= ~0u << (idx & 31);
      const uint64_t m = __ballot(bw != 0u);
      if (m) {
        const int l = __builtin_ctzll(m);
        p0 = ((base + (uint32_t)l) << 5) + (uint32_t)__builtin_ctz((uint32_t)__builtin_amdgcn_readlane((int)bw, l));
        break;
      }
    }
    if (p0 >= G) break;
    const uint32_t p = p0 + lane;
    const bool act = p < G && ((R[p >> 5] >> (p & 31)) & 1u);
    uint32_t g = 0xFFFFFFFFu, len = 0;
    if (act) {
      g = gc[p];
      len = WL[p + n] - WL[p];
    }
    const bool seen0 =
        act && ((__hip_atomic_load(&sn[g >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (g & 31)) & 1u);
    uint64_t A = __ballot(act), S = __ballot(seen0), cnt = 0, fv = 0;
    uint32_t next = p0 + 64;
    while (A) {
      const uint32_t k = (uint32_t)__builtin_ctzll(A);
      if ((S >> k) & 1ull) {
        cnt |= 1ull << k;
        const uint32_t j = k + n;
        A = j >= 64 ? 0ull : (A & (~0ull << j));
        if (p0 + j > next) next = p0 + j;
      } else {
        fv |= 1ull << k;
        S |= __ballot(g == (uint32_t)__builtin_amdgcn_readlane((int)g, (int)k));
        A &= A - 1;
      }
    }
    if ((fv >> lane) & 1ull) atomicOr(&sn[g >> 5], 1u << (g & 31));
    uint32_t add = ((cnt >> lane) & 1ull) ? len : 0u;
    for (int o = 32; o > 0; o >>= 1) add += (uint32_t)__shfl_xor((int)add, o);
    rep += add;
    // the next window's seen loads (other lanes) must observe these bits
    // (same wave, same CU: a workgroup-scope fence waits for the atomics; the seen loads read L2)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    idx = next;
  }
  return rep;
#else
  (void)par;
  return dup_walk(G, n, gc, R, sn, WL);
#endif
}

TB_HD uint64_t span_hash(uint64_t pa, uint64_t pb, uint64_t blen_pow) {
  return pb - pa * blen_pow;
}

// Sentence count of split_into_sentences() over code points [s, e) (already trimmed text),
// saturated: sentences are counted chunk by chunk and counting stops after the chunk
// that reaches `limit`, so the result is exact below `limit` and >= limit otherwise (C4's
// min_num_sentences test and its reason string only use counts below the limit). A chunk's
// breaks are compacted, every segment with a non-whitespace code point counts once; the part
// before the chunk's first break continues the previous chunk's last segment (`seen`: that
// segment already counted).
template <class P>
TB_HD uint32_t count_sentences_upto(DocCtx<P>& x, const Cps& c, uint32_t s, uint32_t e, uint32_t limit) {
  const uint32_t m = e - s;
  if (m == 0 || limit == 0) return 0;
  constexpr uint32_t kChunk = 256;
  const auto mark = x.mark();
  uint32_t* starts = x.template alloc_hot<uint32_t>(kChunk + 1);
  uint32_t* segf = x.template alloc_hot<uint32_t>(kChunk + 1);
  if (x.overflow) return 0;
  const PropArr prop = c.props() + s;
  CpsAcc acc{prop};
  uint32_t cnt = 0;
  bool seen = false;
  for (uint32_t base = 0; base < m && cnt < limit; base += kChunk) {
    const uint32_t len = m - base < kChunk ? m - base : kChunk;
    const uint32_t NS = x.par.template compact<int>(
        len, [&](uint32_t i, int&) { const uint32_t g = base + i; return g == 0 || sb_break(acc, (int)m, (int)g); },
        [&](uint32_t i, uint32_t k, int&) { starts[k] = i; });
    x.par.sync();
    const uint32_t first = NS ? starts[0] : len;
    const bool lead_any = x.par.template sum<uint32_t>(first, [&](uint32_t i) {
      return is_ws(prop[base + i]) ? 0u : 1u;
    }) != 0;
    const uint32_t segs = x.par.template sum<uint32_t>(NS, [&](uint32_t k) {
      const uint32_t a = starts[k], bnd = k + 1 < NS ? starts[k + 1] : len;
      uint32_t f = 0;
      for (uint32_t j = a; j < bnd; ++j) if (!is_ws(prop[base + j])) { f = 1; break; }
      segf[k] = f;
      return f;
    });
    x.par.sync();
    if (!seen && lead_any) ++cnt;
    cnt += segs;
    seen = NS ? segf[NS - 1] != 0 : (seen || lead_any);
    x.par.sync();
  }
  x.reset(mark);
  return cnt;
}

template <class P>
TB_HD void gopher_rep_record(DocCtx<P>& x, const DevStep& ds, const uint8_t* b, const Cps& c,
                             const PHView& ph, const Words& w, int64_t* r, bool release_props = false,
                             GrExport* ex = nullptr, const PreDoc* pre = nullptr,
                             const uint8_t* b_export = nullptr, Lines lines = Lines{}) {
  const uint32_t C = c.n;
  const PropArr prop = c.props();
  const OffArr off = c.offs();
  const int width = ds.width;
  uint32_t tcs, tce;
  trim_span(x, prop, C, tcs, tce);
  if (tcs >= tce) {
    x.par.single([&]() {
      for (int k = 0; k < width; ++k) r[k] = 0;
      r[0] = -1;
    });
    return;
  }
  const auto mark = x.mark();
  const uint32_t span = tce - tcs;
  uint32_t* rs;
  uint32_t* rl;
  uint32_t NR;
  if (pre) {
    // the pre-pass listed every run of '\n' (position, length): the runs inside [tcs, tce) are
    // a contiguous part of that list (a run starts after a non-'\n' code point, so none at tcs)
    const uint32_t a = pre->nl_a, e = pre->nl_e;  // (k_pre_wb: the runs inside [tcs, tce))
    rs = pre->nl_pos + a;
    rl = pre->nl_len + a;
    NR = e - a;
  } else if (lines.n > 0) {
    // From the stage's Rust lines (`lines`: their starts, ls[k] = one past a '\n' for k >= 1):
    // the line feeds are exactly the code points ls[k] - 1, and a run continues while the next
    // line is empty (ls[k + 1] == ls[k] + 1). The runs inside the trimmed span [tcs, tce) are
    // whole (its ends are not whitespace), and the '\n' a text may end with is outside it. One
    // compaction over the lines instead of one over the code points.
    const uint32_t* ls = lines.ls;
    const uint32_t NL = lines.n;
    // (workgroup documents: HBM, so that split mode can hand them to k_gr_dup_split)
    rs = P::kWaves == 1 ? x.template alloc_hot<uint32_t>(NL + 1) : x.template alloc<uint32_t>(NL + 1);
    rl = P::kWaves == 1 ? x.template alloc_hot<uint32_t>(NL + 1) : x.template alloc<uint32_t>(NL + 1);
    if (x.overflow) return;
    NR = x.par.template compact<int>(
        NL,
        [&](uint32_t k, int&) {
          if (k == 0) return false;
          const uint32_t p = ls[k] - 1;
          return p >= tcs && p < tce && (k == 1 || ls[k - 1] != p);
        },
        [&](uint32_t k, uint32_t q, int&) {
          uint32_t e = k;
          while (e + 1 < NL && ls[e + 1] == ls[e] + 1) ++e;
          rs[q] = ls[k] - 1;
          rl[q] = e - k + 1;
        });
    x.par.sync();
  } else {
    rs = x.template alloc<uint32_t>(span + 1);
    rl = x.template alloc<uint32_t>(span + 1);
    if (x.overflow) return;
    NR = x.par.template compact<int>(
        span,
        [&](uint32_t i, int&) {
          const uint32_t j = tcs + i;
          return c.is_lf(j) && !c.is_lf(j - 1);
        },
        [&](uint32_t i, uint32_t k, int&) {
          uint32_t j = tcs + i, q = j;
          while (c.is_lf(q)) ++q;
          rs[k] = j;
          rl[k] = q - j;
        });
    x.par.sync();
  }
  x.stamp(PH_GR_NL);
  uint32_t* prs = x.template alloc<uint32_t>(NR + 1);
  if (x.overflow) return;
  int64_t line_dup = 0, line_dup_b = 0, para_dup = 0, para_dup_b = 0;
  // split mode: the duplicated line / paragraph statistics go to k_gr_dup_split when everything
  // they read is in HBM (it outlives this kernel)
#ifdef TB_NO_SPLIT_LINES
  const bool split_lines = false;
#else
  // (wave documents never: their split kernels run only the n-gram orders)
  const bool split_lines = ex && P::kWaves != 1 && !x.in_lds(rs) && !x.in_lds(rl) && !x.in_lds(prs) &&
                           !x.in_lds(ph.ph8) && !x.in_lds(c.ent) && !x.in_lds(c.off);
#endif
  if (!split_lines)
    dup_spans(x, b, ph, NR + 1,
              [&](uint32_t k, uint32_t& s0, uint32_t& e0) { gr_line_span(rs, rl, off, tcs, tce, NR, k, s0, e0); },
              &line_dup, &line_dup_b);
  x.stamp(PH_GR_LINE_DUP);
  const uint32_t NPR = x.par.template compact<int>(
      NR, [&](uint32_t k, int&) { return rl[k] >= 2; }, [&](uint32_t k, uint32_t q, int&) { prs[q] = k; });
  x.par.sync();
  if (!split_lines)
    dup_spans(x, b, ph, NPR + 1,
              [&](uint32_t q, uint32_t& s0, uint32_t& e0) {
                gr_para_span(rs, rl, prs, off, tcs, tce, NPR, q, s0, e0);
              },
              &para_dup, &para_dup_b);
  if (ex) {
    x.par.single([&]() {
      ex->rs = rs; ex->rl = rl; ex->prs = prs; ex->off = off; ex->ph = ph;
      ex->NR = NR; ex->NPR = NPR; ex->tcs = tcs; ex->tce = tce;
      ex->lines_valid = split_lines ? 1u : 0u;
    });
  }
  x.stamp(PH_GR_LINES);
  x.par.single([&]() {
    r[0] = span;
    r[1] = NPR + 1;
    r[2] = para_dup;
    r[3] = para_dup_b;
    r[4] = NR + 1;
    r[5] = line_dup;
    r[6] = line_dup_b;
  });
  // ---- n-gram statistics over the words ----
  // Word-level arrays (LDS while they fit): wid = canonical word id (smallest index of an equal
  // word), WL = byte prefix of word lengths, and for concatenation hashes of any word run
  //   K[k] = sum_{j<k} H(word j) * B^-WL[j+1],  PB[k] = B^WL[k]
  //   H(words p .. p+n-1 concatenated) = PB[p+n] * (K[p+n] - K[p])
  // (the Horner hash of the concatenation), so a run costs one multiplication and no power
  // lookup; the powers are read once per word instead of once per (n, position). They are built
  // while the prefix hashes are still on chip; then the code point arrays and prefix hashes (top
  // of the LDS slice) are released, so the n-gram tables get that space.
  const uint32_t W = w.n;
  const bool ngrams = ds.n_top + ds.n_dup > 0;
  if constexpr (P::kWaves == 1) {
    if (ngrams && W >= kWave16) {
      x.set_flag(DOC_NEEDS_CPU);
      return;
    }
  }
  uint32_t* wid = nullptr;
  uint32_t* WL = nullptr;
  uint64_t* K = nullptr;
  uint64_t* PB = nullptr;
  if (ngrams && pre && pre->wready) {
    // built by many workgroups before this one (k_pre_wcanon); a hash collision between unequal
    // words has flagged the document for the CPU path there
    wid = pre->wid;
    WL = pre->wl;
    K = pre->wk;
    PB = pre->wpb;
  } else if (ngrams) {
    // LDS only while a canonicalisation table for W elements (~6 W bytes) still fits next to them
    // (split mode: HBM, they outlive this kernel)
    const uint64_t tab_bytes = 6ull * W + 64;
    wid = ex ? x.template alloc<uint32_t>(W + 1) : x.template alloc_hot_keep<uint32_t>(W + 1, tab_bytes);
    WL = ex ? x.template alloc<uint32_t>(W + 1) : x.template alloc_hot_keep<uint32_t>(W + 1, tab_bytes);
    K = ex ? x.template alloc<uint64_t>(W + 1) : x.template alloc_hot_keep<uint64_t>(W + 1, tab_bytes);
    PB = ex ? x.template alloc<uint64_t>(W + 1) : x.template alloc_hot_keep<uint64_t>(W + 1, tab_bytes);
    // One-wave documents export these arrays and read neither the code point arrays nor the prefix
    // hashes (the top of the LDS slice) after the word hashes: the slice's top is released right
    // there, so the word canonicalisation table lands in the LDS (it was in HBM for most ~1 KB
    // documents) and the hashes go to the bottom.
    const bool early = P::kWaves == 1 && release_props && ex != nullptr;
    const auto mw = x.mark();
    uint64_t* wh = early ? x.template alloc_hot<uint64_t>(W + 1) : x.template alloc_hot_hi<uint64_t>(W + 1);
    if (x.overflow) return;
    x.par.for_n(W, [&](uint32_t k) { wh[k] = span_hash8(x, ph, w.bs[k], w.be[k]); });
    x.par.sync();
    if (early) x.release_hi();
    x.stamp(PH_GR_WH);
    canonicalize(
        x, W, [&](uint32_t k) { return dev_key(wh[k], w.be[k] - w.bs[k]); },
        [&](uint32_t i, uint32_t j) { return bytes_eq<P>(b, w.bs[i], w.be[i], w.bs[j], w.be[j]); }, wid);
    x.stamp(PH_GR_WCANON);
    const uint32_t totl = x.par.template scan<uint32_t>(
        W, 0u, [](uint32_t a, uint32_t c2) { return a + c2; },
        [&](uint32_t k) { return w.be[k] - w.bs[k]; }, [&](uint32_t k, uint32_t e) { WL[k] = e; });
    x.par.single([&]() { WL[W] = totl; });
    x.par.sync();
    x.par.for_n(W + 1, [&](uint32_t k) { PB[k] = x.powb(WL[k]); });
    const uint64_t ktot = x.par.template scan<uint64_t>(
        W, 0ull, [](uint64_t a, uint64_t c2) { return a + c2; },
        [&](uint32_t j) { return wh[j] * x.ipowb(WL[j + 1]); }, [&](uint32_t k, uint64_t e) { K[k] = e; });
    x.par.single([&]() { K[W] = ktot; });
    x.par.sync();
    x.reset(mw);  // wh
    if (x.overflow) return;
  }
  x.stamp(PH_GR_WORDS);
  // the n-gram statistics read words, bytes and the arrays above only: the top of the LDS slice
  // (code point arrays, prefix hashes) goes to their hash tables
  if (release_props) x.release_hi();
  if (ngrams) {
    const DupGrams dg{wid, WL, K, PB, w.bs, w.be, b};
    // Top n-grams (space-joined grams: equal iff their word sequences are equal). Canonical ids
    // of the n-grams are built incrementally: the n-gram at p is the pair (id of the (n-1)-gram
    // at p, id of word p+n-1), so each order is one exact pair canonicalisation (O(1) equality,
    // no hashing of the gram text).
    if (ds.n_top > 0 && ex) {
      // split mode: k_gr_dup_split computes each top order in its own workgroup
      x.par.single([&]() { for (int t = 0; t < ds.n_top; ++t) r[rec_gr_fixed() + t] = 0; });
    } else if (ds.n_top > 0) {
      int max_top = 0;
      for (int t = 0; t < ds.n_top; ++t) max_top = ds.top_n[t] > max_top ? ds.top_n[t] : max_top;
      const auto m2 = x.mark();
      // two id arrays in turn; the counts of order n go to the one the (n-1)-gram ids used
      uint32_t* ga = x.template alloc_hot_keep<uint32_t>(W + 1, 6ull * W + 64);
      uint32_t* gb = x.template alloc_hot_keep<uint32_t>(W + 1, 6ull * W + 64);
      if (x.overflow) return;
      x.par.single([&]() { for (int t = 0; t < ds.n_top; ++t) r[rec_gr_fixed() + t] = 0; });
      const uint32_t* gprev = wid;
      for (uint32_t n = 1; n <= (uint32_t)max_top && W >= n; ++n) {
        const uint32_t G = W - n + 1;
        const uint32_t* gc = wid;
        uint32_t* cnt = (n == 1 || !(n & 1)) ? ga : gb;
        if (n > 1) {
          uint32_t* gcur = (n & 1) ? ga : gb;
          canonicalize(
              x, G, [&](uint32_t p) { return mix64(((uint64_t)gprev[p] << 32) ^ (uint64_t)wid[p + n - 1] ^ ((uint64_t)n << 60)); },
              [&](uint32_t p, uint32_t q) { return gprev[p] == gprev[q] && wid[p + n - 1] == wid[q + n - 1]; }, gcur);
          gc = gcur;
          gprev = gcur;
          x.stamp(PH_GR_TOP_CANON);
        }
        bool wanted = false;
        for (int t = 0; t < ds.n_top; ++t) wanted |= ds.top_n[t] == (int32_t)n;
        if (!wanted) continue;
        x.par.for_n(G, [&](uint32_t p) { cnt[p] = 0; });
        x.par.sync();
        x.par.for_n(G, [&](uint32_t p) { P::add32(&cnt[gc[p]], 1u); });
        x.par.sync();
        const uint32_t maxc = x.par.template max<uint32_t>(G, 0u, [&](uint32_t p) { return cnt[p]; });
        int64_t v = 0;
        if (maxc > 1) {
          const uint32_t maxlen = x.par.template max<uint32_t>(G, 0u, [&](uint32_t p) {
            return cnt[p] == maxc ? (WL[p + n] - WL[p] + n - 1) : 0u;
          });
          v = (int64_t)maxlen * (int64_t)maxc;
        }
        x.par.single([&]() {
          for (int t = 0; t < ds.n_top; ++t) if (ds.top_n[t] == (int32_t)n) r[rec_gr_fixed() + t] = v;
        });
        x.par.sync();
      }
      x.reset(m2);
    }
    x.stamp(PH_GR_TOP);
    if (ex) {
      // split mode: export the word arrays; k_gr_dup_split finishes every order (top and
      // duplicated) in its own workgroup and writes the n-gram fields
      const uint64_t base = (x.used + 255) & ~255ull;
      x.par.single([&]() {
        for (int t = 0; t < ds.n_dup; ++t) r[rec_gr_fixed() + ds.n_top + t] = 0;
        ex->wid = wid; ex->WL = WL; ex->K = K; ex->PB = PB; ex->bs = w.bs; ex->be = w.be;
        ex->b = b_export ? b_export : b;
        ex->free_base = x.scr + base;
        ex->free_cap = x.cap > base ? x.cap - base : 0;
        ex->W = W;
        ex->valid = x.overflow ? 0u : 1u;
      });
      x.par.sync();
    } else if (ds.n_dup > 0) {
      // Two phases over all requested orders n (reference find_all_duplicate,
      // utils/text.rs:241-259):
      //   1. per n: canonicalise the n-gram concatenations into gc_n (exact: hash groups, then
      //      word-id / byte equality) and mark repeated positions in R_n (p with gc[p] != p, and
      //      their first occurrence gc[p]);
      //   2. the greedy walks of all orders run at once, one lane each (they are independent
      //      and sequential, so n walks cost about the longest one instead of their sum).
      // Arrays of all orders are packed back to back: gc_n at gbase(t), bitmaps at t * 2 * SW.
      const uint32_t SW = (W + 31) / 32 + 1;
      const int nd = ds.n_dup;
      auto gsize = [&](int t) -> uint32_t {
        const uint32_t n = (uint32_t)ds.dup_n[t];
        return (n == 0 || W < n) ? 0u : W - n + 1;
      };
      uint32_t gtot = 0;
      for (int t = 0; t < nd; ++t) gtot += gsize(t);
      const auto m3 = x.mark();
      uint32_t* bits = x.template alloc_hot<uint32_t>(2 * (uint64_t)SW * (uint64_t)nd);  // [sn | R] per order
      // wave documents keep the canonical ids in 16 bits (half the slice; W < kWave16)
      using GcT = std::conditional_t<P::kWaves == 1, uint16_t, uint32_t>;
      GcT* gcall = x.template alloc_hot_keep<GcT>((uint64_t)gtot + 1, 6ull * W + 64);
      if (x.overflow) return;
      x.par.for_n(2 * SW * (uint32_t)nd, [&](uint32_t i) { bits[i] = 0; });
      x.par.sync();
      uint32_t gb = 0;
      for (int t = 0; t < nd; ++t) {
        const uint32_t n = (uint32_t)ds.dup_n[t];
        const uint32_t G = gsize(t);
        if (G == 0) continue;
        GcT* gc = gcall + gb;
        uint32_t* R = bits + (uint32_t)t * 2 * SW + SW;
        gb += G;
        auto mark_rep = [&](uint32_t p, uint32_t g) {
          if (g != p) {  // repeated: the position and its first occurrence
            P::or32(&R[p >> 5], 1u << (p & 31));
            P::or32(&R[g >> 5], 1u << (g & 31));
          }
        };
        if constexpr (P::kWaves != 1) {
          // fused into the canonicalisation's last pass
          canonicalize_res(
              x, G, [&](uint32_t p) { return dg.key(p, n); }, [&](uint32_t p, uint32_t q) { return dg.eq(p, q, n); },
              gc, mark_rep);
          x.stamp(PH_GR_DUP_CANON);
        } else {
          // own pass in the one-wave kernel (the fused form costs it registers)
          canonicalize(
              x, G, [&](uint32_t p) { return dg.key(p, n); }, [&](uint32_t p, uint32_t q) { return dg.eq(p, q, n); },
              gc);
          x.stamp(PH_GR_DUP_CANON);
          x.par.for_n(G, [&](uint32_t p) { mark_rep(p, gc[p]); });
          x.par.sync();
        }
      }
      auto walk = [&](uint32_t t, bool wave) -> int64_t {
        const uint32_t G = gsize((int)t);
        if (G == 0) return 0;
        uint32_t base = 0;
        for (uint32_t u = 0; u < t; ++u) base += gsize((int)u);
        uint32_t* sn = bits + t * 2 * SW;
        const uint32_t n = (uint32_t)ds.dup_n[t];
        return wave ? dup_walk_wave(x.par, G, n, gcall + base, sn + SW, sn, WL)
                    : dup_walk(G, n, gcall + base, sn + SW, sn, WL);
      };
      if constexpr (P::kWaves > 1) {
        // one wave per order (whole-wave walks)
        for (uint32_t t = x.par.wave_index(); t < (uint32_t)nd; t += P::kWaves) {
          const int64_t rep = walk(t, true);
          if (x.par.lane == 0) r[rec_gr_fixed() + ds.n_top + t] = rep;
        }
      } else {
        // one lane per order: the orders' walks overlap (the whole-wave walk would run them
        // one after another)
        x.par.for_n((uint32_t)nd, [&](uint32_t t) { r[rec_gr_fixed() + ds.n_top + t] = walk(t, false); });
      }
      x.par.sync();
      x.stamp(PH_GR_DUP_WALK);
      x.reset(m3);
      x.stamp(PH_GR_DUP);
    }
  }
  x.reset(mark);
}

// Repeat candidates of n elements: a superset of the elements equal to some other element. Every
// element sets bit h(key) of a bitmap (fetch-or); one that finds its bit already set sets it in a
// second bitmap. Equal elements have equal keys, so every repeated element lands on a bit of the
// second bitmap; an element whose bit no other element set is unique, and only the candidates need
// the exact canonicalisation (with 8 bitmap bits per element a unique one is a false candidate
// with probability ~1/8). Candidate indices go to list[0, nc) in increasing order; returns nc.
// `bm` holds 2 * bw words (bw a power of two), zeroed here.
template <class P, class KeyF>
TB_HD uint32_t repeat_candidates(DocCtx<P>& x, uint32_t n, KeyF&& key, uint32_t* bm, uint32_t bw, uint32_t* list) {
  const uint32_t mask = bw * 32u - 1u;
  uint32_t* once = bm;
  uint32_t* twice = bm + bw;
  x.par.for_n(2 * bw, [&](uint32_t i) { bm[i] = 0; });
  x.par.sync();
  x.par.for_n(n, [&](uint32_t i) {
    const uint32_t h = (uint32_t)(key(i) >> 20) & mask;
    const uint32_t bit = 1u << (h & 31u);
    if (P::fetch_or32(&once[h >> 5], bit) & bit) P::or32(&twice[h >> 5], bit);
  });
  x.par.sync();
  const uint32_t nc = x.par.template compact<int>(
      n,
      [&](uint32_t i, int&) {
        const uint32_t h = (uint32_t)(key(i) >> 20) & mask;
        return ((twice[h >> 5] >> (h & 31u)) & 1u) != 0;
      },
      [&](uint32_t i, uint32_t k, int&) { list[k] = i; });
  x.par.sync();
  return nc;
}

// Bitmap words of repeat_candidates for n elements (>= 8 bits per element, a power of two) and the
// scratch bytes the candidate path may take beyond the order's own arrays, for the capacity test
// that picks it (the full canonicalisation otherwise: results are the same either way).
TB_HD uint32_t cand_bitmap_words(uint32_t n) {
  uint32_t w = 32;
  while (w * 4u < n) w <<= 1;
  return w;
}
TB_HD uint64_t cand_path_bytes(uint32_t n) { return 8ull * cand_bitmap_words(n) + 16ull * n + 256; }
// (workgroup documents keep the full canonicalisation: with the candidate path their
// partitioned-table runs gave wrong top n-gram records on the GPU, unexplained; the sequential
// emulation of the same code, partitioned tables included, is exact)
#ifndef TB_CAND_BLK
#define TB_CAND_BLK 0
#endif
template <class P>
TB_HD bool cand_path_fits(const DocCtx<P>& x, uint32_t n) {
  if (!TB_CAND_BLK && P::kWaves > 1) return false;
  const uint64_t need = cand_path_bytes(n);
  return x.cap >= x.used + need + 64 || (uint64_t)x.lds_free() >= need;
}

// Duplicated lines (which = 0: r[5], r[6]) or paragraphs (which = 1: r[2], r[3]) of a split
// document (k_gr_dup_split), over the arrays gopher_rep_record exported.
template <class P>
TB_HD void gr_lines_split(DocCtx<P>& x, int which, const GrExport& e, int64_t* r) {
  if (!e.lines_valid) return;  // computed in the stage
  int64_t elems = 0, bytes = 0;
  if (which == 0)
    dup_spans(x, e.b, e.ph, e.NR + 1,
              [&](uint32_t k, uint32_t& s0, uint32_t& e0) { gr_line_span(e.rs, e.rl, e.off, e.tcs, e.tce, e.NR, k, s0, e0); },
              &elems, &bytes);
  else
    dup_spans(x, e.b, e.ph, e.NPR + 1,
              [&](uint32_t q, uint32_t& s0, uint32_t& e0) {
                gr_para_span(e.rs, e.rl, e.prs, e.off, e.tcs, e.tce, e.NPR, q, s0, e0);
              },
              &elems, &bytes);
  if (x.overflow) return;
  x.par.single([&]() {
    r[which == 0 ? 5 : 2] = elems;
    r[which == 0 ? 6 : 3] = bytes;
  });
  x.par.sync();
}

// One top n-gram order of a split document (k_gr_dup_split): the n-grams of order n are grouped
// by their word-id tuples directly (equal space-joined grams <=> equal word sequences), so the
// orders are independent of each other (the in-stage path chains order n on order n - 1 instead).
// Writes r[7 + t], the same value as the in-stage path.
template <class P>
TB_HD void gr_top_one_order(DocCtx<P>& x, const DevStep& ds, int t, const GrExport& e, int64_t* r) {
  const uint32_t W = e.W, n = (uint32_t)ds.top_n[t];
  int64_t* out = r + rec_gr_fixed() + t;
  if (n == 0 || W < n) {
    x.par.single([&]() { *out = 0; });
    return;
  }
  const uint32_t G = W - n + 1;
  const uint32_t* wid = e.wid;
  const uint32_t* WL = e.WL;
  const auto mark = x.mark();
  auto key = [&](uint32_t p) {
    uint64_t h = (uint64_t)n << 56;
    for (uint32_t k = 0; k < n; ++k) h = (h ^ wid[p + k]) * 0x9E3779B97F4A7C15ull + k;
    return mix64(h);
  };
  auto eq = [&](uint32_t p, uint32_t q) {
    uint32_t dw = 0;
    for (uint32_t k = 0; k < n; ++k) dw |= wid[p + k] ^ wid[q + k];
    return dw == 0;
  };
  // Only the repeat candidates are grouped (every other gram occurs once): pos[c] = position of
  // candidate c, gc[c] = its canonical candidate, cnt[c] = the class size at the canonical one.
  // Without room for the candidate arrays every position is a candidate (the full grouping).
  uint32_t NC = G;
  const uint32_t* pos = nullptr;
  if (cand_path_fits(x, G)) {
    const uint32_t bw = cand_bitmap_words(G);
#ifdef TB_CAND_GLOBAL
    uint32_t* bm = x.template alloc_global<uint32_t>(2 * bw);
    uint32_t* list = x.template alloc_global<uint32_t>((uint64_t)G + 1);
#else
    uint32_t* bm = x.template alloc_hot<uint32_t>(2 * bw);
    uint32_t* list = x.template alloc_hot<uint32_t>((uint64_t)G + 1);
#endif
    if (x.overflow) return;
    NC = repeat_candidates(x, G, key, bm, bw, list);
    pos = list;
  }
  int64_t v = 0;
  if (NC >= 2) {
    uint32_t* gc = x.template alloc_hot_keep<uint32_t>((uint64_t)NC + 1, 6ull * NC + 64);
    uint32_t* cnt = x.template alloc_hot_keep<uint32_t>((uint64_t)NC + 1, 6ull * NC + 64);
    if (x.overflow) return;
    auto at = [&](uint32_t c) { return pos ? pos[c] : c; };
    canonicalize(
        x, NC, [&](uint32_t c) { return key(at(c)); }, [&](uint32_t c, uint32_t d) { return eq(at(c), at(d)); },
        gc);
    if (x.overflow) return;
    x.par.for_n(NC, [&](uint32_t c) { cnt[c] = 0; });
    x.par.sync();
    x.par.for_n(NC, [&](uint32_t c) { P::add32(&cnt[gc[c]], 1u); });
    x.par.sync();
    const uint32_t maxc = x.par.template max<uint32_t>(NC, 0u, [&](uint32_t c) { return cnt[c]; });
    if (maxc > 1) {
      const uint32_t maxlen = x.par.template max<uint32_t>(NC, 0u, [&](uint32_t c) {
        const uint32_t p = at(c);
        return cnt[c] == maxc ? (WL[p + n] - WL[p] + n - 1) : 0u;
      });
      v = (int64_t)maxlen * (int64_t)maxc;
    }
  }
  x.par.single([&]() { *out = v; });
  x.par.sync();
  x.reset(mark);
}

// One duplicated n-gram order of a split document (k_gr_dup_split): the in-stage dup phase for
// order t alone, over the arrays the stage workgroup exported. Writes r[7 + n_top + t].
template <class P>
TB_HD void gr_dup_one_order(DocCtx<P>& x, const DevStep& ds, int t, const GrExport& e, int64_t* r) {
  const uint32_t W = e.W, n = (uint32_t)ds.dup_n[t];
  const uint32_t G = (n == 0 || W < n) ? 0u : W - n + 1;
  int64_t* out = r + rec_gr_fixed() + ds.n_top + t;
  if (G == 0) {
    x.par.single([&]() { *out = 0; });
    return;
  }
  const DupGrams dg{e.wid, e.WL, e.K, e.PB, e.bs, e.be, e.b};
  const uint32_t SW = (G + 31) / 32 + 1;
  const auto mark = x.mark();
  uint32_t* bits = x.template alloc_hot<uint32_t>(2 * (uint64_t)SW);  // [sn | R]
  uint32_t* gc = x.template alloc_hot_keep<uint32_t>((uint64_t)G + 1, 6ull * G + 64);
  if (x.overflow) return;
  x.par.for_n(2 * SW, [&](uint32_t i) { bits[i] = 0; });
  x.par.sync();
  uint32_t* R = bits + SW;
  auto key = [&](uint32_t p) { return dg.key(p, n); };
  // Only the repeat candidates are canonicalised: a gram that is not a candidate occurs once, so
  // its position is never repeated and the walk never reads its gc entry. gc of a candidate
  // position = the class id (its canonical candidate's index).
  if (cand_path_fits(x, G)) {
    const uint32_t bw = cand_bitmap_words(G);
    uint32_t* bm = x.template alloc_hot<uint32_t>(2 * bw);
    uint32_t* list = x.template alloc_hot<uint32_t>((uint64_t)G + 1);
    if (x.overflow) return;
    const uint32_t nc = repeat_candidates(x, G, key, bm, bw, list);
    if (nc >= 2) {
      uint32_t* cc = x.template alloc_hot_keep<uint32_t>((uint64_t)nc + 1, 6ull * nc + 64);
      if (x.overflow) return;
      canonicalize_res(
          x, nc, [&](uint32_t c) { return key(list[c]); },
          [&](uint32_t c, uint32_t d) { return dg.eq(list[c], list[d], n); }, cc,
          [&](uint32_t c, uint32_t g) {
            const uint32_t p = list[c];
            gc[p] = g;
            if (g != c) {
              const uint32_t q = list[g];
              P::or32(&R[p >> 5], 1u << (p & 31));
              P::or32(&R[q >> 5], 1u << (q & 31));
            }
          });
    }
  } else {
    canonicalize_res(
        x, G, key, [&](uint32_t p, uint32_t q) { return dg.eq(p, q, n); }, gc,
        [&](uint32_t p, uint32_t g) {
          if (g != p) {
            P::or32(&R[p >> 5], 1u << (p & 31));
            P::or32(&R[g >> 5], 1u << (g & 31));
          }
        });
  }
  if (x.overflow) return;
  x.par.sync();
  if constexpr (P::kWaves > 0) {
    if (x.par.wave_index() == 0) {
      const int64_t rep = dup_walk_wave(x.par, G, n, gc, R, bits, e.WL);
      if (x.par.lane == 0) *out = rep;
    }
  } else {
    x.par.single([&]() { *out = dup_walk(G, n, gc, R, bits, e.WL); });
  }
  x.par.sync();
  x.reset(mark);
}

// Language-id record straight from the UTF-8 bytes: every code point position (a UTF-8 lead
// byte, as decode() defines them) of the first kLidMaxCps code points, plus the virtual end
// position, emits the 1..4-grams ending there (lid_grams_at); their int16 logit rows are summed
// exactly. Neighbouring letters are found by stepping back to the previous lead bytes, so no
// per-code-point arrays are needed. The device runs its own kernel for this (k_langid_mfma,
// same sums); this version runs inside the stage emulation on the host.
template <class P, int D>
TB_HD void langid_sums(DocCtx<P>& x, const uint8_t* b, uint32_t n, const LidTables& lt, int64_t* sums) {
  const UcdView ucd = x.ucd;
  const auto mark = x.mark();
  int32_t* tmp = x.template alloc_hot<int32_t>(64 * D);
  uint32_t* limb = x.template alloc_hot<uint32_t>(1);
  if (x.overflow) return;
  // byte offset of code point kLidMaxCps (the cut), or n
  x.par.single([&]() { *limb = n; });
  x.par.sync();
  if (n > (uint32_t)kLidMaxCps) {
    x.par.template compact<int>(
        n, [&](uint32_t i, int&) { return utf8_is_lead(b[i]); },
        [&](uint32_t i, uint32_t k, int&) { if (k == (uint32_t)kLidMaxCps) *limb = i; });
    x.par.sync();
  }
  const uint32_t lim = *limb;
  // A lane visits ceil((lim + 1) / 64) <= 257 byte positions (lim <= 4 * kLidMaxCps) with at most
  // 4 grams each and |row value| <= 2^15: int32 partials cannot overflow.
  x.par.template accum_rows<D>(
      lim + 1,
      [&](uint32_t s, int32_t* part) {
        if (s < lim && !utf8_is_lead(b[s])) return;
        const uint32_t l0 = s < lim ? lid_letter(ucd, b, n, s) : 0u;
        const int64_t p1 = prev_lead(b, s);
        const int64_t p2 = p1 >= 0 ? prev_lead(b, p1) : -1;
        const int64_t p3 = p2 >= 0 ? prev_lead(b, p2) : -1;
        part[D - 1] += lid_grams_n(lid_letter(ucd, b, n, p3), lid_letter(ucd, b, n, p2),
                                   lid_letter(ucd, b, n, p1), l0, [&](uint32_t g, int order) {
                                     lid_add_emb(lt.E, g, order, part);
                                   });
      },
      tmp, sums);
  x.reset(mark);
}

// Language-id record straight from the UTF-8 bytes: every code point position (a UTF-8 lead
// byte, as decode() defines them) of the first kLidMaxCps code points, plus the virtual end
// position, emits the 1..4-grams ending there (lid_grams_at); their int8 embedding rows are summed
// exactly, then decided (lid_record_v3, the same integers as the device's MFMA tile). Neighbouring letters are found by stepping back to the previous lead
// bytes, so no per-code-point arrays are needed. The device runs its own kernel for this
// (k_langid_mfma, same records); this version runs inside the stage
// emulation on the host.
template <class P>
TB_HD void langid_record(DocCtx<P>& x, const uint8_t* b, uint32_t n, const LidTables& lt, int64_t* r) {
  const auto mark = x.mark();
  int64_t* sums = x.template alloc_hot<int64_t>(kLidDim + 1);  // shared by the lanes
  if (x.overflow) return;
  langid_sums<P, kLidDim + 1>(x, b, n, lt, sums);
  if (x.overflow) return;
  x.par.single([&]() { lid_record_v3(sums, sums[kLidDim], lt, r); });
  x.par.sync();
  x.reset(mark);
}

// ---------------------------------------------------------------------------------------------
// C4QualityFilter, pass A: decisions + rewritten text in scratch (reference c4_filters.rs:147-295).
// rec: LOREM, CURLY, TOO_LONG, NO_PUNCT, TOO_FEW, SENTENCES, NEW_LEN
// src: (byte offset of the new text in the doc's scratch, or -1 = unchanged original; length)
TB_HD bool end_punct(uint32_t c) {
  return c == '.' || c == '!' || c == '?' || c == '"' || c == '\'' || c == 0x201D;
}

// Case-insensitive prefix test with the same folding as ci_contains (ASCII letters, and
// U+212A KELVIN SIGN as 'k'): does `pat` start at b[0] within n bytes?
TB_HD bool ci_starts_with(const uint8_t* b, uint32_t n, const char* pat, int plen) {
  uint32_t i = 0;
  for (int j = 0; j < plen; ++j) {
    if (i >= n) return false;
    const char pc = pat[j];
    uint8_t c = b[i];
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
    if (c == (uint8_t)pc) { ++i; continue; }
    if (pc == 'k' && i + 2 < n && b[i] == 0xE2 && b[i + 1] == 0x84 && b[i + 2] == 0xAA) { i += 3; continue; }
    return false;
  }
  return true;
}

// The first three bytes at b (n available), ASCII-lowercased, little endian (0 past the end):
// three independent loads. Every C4 phrase starts with three ASCII letters other than 'k' (the
// only pattern letter with a multi-byte match, the Kelvin sign), so a phrase can only match where
// this equals its packed prefix.
TB_HD uint32_t lower3(const uint8_t* b, uint32_t n) {
  uint32_t w = 0;
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    uint32_t c = k < n ? b[k] : 0u;
    if (c >= 'A' && c <= 'Z') c += 32;
    w |= c << (8 * k);
  }
  return w;
}
TB_HD constexpr uint32_t pack3(const char* p) {
  return (uint32_t)(uint8_t)p[0] | ((uint32_t)(uint8_t)p[1] << 8) | ((uint32_t)(uint8_t)p[2] << 16);
}

// Bits of the per-line pattern flags (c4_pass_a)
enum : uint32_t { C4F_JS = 1, C4F_POLICY = 2 };

// C4 pass A's first pass over the bytes (c4_byte_scan): the whole-document filters, a possible
// citation, and whether a javascript / policy phrase starts anywhere (C4F_JS / C4F_POLICY).
enum : uint32_t { C4S_LOREM = 4, C4S_CURLY = 8, C4S_CITE = 16 };

// The pattern bits (C4F_JS | C4F_POLICY) of the phrases starting at byte s (case-folded).
TB_HD uint32_t c4_phrases_at(const DevC4& c4, const uint8_t* b, uint32_t n, uint32_t s) {
  uint8_t c0 = b[s];
  if (c0 >= 'A' && c0 <= 'Z') c0 = (uint8_t)(c0 + 32);
  if (c0 != 'j' && c0 != 't' && c0 != 'p' && c0 != 'c' && c0 != 'u') return 0;
  const char* const kPol[6] = {"terms of use", "privacy policy", "cookie policy",
                               "uses cookies", "use of cookies", "use cookies"};
  const int kPolLen[6] = {12, 14, 13, 12, 14, 11};
  uint32_t bits = 0;
  const uint32_t w3 = lower3(b + s, n - s);
  auto pre = [&](const char* pat) { return w3 == pack3(pat); };
  if (c4.filter_javascript && c0 == 'j' && pre("javascript") && ci_starts_with(b + s, n - s, "javascript", 10))
    bits |= C4F_JS;
  if (c4.filter_policy)
    for (int t = 0; t < 6; ++t)
      if (kPol[t][0] == (char)c0 && pre(kPol[t]) && ci_starts_with(b + s, n - s, kPol[t], kPolLen[t])) {
        bits |= C4F_POLICY;
        break;
      }
  return bits;
}

// Bytes of v equal to c: bit 7 of each such byte set (exact, no carries between bytes).
TB_HD uint32_t swar_eq_mask(uint32_t v, uint32_t c) {
  const uint32_t t = v ^ (c * 0x01010101u);
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}

// GopherQuality's byte counts of b[0, n): '#' bytes (high half) and ellipses (low half: every
// U+2026 plus len / 3 for each maximal run of '.'). Items are groups of four aligned dwords (one
// dword of look-behind and one of look-ahead, issued together); a dword without '.' or 0xE2 costs
// three SWAR compares and a popcount. Same counts as the per-byte definition.
template <class P>
TB_HD uint64_t gq_byte_counts(DocCtx<P>& x, const uint8_t* b, uint32_t n) {
  const uintptr_t a0 = (uintptr_t)b & ~(uintptr_t)3;
  const uint32_t head = (uint32_t)((uintptr_t)b - a0);
  const uint32_t nd = (head + n + 3) >> 2;
  const uint32_t* w = (const uint32_t*)a0;
  auto dw = [&](int64_t k) -> uint32_t {  // dword k of the aligned stream, bytes outside the text zero
    if (k < 0 || k >= (int64_t)nd) return 0u;
    const int64_t e = 4 * k + 4 - head;
    if (e <= (int64_t)n && 4 * k >= (int64_t)head) return w[k];
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const int64_t sj = 4 * k + j - head;
      if (sj >= 0 && sj < (int64_t)n) v |= (uint32_t)b[sj] << (8 * j);
    }
    return v;
  };
  return x.par.template sum<uint64_t>((nd + 3) >> 2, [&](uint32_t g) {
    uint32_t d[6];  // d[0]: dword 4g - 1, d[1..4]: the group, d[5]: dword 4g + 4
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) d[i] = dw((int64_t)4 * g + i - 1);
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t v = d[i + 1];
      acc += (uint64_t)__builtin_popcount(swar_eq_mask(v, '#')) << 32;
      const uint32_t dots = swar_eq_mask(v, '.'), e2 = swar_eq_mask(v, 0xE2);
      if ((dots | e2) == 0) continue;
      const uint64_t v64 = (uint64_t)v | ((uint64_t)d[i + 2] << 32);
      for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t c0 = (v >> (8 * r)) & 0xFFu;
        if (c0 == 0xE2) {
          acc += ((v64 >> (8 * r + 8)) & 0xFFFFu) == 0xA680u ? 1u : 0u;
          continue;
        }
        if (c0 != '.') continue;
        const uint32_t prev = r ? (v >> (8 * r - 8)) & 0xFFu : d[i] >> 24;
        if (prev == '.') continue;  // not the start of its run
        uint32_t len = 1;
        while (r + len < 8 && ((v64 >> (8 * (r + len))) & 0xFFu) == '.') ++len;
        if (r + len == 8) {  // the run goes past the window: the rest byte by byte
          int64_t j = 4 * ((int64_t)4 * g + i) + r + len - head;
          while (j < (int64_t)n && b[j] == '.') { ++j; ++len; }
        }
        acc += len / 3;
      }
    }
    return acc;
  });
}

// ASCII 'A'..'Z' -> 'a'..'z' in all 8 bytes of v (other bytes unchanged).
TB_HD uint64_t swar_lower8(uint64_t v) {
  constexpr uint64_t k7F = 0x7F7F7F7F7F7F7F7Full, k80 = 0x8080808080808080ull;
  const uint64_t ge_a = (v & k7F) + 0x3F3F3F3F3F3F3F3Full;  // bit 7 set: byte & 0x7F >= 'A'
  const uint64_t gt_z = (v & k7F) + 0x2525252525252525ull;  // bit 7 set: byte & 0x7F > 'Z'
  const uint64_t upper = ge_a & ~gt_z & ~v & k80;
  return v | (upper >> 2);
}

// Every byte position s of b[0, n) visited as f(s, c0, c1, l3): its byte, the next one (0 past the
// end) and the three bytes from s ASCII-lowercased (l3, little endian). Items are four aligned
// dwords whose five loads (one of look-ahead) are issued together, and the lowercase windows
// come from SWAR shifts: one memory round trip per 16 bytes, no per-byte loads.
template <class P, class F>
TB_HD void scan_bytes16(DocCtx<P>& x, const uint8_t* b, uint32_t n, F&& f) {
  const uintptr_t a0 = (uintptr_t)b & ~(uintptr_t)3;
  const uint32_t head = (uint32_t)((uintptr_t)b - a0);
  const uint32_t nd = (head + n + 3) >> 2;
  const uint32_t* w = (const uint32_t*)a0;
  auto dw = [&](uint32_t k) -> uint32_t {  // dword k of the aligned stream, bytes past the text zero
    if (k >= nd) return 0u;
    const int64_t e = (int64_t)4 * k + 4 - head;  // doc position one past its last byte
    if (e <= (int64_t)n && 4 * k >= head) return w[k];
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const int64_t sj = (int64_t)4 * k + j - head;
      if (sj >= 0 && sj < (int64_t)n) v |= (uint32_t)b[sj] << (8 * j);
    }
    return v;
  };
  x.par.for_n((nd + 3) >> 2, [&](uint32_t g) {
    uint32_t d[5];
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i) d[i] = dw(4 * g + i);
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = 4 * g + i;
      const uint64_t v = (uint64_t)d[i] | ((uint64_t)d[i + 1] << 32);
      const uint64_t lo = swar_lower8(v);
      for (uint32_t r = 0; r < 4; ++r) {
        const int64_t sp = (int64_t)4 * k + r - head;
        if (sp < 0 || sp >= (int64_t)n) continue;
        f((uint32_t)sp, (uint32_t)(v >> (8 * r)) & 0xFFu, (uint32_t)(v >> (8 * r + 8)) & 0xFFu,
          (uint32_t)(lo >> (8 * r)) & 0xFFFFFFu);
      }
    }
  });
}

// Could a javascript / policy phrase start here (its case-folded 3-byte prefix)?
TB_HD bool c4_phrase_prefix(uint32_t l3) {
  return l3 == pack3("jav") || l3 == pack3("ter") || l3 == pack3("pri") || l3 == pack3("coo") || l3 == pack3("use");
}

// One pass over the bytes: lorem ipsum and curly brackets (lowercase().contains("lorem ipsum") ==
// the pattern starts, case-folded, at some 'l'), a possible citation ('[' followed by a digit:
// a non-ASCII byte after the '[' counts too, so the test is conservative) and the phrase bits;
// only a position whose 3-byte prefix matches runs the exact comparison (ci_starts_with).
template <class P>
TB_HD uint32_t c4_byte_scan(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n) {
  uint32_t acc = 0;
  const bool phrases = c4.filter_javascript || c4.filter_policy;
  scan_bytes16(x, b, n, [&](uint32_t s, uint32_t c0, uint32_t c1, uint32_t l3) {
    if (c4.filter_curly_bracket && (c0 == '{' || c0 == '}')) acc |= C4S_CURLY;
    if (c0 == '[' && ((c1 >= '0' && c1 <= '9') || c1 >= 0x80)) acc |= C4S_CITE;
    if (c4.filter_lorem_ipsum && l3 == pack3("lor") && ci_starts_with(b + s, n - s, "lorem ipsum", 11))
      acc |= C4S_LOREM;
    if (phrases && c4_phrase_prefix(l3)) acc |= c4_phrases_at(c4, b, n, s);
  });
  return x.par.reduce_or(acc);
}

// C4 pass A, common end: the joined kept lines Jb[0, Jtot) are trimmed and their sentences counted
// (saturated at min_num_sentences), then the record and the rewritten text's source are written.
template <class P>
TB_HD void c4_finish(DocCtx<P>& x, const DevC4& c4, uint32_t n, uint8_t* Jb, uint32_t Jtot, int64_t s_long,
                     int64_t s_punct, int64_t s_few, int64_t* r, int64_t* src) {
  Cps jc = decode(x, Jb, Jtot);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  const uint32_t JC = jc.n;
  const PropArr jprop = jc.props();
  uint32_t tcs, tce;
  trim_span(x, jprop, JC, tcs, tce);
  uint32_t nsent = 0, bstart = 0, blen = 0;
  if (tcs < tce) {
    const uint32_t lim = c4.min_num_sentences > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)c4.min_num_sentences;
    nsent = count_sentences_upto(x, jc, tcs, tce, lim);
    bstart = jc.o(tcs);
    blen = jc.o(tce) - jc.o(tcs);
  }
  x.stamp(PH_C4_SENT);
  const int64_t jrel = (int64_t)((const char*)Jb - x.scr) + bstart;
  // The rewrite can only grow a document by one '\n' per sentence not followed by whitespace
  // (split_paragraph=false). Bounding the growth to kC4MaxGrowth bytes lets the host size the
  // next version's buffer (and its D2H copy) up front without a sync; the rare document that
  // would exceed it is recomputed on the CPU path.
  if (blen > n + kC4MaxGrowth) {
    x.set_flag(DOC_NEEDS_CPU);
    x.par.single([&]() { src[0] = 0; src[1] = 0; });
    return;
  }
  x.par.single([&]() {
    r[0] = 0; r[1] = 0; r[2] = s_long; r[3] = s_punct; r[4] = s_few; r[5] = nsent; r[6] = blen;
    src[0] = jrel;
    src[1] = blen;
  });
}

// The code point that ends the non-empty byte span [s, e) of b[0, n).
TB_HD uint32_t last_cp(const uint8_t* b, uint32_t s, uint32_t e, uint32_t n) {
  uint32_t p = e - 1;
  while (p > s && !utf8_is_lead(b[p])) --p;
  int len;
  return utf8_decode(b, p, n, &len);
}

// C4 pass A for a document with no citation to remove: every processed line is its trimmed
// original line, so the processed text Pb, the per-code-point line ids and the kept-byte prefix
// of the general path are not built. The lines come as trimmed byte spans [lbs[k], lbe[k])
// (lbs[NLn] = 0xFFFFFFFF) with their word counts and longest words; the phrase search, terminal
// punctuation and the join read the original bytes of each line's span. Same records and
// rewritten text as the general path.
template <class P>
TB_HD void c4_plain_tail(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n, uint32_t NLn,
                         const uint32_t* lbs, const uint32_t* lbe, const uint32_t* nw, const uint32_t* mx,
                         uint32_t phrase_bits, int64_t* r, int64_t* src, uint32_t* wout = nullptr) {
  uint32_t* pf = x.template alloc_hot<uint32_t>(NLn + 1);   // pattern flags per line
  uint8_t* code = x.template alloc_hot<uint8_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  auto line_of_byte = [&](uint32_t bs) {  // last line with byte start <= bs
    uint32_t lo = 0, hi = NLn;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (lbs[mid] <= bs) lo = mid; else hi = mid;
    }
    return lo;
  };
  const bool phrases = NLn > 0 && (phrase_bits & (C4F_JS | C4F_POLICY));
  if (phrases) {
    x.par.for_n(NLn, [&](uint32_t k) { pf[k] = 0; });
    x.par.sync();
    // only when the byte scan saw a phrase somewhere (rare). A phrase (letters and spaces, starting
    // with a letter) that matches at a byte lies inside one line's trimmed span: it cannot cross
    // the line feed or run into trailing whitespace.
    scan_bytes16(x, b, n, [&](uint32_t s, uint32_t, uint32_t, uint32_t l3) {
      if (!c4_phrase_prefix(l3)) return;
      const uint32_t bits = c4_phrases_at(c4, b, n, s);
      if (bits) P::or32(&pf[line_of_byte(s)], bits);
    });
    x.par.sync();
  }
  x.par.for_n(NLn, [&](uint32_t k) {
    const uint32_t s0 = lbs[k], e0 = lbe[k], ln = e0 - s0;
    const uint32_t fl = phrases ? pf[k] : 0u;
    uint8_t cd = 0;
    if (c4.max_word_length > 0 && (int64_t)mx[k] > c4.max_word_length) {
      cd = 1;
    } else if (c4.filter_no_terminal_punct) {
      const bool term = ln > 0 && end_punct(last_cp(b, s0, e0, n));
      const bool ell = ln >= 3 && b[e0 - 1] == '.' && b[e0 - 2] == '.' && b[e0 - 3] == '.';
      if (!term || ell) cd = 2;
    }
    if (cd == 0 && c4.min_words_per_line > 0 && (int64_t)nw[k] < c4.min_words_per_line) cd = 3;
    if (cd == 0 && c4.filter_javascript && (fl & C4F_JS)) cd = 4;
    if (cd == 0 && c4.filter_policy && (fl & C4F_POLICY)) cd = 5;
    code[k] = cd;
  });
  x.par.sync();
  const uint64_t s12 = x.par.template sum<uint64_t>(NLn, [&](uint32_t k) {
    return (uint64_t)(code[k] == 1) | ((uint64_t)(code[k] == 2) << 32);
  });
  const int64_t s_long = (int64_t)(s12 & 0xFFFFFFFFull), s_punct = (int64_t)(s12 >> 32);
  const int64_t s_few = x.par.template sum<int64_t>(NLn, [&](uint32_t k) { return (int64_t)(code[k] == 3); });
  if (wout) {
    // words of the rewrite (the kept lines joined by '\n', trimmed): words never cross a line
    // feed, so they are the kept lines' words (StageOut::dict_words of the next version)
    const uint32_t wk = x.par.template sum<uint32_t>(NLn, [&](uint32_t k) { return code[k] == 0 ? nw[k] : 0u; });
    x.par.single([&]() { *wout = wk; });
  }
  x.stamp(PH_C4_CODES);
  // ---- joined kept lines (HBM: read back by pass B), copied byte by byte ----
  uint32_t* joff = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  uint32_t Jtot = x.par.template scan<uint32_t>(
      NLn, 0u, [](uint32_t a, uint32_t b2) { return a + b2; },
      [&](uint32_t k) { return code[k] == 0 ? lbe[k] - lbs[k] + 1 : 0u; },
      [&](uint32_t k, uint32_t e) { joff[k] = e; });
  if (Jtot > 0) Jtot -= 1;
  uint8_t* Jb = x.template alloc_global<uint8_t>(Jtot + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.sync();
  if (NLn > 0) {
    x.par.for_n(n, [&](uint32_t i) {
      const uint32_t k = line_of_byte(i);
      if (code[k] != 0 || i < lbs[k] || i >= lbe[k]) return;
      Jb[joff[k] + (i - lbs[k])] = b[i];
    });
    x.par.for_n(NLn, [&](uint32_t k) {
      const uint32_t ln = lbe[k] - lbs[k];
      if (code[k] == 0 && joff[k] + ln < Jtot) Jb[joff[k] + ln] = '\n';
    });
  }
  x.par.sync();
  x.stamp(PH_C4_JOIN);
  c4_finish(x, c4, n, Jb, Jtot, s_long, s_punct, s_few, r, src);
}

// The plain path from this pass's own decode and lines [la, lb) (code points): words come from
// one segmentation of the whole text — the words of a trimmed line are exactly the document's
// words inside its span (UAX#29 always breaks around a line feed, WB3a/b, and trimming only
// drops whitespace, which no word contains) — assigned to lines by their first code point.
template <class P>
TB_HD void c4_pass_a_plain(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n, const Cps& c,
                           const uint32_t* la, const uint32_t* lb, uint32_t NLn, int64_t* r, int64_t* src,
                           uint32_t phrase_bits) {
  const OffArr off = c.offs();
  uint32_t* lbs = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* lbe = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* nw = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* mx = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.for_n(NLn, [&](uint32_t k) { lbs[k] = off[la[k]]; lbe[k] = off[lb[k]]; nw[k] = 0; mx[k] = 0; });
  x.par.single([&]() { lbs[NLn] = 0xFFFFFFFFu; });
  x.par.sync();
  x.stamp(PH_C4_CITE);
  if (NLn > 0) {
    auto line_of_cp = [&](uint32_t cs) {  // last line with la <= cs
      uint32_t lo = 0, hi = NLn;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (la[mid] <= cs) lo = mid; else hi = mid;
      }
      return lo;
    };
    const auto mw = x.mark();
    Words wd = words(x, c);
    if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    x.par.for_n(wd.n, [&](uint32_t q) {
      const uint32_t k = line_of_cp(wd.cs[q]);
      P::add32(&nw[k], 1u);
      P::max32(&mx[k], wd.ce[q] - wd.cs[q]);
    });
    x.par.sync();
    x.reset(mw);
  }
  x.stamp(PH_C4_WORDS);
  c4_plain_tail(x, c4, b, n, NLn, lbs, lbe, nw, mx, phrase_bits, r, src);
}

// The plain path from the stage's line export (LineStat region, header = line count): no decode,
// lines or words here.
template <class P>
TB_HD void c4_pass_a_export(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n, const uint32_t* region,
                            uint32_t NLn, int64_t* r, int64_t* src, uint32_t phrase_bits, uint32_t* wout = nullptr) {
  const LineStat* ls = (const LineStat*)(region + 4);
  uint32_t* lbs = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* lbe = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* nw = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* mx = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.for_n(NLn, [&](uint32_t k) {
    const LineStat e = ls[k];
    lbs[k] = e.bs; lbe[k] = e.be; nw[k] = e.nw; mx[k] = e.mx;
  });
  x.par.single([&]() { lbs[NLn] = 0xFFFFFFFFu; });
  x.par.sync();
  x.stamp(PH_C4_WORDS);
  c4_plain_tail(x, c4, b, n, NLn, lbs, lbe, nw, mx, phrase_bits, r, src, wout);
}

// The byte past a citation starting at b[i] == '[' inside [i, e) (a trimmed line), 0 when none
// starts there, 0xFFFFFFFF when the match depends on a non-ASCII byte (a Unicode digit or space).
TB_HD uint32_t c4_cite_end_bytes(const UcdView& ucd, const uint8_t* b, uint32_t i, uint32_t e) {
  uint32_t p = i + 1;
  if (p >= e) return 0;
  if (b[p] >= 0x80) return 0xFFFFFFFFu;
  if (b[p] < '0' || b[p] > '9') return 0;
  while (p < e && b[p] >= '0' && b[p] <= '9') ++p;
  while (true) {
    if (p < e && b[p] >= 0x80) return 0xFFFFFFFFu;  // a non-ASCII digit could continue \d+
    if (!(p < e && b[p] == ',')) break;
    uint32_t q = p + 1;
    while (q < e && b[q] < 0x80 && (ucd.props(b[q]) & P_WS)) ++q;
    if (q < e && b[q] >= 0x80) return 0xFFFFFFFFu;  // Unicode whitespace or digit
    if (!(q < e && b[q] >= '0' && b[q] <= '9')) break;
    while (q < e && b[q] >= '0' && b[q] <= '9') ++q;
    p = q;
  }
  return (p < e && b[p] == ']') ? p + 1 : 0;
}

// C4 pass A for a document with a possible citation, from the stage's line export: the
// citations (reference CITATION_REGEX, c4_filters.rs:33, applied to each trimmed line) are found on
// the bytes of the exported trimmed line spans, the processed lines Pb are built byte-parallel
// (a removed-byte bitmap and its prefix popcounts give every kept byte's place), and only the lines
// that lost a citation are segmented again; no decode, no Rust lines, no per-code-point line ids.
// Returns false without writing anything when a candidate needs Unicode classes (a non-ASCII byte
// where \d or \s could continue the match): the general path runs then.
template <class P>
TB_HD bool c4_pass_a_cite_export(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n, const uint32_t* region,
                                 uint32_t NLn, int64_t* r, int64_t* src) {
  const LineStat* ls = (const LineStat*)(region + 4);
  const auto mark0 = x.mark();
  const uint32_t nwd = (n + 31) / 32 + 1;
  uint32_t* lbs = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* lbe = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* nw = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* mx = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* plen = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* poff = x.template alloc_hot<uint32_t>(NLn + 1);
  uint8_t* code = x.template alloc_hot<uint8_t>(NLn + 1);    // 1: the line lost a citation (then the codes)
  uint32_t* pf = x.template alloc_hot<uint32_t>(NLn + 1);    // pattern flags per line
  uint32_t* rmb = x.template alloc_hot<uint32_t>(nwd);       // removed bytes
  uint32_t* wr = x.template alloc_hot<uint32_t>(nwd + 1);    // exclusive popcount prefix of rmb
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
  x.par.for_n(NLn, [&](uint32_t k) {
    const LineStat e = ls[k];
    lbs[k] = e.bs; lbe[k] = e.be; nw[k] = e.nw; mx[k] = e.mx; code[k] = 0; pf[k] = 0;
  });
  x.par.for_n(nwd, [&](uint32_t w) { rmb[w] = 0; });
  x.par.single([&]() { lbs[NLn] = 0xFFFFFFFFu; });
  x.par.sync();
  auto line_of_byte = [&](uint32_t bs) {  // last line with byte start <= bs
    uint32_t lo = 0, hi = NLn;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (lbs[mid] <= bs) lo = mid; else hi = mid;
    }
    return lo;
  };
  uint32_t bad = 0;
  x.par.for_n(n, [&](uint32_t i) {
    if (b[i] != '[') return;
    const uint32_t k = line_of_byte(i), e = lbe[k];
    if (i < lbs[k] || i >= e) return;
    const uint32_t ce = c4_cite_end_bytes(x.ucd, b, i, e);
    if (ce == 0xFFFFFFFFu) { bad = 1; return; }
    if (ce == 0) return;
    for (uint32_t q = i; q < ce; ++q) P::or32(&rmb[q >> 5], 1u << (q & 31));
    code[k] = 1;
  });
  x.par.sync();
  if (x.par.reduce_or(bad)) {
    x.reset(mark0);
    return false;
  }
  x.par.template scan<uint32_t>(
      nwd, 0u, [](uint32_t a, uint32_t c2) { return a + c2; }, [&](uint32_t w) { return (uint32_t)__builtin_popcount(rmb[w]); },
      [&](uint32_t w, uint32_t e) { wr[w] = e; });
  x.par.sync();
  auto rank = [&](uint32_t i) {  // removed bytes before byte i
    return wr[i >> 5] + (uint32_t)__builtin_popcount(rmb[i >> 5] & ((1u << (i & 31)) - 1u));
  };
  auto removed = [&](uint32_t i) { return (rmb[i >> 5] >> (i & 31)) & 1u; };
  x.par.for_n(NLn, [&](uint32_t k) { plen[k] = (lbe[k] - lbs[k]) - (rank(lbe[k]) - rank(lbs[k])); });
  x.par.sync();
  const uint32_t Ptot = x.par.template scan<uint32_t>(
      NLn, 0u, [](uint32_t a, uint32_t c2) { return a + c2; }, [&](uint32_t k) { return plen[k] + 1u; },
      [&](uint32_t k, uint32_t e) { poff[k] = e; });
  uint8_t* Pb = x.template alloc<uint8_t>(Ptot + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
  x.par.sync();
  x.par.for_n(n, [&](uint32_t i) {
    const uint32_t k = line_of_byte(i);
    if (i < lbs[k] || i >= lbe[k] || removed(i)) return;
    Pb[poff[k] + (i - lbs[k]) - (rank(i) - rank(lbs[k]))] = b[i];
  });
  x.par.for_n(NLn, [&](uint32_t k) { Pb[poff[k] + plen[k]] = '\n'; });
  x.par.single([&]() { poff[NLn] = Ptot; });
  x.par.sync();
  x.stamp(PH_C4_CITE);
  auto line_of_p = [&](uint32_t bs) {  // last line with poff <= bs
    uint32_t lo = 0, hi = NLn;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (poff[mid] <= bs) lo = mid; else hi = mid;
    }
    return lo;
  };
  // words of the lines that lost a citation (joined with '\n', so no word spans two lines)
  {
    uint32_t* coff = x.template alloc_hot<uint32_t>(NLn + 1);
    if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
    const uint32_t Ctot = x.par.template scan<uint32_t>(
        NLn, 0u, [](uint32_t a, uint32_t c2) { return a + c2; },
        [&](uint32_t k) { return code[k] ? plen[k] + 1 : 0u; }, [&](uint32_t k, uint32_t e) { coff[k] = e; });
    x.par.for_n(NLn, [&](uint32_t k) { if (code[k]) { nw[k] = 0; mx[k] = 0; } });
    x.par.sync();
    if (Ctot > 0) {
      const auto mc = x.mark();
      uint8_t* Pc = x.template alloc<uint8_t>(Ctot + 1);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
      x.par.for_n(Ptot, [&](uint32_t i) {
        const uint32_t k = line_of_p(i);
        if (code[k] && i - poff[k] <= plen[k]) Pc[coff[k] + (i - poff[k])] = Pb[i];  // (its '\n' too)
      });
      x.par.sync();
      uint32_t dict = 0;
      Cps cc = decode(x, Pc, Ctot, false, &dict);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
      if (dict) {  // dictionary-script text in a cited line: its words need ICU
        x.set_flag(DOC_NEEDS_CPU);
        return true;
      }
      Words cw = words(x, cc);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
      x.par.for_n(cw.n, [&](uint32_t q) {
        const uint32_t bs = cw.bs[q];
        uint32_t lo = 0, hi = NLn;  // last line with coff <= bs: the cited line holding the word
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (coff[mid] <= bs) lo = mid; else hi = mid;
        }
        P::add32(&nw[lo], 1u);
        P::max32(&mx[lo], cw.ce[q] - cw.cs[q]);
      });
      x.par.sync();
      x.reset(mc);
    }
  }
  x.stamp(PH_C4_WORDS);
  if (c4.filter_javascript || c4.filter_policy) {
    scan_bytes16(x, Pb, Ptot, [&](uint32_t s, uint32_t, uint32_t, uint32_t l3) {
      if (!c4_phrase_prefix(l3)) return;
      const uint32_t bits = c4_phrases_at(c4, Pb, Ptot, s);
      if (bits) P::or32(&pf[line_of_p(s)], bits);
    });
  }
  x.par.sync();
  x.par.for_n(NLn, [&](uint32_t k) {
    const uint8_t* lp = Pb + poff[k];
    const uint32_t ln = plen[k];
    uint8_t cd = 0;
    if (c4.max_word_length > 0 && (int64_t)mx[k] > c4.max_word_length) {
      cd = 1;
    } else if (c4.filter_no_terminal_punct) {
      bool term = false;
      if (ln > 0) {
        uint32_t st = ln - 1;
        while (st > 0 && (lp[st] & 0xC0) == 0x80) --st;
        int len;
        term = end_punct(utf8_decode(lp, st, ln, &len));
      }
      const bool ell = ln >= 3 && lp[ln - 1] == '.' && lp[ln - 2] == '.' && lp[ln - 3] == '.';
      if (!term || ell) cd = 2;
    }
    if (cd == 0 && c4.min_words_per_line > 0 && (int64_t)nw[k] < c4.min_words_per_line) cd = 3;
    if (cd == 0 && c4.filter_javascript && (pf[k] & C4F_JS)) cd = 4;
    if (cd == 0 && c4.filter_policy && (pf[k] & C4F_POLICY)) cd = 5;
    code[k] = cd;
  });
  x.par.sync();
  const uint64_t s12 = x.par.template sum<uint64_t>(NLn, [&](uint32_t k) {
    return (uint64_t)(code[k] == 1) | ((uint64_t)(code[k] == 2) << 32);
  });
  const int64_t s_long = (int64_t)(s12 & 0xFFFFFFFFull), s_punct = (int64_t)(s12 >> 32);
  const int64_t s_few = x.par.template sum<int64_t>(NLn, [&](uint32_t k) { return (int64_t)(code[k] == 3); });
  x.stamp(PH_C4_CODES);
  // ---- joined kept lines (HBM: read back by pass B), copied from Pb ----
  uint32_t* joff = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
  uint32_t Jtot = x.par.template scan<uint32_t>(
      NLn, 0u, [](uint32_t a, uint32_t b2) { return a + b2; },
      [&](uint32_t k) { return code[k] == 0 ? plen[k] + 1 : 0u; }, [&](uint32_t k, uint32_t e) { joff[k] = e; });
  if (Jtot > 0) Jtot -= 1;
  uint8_t* Jb = x.template alloc_global<uint8_t>(Jtot + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return true; }
  x.par.sync();
  x.par.for_n(Ptot, [&](uint32_t i) {
    const uint32_t k = line_of_p(i);
    const uint32_t j = i - poff[k];
    if (code[k] != 0 || j >= plen[k]) return;
    Jb[joff[k] + j] = Pb[i];
  });
  x.par.for_n(NLn, [&](uint32_t k) {
    if (code[k] == 0 && joff[k] + plen[k] < Jtot) Jb[joff[k] + plen[k]] = '\n';
  });
  x.par.sync();
  x.stamp(PH_C4_JOIN);
  c4_finish(x, c4, n, Jb, Jtot, s_long, s_punct, s_few, r, src);
  return true;
}

// `wout` (optional): the rewrite's word count when it comes from the stage's line export (the
// only path a dictionary-script document takes here; kNoWords stays otherwise)
// `hls` (optional): a dictionary-script document's per-line word statistics from the host (ICU,
// text.h dict_c4_lines: [NL, nw_0, mx_0, ...]) in place of segmenting its processed lines here.
template <class P>
TB_HD void c4_pass_a(DocCtx<P>& x, const DevC4& c4, const uint8_t* b, uint32_t n, int64_t* r, int64_t* src,
                     const uint32_t* line_stats = nullptr, uint32_t* wout = nullptr, const uint32_t* hls = nullptr) {
  x.stamp(PH_START);
  const uint32_t scan = c4_byte_scan(x, c4, b, n);
  const bool lorem = scan & C4S_LOREM, curly = scan & C4S_CURLY;
  if (lorem || curly) {
    x.par.single([&]() {
      r[0] = lorem; r[1] = curly; r[2] = r[3] = r[4] = r[5] = 0; r[6] = n;
      src[0] = -1; src[1] = n;
    });
    return;
  }
  x.stamp(PH_C4_LOREM);
#ifndef TB_C4_PLAIN
#define TB_C4_PLAIN 1
#endif
  // A citation needs a '[' followed by a digit: without one (the common case) every processed
  // line is its trimmed original line and the plain path runs on the original bytes.
  const bool maybe_cite = c4.remove_citations != 0 && (scan & C4S_CITE);
  if (TB_C4_PLAIN && line_stats && c4.split_paragraph) {
    const uint32_t NL = line_stats[0];  // the stage kernel of this content version wrote it
    if (NL != kLineStatsNone) {
      if (!maybe_cite) {
        c4_pass_a_export(x, c4, b, n, line_stats, NL, r, src, scan, wout);
        return;
      }
      // (documents with host line statistics, i.e. dictionary-script lines, take the general
      // path, which has the ICU statistics of every processed line; workgroup documents too:
      // k_c4_pass_a_blk 1.09 -> 0.57 ms/step, profiles/r10_ab_citeblk)
      if (!hls && NL > 0 && c4_pass_a_cite_export(x, c4, b, n, line_stats, NL, r, src)) return;
    }
  }
  uint32_t dict = 0;
  Cps c = decode(x, b, n, false, &dict);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.stamp(PH_C4_DECODE);
  const uint32_t C = c.n;
  const PropArr prop = c.props();
  const OffArr off = c.offs();
  if (!dict) hls = nullptr;
  if (dict && (!hls || !c4.split_paragraph)) {
    x.set_flag(DOC_NEEDS_CPU);
    return;
  }
  // ---- line spans [la, lb) in code points, trimmed ----
  uint32_t* la = x.template alloc<uint32_t>(C + 1);
  uint32_t* lb = x.template alloc<uint32_t>(C + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  uint32_t NLn = 0;
  if (c4.split_paragraph) {
    Lines L = rust_lines(x, c);
    if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    NLn = L.n;
    x.par.for_n(NLn, [&](uint32_t k) {
      uint32_t s = L.ls[k], e = L.le[k];
      while (s < e && is_ws(prop[s])) ++s;
      while (e > s && is_ws(prop[e - 1])) --e;
      la[k] = s;
      lb[k] = e;
    });
  } else {
    uint32_t tcs, tce;
    trim_span(x, prop, C, tcs, tce);
    if (tcs < tce) {
      const uint32_t m = tce - tcs;
      uint32_t* st = x.template alloc<uint32_t>(m + 1);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
      CpsAcc acc{prop + tcs};
      const uint32_t NS = x.par.template compact<int>(
          m, [&](uint32_t i, int&) { return i == 0 || sb_break(acc, (int)m, (int)i); },
          [&](uint32_t i, uint32_t k, int&) { st[k] = i; });
      x.par.sync();
      struct SS { uint32_t s, e; };
      NLn = x.par.template compact<SS>(
          NS,
          [&](uint32_t k, SS& ss) {
            uint32_t s = tcs + st[k], e = tcs + (k + 1 < NS ? st[k + 1] : m);
            while (s < e && is_ws(prop[s])) ++s;
            while (e > s && is_ws(prop[e - 1])) --e;
            ss.s = s;
            ss.e = e;
            return s < e;
          },
          [&](uint32_t, uint32_t q, SS& ss) { la[q] = ss.s; lb[q] = ss.e; });
    }
  }
  x.par.sync();
  x.stamp(PH_C4_LINES);
  if (hls && hls[0] != NLn) {  // (never: the host splits the same Rust lines)
    x.set_flag(DOC_NEEDS_CPU);
    return;
  }
  if (TB_C4_PLAIN && !maybe_cite && !hls) {
    c4_pass_a_plain(x, c4, b, n, c, la, lb, NLn, r, src, scan);
    return;
  }
  // ---- citation removal -> processed lines Pb (every step parallel over code points) ----
  // lid[j]: the line whose trimmed span holds code point j (kNoLine otherwise), by a max-scan
  // of line-start markers (lines are ordered and disjoint).
  constexpr uint32_t kNoLine = 0xFFFFFFFFu;
  uint32_t* lid = x.template alloc<uint32_t>(C + 1);
  uint32_t* Pw = x.template alloc<uint32_t>(C + 1);   // exclusive prefix of kept bytes
  uint8_t* rm = x.template alloc<uint8_t>(C + 1);     // inside a removed citation
  uint32_t* plen = x.template alloc_hot<uint32_t>(NLn + 1);
  uint32_t* poff = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.for_n(C, [&](uint32_t j) { lid[j] = 0; rm[j] = 0; });
  x.par.sync();
  x.par.for_n(NLn, [&](uint32_t k) { if (la[k] < lb[k]) lid[la[k]] = k + 1; });
  x.par.sync();
  x.par.template scan<uint32_t>(
      C, 0u, [](uint32_t a, uint32_t b2) { return a > b2 ? a : b2; }, [&](uint32_t j) { return lid[j]; },
      [&](uint32_t j, uint32_t e) {
        const uint32_t cur = e > lid[j] ? e : lid[j];  // inclusive max
        lid[j] = (cur > 0 && j < lb[cur - 1]) ? cur - 1 : kNoLine;
      });
  x.par.sync();
  auto cite_end = [&](uint32_t j, uint32_t e) -> uint32_t {  // cp index past a citation at j, or 0
    if (c.lead(j) != '[') return 0;
    uint32_t p = j + 1;
    if (p >= e || !(prop[p] & P_DIGIT)) return 0;
    while (p < e && (prop[p] & P_DIGIT)) ++p;
    while (p < e && c.lead(p) == ',') {
      uint32_t q = p + 1;
      while (q < e && (prop[q] & P_WS)) ++q;
      if (q < e && (prop[q] & P_DIGIT)) {
        while (q < e && (prop[q] & P_DIGIT)) ++q;
        p = q;
      } else {
        break;
      }
    }
    return (p < e && c.lead(p) == ']') ? p + 1 : 0;
  };
  const bool rmc = c4.remove_citations != 0;
  if (rmc) {
    // a citation holds only digits, commas, whitespace and ']': no '[' inside one, so every
    // '[' can be tested independently (same result as the left-to-right scan)
    x.par.for_n(C, [&](uint32_t j) {
      if (c.lead(j) != '[' || lid[j] == kNoLine) return;
      const uint32_t ce = cite_end(j, lb[lid[j]]);
      for (uint32_t q = j; q < ce; ++q) rm[q] = 1;
    });
    x.par.sync();
  }
  auto kept_bytes = [&](uint32_t j) -> uint32_t {
    return (lid[j] != kNoLine && !rm[j]) ? off[j + 1] - off[j] : 0u;
  };
  const uint32_t Ktot = x.par.template scan<uint32_t>(
      C, 0u, [](uint32_t a, uint32_t b2) { return a + b2; }, kept_bytes, [&](uint32_t j, uint32_t e) { Pw[j] = e; });
  x.par.single([&]() { Pw[C] = Ktot; });
  x.par.sync();
  x.par.for_n(NLn, [&](uint32_t k) {
    plen[k] = Pw[lb[k]] - Pw[la[k]];
    poff[k] = Pw[la[k]] + k;  // kept bytes of the earlier lines + one '\n' per earlier line
  });
  const uint32_t Ptot = Ktot + NLn;
  uint8_t* Pb = x.template alloc<uint8_t>(Ptot + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.sync();
  x.par.for_n(C, [&](uint32_t j) {
    const uint32_t nb = kept_bytes(j);
    if (!nb) return;
    uint8_t* d = Pb + Pw[j] + lid[j];
    for (uint32_t q = 0; q < nb; ++q) d[q] = b[off[j] + q];
  });
  x.par.for_n(NLn, [&](uint32_t k) { Pb[poff[k] + plen[k]] = '\n'; });
  x.par.single([&]() { poff[NLn] = Ptot; });
  x.stamp(PH_C4_CITE);
  // ---- words of the processed lines ----
  uint32_t* nw = nullptr;
  uint32_t* mx = nullptr;
  uint32_t* pf = nullptr;  // pattern flags per line
  uint8_t* code = nullptr;
  auto line_arrays = [&]() {
    nw = x.template alloc_hot<uint32_t>(NLn + 1);
    mx = x.template alloc_hot<uint32_t>(NLn + 1);
    pf = x.template alloc_hot<uint32_t>(NLn + 1);
    code = x.template alloc_hot<uint8_t>(NLn + 1);
    if (x.overflow) return false;
    x.par.for_n(NLn, [&](uint32_t k) { nw[k] = 0; mx[k] = 0; pf[k] = 0; code[k] = 0; });
    x.par.sync();
    return true;
  };
  auto line_of_byte = [&](uint32_t bs) {  // last line with poff <= bs
    uint32_t lo = 0, hi = NLn;
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (poff[mid] <= bs) lo = mid; else hi = mid;
    }
    return lo;
  };
  // (one-wave documents only: in the workgroup kernel the per-byte line lookups of the cited-line
  // copy cost more than segmenting the whole processed text, measured)
  const bool from_export = P::kWaves == 1 && TB_C4_PLAIN && line_stats && c4.split_paragraph && NLn > 0 &&
                           line_stats[0] == NLn;
  if (hls) {
    if (!line_arrays()) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    x.par.for_n(NLn, [&](uint32_t k) { nw[k] = hls[1 + 2 * k]; mx[k] = hls[2 + 2 * k]; });
    x.par.sync();
  } else if (from_export) {
    if (!line_arrays()) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    // Lines that lost no citation are their trimmed original lines: their counts come from the
    // stage's line export. Only the processed text of the lines that lost one (code[k] = 1 marks
    // them here) is segmented, joined with '\n' so that no word spans two lines.
    const LineStat* ls = (const LineStat*)(line_stats + 4);
    x.par.for_n(C, [&](uint32_t j) { if (rm[j] && lid[j] != kNoLine) code[lid[j]] = 1; });
    x.par.sync();
    uint32_t* coff = x.template alloc_hot<uint32_t>(NLn + 1);
    if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    const uint32_t Ctot = x.par.template scan<uint32_t>(
        NLn, 0u, [](uint32_t a, uint32_t b2) { return a + b2; },
        [&](uint32_t k) { return code[k] ? plen[k] + 1 : 0u; }, [&](uint32_t k, uint32_t e) { coff[k] = e; });
    x.par.for_n(NLn, [&](uint32_t k) {
      if (!code[k]) { nw[k] = ls[k].nw; mx[k] = ls[k].mx; }
    });
    x.par.sync();
    if (Ctot > 0) {
      const auto mc = x.mark();
      uint8_t* Pc = x.template alloc<uint8_t>(Ctot + 1);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
      x.par.for_n(Ptot, [&](uint32_t i) {
        const uint32_t k = line_of_byte(i);
        if (code[k] && i - poff[k] <= plen[k]) Pc[coff[k] + (i - poff[k])] = Pb[i];  // (its '\n' too)
      });
      x.par.sync();
      Cps cc = decode(x, Pc, Ctot);
      Words cw = words(x, cc);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
      x.par.for_n(cw.n, [&](uint32_t q) {
        const uint32_t bs = cw.bs[q];
        uint32_t lo = 0, hi = NLn;  // last line with coff <= bs: the cited line holding the word
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (coff[mid] <= bs) lo = mid; else hi = mid;
        }
        P::add32(&nw[lo], 1u);
        P::max32(&mx[lo], cw.ce[q] - cw.cs[q]);
      });
      x.par.sync();
      x.reset(mc);
    }
  } else {
    Cps pc = decode(x, Pb, Ptot);
    Words pwd = words(x, pc);
    if (!line_arrays() || x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
    x.par.for_n(pwd.n, [&](uint32_t q) {
      const uint32_t lo = line_of_byte(pwd.bs[q]);
      P::add32(&nw[lo], 1u);
      P::max32(&mx[lo], pwd.ce[q] - pwd.cs[q]);
    });
  }
  x.stamp(PH_C4_WORDS);
  // javascript / policy phrases: to_lowercase().contains() per line == a case-folded match
  // starting at some byte of the line; every byte position is tested in parallel.
  if (c4.filter_javascript || c4.filter_policy) {
    // The phrases hold letters and spaces only, so a match never runs over the '\n' that ends
    // its line: match against the rest of Pb first, look the line up only on a match.
    scan_bytes16(x, Pb, Ptot, [&](uint32_t s, uint32_t, uint32_t, uint32_t l3) {
      if (!c4_phrase_prefix(l3)) return;
      const uint32_t bits = c4_phrases_at(c4, Pb, Ptot, s);
      if (bits) P::or32(&pf[line_of_byte(s)], bits);
    });
  }
  x.par.sync();
  x.par.for_n(NLn, [&](uint32_t k) {
    const uint8_t* lp = Pb + poff[k];
    const uint32_t ln = plen[k];
    uint8_t cd = 0;
    if (c4.max_word_length > 0 && (int64_t)mx[k] > c4.max_word_length) {
      cd = 1;
    } else if (c4.filter_no_terminal_punct) {
      bool term = false;
      if (ln > 0) {
        uint32_t st = ln - 1;
        while (st > 0 && (lp[st] & 0xC0) == 0x80) --st;
        int len;
        term = end_punct(utf8_decode(lp, st, ln, &len));
      }
      const bool ell = ln >= 3 && lp[ln - 1] == '.' && lp[ln - 2] == '.' && lp[ln - 3] == '.';
      if (!term || ell) cd = 2;
    }
    if (cd == 0 && c4.min_words_per_line > 0 && (int64_t)nw[k] < c4.min_words_per_line) cd = 3;
    if (cd == 0 && c4.filter_javascript && (pf[k] & C4F_JS)) cd = 4;
    if (cd == 0 && c4.filter_policy && (pf[k] & C4F_POLICY)) cd = 5;
    code[k] = cd;
  });
  x.par.sync();
  const int64_t s_long = x.par.template sum<int64_t>(NLn, [&](uint32_t k) { return (int64_t)(code[k] == 1); });
  const int64_t s_punct = x.par.template sum<int64_t>(NLn, [&](uint32_t k) { return (int64_t)(code[k] == 2); });
  const int64_t s_few = x.par.template sum<int64_t>(NLn, [&](uint32_t k) { return (int64_t)(code[k] == 3); });
  if (wout && hls) {  // words of the rewrite: the kept lines' (see c4_plain_tail)
    const uint32_t wk = x.par.template sum<uint32_t>(NLn, [&](uint32_t k) { return code[k] == 0 ? nw[k] : 0u; });
    x.par.single([&]() { *wout = wk; });
  }
  x.stamp(PH_C4_CODES);
  // ---- joined kept lines (HBM: read back by pass B), scattered per code point ----
  uint32_t* joff = x.template alloc_hot<uint32_t>(NLn + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  uint32_t Jtot = x.par.template scan<uint32_t>(
      NLn, 0u, [](uint32_t a, uint32_t b2) { return a + b2; },
      [&](uint32_t k) { return code[k] == 0 ? plen[k] + 1 : 0u; }, [&](uint32_t k, uint32_t e) { joff[k] = e; });
  if (Jtot > 0) Jtot -= 1;
  uint8_t* Jb = x.template alloc_global<uint8_t>(Jtot + 1);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.par.sync();
  x.par.for_n(C, [&](uint32_t j) {
    const uint32_t nb = kept_bytes(j);
    if (!nb || code[lid[j]] != 0) return;
    const uint32_t k = lid[j];
    uint8_t* d = Jb + joff[k] + (Pw[j] - Pw[la[k]]);
    for (uint32_t q = 0; q < nb; ++q) d[q] = b[off[j] + q];
  });
  x.par.for_n(NLn, [&](uint32_t k) {
    if (code[k] == 0 && joff[k] + plen[k] < Jtot) Jb[joff[k] + plen[k]] = '\n';
  });
  x.par.sync();
  x.stamp(PH_C4_JOIN);
  c4_finish(x, c4, n, Jb, Jtot, s_long, s_punct, s_few, r, src);
}

// ---------------------------------------------------------------------------------------------
// Stage analysis for one content version: writes the records of every step of the stage.

#ifndef TB_HOT_PROPS
#define TB_HOT_PROPS 1
#endif
constexpr bool kHotProps = TB_HOT_PROPS != 0;

// kPre: the document comes with its pre-pass (StageOut::pre: code points, words, runs of '\n');
// a separate instantiation, so the common kernel carries no branch for it (a runtime branch
// doubled the workgroup kernel's register spill).
template <class P, bool kWithLid = true, bool kPre = false>
TB_HD void analyze_stage(DocCtx<P>& x, const DevStage& st, const DevPlan& plan,
                         const LidTables& lid, const uint8_t* b, uint32_t n, StageOut& out) {
  bool need_words = false, need_lines = false, need_ph = false, need_lid = false;
  for (int s = 0; s < st.n_steps; ++s) {
    const int k = st.steps[s].kind;
    if (k == DK_GOPHER_QUALITY) need_words = need_lines = true;
    if (k == DK_GOPHER_REP) need_words = need_ph = true;
    if (k == DK_FINEWEB) need_words = need_lines = need_ph = true;
    if (k == DK_LANGID) need_lid = true;
  }
  x.stamp(PH_START);
  if (out.line_stats) x.par.single([&]() { out.line_stats[0] = kLineStatsNone; });
  uint32_t ndict = 0;
  Cps c;
  if constexpr (kPre) {
    c.n = out.pre->C;
    c.off = out.pre->off;
    c.prop = out.pre->prop;
    c.b = b;
    c.nb = n;
    ndict = out.pre->dict;
  } else {
    c = decode(x, b, n, kHotProps, &ndict);
  }
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.stamp(PH_DECODE);
  const uint32_t C = c.n;
  // Documents with dictionary-segmented scripts go to the ICU path (host): their records are
  // recomputed there, so nothing else is analysed on the device. The language record needs no
  // segmentation and is exact for every script (the device computes it in its own kernel, and a
  // document the language gate filters is not delegated), so the emulation still produces it.
  // Dictionary-script documents: their words come from the host's ICU segmentation (the word
  // marks of the original text), or — for a stage after C4 whose only word reader is FineWeb,
  // which needs just the count — from the word count C4 pass A left for the rewrite. Otherwise
  // (no marks, GopherQuality / GopherRepetition on a rewritten version, a pre-pass document) the
  // document goes to the ICU path (host) and is recomputed there, so nothing else is analysed
  // here. The language record needs no segmentation and is exact for every script (the device
  // computes it in its own kernel, and a document the language gate filters is not delegated),
  // so the emulation still produces it.
  // wfix: the word count a count-only document's FineWeb record takes (kNoWords: none); it is
  // applied after the steps, so no branch on it sits in the analysis (a branch there made the
  // compiler duplicate the step loop: 4x the register spills)
  const uint32_t* dict_marks = nullptr;
  uint32_t wfix = kNoWords;
  if (ndict && need_words) {  // (a stage without word segmentation reads no script-dependent data)
    bool fw_only = true;
    for (int s = 0; s < st.n_steps; ++s)
      fw_only &= st.steps[s].kind != DK_GOPHER_QUALITY && st.steps[s].kind != DK_GOPHER_REP;
    if (!kPre) dict_marks = out.dict.marks(out.doc);
    if (!kPre && !dict_marks && fw_only) wfix = out.dict.nwords(out.doc);
    if (!dict_marks && wfix == kNoWords) {
      if constexpr (kWithLid) {
        for (int s = 0; s < st.n_steps; ++s) {
          const DevStep& ds = st.steps[s];
          if (ds.kind == DK_LANGID && lid.E)
            langid_record(x, b, n, lid, out.rec + (int64_t)ds.rec_prefix * out.ndocs + (int64_t)out.doc * ds.width);
        }
      }
      x.set_flag(DOC_NEEDS_CPU);
      return;
    }
  }
  x.stamp(PH_DICT);
  PHView ph;
  if (need_ph) ph = prefix_hash8(x, b, n);
  x.stamp(PH_PREFIX_HASH);
  Words w;
  if (need_words) {
    w = words(x, c, kPre ? out.pre : nullptr, dict_marks);
  }
  x.stamp(PH_WORDS);
  Lines L;
  if (need_lines) L = rust_lines(x, c);
  if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  x.stamp(PH_RUST_LINES);
  if (out.line_stats && need_words && need_lines) export_line_stats(x, c, w, L, n, out.line_stats);
  x.stamp(PH_LINES);
  const uint32_t W = w.n;
  const PropArr prop = c.props();
  const OffArr off = c.offs();

  // Records are independent: GopherRepetition runs after the other steps so that its n-gram
  // phase (the last user of the code point properties) can hand their LDS to its hash tables.
  int n_gr = 0;
  for (int s = 0; s < st.n_steps; ++s) n_gr += st.steps[s].kind == DK_GOPHER_REP;
  int gr_seen = 0;
  for (int so = 0; so < 2 * st.n_steps; ++so) {
    const int s = so % st.n_steps;
    const DevStep& ds = st.steps[s];
    if ((so < st.n_steps) == (ds.kind == DK_GOPHER_REP)) continue;
    int64_t* r = out.rec + (int64_t)ds.rec_prefix * out.ndocs + (int64_t)out.doc * ds.width;
    if (ds.kind == DK_GOPHER_QUALITY) {
      const DevStopSet& ss = plan.stops[ds.stop_set];
      const UcdView ucd = x.ucd;
      // Counts are packed two per 64-bit sum (each < 2^32: a document is < 4 GiB), so the seven
      // statistics take one pass over the words, one over the code points and one over the lines.
      auto lo32 = [](uint64_t v) { return (int64_t)(v & 0xFFFFFFFFull); };
      auto hi32 = [](uint64_t v) { return (int64_t)(v >> 32); };
      int64_t sum_chars = 0;
      const uint64_t as = x.par.template sum<uint64_t>(W, [&](uint32_t k) {
        const uint32_t a = w.cs[k], e = w.ce[k];
        return ((uint64_t)(e - a) << 32) | ((uint64_t)w.alpha[k] << 16) |
               (uint64_t)is_stop_word(ucd, ss, c, a, e, w.bs[k], w.be[k]);
      });
      // fields: chars (bits 32..63, <= C), alphabetic words (16..31) and stop words (0..15), both
      // <= W; documents with 2^16 words or more are counted field by field
      int64_t alpha, stop;
      if (W < 65536u) {
        sum_chars = hi32(as);
        alpha = (int64_t)((as >> 16) & 0xFFFFull);
        stop = (int64_t)(as & 0xFFFFull);
      } else {
        sum_chars = x.par.template sum<int64_t>(W, [&](uint32_t k) { return (int64_t)(w.ce[k] - w.cs[k]); });
        alpha = x.par.template sum<int64_t>(W, [&](uint32_t k) { return (int64_t)w.alpha[k]; });
        stop = x.par.template sum<int64_t>(W, [&](uint32_t k) {
          return (int64_t)is_stop_word(ucd, ss, c, w.cs[k], w.ce[k], w.bs[k], w.be[k]);
        });
      }
      x.stamp(PH_GQ_WORDS);
      // the same counts over the bytes ('#' and '.' are ASCII, U+2026 is E2 80 A6 and E2 is
      // always a lead byte): no code point offset loads, four bytes per SWAR test
      // (workgroup documents: the per-byte form, the SWAR groups cost their kernels ~50 spilled VGPRs)
      const uint64_t he = P::kWaves <= 1 ? gq_byte_counts(x, b, n) : x.par.template sum<uint64_t>(n, [&](uint32_t i) {
        const uint32_t c0 = b[i];
        if (c0 == '#') return (uint64_t)1 << 32;
        if (c0 == 0xE2) return (uint64_t)(i + 2 < n && b[i + 1] == 0x80 && b[i + 2] == 0xA6);
        if (c0 != '.' || (i > 0 && b[i - 1] == '.')) return (uint64_t)0;
        uint32_t j = i;
        while (j < n && b[j] == '.') ++j;
        return (uint64_t)((j - i) / 3);
      });
      x.stamp(PH_GQ_BYTES);
      const int64_t nhash = hi32(he), nell = lo32(he);
      const uint64_t be = x.par.template sum<uint64_t>(L.n, [&](uint32_t k) {
        const uint32_t ls = L.ls[k], le = L.le[k];
        uint32_t j = ls;
        while (j < le && is_ws(prop[j])) ++j;
        const uint32_t l0 = j < le ? c.lead(j) : 0u;
        const uint64_t bul = (l0 == '-' || (l0 == 0xE2 && c.cp(j) == 0x2022)) ? 1 : 0;
        j = le;
        while (j > ls && is_ws(prop[j - 1])) --j;
        const uint32_t E = off[j], S = off[ls];
        uint64_t ell = 0;
        if (E - S >= 3) {
          const bool dots = b[E - 3] == '.' && b[E - 2] == '.' && b[E - 1] == '.';
          const bool uell = b[E - 3] == 0xE2 && b[E - 2] == 0x80 && b[E - 1] == 0xA6;
          ell = (dots || uell) ? 1 : 0;
        }
        return (bul << 32) | ell;
      });
      const int64_t bullet = hi32(be), ell_lines = lo32(be);
      x.par.single([&]() {
        r[0] = W; r[1] = sum_chars; r[2] = nhash; r[3] = nell; r[4] = L.n;
        r[5] = bullet; r[6] = ell_lines; r[7] = alpha; r[8] = stop;
      });
      x.stamp(PH_GQ);
    } else if (ds.kind == DK_GOPHER_REP) {
      ++gr_seen;
      gopher_rep_record(x, ds, b, c, ph, w, r, kHotProps && gr_seen == n_gr, n_gr == 1 ? out.gr_export : nullptr,
                        kPre ? out.pre : nullptr, out.b_global, L);
    } else if (ds.kind == DK_FINEWEB) {
      const auto mark = x.mark();
      uint32_t* nb = x.template alloc<uint32_t>(L.n + 1);
      if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
      const uint32_t NB = x.par.template compact<int>(
          L.n,
          [&](uint32_t k, int&) {
            for (uint32_t j = L.ls[k]; j < L.le[k]; ++j) if (!is_ws(prop[j])) return true;
            return false;
          },
          [&](uint32_t k, uint32_t q, int&) { nb[q] = k; });
      x.par.sync();
      int64_t stop_end = x.par.template sum<int64_t>(NB, [&](uint32_t q) {
        uint32_t k = nb[q];
        uint32_t j = L.le[k];
        while (j > L.ls[k] && is_ws(prop[j - 1])) --j;
        uint32_t last = c.cp(j - 1);
        for (int t = 0; t < ds.n_stop_chars; ++t) if (ds.stop_chars[t] == last) return (int64_t)1;
        return (int64_t)0;
      });
      int64_t shrt = x.par.template sum<int64_t>(NB, [&](uint32_t q) {
        uint32_t k = nb[q];
        return (int64_t)((int64_t)(L.le[k] - L.ls[k]) <= ds.short_line_length);
      });
      int64_t dup_e = 0, dup_b = 0;
      dup_spans(x, b, ph, NB,
                [&](uint32_t q, uint32_t& s0, uint32_t& e0) { s0 = off[L.ls[nb[q]]]; e0 = off[L.le[nb[q]]]; },
                &dup_e, &dup_b);
      int64_t nl = x.par.template sum<int64_t>(C, [&](uint32_t i) { return (int64_t)c.is_lf(i); });
      x.par.single([&]() {
        r[0] = NB; r[1] = stop_end; r[2] = shrt; r[3] = dup_b; r[4] = (int64_t)C - nl; r[5] = nl; r[6] = W;
      });
      x.reset(mark);
      x.stamp(PH_FW);
    } else if (ds.kind == DK_LANGID) {
      // on the device this runs as a separate kernel (k_langid_mfma): lid.E == nullptr
      if constexpr (kWithLid)
        if (lid.E) langid_record(x, b, n, lid, r);
      x.stamp(PH_LID);
    }
    if (x.overflow) { x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); return; }
  }
  if (wfix != kNoWords) {
    // a count-only document (dictionary script, FineWeb after C4): its words were segmented by the
    // rules above; FineWeb's word count is C4's ICU-based one, and its line export is withdrawn
    x.par.sync();
    x.par.single([&]() {
      for (int s = 0; s < st.n_steps; ++s) {
        const DevStep& ds = st.steps[s];
        if (ds.kind == DK_FINEWEB) out.rec[(int64_t)ds.rec_prefix * out.ndocs + (int64_t)out.doc * ds.width + 6] = wfix;
      }
      if (out.line_stats) out.line_stats[0] = kLineStatsNone;
    });
  }
}

}  // namespace tb
