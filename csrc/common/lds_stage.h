// LDS-resident stage analysis for short documents (one wavefront per document, every working
// array in the wave's LDS slice, no HBM scratch): the records of GopherQuality, GopherRepetition
// and FineWeb steps, bit-identical to analyze_stage (docproc.h), from a different memory design.
//
// Why a second implementation: analyze_stage addresses its arrays through generic pointers that
// may point to LDS or to the HBM scratch arena, so every access is a FLAT instruction that waits
// on both the LDS and the vector-memory counters, and the per-code-point arrays (words, lines,
// n-gram keys) spill to HBM: the round-2 profile measured 928 flat instructions in the kernel
// body and 58.7% of wave cycles waiting (profiles/r3_start/pmc_per_kernel.txt). Here
//   * every array is an address-space-3 pointer (TB_LDS): ds_read/ds_write only;
//   * arrays are sized by the counts they hold (words, lines, newline runs) and packed in 16-bit
//     fields (documents are < 64 KiB): words are one u32 (byte start | byte end << 16);
//   * span equality keys are hashed straight from the LDS text (no prefix-hash table);
//   * duplicated n-gram keys use a bigram-sum key over the concatenated words (a prefix sum per
//     word: no modular powers), and every requested order is canonicalised in ONE shared table
//     pass (orders grouped only when the slice is short);
//   * a document whose arrays do not fit its slice is not spilled: the kernel reports it, and the
//     generic kernel (analyze_stage over HBM scratch) recomputes it.
// The algorithm is templated on the parallel policy, so the host runs it sequentially
// (emulate_stage_lds) and CPU tests compare it with analyze_stage record for record.
//
// Reference hot loops: src/utils/text.rs:184-259 (find_duplicates / find_top_duplicate /
// find_all_duplicate), src/pipeline/filters/gopher_rep.rs:52-220, gopher_quality.rs:69-187,
// fineweb_quality.rs:71-189.
#pragma once
#include "docproc.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define TB_LDS __attribute__((address_space(3)))
#else
#define TB_LDS
#endif

namespace tb {

constexpr uint32_t kLdsMaxDoc = 65535;  // 16-bit byte offsets
#ifndef TB_LDS_SCAN_WORDS
#define TB_LDS_SCAN_WORDS 0
#endif
// 1: the segmented-scan word pass for every policy (A/B against the chunked-ballot pass)
constexpr bool kLdsScanWords = TB_LDS_SCAN_WORDS != 0;

// ---- LDS atomics (relaxed, workgroup scope; lanes of one instruction serialise per address) ----
TB_HD uint32_t l_cas(TB_LDS uint32_t* p, uint32_t cmp, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return cmp;
#else
  const uint32_t o = *p;
  if (o == cmp) *p = v;
  return o;
#endif
}
TB_HD void l_min(TB_LDS uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  if (v < *p) *p = v;
#endif
}
TB_HD void l_add(TB_LDS uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  *p += v;
#endif
}
TB_HD void l_or(TB_LDS uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  *p |= v;
#endif
}

// Little-endian u32 of bytes [i, i+4) of a 4-aligned LDS text (padded with >= 8 zero bytes).
TB_HD uint32_t l_ld32(TB_LDS const uint8_t* b, uint32_t i) {
  const uint32_t a = i & ~3u, sh = i & 3u;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = *(TB_LDS const uint32_t*)(b + a);
  if (!sh) return lo;
  const uint32_t hi = *(TB_LDS const uint32_t*)(b + a + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, sh);  // byte shift
#else
  uint64_t v = 0;
  __builtin_memcpy(&v, b + a, 8);
  return (uint32_t)(v >> (8 * sh));
#endif
}

TB_HD uint32_t l_utf8_decode(TB_LDS const uint8_t* s, uint32_t i, uint32_t n, int* len) {
  const uint32_t c = s[i];
  if (c < 0x80) { *len = 1; return c; }
  if ((c >> 5) == 6 && i + 1 < n) { *len = 2; return ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); }
  if ((c >> 4) == 14 && i + 2 < n) {
    *len = 3;
    return ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
  }
  if (i + 3 < n) {
    *len = 4;
    return ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
  }
  *len = 1;
  return 0xFFFD;
}

// 64-bit key of the bytes [s, e): equal byte strings have equal keys (hash table grouping; every
// match is verified with l_bytes_eq). Four bytes per step from two aligned LDS reads.
TB_HD uint64_t l_span_key(TB_LDS const uint8_t* b, uint32_t s, uint32_t e) {
  uint64_t h = 0x243F6A8885A308D3ull ^ ((uint64_t)(e - s) * 0x9E3779B97F4A7C15ull);
  uint32_t i = s;
  auto step = [&](uint32_t u) {
    h ^= u;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 31;
  };
  // 16 bytes per iteration: four independent LDS reads in flight before the (serial) mixing
  for (; i + 16 <= e; i += 16) {
    const uint32_t u0 = l_ld32(b, i), u1 = l_ld32(b, i + 4), u2 = l_ld32(b, i + 8), u3 = l_ld32(b, i + 12);
    step(u0);
    step(u1);
    step(u2);
    step(u3);
  }
  for (; i + 4 <= e; i += 4) step(l_ld32(b, i));
  if (i < e) {
    const uint32_t r = e - i;
    h ^= (uint64_t)(l_ld32(b, i) & (0xFFFFFFFFu >> (32 - 8 * r))) | ((uint64_t)r << 40);
    h *= 0xc4ceb9fe1a85ec53ull;
  }
  return mix64(h) | 1ull;
}

TB_HD bool l_bytes_eq(TB_LDS const uint8_t* b, uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
  if (a1 - a0 != b1 - b0) return false;
  const uint32_t n = a1 - a0;
  uint32_t i = 0;
  for (; i + 16 <= n; i += 16) {
    const uint32_t d = (l_ld32(b, a0 + i) ^ l_ld32(b, b0 + i)) | (l_ld32(b, a0 + i + 4) ^ l_ld32(b, b0 + i + 4)) |
                       (l_ld32(b, a0 + i + 8) ^ l_ld32(b, b0 + i + 8)) |
                       (l_ld32(b, a0 + i + 12) ^ l_ld32(b, b0 + i + 12));
    if (d) return false;
  }
  for (; i + 4 <= n; i += 4)
    if (l_ld32(b, a0 + i) != l_ld32(b, b0 + i)) return false;
  if (i < n) {
    const uint32_t m = 0xFFFFFFFFu >> (32 - 8 * (n - i));
    if ((l_ld32(b, a0 + i) & m) != (l_ld32(b, b0 + i) & m)) return false;
  }
  return true;
}

// Bigram term of the duplicated n-gram keys (murmur3 fmix32: a bijection, so distinct byte pairs
// give distinct terms).
TB_HD uint32_t l_pair(uint32_t x, uint32_t y) {
  uint32_t h = ((x << 8) | y) + 0x7F4A7C15u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// Bump allocator over the wave's LDS slice: `lo` grows up (arrays that live to the end of a
// phase), `hi` grows down (short-lived tables and the code point array, released as a stack).
struct LArena {
  TB_LDS char* base = nullptr;
  uint32_t cap = 0, lo = 0, hi = 0;
  bool ovf = false;
  template <class T>
  TB_HD TB_LDS T* get(uint32_t count) {
    const uint32_t a = (lo + 7u) & ~7u;
    const uint64_t e = (uint64_t)a + (uint64_t)count * sizeof(T);
    if (e + hi > cap) {
      ovf = true;
      return (TB_LDS T*)base;
    }
    lo = (uint32_t)e;
    return (TB_LDS T*)(base + a);
  }
  template <class T>
  TB_HD TB_LDS T* get_hi(uint32_t count) {
    const uint64_t bytes = ((uint64_t)count * sizeof(T) + 7u) & ~7ull;
    if ((uint64_t)((lo + 7u) & ~7u) + hi + bytes > cap) {
      ovf = true;
      return (TB_LDS T*)base;
    }
    hi += (uint32_t)bytes;
    return (TB_LDS T*)(base + (cap - hi));
  }
  TB_HD uint32_t free_bytes() const {
    const uint32_t a = (lo + 7u) & ~7u;
    return a + hi >= cap ? 0u : cap - a - hi;
  }
  struct Mark { uint32_t lo, hi; };
  TB_HD Mark mark() const { return Mark{lo, hi}; }
  TB_HD void reset(Mark m) { lo = m.lo; hi = m.hi; }
};

template <class P>
struct LCtx {
  P par;
  LArena a;
  UcdView ucd;
  TB_LDS const uint16_t* asc = nullptr;  // compact properties of the ASCII code points
  uint32_t* flag = nullptr;              // per-document status word (global)
  uint64_t* prof = nullptr;
  uint64_t t_last = 0;
  TB_HD void stamp(int id) {
    if (!prof) return;
    const uint64_t t = P::clock();
    if (t_last && par.leader()) prof[id] += t - t_last;
    t_last = t;
  }
  TB_HD void set_flag(uint32_t f) {
    if (flag) P::or32(flag, f);
  }
};

enum : int { LDS_OK = 0, LDS_RETRY = 1 };

// Code points of the LDS text: ent[i] = byte offset | compact properties << 16 (ent[C] = n).
struct LCps {
  uint32_t n = 0;  // code points
  TB_LDS const uint32_t* ent = nullptr;
  TB_LDS const uint8_t* b = nullptr;
  uint32_t nb = 0;
  TB_HD uint32_t o(uint32_t i) const { return ent[i] & 0xFFFFu; }
  TB_HD uint32_t p(uint32_t i) const { return ent[i] >> 16; }
  TB_HD uint32_t lead(uint32_t i) const { return b[o(i)]; }
  TB_HD uint32_t cp(uint32_t i) const {
    int len;
    return l_utf8_decode(b, o(i), nb, &len);
  }
};
struct LAcc {  // UAX#29 rule accessor (uax29.h)
  TB_LDS const uint32_t* ent;
  TB_HD uint32_t p(int i) const { return ent[i] >> 16; }
};

template <class P>
TB_HD uint32_t l_decode(LCtx<P>& x, TB_LDS const uint8_t* b, uint32_t n, TB_LDS uint32_t* ent, uint32_t* dict) {
  uint32_t dl = 0;
  const uint32_t C = x.par.template compact<int>(
      n, [&](uint32_t i, int&) { return utf8_is_lead(b[i]); },
      [&](uint32_t i, uint32_t k, int&) {
        const uint32_t c0 = b[i];
        uint32_t p16;
        if (c0 < 0x80u) {
          p16 = x.asc[c0];
        } else {
          int len;
          const uint32_t p = x.ucd.props(l_utf8_decode(b, i, n, &len));
          dl |= (p & P_DICT) ? 1u : 0u;
          p16 = compact_prop(p);
        }
        ent[k] = i | (p16 << 16);
      });
  x.par.single([&]() { ent[C] = n; });
  *dict = x.par.reduce_or(dl);
  x.par.sync();
  return C;
}

// Stop-word test of a word given by its bytes [s, e) and its code point count (gopher_quality.rs
// lowercases the word: Rust str::to_lowercase, final sigma included).
template <class F>
TB_HD void l_lower_bytes(const UcdView& ucd, TB_LDS const uint8_t* b, uint32_t nb, uint32_t s, uint32_t e, F&& push) {
  for (uint32_t i = s; i < e;) {
    int len;
    const uint32_t c = l_utf8_decode(b, i, nb, &len);
    uint32_t lc;
    if (c == 0x3A3) {
      bool before = false, after = false;
      for (uint32_t j = i; j > s;) {  // previous code points of the word
        uint32_t q = j - 1;
        while (q > s && !utf8_is_lead(b[q])) --q;
        int l2;
        const uint32_t p = ucd.props(l_utf8_decode(b, q, nb, &l2));
        j = q;
        if (p & P_CASE_IGN) continue;
        before = (p & P_CASED) != 0;
        break;
      }
      for (uint32_t j = i + (uint32_t)len; j < e;) {
        int l2;
        const uint32_t p = ucd.props(l_utf8_decode(b, j, nb, &l2));
        j += (uint32_t)l2;
        if (p & P_CASE_IGN) continue;
        after = (p & P_CASED) != 0;
        break;
      }
      lc = (before && !after) ? 0x3C2 : 0x3C3;
    } else {
      lc = ucd.lower(c);
    }
    // UTF-8 of lc straight into push (no byte array: a dynamically indexed array would live in
    // scratch memory)
    if (lc < 0x80) {
      push((uint8_t)lc);
    } else if (lc < 0x800) {
      push((uint8_t)(0xC0 | (lc >> 6)));
      push((uint8_t)(0x80 | (lc & 0x3F)));
    } else if (lc < 0x10000) {
      push((uint8_t)(0xE0 | (lc >> 12)));
      push((uint8_t)(0x80 | ((lc >> 6) & 0x3F)));
      push((uint8_t)(0x80 | (lc & 0x3F)));
    } else {
      push((uint8_t)(0xF0 | (lc >> 18)));
      push((uint8_t)(0x80 | ((lc >> 12) & 0x3F)));
      push((uint8_t)(0x80 | ((lc >> 6) & 0x3F)));
      push((uint8_t)(0x80 | (lc & 0x3F)));
    }
    if (c == 0x130) { push(0xCC); push(0x87); }
    i += (uint32_t)len;
  }
}

TB_HD bool l_is_stop(const UcdView& ucd, const DevStopSet& ss, TB_LDS const uint8_t* b, uint32_t nb, uint32_t s,
                     uint32_t e, uint32_t ncp) {
  if (ss.n == 0 || (int32_t)ncp > ss.max_len) return false;
  uint64_t h = 0;
  uint32_t len = 0;
  l_lower_bytes(ucd, b, nb, s, e, [&](uint8_t v) { h = hash_push(h, v); ++len; });
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
      l_lower_bytes(ucd, b, nb, s, e, [&](uint8_t v) { ok = ok && ss.blob[pos++] == v; });
      return ok;
    }
    slot = (slot + 1) & (kStopTableSize - 1);
  }
}

// The stop-word set in the wave's slice (DevStopSet lite form): slots, word offsets, words.
struct LStop {
  uint32_t nslots = 0;
  int32_t max_len = 0;
  TB_LDS const uint64_t* fast = nullptr;
  TB_LDS const uint32_t* slots = nullptr;
  TB_LDS const uint16_t* off = nullptr;
  TB_LDS const uint8_t* blob = nullptr;
};

template <class P>
TB_HD bool l_stop_load(LCtx<P>& x, const DevStopSet& ss, LStop& out) {
  const uint32_t ns = (uint32_t)ss.lite_nslots, nw = (uint32_t)ss.n, nb = (uint32_t)ss.off[nw];
  TB_LDS uint64_t* fk = x.a.template get<uint64_t>(ns);
  TB_LDS uint32_t* sl = x.a.template get<uint32_t>(ns);
  TB_LDS uint16_t* of = x.a.template get<uint16_t>(nw + 1);
  TB_LDS uint8_t* bl = x.a.template get<uint8_t>(nb + 1);
  if (x.a.ovf) return false;
  x.par.for_n(ns, [&](uint32_t i) {
    sl[i] = ss.lite_slots[i];
    fk[i] = ss.fast_keys[i];
  });
  x.par.for_n(nw + 1, [&](uint32_t i) { of[i] = (uint16_t)ss.off[i]; });
  x.par.for_n(nb, [&](uint32_t i) { bl[i] = ss.blob[i]; });
  x.par.sync();
  out.nslots = ns;
  out.max_len = ss.max_len;
  out.slots = sl;
  out.fast = fk;
  out.off = of;
  out.blob = bl;
  return true;
}

// Is the lowercased word (bytes [s, e), ncp code points) in the set?
TB_HD bool l_is_stop_lite(const UcdView& ucd, const LStop& st, TB_LDS const uint8_t* b, uint32_t nb, uint32_t s,
                          uint32_t e, uint32_t ncp) {
  if (st.nslots == 0 || (int32_t)ncp > st.max_len) return false;
  if (e - s <= 7) {
    // ASCII words of <= 7 bytes: lowercase 8 bytes at once (SWAR) and look the key up
    const uint32_t len = e - s;
    uint64_t v = (uint64_t)l_ld32(b, s) | ((uint64_t)l_ld32(b, s + 4) << 32);
    v &= len ? (~0ull >> (64 - 8 * len)) : 0ull;
    if ((v & 0x8080808080808080ull) == 0) {
      const uint64_t hb = 0x8080808080808080ull;
      const uint64_t ge_a = (v | hb) - 0x4141414141414141ull;  // high bit: byte >= 'A'
      const uint64_t ge_z = (v | hb) - 0x5B5B5B5B5B5B5B5Bull;  // high bit: byte > 'Z'
      const uint64_t up = ge_a & ~ge_z & hb;
      const uint64_t key = (v | (up >> 2)) | ((uint64_t)len << 56);
      uint32_t slot = stop_fast_slot(key, st.nslots);
      while (true) {
        const uint64_t k = st.fast[slot];
        if (k == key) return true;
        if (k == 0) return false;
        slot = (slot + 1) & (st.nslots - 1);
      }
    }
  }
  uint32_t h = kStopLiteHash0, len = 0;
  l_lower_bytes(ucd, b, nb, s, e, [&](uint8_t v) { h = stop_lite_hash_push(h, v); ++len; });
  uint32_t slot = stop_lite_slot(h, st.nslots);
  while (true) {
    const uint32_t en = st.slots[slot];
    if (en == 0) return false;
    if ((en >> 16) == (h >> 16)) {
      const uint32_t w = (en & 0xFFFFu) - 1;
      const uint32_t o0 = st.off[w], o1 = st.off[w + 1];
      if (o1 - o0 == len) {
        uint32_t pos = o0;
        bool ok = true;
        l_lower_bytes(ucd, b, nb, s, e, [&](uint8_t v) { ok = ok && st.blob[pos++] == v; });
        if (ok) return true;
      }
    }
    slot = (slot + 1) & (st.nslots - 1);
  }
}

// canon[i] = smallest j < N with item j == item i, N < 43000 (16-bit slots and indices; an item
// whose key is 0 is not inserted and stays its own class). Open
// addressing in an LDS table of 1.5 N + 2 packed slots (16-bit fingerprint | index + 1; 0 empty);
// a fingerprint match joins a slot only after eq() confirms it (exact grouping), a 32-bit atomic
// min keeps the smallest index. The table lives on the hi stack for the duration of the call.
template <class P, class KeyF, class EqF>
TB_HD bool l_canon(LCtx<P>& x, uint32_t N, KeyF&& key, EqF&& eq, TB_LDS uint16_t* canon) {
  if (N == 0) return true;
  if (N >= 43000u) return false;  // 16-bit slot numbers
  const auto m = x.a.mark();
  const uint32_t capn = N + (N >> 1) + 2;
  TB_LDS uint32_t* tab = x.a.template get_hi<uint32_t>(capn);
  if (x.a.ovf) return false;
  x.par.for_n(capn, [&](uint32_t i) { tab[i] = 0; });
  x.par.sync();
  x.par.for_n(N, [&](uint32_t i) {
    const uint64_t k = key(i);
    if (k == 0) {  // not an item: its own class
      canon[i] = 0xFFFFu;
      return;
    }
    const uint32_t fp = (uint32_t)(k >> 48);
    const uint32_t mine = (fp << 16) | (i + 1);
    uint32_t slot = (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
    while (true) {
      uint32_t cur = tab[slot];
      if (cur == 0) {
        cur = l_cas(&tab[slot], 0u, mine);
        if (cur == 0) break;
      }
      if ((cur >> 16) == fp && eq(i, (cur & 0xFFFFu) - 1u)) {
        l_min(&tab[slot], mine);
        break;
      }
      if (++slot == capn) slot = 0;
    }
    canon[i] = (uint16_t)slot;
  });
  x.par.sync();
  x.par.for_n(N, [&](uint32_t i) {
    const uint32_t sl = canon[i];
    canon[i] = (uint16_t)(sl == 0xFFFFu ? i : (tab[sl] & 0xFFFFu) - 1u);
  });
  x.par.sync();
  x.a.reset(m);
  return true;
}

// Classes of N items without the resolve pass: cls[i] = the table slot of i's class (a
// canonical identifier: equal items <-> equal slot, < capn), and cnt[slot] = the class size.
// tab / cnt hold >= capn = N + N/2 + 2 entries (the caller's arrays).
template <class P, class KeyF, class EqF>
TB_HD void l_classes(LCtx<P>& x, uint32_t N, KeyF&& key, EqF&& eq, TB_LDS uint32_t* tab, TB_LDS uint32_t* cnt,
                     TB_LDS uint16_t* cls) {
  const uint32_t capn = N + (N >> 1) + 2;
  x.par.for_n(capn, [&](uint32_t i) {
    tab[i] = 0;
    cnt[i] = 0;
  });
  x.par.sync();
  x.par.for_n(N, [&](uint32_t i) {
    const uint64_t k = key(i);
    const uint32_t fp = (uint32_t)(k >> 48);
    const uint32_t mine = (fp << 16) | (i + 1);
    uint32_t slot = (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
    while (true) {
      uint32_t cur = tab[slot];
      if (cur == 0) {
        cur = l_cas(&tab[slot], 0u, mine);
        if (cur == 0) break;
      }
      if ((cur >> 16) == fp && eq(i, (cur & 0xFFFFu) - 1u)) break;
      if (++slot == capn) slot = 0;
    }
    l_add(&cnt[slot], 1u);
    cls[i] = (uint16_t)slot;
  });
  x.par.sync();
}

// find_duplicates over N byte spans: (#repeats, sum of repeat byte lengths).
template <class P, class SpanF>
TB_HD bool l_dup_spans(LCtx<P>& x, TB_LDS const uint8_t* b, uint32_t N, SpanF&& span, int64_t* elems, int64_t* bytes) {
  const auto m = x.a.mark();
  TB_LDS uint16_t* canon = x.a.template get_hi<uint16_t>(N + 1);
  if (x.a.ovf) return false;
  const bool ok = l_canon(
      x, N,
      [&](uint32_t i) {
        uint32_t s, e;
        span(i, s, e);
        return l_span_key(b, s, e);
      },
      [&](uint32_t i, uint32_t j) {
        uint32_t s0, e0, s1, e1;
        span(i, s0, e0);
        span(j, s1, e1);
        return l_bytes_eq(b, s0, e0, s1, e1);
      },
      canon);
  if (!ok) return false;
  const uint64_t v = x.par.template sum<uint64_t>(N, [&](uint32_t i) {
    if (canon[i] == i) return (uint64_t)0;
    uint32_t s, e;
    span(i, s, e);
    return ((uint64_t)1 << 40) | (uint64_t)(e - s);  // count in the high bits (bytes < 2^40)
  });
  *elems = (int64_t)(v >> 40);
  *bytes = (int64_t)(v & ((1ull << 40) - 1));
  x.a.reset(m);
  return true;
}

// Greedy duplicated-n-gram walk of one order (see dup_walk in docproc.h), LDS arrays.
TB_HD int64_t l_dup_walk(uint32_t G, uint32_t n, TB_LDS const uint16_t* gc, uint32_t stride, TB_LDS const uint32_t* R,
                         TB_LDS uint32_t* sn, TB_LDS const uint16_t* WL) {
  const uint32_t nw = (G + 31) >> 5;
  auto next_rep = [&](uint32_t from) -> uint32_t {
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
    const uint32_t g = gc[idx * stride];
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

// Words of the code points: W, and (optionally) their byte spans and the GopherQuality word sums.
struct LWords {
  uint32_t n = 0;
  TB_LDS uint32_t* w = nullptr;  // byte start | byte end << 16
  int64_t chars = 0, alpha = 0, stop = 0;
};

template <class P>
TB_HD bool l_words_chunks(LCtx<P>& x, const LCps& c, bool store, const DevStopSet* ss, LWords& out, bool use_lite,
                          LStop lite);

template <class P>
TB_HD bool l_words(LCtx<P>& x, const LCps& c, bool store, const DevStopSet* ss, LWords& out,
                   bool use_lite = false, LStop lite = LStop{}) {
  if constexpr (P::kChunks) {
    if (!kLdsScanWords) return l_words_chunks(x, c, store, ss, out, use_lite, lite);
  }
  const uint32_t C = c.n;
  const auto m = x.a.mark();
  TB_LDS uint32_t* wbm = x.a.template get_hi<uint32_t>(mask_words(C + 1));
  if (x.a.ovf) return false;
  const LAcc acc{c.ent};
  // the window i-2 .. i+1 comes from four independent LDS reads; the look-around of wb_break
  // runs only where the window holds Extend/Format/ZWJ/RI
  x.par.mask_store(
      C + 1,
      [&](uint32_t i) {
        if (i == 0 || i >= C) return true;
        const uint32_t pm2 = i >= 2 ? c.p(i - 2) : 0xFFFFFFFFu;
        const uint32_t pp1 = i + 1 < C ? c.p(i + 1) : 0xFFFFFFFFu;
        const int r = wb_break_ctx(pm2, c.p(i - 1), c.p(i), pp1);
        return r == 2 ? wb_break(acc, (int)C, (int)i) : r != 0;
      },
      [&](uint32_t w, uint32_t v) { wbm[w] = v; });
  x.par.sync();
  x.stamp(PH_W_MASK);
  auto bit = [&](uint32_t i) { return (wbm[i >> 5] >> (i & 31)) & 1u; };
  TB_LDS uint32_t* words = nullptr;
  if (store) {
    // W <= segments = set bits - 1 (the breaks at 0 and C are both set)
    const uint32_t nseg = x.par.template sum<uint32_t>(mask_words(C + 1), [&](uint32_t w) {
      return (uint32_t)__builtin_popcount(wbm[w]);
    });
    // words go below the break mask: allocated from `lo` after the mask is done with `hi`
    words = x.a.template get<uint32_t>(nseg + 1);
    if (x.a.ovf) return false;
  }
  const uint32_t nb = c.nb;
  TB_LDS const uint8_t* b = c.b;
  uint32_t chars = 0, alpha = 0, stop = 0;
  const UcdView ucd = x.ucd;
  out.n = x.par.template scan_compact<WSeg>(
      C, WSeg{0u, 0xFFFFFFFFu, 0u}, wseg_op,
      [&](uint32_t j) {
        const uint32_t p = c.p(j);
        const bool ws = is_ws(p);
        WSeg e;
        e.bits = bit(j) | ((!(p & P_PUNCT) && !ws) ? 2u : 0u) | ((p & P_ALPHA) ? 4u : 0u);
        e.first = ws ? 0xFFFFFFFFu : j;
        e.last = ws ? 0u : j + 1;
        return e;
      },
      [&](uint32_t j, const WSeg& in) { return bit(j + 1) && (in.bits & 2u); },
      [&](uint32_t, uint32_t k, const WSeg& in) {
        const uint32_t bs = c.o(in.first), be = c.o(in.last);
        if (store) words[k] = bs | (be << 16);
        if (ss) {
          chars += in.last - in.first;
          alpha += (in.bits & 4u) ? 1u : 0u;
          const bool st = use_lite ? l_is_stop_lite(ucd, lite, b, nb, bs, be, in.last - in.first)
                               : l_is_stop(ucd, *ss, b, nb, bs, be, in.last - in.first);
          stop += st ? 1u : 0u;
        }
      });
  if (ss) {
    out.chars = x.par.reduce_add((int64_t)chars);
    out.alpha = x.par.reduce_add((int64_t)alpha);
    out.stop = x.par.reduce_add((int64_t)stop);
  }
  x.par.sync();
  // release the mask (the words, if stored, stay: they were allocated after the mark's lo)
  x.a.hi = m.hi;
  out.w = words;
  return true;
}

// l_words by chunked ballots (policies with P::kChunks): per chunk of 64 code points four
// 64-bit masks (break before, non-whitespace, word char, alphabetic) and per-lane bit arithmetic
// replace the segmented scan over a 12-byte state: a word is a segment (between consecutive
// breaks) with a word char, trimmed to its first and last non-whitespace code point. The segment
// still open at a chunk's end is carried in uniform state. Pass 1 finds the breaks (stored as a
// bitmask) and counts the words (one per segment: its first word char); pass 2 emits them.
TB_HD uint64_t lmask(uint32_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }  // bits [0, k)
TB_HD uint32_t hibit(uint64_t v) { return 63u - (uint32_t)__builtin_clzll(v); }
TB_HD uint32_t lobit(uint64_t v) { return (uint32_t)__builtin_ctzll(v); }

template <class P>
TB_HD bool l_words_chunks(LCtx<P>& x, const LCps& c, bool store, const DevStopSet* ss, LWords& out, bool use_lite,
                          LStop lite) {
  const uint32_t C = c.n;
  const auto m = x.a.mark();
  const uint32_t nwm = mask_words(C + 1);
  TB_LDS uint32_t* wbm = x.a.template get_hi<uint32_t>(nwm);
  if (x.a.ovf) return false;
  const LAcc acc{c.ent};
  // ---- pass 1: break mask + word count ----
  bool open_wc = false;
  const uint32_t W = x.par.chunks(
      C,
      [&](uint32_t i) -> uint32_t {
        const uint32_t p0 = c.p(i);
        bool brk = true;
        if (i > 0) {
          const uint32_t pm2 = i >= 2 ? c.p(i - 2) : 0xFFFFFFFFu;
          const uint32_t pp1 = i + 1 < C ? c.p(i + 1) : 0xFFFFFFFFu;
          const int r = wb_break_ctx(pm2, c.p(i - 1), p0, pp1);
          brk = r == 2 ? wb_break(acc, (int)C, (int)i) : r != 0;
        }
        const bool ws = is_ws(p0);
        const bool wc = !(p0 & P_PUNCT) && !ws;
        return (brk ? 1u : 0u) | (wc ? 2u : 0u);
      },
      [&](uint32_t, uint32_t l, const uint64_t* mm) {  // the first word char of its segment
        if (!((mm[1] >> l) & 1u)) return false;
        const uint64_t below = mm[0] & lmask(l + 1);
        if (below) return (mm[1] & lmask(l) & ~lmask(hibit(below))) == 0;
        return !open_wc && (mm[1] & lmask(l)) == 0;
      },
      [&](uint32_t, uint32_t, const uint64_t*, uint32_t) {},
      [&](uint32_t base, const uint64_t* mm) {
        x.par.single([&]() {
          wbm[base >> 5] = (uint32_t)mm[0];
          wbm[(base >> 5) + 1] = (uint32_t)(mm[0] >> 32);
        });
        if (mm[0]) open_wc = (mm[1] & ~lmask(hibit(mm[0]))) != 0;
        else open_wc = open_wc || mm[1] != 0;
      });
  x.par.single([&]() {  // the end-of-text break (bit C), in a word pass 1 may not have written
    if ((C & 63u) == 0) {
      wbm[C >> 5] = 0;
      wbm[(C >> 5) + 1] = 0;
    }
    wbm[C >> 5] |= 1u << (C & 31);
  });
  x.par.sync();
  x.stamp(PH_W_MASK);
  TB_LDS uint32_t* words = nullptr;
  if (store) {
    words = x.a.template get<uint32_t>(W + 1);
    if (x.a.ovf) return false;
  }
  // ---- pass 2: emit (spans, GopherQuality sums) ----
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  uint32_t o_first = kNone, o_last = 0;
  bool o_wc = false, o_al = false;
  const uint32_t nb = c.nb;
  TB_LDS const uint8_t* b = c.b;
  uint32_t chars = 0, alpha = 0, stop = 0;
  const UcdView ucd = x.ucd;
  auto bmask = [&](uint32_t base) {
    return (uint64_t)wbm[base >> 5] | ((uint64_t)wbm[(base >> 5) + 1] << 32);
  };
  auto next_brk = [&](uint32_t base) { return base + 64 <= C ? (wbm[(base + 64) >> 5] & 1u) : 1u; };
  // the segment ending at lane l: first / last non-whitespace code point, word char, alphabetic
  auto segment = [&](uint32_t base, uint32_t l, const uint64_t* mm, uint32_t& first, uint32_t& last, bool& wc,
                     bool& al) {
    const uint64_t B = bmask(base);
    const uint64_t below = B & lmask(l + 1);
    const bool carried = below == 0;
    const uint64_t seg = lmask(l + 1) & (carried ? ~0ull : ~lmask(hibit(below)));
    const uint64_t nws = mm[0] & seg;
    wc = (mm[1] & seg) != 0 || (carried && o_wc);
    al = (mm[2] & seg) != 0 || (carried && o_al);
    first = (carried && o_first != kNone) ? o_first : (nws ? base + lobit(nws) : kNone);
    last = nws ? base + hibit(nws) + 1 : (carried ? o_last : 0u);
  };
  const uint32_t got = x.par.chunks(
      C,
      [&](uint32_t i) -> uint32_t {
        const uint32_t p0 = c.p(i);
        const bool ws = is_ws(p0);
        return (ws ? 0u : 1u) | ((!(p0 & P_PUNCT) && !ws) ? 2u : 0u) | ((p0 & P_ALPHA) ? 4u : 0u);
      },
      [&](uint32_t i, uint32_t l, const uint64_t* mm) {
        const uint32_t base = i - l;
        const uint64_t E = (bmask(base) >> 1) | ((uint64_t)next_brk(base) << 63);
        if (!((E >> l) & 1u)) return false;
        uint32_t first, last;
        bool wc, al;
        segment(base, l, mm, first, last, wc, al);
        return wc;
      },
      [&](uint32_t i, uint32_t l, const uint64_t* mm, uint32_t k) {
        uint32_t first, last;
        bool wc, al;
        segment(i - l, l, mm, first, last, wc, al);
        const uint32_t bs = c.o(first), be = c.o(last);
        if (store && k < W) words[k] = bs | (be << 16);
        if (ss) {
          chars += last - first;
          alpha += al ? 1u : 0u;
          const bool st = use_lite ? l_is_stop_lite(ucd, lite, b, nb, bs, be, last - first)
                                   : l_is_stop(ucd, *ss, b, nb, bs, be, last - first);
          stop += st ? 1u : 0u;
        }
      },
      [&](uint32_t base, const uint64_t* mm) {
        if (next_brk(base)) {  // the next chunk starts a new segment
          o_first = kNone;
          o_last = 0;
          o_wc = o_al = false;
          return;
        }
        const uint64_t B = bmask(base);
        uint64_t seg = ~0ull;
        if (B) {
          seg = ~lmask(hibit(B));
          o_first = kNone;
          o_last = 0;
          o_wc = o_al = false;
        }
        const uint64_t nws = mm[0] & seg;
        o_wc = o_wc || (mm[1] & seg) != 0;
        o_al = o_al || (mm[2] & seg) != 0;
        if (nws) {
          if (o_first == kNone) o_first = base + lobit(nws);
          o_last = base + hibit(nws) + 1;
        }
      });
  if (got != W) return false;  // the passes disagree: never expected; the generic path decides
  if (ss) {
    out.chars = x.par.reduce_add((int64_t)chars);
    out.alpha = x.par.reduce_add((int64_t)alpha);
    out.stop = x.par.reduce_add((int64_t)stop);
  }
  x.par.sync();
  x.a.hi = m.hi;
  out.n = W;
  out.w = words;
  return true;
}

// Rust str::lines() of the code points: line i = [ls, le) packed as ls | le << 16.
struct LLines {
  uint32_t n = 0;
  TB_LDS uint32_t* l = nullptr;
  TB_HD uint32_t s(uint32_t k) const { return l[k] & 0xFFFFu; }
  TB_HD uint32_t e(uint32_t k) const { return l[k] >> 16; }
};

template <class P>
TB_HD bool l_lines(LCtx<P>& x, const LCps& c, uint32_t nl, LLines& L) {
  const uint32_t C = c.n;
  if (C == 0) {
    L.n = 0;
    return true;
  }
  const uint32_t NL = 1 + nl - (c.lead(C - 1) == '\n' ? 1u : 0u);
  TB_LDS uint32_t* l = x.a.template get<uint32_t>(NL + 1);
  if (x.a.ovf) return false;
  const uint32_t got = x.par.template compact<int>(
      C, [&](uint32_t i, int&) { return i == 0 || c.lead(i - 1) == '\n'; },
      [&](uint32_t i, uint32_t k, int&) { l[k] = i; });
  x.par.sync();
  x.par.for_n(got, [&](uint32_t k) {
    const uint32_t ls = l[k];
    const uint32_t e = (k + 1 < got) ? (l[k + 1] & 0xFFFFu) - 1 : (c.lead(C - 1) == '\n' ? C - 1 : C);
    uint32_t ce = e;
    if (e < C && ce > ls && c.lead(ce - 1) == '\r') --ce;
    l[k] = ls | (ce << 16);
  });
  x.par.sync();
  L.n = got;
  L.l = l;
  return true;
}

// GopherRepetition record (gopher_rep_record in docproc.h): lines/paragraphs and the n-gram
// statistics. `words` holds the stored words; `ent_mark` is the hi-stack level that releases the
// code point array before the n-gram tables.
template <class P>
TB_HD bool l_gopher_rep(LCtx<P>& x, const DevStep& ds, const LCps& c, const LWords& wd, uint32_t nl, int64_t* r,
                        bool release_cps, uint32_t cps_hi_mark) {
  const uint32_t C = c.n;
  TB_LDS const uint8_t* b = c.b;
  const int width = ds.width;
  const uint32_t tcs = x.par.template min<uint32_t>(C, C, [&](uint32_t i) { return is_ws(c.p(i)) ? C : i; });
  const uint32_t tce = x.par.template max<uint32_t>(C, 0u, [&](uint32_t i) { return is_ws(c.p(i)) ? 0u : i + 1; });
  if (tcs >= tce) {
    x.par.single([&]() {
      for (int k = 0; k < width; ++k) r[k] = 0;
      r[0] = -1;
    });
    return true;
  }
  const auto m0 = x.a.mark();
  const uint32_t span = tce - tcs;
  // newline runs inside the trimmed text: rs | rl << 16
  TB_LDS uint32_t* runs = x.a.template get<uint32_t>(nl + 1);
  TB_LDS uint16_t* prs = x.a.template get<uint16_t>(nl + 1);
  if (x.a.ovf) return false;
  const uint32_t NR = x.par.template compact<int>(
      span,
      [&](uint32_t i, int&) {
        const uint32_t j = tcs + i;
        return c.lead(j) == '\n' && c.lead(j - 1) != '\n';
      },
      [&](uint32_t i, uint32_t k, int&) {
        const uint32_t j = tcs + i;
        uint32_t q = j;
        while (c.lead(q) == '\n') ++q;
        runs[k] = j | ((q - j) << 16);
      });
  x.par.sync();
  x.stamp(PH_GR_RUNS);
  auto rs = [&](uint32_t k) { return runs[k] & 0xFFFFu; };
  auto rl = [&](uint32_t k) { return runs[k] >> 16; };
  int64_t line_dup = 0, line_dup_b = 0, para_dup = 0, para_dup_b = 0;
  if (!l_dup_spans(
          x, b, NR + 1,
          [&](uint32_t k, uint32_t& s0, uint32_t& e0) {
            const uint32_t cs = k == 0 ? tcs : rs(k - 1) + rl(k - 1);
            const uint32_t ce = k == NR ? tce : rs(k);
            s0 = c.o(cs);
            e0 = c.o(ce);
          },
          &line_dup, &line_dup_b))
    return false;
  x.stamp(PH_GR_LINEDUP);
  const uint32_t NPR = x.par.template compact<int>(
      NR, [&](uint32_t k, int&) { return rl(k) >= 2; }, [&](uint32_t k, uint32_t q, int&) { prs[q] = (uint16_t)k; });
  x.par.sync();
  if (!l_dup_spans(
          x, b, NPR + 1,
          [&](uint32_t q, uint32_t& s0, uint32_t& e0) {
            const uint32_t cs = q == 0 ? tcs : rs(prs[q - 1]) + rl(prs[q - 1]);
            const uint32_t ce = q == NPR ? tce : rs(prs[q]);
            s0 = c.o(cs);
            e0 = c.o(ce);
          },
          &para_dup, &para_dup_b))
    return false;
  x.stamp(PH_GR_LINES);
  x.par.single([&]() {
    r[0] = span;
    r[1] = NPR + 1;
    r[2] = para_dup;
    r[3] = para_dup_b;
    r[4] = NR + 1;
    r[5] = line_dup;
    r[6] = line_dup_b;
    for (int k = rec_gr_fixed(); k < width; ++k) r[k] = 0;
  });
  x.a.reset(m0);  // runs, prs
  if (ds.n_top + ds.n_dup == 0) return true;
  // the n-gram statistics read words and bytes only: the code point array (bottom of the hi
  // stack, nothing above it now) goes to their tables
  if (release_cps) x.a.hi = cps_hi_mark;
  // ---- n-gram statistics over the words ----
  const uint32_t W = wd.n;
  TB_LDS const uint32_t* words = wd.w;
  auto ws = [&](uint32_t k) { return words[k] & 0xFFFFu; };
  auto we = [&](uint32_t k) { return words[k] >> 16; };
  // wid: canonical word id; WL: byte prefix of word lengths; SK / CR: bigram-sum prefix of the
  // concatenated words (SK[k] = sum_{j<k} inner_j + cross_{j-1}, CR[j] = cross_{j-1}), so the key
  // of the concatenation of words p..p+n-1 is SK[p+n] - SK[p] - CR[p]
  TB_LDS uint16_t* wid = x.a.template get<uint16_t>(W + 1);
  TB_LDS uint16_t* WL = x.a.template get<uint16_t>(W + 1);
  TB_LDS uint32_t* SK = x.a.template get<uint32_t>(W + 1);
  TB_LDS uint32_t* CR = x.a.template get<uint32_t>(W + 1);
  if (x.a.ovf) return false;
  if (!l_canon(
          x, W, [&](uint32_t k) { return l_span_key(b, ws(k), we(k)); },
          [&](uint32_t i, uint32_t j) { return l_bytes_eq(b, ws(i), we(i), ws(j), we(j)); }, wid))
    return false;
  x.stamp(PH_WORD_CANON);
  const uint32_t totl = x.par.template scan<uint32_t>(
      W, 0u, [](uint32_t a, uint32_t c2) { return a + c2; }, [&](uint32_t k) { return we(k) - ws(k); },
      [&](uint32_t k, uint32_t e) { WL[k] = (uint16_t)e; });
  x.par.single([&]() { WL[W] = (uint16_t)totl; });
  x.par.for_n(W, [&](uint32_t j) {
    const uint32_t s = ws(j), e = we(j);
    uint32_t inner = 0;
    for (uint32_t q = s; q + 1 < e; ++q) inner += l_pair(b[q], b[q + 1]);
    CR[j] = j > 0 ? l_pair(b[we(j - 1) - 1], b[s]) : 0u;
    SK[j] = inner;  // element of the scan below
  });
  x.par.sync();
  const uint32_t sktot = x.par.template scan<uint32_t>(
      W, 0u, [](uint32_t a, uint32_t c2) { return a + c2; }, [&](uint32_t j) { return SK[j] + CR[j]; },
      [&](uint32_t k, uint32_t e) { SK[k] = e; });
  x.par.single([&]() { SK[W] = sktot; });
  x.par.sync();
  x.stamp(PH_GR_WORDS);
  // Top n-grams: the n-gram at p is the pair (class of the (n-1)-gram at p, id of word p+n-1):
  // per order one exact pair classification that also counts the classes (l_classes: the table
  // slot is the class id, no resolve pass), then two reductions.
  if (ds.n_top > 0) {
    int max_top = 0;
    for (int t = 0; t < ds.n_top; ++t) max_top = ds.top_n[t] > max_top ? ds.top_n[t] : max_top;
    const auto m2 = x.a.mark();
    const uint32_t capw = W + (W >> 1) + 2;
    TB_LDS uint16_t* ga = x.a.template get<uint16_t>(W + 1);
    TB_LDS uint16_t* gb = x.a.template get<uint16_t>(W + 1);
    TB_LDS uint32_t* cnt = x.a.template get<uint32_t>(capw);
    TB_LDS uint32_t* tab = x.a.template get_hi<uint32_t>(capw);
    if (x.a.ovf || W >= 43000u) return false;
    TB_LDS const uint16_t* gprev = wid;
    for (uint32_t n = 1; n <= (uint32_t)max_top && W >= n; ++n) {
      const uint32_t G = W - n + 1;
      TB_LDS const uint16_t* gc = wid;
      uint32_t ncls;  // class ids are < ncls
      if (n == 1) {
        // words: classes = canonical word ids; counted directly
        x.par.for_n(W, [&](uint32_t p) { cnt[p] = 0; });
        x.par.sync();
        x.par.for_n(W, [&](uint32_t p) { l_add(&cnt[wid[p]], 1u); });
        x.par.sync();
        ncls = W;
      } else {
        TB_LDS uint16_t* gcur = (n & 1) ? ga : gb;
        l_classes(
            x, G,
            [&](uint32_t p) {
              return mix64(((uint64_t)gprev[p] << 32) ^ (uint64_t)wid[p + n - 1] ^ ((uint64_t)n << 60));
            },
            [&](uint32_t p, uint32_t q) { return gprev[p] == gprev[q] && wid[p + n - 1] == wid[q + n - 1]; },
            tab, cnt, gcur);
        gc = gcur;
        gprev = gcur;
        ncls = G + (G >> 1) + 2;
        x.stamp(PH_GR_TOP_CANON);
      }
      bool wanted = false;
      for (int t = 0; t < ds.n_top; ++t) wanted |= ds.top_n[t] == (int32_t)n;
      if (!wanted) continue;
      const uint32_t maxc = x.par.template max<uint32_t>(ncls, 0u, [&](uint32_t k) { return cnt[k]; });
      int64_t v = 0;
      if (maxc > 1) {
        // the longest gram among the most frequent (equal grams have equal lengths)
        const uint32_t maxlen = x.par.template max<uint32_t>(G, 0u, [&](uint32_t p) {
          return cnt[gc[p]] == maxc ? ((uint32_t)WL[p + n] - (uint32_t)WL[p] + n - 1) : 0u;
        });
        v = (int64_t)maxlen * (int64_t)maxc;
      }
      x.par.single([&]() {
        for (int t = 0; t < ds.n_top; ++t) if (ds.top_n[t] == (int32_t)n) r[rec_gr_fixed() + t] = v;
      });
      x.par.sync();
    }
    x.a.reset(m2);
  }
  x.stamp(PH_GR_TOP);
  if (ds.n_dup > 0) {
    // Duplicated n-grams (find_all_duplicate): grams of order n are equal iff their
    // concatenations are. The grams of all orders are canonicalised in one table pass (orders are
    // grouped only when that table does not fit the slice), interleaved: item i of a group of ng
    // orders is the gram at position i / ng of order t0 + i % ng (no per-lane order tables), then
    // the greedy walks of all orders run concurrently, one lane each.
    const uint32_t nd = (uint32_t)ds.n_dup;
    uint32_t nmin = 0xFFFFFFFFu;
    for (uint32_t t = 0; t < nd; ++t) nmin = (uint32_t)ds.dup_n[t] < nmin ? (uint32_t)ds.dup_n[t] : nmin;
    const uint32_t Gmax = (nmin == 0 || W < nmin) ? 0u : W - nmin + 1;
    const uint32_t SW = (W + 31) / 32 + 1;
    const auto m3 = x.a.mark();
    TB_LDS uint32_t* dn = x.a.template get<uint32_t>(nd);
    TB_LDS uint16_t* gc = x.a.template get<uint16_t>(Gmax * nd + 1);  // [p * nd + t]
    TB_LDS uint32_t* bits = x.a.template get<uint32_t>(2 * SW * nd);  // [sn | R] per order
    if (x.a.ovf) return false;
    x.par.for_n(nd, [&](uint32_t t) { dn[t] = (uint32_t)ds.dup_n[t]; });
    x.par.for_n(2 * SW * nd, [&](uint32_t i) { bits[i] = 0; });
    x.par.sync();
    for (uint32_t t0 = 0; t0 < nd;) {
      // largest group of orders [t0, t1) whose table (4 bytes x 1.5 slots per item) and
      // canonical-index array (2 bytes per item) fit what is left of the slice
      uint32_t t1 = t0 + 1;
      while (t1 < nd) {
        const uint64_t items = (uint64_t)(t1 + 1 - t0) * Gmax;
        if (items >= 43000u || 8ull * items + 32 > (uint64_t)x.a.free_bytes()) break;
        ++t1;
      }
      const uint32_t ng = t1 - t0, items = ng * Gmax;
      if (items >= 43000u) return false;
      const auto mg = x.a.mark();
      TB_LDS uint16_t* cg = x.a.template get_hi<uint16_t>(items + 1);
      if (x.a.ovf) return false;
      auto gram = [&](uint32_t i, uint32_t& t, uint32_t& p, uint32_t& n) {  // item -> order, position
        p = i / ng;
        t = t0 + (i - p * ng);
        n = dn[t];
        return n > 0 && p + n <= W;
      };
      if (!l_canon(
              x, items,
              [&](uint32_t i) -> uint64_t {
                uint32_t t, p, n;
                if (!gram(i, t, p, n)) return 0;  // past the order's last gram: not inserted
                const uint32_t L = (uint32_t)WL[p + n] - (uint32_t)WL[p];
                const uint32_t kk = SK[p + n] - SK[p] - CR[p];
                return mix64((uint64_t)kk ^ ((uint64_t)L << 32) ^ ((uint64_t)b[ws(p)] << 48) ^ ((uint64_t)n << 56)) | 1ull;
              },
              [&](uint32_t i, uint32_t j) {
                uint32_t t, p, n, tq, q, nq;
                gram(i, t, p, n);
                gram(j, tq, q, nq);
                if (tq != t) return false;
                const uint32_t L = (uint32_t)WL[p + n] - (uint32_t)WL[p];
                if ((uint32_t)WL[q + n] - (uint32_t)WL[q] != L) return false;
                uint32_t dw = 0, k = 0;
                for (; k + 4 <= n; k += 4)  // four id pairs per iteration, loads issued together
                  dw |= (uint32_t)((wid[p + k] ^ wid[q + k]) | (wid[p + k + 1] ^ wid[q + k + 1]) |
                                   (wid[p + k + 2] ^ wid[q + k + 2]) | (wid[p + k + 3] ^ wid[q + k + 3]));
                for (; k < n; ++k) dw |= (uint32_t)(wid[p + k] ^ wid[q + k]);
                if (dw == 0) return true;
                // different word splits: compare the concatenations byte by byte
                uint32_t wp = p, wq = q, bp = ws(p), bq = ws(q);
                for (uint32_t i2 = 0; i2 < L; ++i2) {
                  while (bp == we(wp)) { ++wp; bp = ws(wp); }
                  while (bq == we(wq)) { ++wq; bq = ws(wq); }
                  if (b[bp] != b[bq]) return false;
                  ++bp;
                  ++bq;
                }
                return true;
              },
              cg))
        return false;
      x.stamp(PH_GR_DUP_CANON);
      // canonical item -> gram id (its position) per order; repeat bits
      x.par.for_n(items, [&](uint32_t i) {
        uint32_t t, p, n;
        if (!gram(i, t, p, n)) return;
        const uint32_t g = (uint32_t)cg[i] / ng;
        gc[p * nd + t] = (uint16_t)g;
        if (g != p) {
          TB_LDS uint32_t* R = bits + t * 2 * SW + SW;
          l_or(&R[p >> 5], 1u << (p & 31));
          l_or(&R[g >> 5], 1u << (g & 31));
        }
      });
      x.par.sync();
      x.a.reset(mg);
      t0 = t1;
    }
    x.par.for_n(nd, [&](uint32_t t) {
      const uint32_t n = dn[t];
      const uint32_t G = (n == 0 || W < n) ? 0u : W - n + 1;
      int64_t rep = 0;
      if (G > 0) {
        TB_LDS uint32_t* sn = bits + t * 2 * SW;
        rep = l_dup_walk(G, n, gc + t, nd, sn + SW, sn, WL);
      }
      r[rec_gr_fixed() + ds.n_top + t] = rep;
    });
    x.par.sync();
    x.stamp(PH_GR_DUP_WALK);
    x.a.reset(m3);
  }
  return true;
}

// Stage analysis of one document from its LDS text b[0, n) (4-aligned, >= 8 zero bytes of
// padding): writes the records of every GopherQuality / GopherRepetition / FineWeb step of the
// stage (language-id steps run in their own kernel). LDS_RETRY: the arrays did not fit the slice;
// nothing is final and the caller recomputes the document with analyze_stage.
template <class P>
TB_HD int lds_analyze_stage(LCtx<P>& x, const DevStage& st, const DevPlan& plan, TB_LDS const uint8_t* b, uint32_t n,
                            int64_t* rec, uint32_t ndocs, uint32_t doc) {
  bool need_gq = false, need_fw = false, need_gr = false, store_words = false;
  for (int s = 0; s < st.n_steps; ++s) {
    const DevStep& ds = st.steps[s];
    if (ds.kind == DK_GOPHER_QUALITY) need_gq = true;
    if (ds.kind == DK_FINEWEB) need_fw = true;
    if (ds.kind == DK_GOPHER_REP) {
      need_gr = true;
      store_words |= ds.n_top + ds.n_dup > 0;
    }
  }
  if (!need_gq && !need_fw && !need_gr) return LDS_OK;
  x.stamp(PH_START);
  const uint32_t hi0 = x.a.hi;
  TB_LDS uint32_t* ent = x.a.template get_hi<uint32_t>(n + 1);
  if (x.a.ovf) return LDS_RETRY;
  uint32_t dict = 0;
  LCps c;
  c.b = b;
  c.nb = n;
  c.ent = ent;
  c.n = l_decode(x, b, n, ent, &dict);
  x.stamp(PH_DECODE);
  if (dict) {  // dictionary scripts: the ICU path (host) recomputes the document
    x.set_flag(DOC_NEEDS_CPU);
    return LDS_OK;
  }
  const uint32_t C = c.n;
  // GopherQuality's stop-word set (the first GopherQuality step's; one per stage in practice)
  const DevStopSet* ss = nullptr;
  for (int s = 0; s < st.n_steps; ++s)
    if (st.steps[s].kind == DK_GOPHER_QUALITY) { ss = &plan.stops[st.steps[s].stop_set]; break; }
  int n_gq = 0;
  for (int s = 0; s < st.n_steps; ++s) n_gq += st.steps[s].kind == DK_GOPHER_QUALITY;
  LWords wd;
  // the stop-word set goes into the slice when it is small (compact form), else lookups read the
  // plan's table in global memory
  LStop lite;
  const bool use_lite = need_gq && ss->lite_nslots > 0;
  if (use_lite && !l_stop_load(x, *ss, lite)) return LDS_RETRY;
  // the word sums are per stop-word set: with several GopherQuality steps of different sets,
  // the stop counts are taken per step below
  if (!l_words(x, c, store_words, need_gq ? ss : nullptr, wd, use_lite, lite)) return LDS_RETRY;
  x.stamp(PH_WORDS);
  const uint32_t nl = x.par.template sum<uint32_t>(C, [&](uint32_t i) { return c.lead(i) == '\n' ? 1u : 0u; });
  x.stamp(PH_NL_COUNT);
  LLines L;
  if ((need_gq || need_fw) && !l_lines(x, c, nl, L)) return LDS_RETRY;
  x.stamp(PH_LINES);
  const uint32_t W = wd.n;
  int n_gr = 0;
  for (int s = 0; s < st.n_steps; ++s) n_gr += st.steps[s].kind == DK_GOPHER_REP;
  int gr_seen = 0;
  for (int so = 0; so < 2 * st.n_steps; ++so) {
    const int s = so % st.n_steps;
    const DevStep& ds = st.steps[s];
    if ((so < st.n_steps) == (ds.kind == DK_GOPHER_REP)) continue;
    int64_t* r = rec + (int64_t)ds.rec_prefix * ndocs + (int64_t)doc * ds.width;
    if (ds.kind == DK_GOPHER_QUALITY) {
      int64_t stop = wd.stop;
      if (n_gq > 1 && &plan.stops[ds.stop_set] != ss) {
        // another stop-word set: count this step's stop words over the words again
        LWords w2;
        if (!l_words(x, c, false, &plan.stops[ds.stop_set], w2)) return LDS_RETRY;
        stop = w2.stop;
      }
      const uint64_t he = x.par.template sum<uint64_t>(C, [&](uint32_t i) {
        const uint32_t c0 = c.lead(i);
        if (c0 == '#') return (uint64_t)1 << 32;
        if (c0 == 0xE2) return (uint64_t)(c.cp(i) == 0x2026);
        if (c0 != '.' || (i > 0 && c.lead(i - 1) == '.')) return (uint64_t)0;
        uint32_t j = i;
        while (j < C && c.lead(j) == '.') ++j;
        return (uint64_t)((j - i) / 3);
      });
      x.stamp(PH_GQ_CHARS);
      const uint64_t bl = x.par.template sum<uint64_t>(L.n, [&](uint32_t k) {
        const uint32_t ls = L.s(k), le = L.e(k);
        uint32_t j = ls;
        while (j < le && is_ws(c.p(j))) ++j;
        const uint32_t l0 = j < le ? c.lead(j) : 0u;
        const uint64_t bul = (l0 == '-' || (l0 == 0xE2 && c.cp(j) == 0x2022)) ? 1 : 0;
        j = le;
        while (j > ls && is_ws(c.p(j - 1))) --j;
        const uint32_t E = c.o(j), S = c.o(ls);
        uint64_t ell = 0;
        if (E - S >= 3) {
          const bool dots = b[E - 3] == '.' && b[E - 2] == '.' && b[E - 1] == '.';
          const bool uell = b[E - 3] == 0xE2 && b[E - 2] == 0x80 && b[E - 1] == 0xA6;
          ell = (dots || uell) ? 1 : 0;
        }
        return (bul << 32) | ell;
      });
      x.par.single([&]() {
        r[0] = W; r[1] = wd.chars; r[2] = (int64_t)(he >> 32); r[3] = (int64_t)(he & 0xFFFFFFFFull); r[4] = L.n;
        r[5] = (int64_t)(bl >> 32); r[6] = (int64_t)(bl & 0xFFFFFFFFull); r[7] = wd.alpha; r[8] = stop;
      });
      x.par.sync();
      x.stamp(PH_GQ);
    } else if (ds.kind == DK_GOPHER_REP) {
      ++gr_seen;
      // the last GopherRepetition step may release the code point array for its n-gram tables
      if (!l_gopher_rep(x, ds, c, wd, nl, r, gr_seen == n_gr, hi0)) return LDS_RETRY;
    } else if (ds.kind == DK_FINEWEB) {
      const auto m = x.a.mark();
      TB_LDS uint16_t* nbl = x.a.template get<uint16_t>(L.n + 1);
      if (x.a.ovf) return LDS_RETRY;
      const uint32_t NB = x.par.template compact<int>(
          L.n,
          [&](uint32_t k, int&) {
            for (uint32_t j = L.s(k); j < L.e(k); ++j) if (!is_ws(c.p(j))) return true;
            return false;
          },
          [&](uint32_t k, uint32_t q, int&) { nbl[q] = (uint16_t)k; });
      x.par.sync();
      const uint64_t se = x.par.template sum<uint64_t>(NB, [&](uint32_t q) {
        const uint32_t k = nbl[q];
        uint32_t j = L.e(k);
        while (j > L.s(k) && is_ws(c.p(j - 1))) --j;
        const uint32_t last = c.cp(j - 1);
        uint64_t v = ((int64_t)(L.e(k) - L.s(k)) <= ds.short_line_length) ? (1ull << 32) : 0ull;
        for (int t = 0; t < ds.n_stop_chars; ++t)
          if (ds.stop_chars[t] == last) { v |= 1ull; break; }
        return v;
      });
      int64_t dup_e = 0, dup_b = 0;
      if (!l_dup_spans(
              x, b, NB,
              [&](uint32_t q, uint32_t& s0, uint32_t& e0) {
                s0 = c.o(L.s(nbl[q]));
                e0 = c.o(L.e(nbl[q]));
              },
              &dup_e, &dup_b))
        return LDS_RETRY;
      x.par.single([&]() {
        r[0] = NB; r[1] = (int64_t)(se & 0xFFFFFFFFull); r[2] = (int64_t)(se >> 32); r[3] = dup_b;
        r[4] = (int64_t)C - nl; r[5] = nl; r[6] = W;
      });
      x.par.sync();
      x.a.reset(m);
      x.stamp(PH_FW);
    }
    if (x.a.ovf) return LDS_RETRY;
  }
  return LDS_OK;
}

}  // namespace tb
