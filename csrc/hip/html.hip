// K17: HTML character-reference decoding of packed input text on the MI355X (the reference
// reader runs html_escape::decode_html_entities on every text cell, parquet_reader.rs:177-179).
// Same semantics as the host decoder csrc/host/html.cpp (the oracle its tests compare against):
//   &name;  HTML5 named references (hashed lookup table built by ops/html.py)
//   &#DDD; / &#xHHH;  numeric references denoting a Unicode scalar value (NUL included)
//   anything else is copied verbatim.
//
// A matched reference contains no '&', so every '&' can be decided independently. One wave per
// document walks it in 64-byte chunks: each lane decides its byte (plain byte -> 1 output byte;
// '&' that matches -> the replacement; bytes inside a match -> nothing), an exclusive max-scan
// of the match ends marks bytes covered by a match that starts at an earlier lane, and an
// exclusive sum-scan of the emitted counts gives every lane its output position. A match can
// be longer than a chunk (numeric references may carry any number of leading zeros), so the
// furthest match end seen so far is carried across chunks as `skip_until`. The same routine
// sizes the output (pass 1) and writes it (pass 2).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct HtmlTab {
  const uint8_t* names;     // concatenated entity names, sorted bytewise
  const int32_t* name_off;  // [nent + 1]
  const uint8_t* vals;      // concatenated UTF-8 replacements
  const int32_t* val_off;   // [nent + 1]
  int32_t nent;
  const int32_t* slots;     // open-addressing name hash -> entity index (-1 = empty), pow2 size
  uint32_t slot_mask;
};

__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool is_xdigit(uint8_t c) {
  return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
__device__ __forceinline__ bool is_alnum(uint8_t c) {
  return is_digit(c) || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}

// strncmp(table_name, s, len) with "longer table name compares greater" (html.cpp find_entity)
__device__ int cmp_name(const HtmlTab& t, int k, const uint8_t* s, uint32_t len) {
  const uint8_t* a = t.names + t.name_off[k];
  const uint32_t la = (uint32_t)(t.name_off[k + 1] - t.name_off[k]);
  const uint32_t m = la < len ? la : len;
  for (uint32_t i = 0; i < m; ++i)
    if (a[i] != s[i]) return (int)a[i] - (int)s[i];
  return la == len ? 0 : (la > len ? 1 : -1);
}

// FNV-1a of the name; must equal html_name_hash in textblaster_amd/ops/html.py (table builder)
__device__ __forceinline__ uint32_t name_hash(const uint8_t* s, uint32_t len) {
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < len; ++i) h = (h ^ s[i]) * 16777619u;
  return h;
}

// One probe (plus linear probing on collisions) instead of a binary search of dependent loads.
__device__ int find_entity(const HtmlTab& t, const uint8_t* s, uint32_t len) {
  uint32_t k = name_hash(s, len) & t.slot_mask;
  for (;;) {
    const int e = t.slots[k];
    if (e < 0) return -1;
    if (cmp_name(t, e, s, len) == 0) return e;
    k = (k + 1) & t.slot_mask;
  }
}

// Decides the reference starting at the '&' at b[p]. On a match: *end = one past its ';',
// the replacement is either table value *ent (>= 0) or code point *cp (*ent = -1), *olen its
// UTF-8 length. Returns false when the '&' is copied verbatim.
__device__ bool match_ref(const HtmlTab& t, const uint8_t* b, uint32_t n, uint32_t p, uint32_t* end, int* ent,
                          uint32_t* cp, uint32_t* olen) {
  uint32_t q = p + 1;
  if (q < n && b[q] == '#') {
    ++q;
    bool hex = false;
    if (q < n && (b[q] == 'x' || b[q] == 'X')) { hex = true; ++q; }
    const uint32_t ds = q;
    uint64_t v = 0;
    bool overflow = false;
    while (q < n && (hex ? is_xdigit(b[q]) : is_digit(b[q]))) {
      const uint8_t c = b[q];
      const int d = is_digit(c) ? c - '0' : ((c | 0x20) - 'a' + 10);
      v = v * (hex ? 16 : 10) + (uint64_t)d;
      if (v > 0x10FFFF) overflow = true;
      ++q;
    }
    if (q > ds && q < n && b[q] == ';' && !overflow && !(v >= 0xD800 && v < 0xE000)) {
      *end = q + 1;
      *ent = -1;
      *cp = (uint32_t)v;
      *olen = v < 0x80 ? 1u : v < 0x800 ? 2u : v < 0x10000 ? 3u : 4u;
      return true;
    }
    return false;
  }
  const uint32_t ns = q;
  while (q < n && is_alnum(b[q]) && q - ns < 40) ++q;
  if (q > ns && q < n && b[q] == ';') {
    const int e = find_entity(t, b + ns, q - ns);
    if (e >= 0) {
      *end = q + 1;
      *ent = e;
      *olen = (uint32_t)(t.val_off[e + 1] - t.val_off[e]);
      return true;
    }
  }
  return false;
}

template <class T, class Op>
__device__ __forceinline__ T wave_scan_incl(T v, uint32_t lane, Op op) {
  for (int o = 1; o < 64; o <<= 1) {
    const T u = (T)__shfl_up((int)v, o);
    if (lane >= (uint32_t)o) v = op(v, u);
  }
  return v;
}

// Decodes one document (one wave). WRITE=false: returns the output length only.
template <bool WRITE>
__device__ uint32_t decode_doc(const HtmlTab& t, const uint8_t* b, uint32_t n, uint8_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t out_base = 0, skip_until = 0;
  for (uint32_t base = 0; base < n; base += 64) {  // wave-uniform
    const uint32_t i = base + lane;
    const uint8_t c = i < n ? b[i] : 0;
    if (__ballot(c == '&') == 0 && skip_until <= base) {  // plain chunk: straight copy
      const uint32_t cnt = n - base < 64u ? n - base : 64u;
      if (WRITE && i < n) out[out_base + lane] = c;
      out_base += cnt;
      continue;
    }
    uint32_t end = 0, cp = 0, olen = 0;
    int ent = -1;
    const bool m = c == '&' && match_ref(t, b, n, i, &end, &ent, &cp, &olen);
    // end of the furthest match that starts at an earlier lane of this chunk
    const uint32_t mend = m ? end : 0u;
    const uint32_t incl = wave_scan_incl<uint32_t>(mend, lane, [](uint32_t a, uint32_t x) { return a > x ? a : x; });
    uint32_t excl = (uint32_t)__shfl_up((int)incl, 1);
    if (lane == 0) excl = 0;
    const bool covered = i < skip_until || i < excl;
    const uint32_t emit = i >= n || covered ? 0u : (m ? olen : 1u);
    const uint32_t esum = wave_scan_incl<uint32_t>(emit, lane, [](uint32_t a, uint32_t x) { return a + x; });
    if (WRITE && emit) {
      uint8_t* o = out + out_base + esum - emit;
      if (!m) {
        o[0] = c;
      } else if (ent >= 0) {
        const uint8_t* v = t.vals + t.val_off[ent];
        for (uint32_t k = 0; k < olen; ++k) o[k] = v[k];
      } else if (olen == 1) {
        o[0] = (uint8_t)cp;
      } else if (olen == 2) {
        o[0] = (uint8_t)(0xC0 | (cp >> 6)); o[1] = (uint8_t)(0x80 | (cp & 0x3F));
      } else if (olen == 3) {
        o[0] = (uint8_t)(0xE0 | (cp >> 12)); o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
        o[2] = (uint8_t)(0x80 | (cp & 0x3F));
      } else {
        o[0] = (uint8_t)(0xF0 | (cp >> 18)); o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
        o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (uint8_t)(0x80 | (cp & 0x3F));
      }
    }
    out_base += (uint32_t)__shfl((int)esum, 63);
    const uint32_t cend = (uint32_t)__shfl((int)incl, 63);
    skip_until = skip_until > cend ? skip_until : cend;
  }
  return out_base;
}

// Pass 1: output length per document.
__global__ __launch_bounds__(64) void k_html_sizes(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
                                                   int32_t ndocs, HtmlTab t, int64_t* out_len) {
  const int doc = (int)blockIdx.x;
  if (doc >= ndocs) return;
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  const uint32_t len = decode_doc<false>(t, b, n, nullptr);
  if ((threadIdx.x & 63u) == 0) out_len[doc] = (int64_t)len;
}

// Pass 2: decoded bytes at out + out_off[doc].
__global__ __launch_bounds__(64) void k_html_scatter(const uint8_t* __restrict__ bytes,
                                                     const int64_t* __restrict__ off, int32_t ndocs, HtmlTab t,
                                                     const int64_t* __restrict__ out_off, uint8_t* out) {
  const int doc = (int)blockIdx.x;
  if (doc >= ndocs) return;
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  (void)decode_doc<true>(t, b, n, out + out_off[doc]);
}

}  // namespace

extern "C" {

int tb_html_sizes(hipStream_t stream, const uint8_t* bytes, const int64_t* off, int32_t ndocs, const uint8_t* names,
                  const int32_t* name_off, const uint8_t* vals, const int32_t* val_off, int32_t nent,
                  const int32_t* slots, uint32_t slot_mask, int64_t* out_len) {
  if (ndocs <= 0) return 0;
  HtmlTab t{names, name_off, vals, val_off, nent, slots, slot_mask};
  hipLaunchKernelGGL(k_html_sizes, dim3(ndocs), dim3(64), 0, stream, bytes, off, ndocs, t, out_len);
  return (int)hipGetLastError();
}

int tb_html_scatter(hipStream_t stream, const uint8_t* bytes, const int64_t* off, int32_t ndocs,
                    const uint8_t* names, const int32_t* name_off, const uint8_t* vals, const int32_t* val_off,
                    int32_t nent, const int32_t* slots, uint32_t slot_mask, const int64_t* out_off,
                    uint8_t* out) {
  if (ndocs <= 0) return 0;
  HtmlTab t{names, name_off, vals, val_off, nent, slots, slot_mask};
  hipLaunchKernelGGL(k_html_scatter, dim3(ndocs), dim3(64), 0, stream, bytes, off, ndocs, t, out_off, out);
  return (int)hipGetLastError();
}

}  // extern "C"
