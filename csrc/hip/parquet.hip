// Parquet text-column decoding on the MI355X: the input side of the reader (reference
// src/data/readers/parquet_reader.rs reads `text` through the parquet crate on the CPU). The host
// parses the column chunk's page headers (csrc/host/parquet_pages.cpp) and uploads the chunk
// as stored; the device does the byte work:
//
//   k_pq_decompress  one wave per page: raw Snappy blocks (Parquet's SNAPPY codec) or stored
//                    pages copied; v2 level bytes are copied verbatim ahead of the values
//   k_pq_dict        one wave per dictionary page: PLAIN entries -> (offset, length)
//   k_pq_values      one wave per data page: definition levels (RLE / bit-packed hybrid, bit
//                    width 1) -> validity, PLAIN lengths or RLE_DICTIONARY indices -> per-row
//                    (offset, length) in the page buffer
//   k_pq_gather      one wave per row: strings into one packed buffer at the scanned offsets
//
// Snappy (one wave per page, snappy_batched below): 64 input positions per step, token starts
// found lane-parallel, the batch's output written 64 bytes at a time from the staged input and
// a 32 KB LDS history ring (older offsets from the output in HBM).
// Every malformed input (bad tag, offset or length, truncated stream, size mismatch) sets the
// error word and the caller decodes the row group with pyarrow instead.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct PqDev {        // one per page (ops/parquet_gpu.py builds them from the page directory)
  int64_t in_off;     // page data in the uploaded chunk
  int64_t out_off;    // its decoded bytes in the page buffer
  int32_t in_size;
  int32_t out_size;   // uncompressed size
  int32_t raw;        // leading bytes stored as is (v2: repetition + definition levels)
  int32_t codec;      // 0 stored, 1 snappy
  int32_t kind;       // 0 dictionary page, 1 data page v1, 2 data page v2
  int32_t num_values; // data pages: values incl. nulls; dictionary: entries
  int32_t encoding;   // 0 PLAIN, 2 PLAIN_DICTIONARY, 8 RLE_DICTIONARY
  int32_t def_len;    // v2: definition-level bytes
  int32_t rep_len;    // v2: repetition-level bytes
  int32_t max_def;    // 0: required column (no levels), 1: optional
  int64_t row0;       // data pages: first row
};
static_assert(sizeof(PqDev) == 64, "PqDev layout (ops/parquet_gpu.py)");

enum : uint32_t { PQE_SNAPPY = 1, PQE_LEVELS = 2, PQE_VALUES = 4, PQE_DICT = 8, PQE_BOUNDS = 16 };

#ifndef TB_PQ_RING
#define TB_PQ_RING 32768
#endif
constexpr uint32_t kRing = TB_PQ_RING;  // LDS output history per wave (bytes, power of two)

__device__ __forceinline__ void set_err(uint32_t* err, uint32_t e) { atomicOr(err, e); }

// in[0, n) -> out[0, n), whole wave: 16 independent byte loads per lane before the stores.
__device__ void copy_wave(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t base = 0; base < n; base += 64 * 16) {
    uint8_t v[16];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint32_t i = base + k * 64 + lane;
      v[k] = i < n ? in[i] : 0;
    }
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint32_t i = base + k * 64 + lane;
      if (i < n) out[i] = v[k];
    }
  }
}

// Batched Snappy decoding (one wave per page): per step the wave looks at the 64 input positions
// [ip, ip + 64) at once. Every lane decodes "a token starting at my position" (its input length L,
// output length O, and literal source or copy offset) from the input staged in LDS; a short
// scalar walk over those lane results (readlane, ~10 SALU per token) picks the real token
// starts; one wave prefix sum gives each token its output position; then the batch's output is
// produced 64 bytes at a time, every lane finding its byte's token by binary search: literal bytes
// come from the staged input, copy bytes from the LDS history ring — a source inside the same
// 64-byte chunk is resolved in a few ballot rounds (sources always lie before their byte). One
// coalesced store per 64 output bytes; ~10x fewer instructions per token than walking tokens
// one by one with the whole wave.
constexpr uint32_t kStage = 4096;  // staged input bytes (LDS)

__device__ bool snappy_batched(const uint8_t* __restrict__ in, uint32_t nin, uint8_t* __restrict__ o, uint32_t nout,
                               uint8_t* ring, uint8_t* inb, uint32_t* tok) {
  const uint32_t lane = threadIdx.x;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t ib = 0, ie = 0;  // staged input range [ib, ie)
  auto stage = [&](uint32_t base) {
    ib = base;
    ie = base + kStage < nin ? base + kStage : nin;
    const uint32_t n = ie - ib;
    for (uint32_t c = 0; c < n; c += 64 * 16) {
      uint32_t v[16];
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t i = c + k * 64 + lane;
        v[k] = i < n ? in[ib + i] : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t i = c + k * 64 + lane;
        // wait for the loads here: gfx9 counts loads and stores on one vmcnt, so a value still
        // pending later would make the token loop wait for every earlier output store
        asm volatile("" : "+v"(v[k]));
        if (i < n) inb[i] = (uint8_t)v[k];
      }
    }
    // zero slack after the staged bytes: header reads near the end see zeros
    inb[ie - ib + lane] = 0;
    __builtin_amdgcn_wave_barrier();
  };
  auto ib_at = [&](uint32_t q) -> uint32_t { return inb[q - ib]; };  // q in [ib, ie + 63]
  stage(0);
  uint32_t ip = 0, ulen = 0;
  for (uint32_t shift = 0;; shift += 7) {
    if (ip >= nin || shift > 28) return false;
    const uint32_t b = ib_at(ip++);
    ulen |= (b & 0x7Fu) << shift;
    if (!(b & 0x80u)) break;
  }
  if (ulen != nout) return false;
  uint32_t op = 0;
  while (ip < nin) {
    if (ip + 64 + 5 > ie && ie < nin) stage(ip);
    // ---- every lane: the token that would start at p = ip + lane ----
    const uint32_t p = ip + lane;
    uint32_t L = 0xFFFFFFFFu, O = 0, src = 0, lit = 0;
    if (p < nin) {
      const uint32_t t = ib_at(p);
      const uint32_t b1 = ib_at(p + 1), b2 = ib_at(p + 2), b3 = ib_at(p + 3), b4 = ib_at(p + 4);
      const uint32_t kind = t & 3u;
      if (kind == 0) {
        uint32_t l = t >> 2, hdr = 1;
        if (l >= 60) {
          const uint32_t nb = l - 59;
          const uint32_t v = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
          l = nb == 4 ? v : (v & ((1u << (8 * nb)) - 1u));
          hdr = 1 + nb;
        }
        const uint64_t len = (uint64_t)l + 1;
        const uint64_t ll = hdr + len;
        L = ll > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)ll;
        O = len > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)len;
        src = p + hdr;
        lit = 1;
      } else if (kind == 1) {
        L = 2; O = 4 + ((t >> 2) & 7u); src = ((t >> 5) << 8) | b1;
      } else if (kind == 2) {
        L = 3; O = (t >> 2) + 1; src = b1 | (b2 << 8);
      } else {
        L = 5; O = (t >> 2) + 1; src = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
      }
    }
    // ---- scalar walk over the lanes' results: the real token starts of this window ----
    uint64_t starts = 0;
    uint32_t pos = 0, Ob = 0, T = 0;
    bool long_lit = false;
    while (pos < 64 && ip + pos < nin) {
      const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)L, (int)pos);
      const uint32_t oo = (uint32_t)__builtin_amdgcn_readlane((int)O, (int)pos);
      const uint32_t lt = (uint32_t)__builtin_amdgcn_readlane((int)lit, (int)pos);
      const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)src, (int)pos);
      if (l > nin - (ip + pos)) return false;                      // token runs past the input
      if ((uint64_t)op + Ob + oo > nout) return false;              // output overflow
      if (lt) {
        if (ip + pos + l > ie) {                                     // literal data not staged
          if (T == 0) long_lit = true;
          break;
        }
      } else if (sv == 0 || sv > op + Ob) {
        return false;                                                // bad copy offset
      }
      starts |= 1ull << pos;
      ++T;
      Ob += oo;
      pos += l;
    }
    if (long_lit) {
      // a literal longer than the staged input: alone, restaging as it goes
      const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)L, 0);
      const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)O, 0);
      uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)src, 0);
      for (uint32_t c = 0; c < len; c += 64) {
        if (q + c + 64 > ie && ie < nin) stage(q + c);
        const uint32_t j = c + lane;
        if (j < len) {
          const uint32_t v = ib_at(q + j);
          ring[(op + j) & (kRing - 1)] = (uint8_t)v;
          o[op + j] = (uint8_t)v;
        }
      }
      op += len;
      ip += l;
      continue;
    }
    if (T == 0) return false;
    // ---- token table: output start, source, kind (by token rank) ----
    const bool is_start = (starts >> lane) & 1ull;
    uint32_t x = is_start ? O : 0u;  // exclusive prefix of output lengths over the starts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d);
      if ((int)lane >= d) x += y;
    }
    const uint32_t excl = x - (is_start ? O : 0u);
    if (is_start) {
      const uint32_t r = (uint32_t)__popcll(starts & below);
      tok[r] = excl;                             // output start (relative to op)
      tok[64 + r] = src;                         // literal: input position; copy: offset
      tok[128 + r] = lit;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- the batch's output, 64 bytes at a time ----
    for (uint32_t c = 0; c < Ob; c += 64) {
      const uint32_t q = c + lane;  // relative to op
      const bool act = q < Ob;
      uint32_t k = 0;
      if (act) {  // last token with start <= q
        uint32_t lo = 0, hi = T;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (tok[mid] <= q) lo = mid; else hi = mid;
        }
        k = lo;
      }
      uint32_t v = 0, sabs = 0;
      bool res = !act;
      if (act) {
        const uint32_t ts = tok[k], sv = tok[64 + k];
        const uint32_t d = q - ts;
        if (tok[128 + k]) {
          v = ib_at(sv + d);
          res = true;
        } else {
          sabs = op + ts - sv + (sv >= 64 ? d : d % sv);  // absolute source (< op + q)
          if (sabs < op + c) {
            if (sv <= kRing - 64) {
              v = ring[sabs & (kRing - 1)];
            } else {
              v = o[sabs];
              asm volatile("" : "+v"(v));
            }
            res = true;
          }
        }
        if (res) ring[(op + q) & (kRing - 1)] = (uint8_t)v;
      }
      // sources inside this chunk: a few ballot rounds (each resolves at least the first pending byte)
      uint64_t done = __ballot(res);
      while (done != ~0ull) {
        __builtin_amdgcn_wave_barrier();
        if (!res && ((done >> (sabs - (op + c))) & 1ull)) {
          v = ring[sabs & (kRing - 1)];
          ring[(op + q) & (kRing - 1)] = (uint8_t)v;
          res = true;
        }
        done = __ballot(res);
      }
      if (act) o[op + q] = (uint8_t)v;
    }
    op += Ob;
    ip += pos;
  }
  return op == nout;
}

__global__ __launch_bounds__(64) void k_pq_decompress(const uint8_t* __restrict__ chunk, const PqDev* __restrict__ pages,
                                                      int32_t npages, uint8_t* __restrict__ pagebuf,
                                                      uint32_t* __restrict__ err) {
  __shared__ uint8_t ring[kRing];
  __shared__ uint8_t inb[kStage + 64];
  __shared__ uint32_t tok[3 * 64];
  const int p = (int)blockIdx.x;
  if (p >= npages) return;
  const PqDev d = pages[p];
  const uint32_t lane = threadIdx.x;
  const uint8_t* in = chunk + d.in_off;
  uint8_t* out = pagebuf + d.out_off;
  const uint32_t raw = (uint32_t)d.raw;
  if (d.codec == 0) {
    copy_wave(in, out, (uint32_t)d.out_size);
    return;
  }
  copy_wave(in, out, raw);
  if (!snappy_batched(in + raw, (uint32_t)d.in_size - raw, out + raw, (uint32_t)d.out_size - raw, ring, inb, tok) &&
      lane == 0)
    set_err(err, PQE_SNAPPY);
}

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Dictionary page (PLAIN BYTE_ARRAY entries): dict_off / dict_len per entry. Lane 0 walks it.
__global__ __launch_bounds__(64) void k_pq_dict(const PqDev* __restrict__ pages, int32_t dict_page,
                                                const uint8_t* __restrict__ pagebuf, int64_t* __restrict__ dict_off,
                                                int32_t* __restrict__ dict_len, uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const PqDev d = pages[dict_page];
  const uint8_t* b = pagebuf + d.out_off;
  const uint32_t n = (uint32_t)d.out_size;
  uint32_t p = 0;
  for (int32_t k = 0; k < d.num_values; ++k) {
    if (p + 4 > n) { set_err(err, PQE_DICT); return; }
    const uint32_t l = ld_u32(b + p);
    if (l > n - p - 4) { set_err(err, PQE_DICT); return; }
    dict_off[k] = d.out_off + p + 4;
    dict_len[k] = (int32_t)l;
    p += 4 + l;
  }
}

// RLE / bit-packed hybrid decoder over b[p, e) (Parquet encodings.md), bit width <= 32: next()
// returns the next value; ok turns false on malformed input.
struct Hybrid {
  const uint8_t* b;
  uint32_t p, e, bw;
  uint32_t run = 0;      // values left in the current run
  bool packed = false;
  uint32_t rle_val = 0;
  uint32_t bitpos = 0;   // packed: bit offset of the next value from p0
  uint32_t p0 = 0;
  bool ok = true;
  __device__ uint32_t varint() {
    uint32_t v = 0;
    for (uint32_t s = 0; s < 35; s += 7) {
      if (p >= e) { ok = false; return 0; }
      const uint32_t c = b[p++];
      v |= (c & 0x7Fu) << s;
      if (!(c & 0x80u)) return v;
    }
    ok = false;
    return 0;
  }
  __device__ uint32_t next() {
    if (!ok) return 0;
    if (run == 0) {
      const uint32_t h = varint();
      if (!ok) return 0;
      if (h & 1u) {
        packed = true;
        run = (h >> 1) * 8u;
        p0 = p;
        bitpos = 0;
        const uint64_t bytes = (uint64_t)(h >> 1) * bw;
        if (bytes > (uint64_t)(e - p)) { ok = false; return 0; }
        p += (uint32_t)bytes;
      } else {
        packed = false;
        run = h >> 1;
        const uint32_t nb = (bw + 7) / 8;
        if (p + nb > e) { ok = false; return 0; }
        rle_val = 0;
        for (uint32_t k = 0; k < nb; ++k) rle_val |= (uint32_t)b[p + k] << (8 * k);
        p += nb;
      }
      if (run == 0) { ok = false; return 0; }
    }
    --run;
    if (!packed) return rle_val;
    uint64_t v = 0;
    const uint32_t byte0 = p0 + (bitpos >> 3), sh = bitpos & 7;
    for (uint32_t k = 0; k < 5 && k * 8 < bw + sh; ++k) v |= (uint64_t)b[byte0 + k] << (8 * k);
    bitpos += bw;
    return (uint32_t)((v >> sh) & ((bw >= 32) ? 0xFFFFFFFFull : ((1ull << bw) - 1)));
  }
};

// Data page -> per row: valid, src (byte offset in the page buffer), len. Lane 0 walks the page
// (about a thousand values per page).
__global__ __launch_bounds__(64) void k_pq_values(const PqDev* __restrict__ pages, const int32_t* __restrict__ data_pages,
                                                  int32_t ndata, const uint8_t* __restrict__ pagebuf,
                                                  const int64_t* __restrict__ dict_off,
                                                  const int32_t* __restrict__ dict_len, int32_t ndict,
                                                  int64_t* __restrict__ src, int64_t* __restrict__ len,
                                                  uint8_t* __restrict__ valid, int64_t nrows,
                                                  uint32_t* __restrict__ err) {
  if (threadIdx.x != 0 || (int)blockIdx.x >= ndata) return;
  const PqDev d = pages[data_pages[blockIdx.x]];
  const uint8_t* b = pagebuf + d.out_off;
  const uint32_t n = (uint32_t)d.out_size;
  const uint32_t nv = (uint32_t)d.num_values;
  if (d.row0 < 0 || d.row0 + (int64_t)nv > nrows) { set_err(err, PQE_BOUNDS); return; }
  uint32_t p = 0;        // values start
  Hybrid lv{b, 0, 0, 1};
  if (d.max_def > 0) {
    if (d.kind == 1) {
      if (n < 4) { set_err(err, PQE_LEVELS); return; }
      const uint32_t ll = ld_u32(b);
      if (ll > n - 4) { set_err(err, PQE_LEVELS); return; }
      lv.p = 4;
      lv.e = 4 + ll;
      p = 4 + ll;
    } else {
      const uint32_t a = (uint32_t)d.rep_len, dl = (uint32_t)d.def_len;
      if ((uint64_t)a + dl > n) { set_err(err, PQE_LEVELS); return; }
      lv.p = a;
      lv.e = a + dl;
      p = a + dl;
    }
  } else if (d.kind == 2) {
    p = (uint32_t)d.rep_len + (uint32_t)d.def_len;
  }
  const bool dict = d.encoding == 2 || d.encoding == 8;
  Hybrid ix{b, 0, n, 0};
  if (dict) {
    if (p >= n) {
      // a page of nulls only may hold no index bytes at all
      ix.ok = true;
      ix.p = n;
    } else {
      ix.bw = b[p];
      ix.p = p + 1;
      if (ix.bw > 32) { set_err(err, PQE_VALUES); return; }
    }
  } else if (d.encoding != 0) {
    set_err(err, PQE_VALUES);
    return;
  }
  for (uint32_t i = 0; i < nv; ++i) {
    const int64_t row = d.row0 + i;
    const bool v = d.max_def > 0 ? lv.next() == 1u : true;
    if (!lv.ok) { set_err(err, PQE_LEVELS); return; }
    valid[row] = v ? 1 : 0;
    if (!v) {
      src[row] = 0;
      len[row] = 0;
      continue;
    }
    if (dict) {
      const uint32_t k = ix.next();
      if (!ix.ok || (int32_t)k >= ndict) { set_err(err, PQE_VALUES); return; }
      src[row] = dict_off[k];
      len[row] = dict_len[k];
    } else {
      if (p + 4 > n) { set_err(err, PQE_VALUES); return; }
      const uint32_t l = ld_u32(b + p);
      if (l > n - p - 4) { set_err(err, PQE_VALUES); return; }
      src[row] = d.out_off + p + 4;
      len[row] = l;
      p += 4 + l;
    }
  }
}

// One wave per row: bytes pagebuf[src, src + len) -> out[off[row], ...).
constexpr int kGatherWaves = 4;
__global__ __launch_bounds__(64 * kGatherWaves) void k_pq_gather(const uint8_t* __restrict__ pagebuf,
                                                                 const int64_t* __restrict__ src,
                                                                 const int64_t* __restrict__ off, int64_t nrows,
                                                                 uint8_t* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * kGatherWaves + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint8_t* s = pagebuf + src[row];
  uint8_t* d = out + off[row];
  const int64_t n = off[row + 1] - off[row];
  for (int64_t i = lane; i < n; i += 64) d[i] = s[i];
}

}  // namespace

extern "C" {

size_t tb_sizeof_pq_page() { return sizeof(PqDev); }

int tb_pq_decompress(hipStream_t stream, const uint8_t* chunk, const void* pages, int32_t npages, uint8_t* pagebuf,
                     uint32_t* err) {
  if (npages <= 0) return 0;
  hipLaunchKernelGGL(k_pq_decompress, dim3(npages), dim3(64), 0, stream, chunk, (const PqDev*)pages, npages, pagebuf,
                     err);
  return (int)hipGetLastError();
}

int tb_pq_dict(hipStream_t stream, const void* pages, int32_t dict_page, const uint8_t* pagebuf, int64_t* dict_off,
               int32_t* dict_len, uint32_t* err) {
  hipLaunchKernelGGL(k_pq_dict, dim3(1), dim3(64), 0, stream, (const PqDev*)pages, dict_page, pagebuf, dict_off,
                     dict_len, err);
  return (int)hipGetLastError();
}

int tb_pq_values(hipStream_t stream, const void* pages, const int32_t* data_pages, int32_t ndata, const uint8_t* pagebuf,
                 const int64_t* dict_off, const int32_t* dict_len, int32_t ndict, int64_t* src, int64_t* len,
                 uint8_t* valid, int64_t nrows, uint32_t* err) {
  if (ndata <= 0) return 0;
  hipLaunchKernelGGL(k_pq_values, dim3(ndata), dim3(64), 0, stream, (const PqDev*)pages, data_pages, ndata, pagebuf,
                     dict_off, dict_len, ndict, src, len, valid, nrows, err);
  return (int)hipGetLastError();
}

int tb_pq_gather(hipStream_t stream, const uint8_t* pagebuf, const int64_t* src, const int64_t* off, int64_t nrows,
                 uint8_t* out) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(k_pq_gather, dim3((uint32_t)((nrows + kGatherWaves - 1) / kGatherWaves)), dim3(64 * kGatherWaves),
                     0, stream, pagebuf, src, off, nrows, out);
  return (int)hipGetLastError();
}

}  // extern "C"
