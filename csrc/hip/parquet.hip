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
// Snappy (one wave per page): the token stream is parsed uniformly by the whole wave from a
// 512-byte register window of the compressed input (bytes fetched with readlane), literal bytes
// are copied lane-parallel out of the window (ds_bpermute), and copies read the last 32 KB of
// output from an LDS ring (older offsets from the output in HBM); a copy shorter than its offset
// is one lane-parallel step, a self-overlapping one replicates its period (lane % offset).
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
constexpr uint32_t kWin = 512;     // register window of the compressed input (8 bytes per lane)

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

// Snappy raw block in[0, nin) -> o[0, nout). Whole-wave (uniform) control flow.
__device__ bool snappy_wave(const uint8_t* __restrict__ in, uint32_t nin, uint8_t* __restrict__ o, uint32_t nout,
                            uint8_t* ring) {
  const uint32_t lane = threadIdx.x;
  uint32_t wb = 0;
  uint32_t wlo = 0, whi = 0;  // bytes [wb + 8 lane, +8) of the input
  auto refill = [&](uint32_t base) {
    wb = base;
    const uint32_t s = base + 8 * lane;
    uint32_t lo = 0, hi = 0;
    if (s + 8 <= nin) {
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) lo |= (uint32_t)in[s + k] << (8 * k);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) hi |= (uint32_t)in[s + 4 + k] << (8 * k);
    } else {
      for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t v = s + k < nin ? (uint32_t)in[s + k] : 0u;
        if (k < 4) lo |= v << (8 * k); else hi |= v << (8 * (k - 4));
      }
    }
    // consume the loads here: gfx9 counts loads and stores on one vmcnt, so a window register
    // still pending at the token loop's head would make every token wait for all earlier
    // output stores (measured: ~1 us per token)
    asm volatile("" ::"v"(lo), "v"(hi));
    wlo = lo;
    whi = hi;
  };
  auto byte_at = [&](uint32_t q) -> uint32_t {  // uniform q in [wb, wb + kWin)
    const uint32_t r = q - wb;
    const uint32_t src = r >> 3;
    const uint32_t w = (r & 4) ? (uint32_t)__builtin_amdgcn_readlane((int)whi, (int)src)
                               : (uint32_t)__builtin_amdgcn_readlane((int)wlo, (int)src);
    return (w >> (8 * (r & 3))) & 0xFFu;
  };
  refill(0);
  // preamble: varint of the uncompressed length
  uint32_t ip = 0, ulen = 0;
  for (uint32_t shift = 0;; shift += 7) {
    if (ip >= nin || shift > 28) return false;
    const uint32_t b = byte_at(ip++);
    ulen |= (b & 0x7Fu) << shift;
    if (!(b & 0x80u)) break;
  }
  if (ulen != nout) return false;
  uint32_t op = 0;
  while (ip < nin) {
    if (ip + 5 > wb + kWin) refill(ip);
    const uint32_t tag = byte_at(ip);
    uint32_t len, off = 0;
    const uint32_t kind = tag & 3u;
    if (kind == 0) {
      uint32_t l = tag >> 2;
      ip += 1;
      if (l >= 60) {
        const uint32_t nb = l - 59;
        if (ip + nb > nin) return false;
        l = 0;
        for (uint32_t k = 0; k < nb; ++k) l |= byte_at(ip + k) << (8 * k);
        ip += nb;
      }
      len = l + 1;
      if (len == 0 || ip + len > nin || op + len > nout) return false;
      // literal: lane-parallel out of the window, 64 bytes per step
      for (uint32_t c = 0; c < len; c += 64) {
        const uint32_t q = ip + c;
        if (q + 64 > wb + kWin) refill(q);
        const uint32_t r = q + lane - wb;
        const int src = (int)((r >> 3) & 63u) << 2;  // byte address of the source lane
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wlo);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)whi);
        const uint32_t w = (r & 4) ? hi : lo;
        const uint32_t v = (w >> (8 * (r & 3))) & 0xFFu;
        const uint32_t j = c + lane;
        if (j < len) {
          o[op + j] = (uint8_t)v;
          ring[(op + j) & (kRing - 1)] = (uint8_t)v;
        }
      }
      ip += len;
      op += len;
      continue;
    }
    if (kind == 1) {
      if (ip + 2 > nin) return false;
      len = 4 + ((tag >> 2) & 7u);
      off = ((tag >> 5) << 8) | byte_at(ip + 1);
      ip += 2;
    } else if (kind == 2) {
      if (ip + 3 > nin) return false;
      len = (tag >> 2) + 1;
      off = byte_at(ip + 1) | (byte_at(ip + 2) << 8);
      ip += 3;
    } else {
      if (ip + 5 > nin) return false;
      len = (tag >> 2) + 1;
      off = byte_at(ip + 1) | (byte_at(ip + 2) << 8) | (byte_at(ip + 3) << 16) | (byte_at(ip + 4) << 24);
      ip += 5;
    }
    if (off == 0 || off > op || op + len > nout) return false;
    // len <= 64: one step; a source position is op - off + (j % off) < op (already written)
    // (two branches, not a select: a pointer select becomes a flat load, which waits for every
    // outstanding output store before it returns)
    const uint32_t s = op - off + (off >= 64 ? lane : lane % off);
    uint32_t v = 0;
    if (off <= kRing - 64) {
      if (lane < len) v = ring[s & (kRing - 1)];
    } else {
      if (lane < len) v = o[s];
      asm volatile("" : "+v"(v));  // wait for this load here, not at the shared store below
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < len) {
      o[op + lane] = (uint8_t)v;
      ring[(op + lane) & (kRing - 1)] = (uint8_t)v;
    }
    __builtin_amdgcn_wave_barrier();
    op += len;
  }
  return op == nout;
}

__global__ __launch_bounds__(64) void k_pq_decompress(const uint8_t* __restrict__ chunk, const PqDev* __restrict__ pages,
                                                      int32_t npages, uint8_t* __restrict__ pagebuf,
                                                      uint32_t* __restrict__ err) {
  __shared__ uint8_t ring[kRing];
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
  if (!snappy_wave(in + raw, (uint32_t)d.in_size - raw, out + raw, (uint32_t)d.out_size - raw, ring) && lane == 0)
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
