// Per-document parallel primitives.
//
// The document algorithms in docproc.h are written against this small interface so the same
// source runs as a wave64 kernel on the MI355X (WavePar: one wavefront per document, lanes
// cooperate through DPP shuffles / ballots, no LDS needed) and sequentially on the host
// (SeqPar: used to differential-test the device algorithms against the ICU oracle on CPU, and
// as a fast ICU-free CPU path).
//
// Contract for algorithm code:
//  * for_n(n, f): f(i) for every i < n, in any order and concurrently; f must not depend on
//    other iterations of the same call.
//  * compact<S>(n, pred, emit): pred(i, S&) computes per-item state and says whether item i
//    is selected; emit(i, k, S&) is then called with k = rank of i among selected items (in i
//    order). Returns the number selected (uniform across lanes).
//  * sum/max/min: reductions (uniform result).
//  * scan<T>(n, id, op, in, out): out(i, exclusive prefix) for every i; returns the total.
//  * mask_bits(n, pred, bits): bit i of the u32 array = pred(i) (mask_words(n) words written).
//  * scan_compact<T>(n, id, op, in, sel, emit): inclusive scan fused with a compaction that
//    selects items by their inclusive prefix; emit(i, k, incl). Returns the number selected.
//  * reduce_or(v): OR of a per-lane value over the document's lanes (uniform result).
//  * sync(): every write before it is visible to every lane after it.
//  * single(f): f() runs once (lane 0).
//  * cas64/min32/min64/add32/add64/max32/or32/fetch_or32: atomics on scratch memory.
#pragma once
#include "langid.h"
#include "tb_common.h"

// Chunks of 64 items whose loads a wave issues together in the latency-bound passes (WavePar).
// 1 since the round-2 kernel rework: serialized stage-kernel time per 262,144-doc step (two
// stages, tools/kernel_ab.sh) 89.1 ms at 1, 90.9 ms at 2, 93.5 ms at 4 (register pressure).
#ifndef TB_UNROLL
#define TB_UNROLL 1
#endif

namespace tb {

// u32 words mask_bits() writes for n items (whole 64-bit chunks).
TB_HD constexpr uint32_t mask_words(uint32_t n) { return ((n + 63) / 64) * 2; }

struct SeqPar {
  static constexpr bool kPartTables = false;  // canonicalize(): LDS-partitioned tables (no LDS here)
  // Wave-cooperative sequential loops (dup_walk_wave): the waves of the document's group, each
  // running whole-wave code; 0 = none (run the scalar version on one lane).
  static constexpr uint32_t kWaves = 0;
  uint32_t wave_index() const { return 0; }
  template <class F>
  void for_n(uint32_t n, F&& f) const {
    for (uint32_t i = 0; i < n; ++i) f(i);
  }
  template <class S, class Pred, class Emit>
  uint32_t compact(uint32_t n, Pred&& pred, Emit&& emit) const {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; ++i) {
      S st{};
      if (pred(i, st)) emit(i, k++, st);
    }
    return k;
  }
  template <class T, class F>
  T sum(uint32_t n, F&& f) const {
    T s = 0;
    for (uint32_t i = 0; i < n; ++i) s += f(i);
    return s;
  }
  template <class T, class F>
  T max(uint32_t n, T init, F&& f) const {
    T s = init;
    for (uint32_t i = 0; i < n; ++i) { T v = f(i); if (v > s) s = v; }
    return s;
  }
  template <class T, class F>
  T min(uint32_t n, T init, F&& f) const {
    T s = init;
    for (uint32_t i = 0; i < n; ++i) { T v = f(i); if (v < s) s = v; }
    return s;
  }
  template <class T, class Op, class In, class Out>
  T scan(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    T acc = id;
    for (uint32_t i = 0; i < n; ++i) {
      const T v = in(i);  // read before out(i) may overwrite what in(i) reads (as on the device)
      out(i, acc);
      acc = op(acc, v);
    }
    return acc;
  }
  template <int K, class T, class Op, class In, class Out>
  T scan_blocked(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    return scan(n, id, op, in, out);
  }
  // bits[i >> 5] bit (i & 31) = pred(i) for i < n; words up to the next multiple of 64 bits
  // are written (callers size `bits` as mask_words(n)).
  template <class Pred>
  void mask_bits(uint32_t n, Pred&& pred, uint32_t* bits) const {
    const uint32_t nw = ((n + 63) / 64) * 2;
    for (uint32_t w = 0; w < nw; ++w) bits[w] = 0;
    for (uint32_t i = 0; i < n; ++i) if (pred(i)) bits[i >> 5] |= 1u << (i & 31);
  }
  // mask_bits with the words handed to store(w, bits) (any destination address space).
  template <class Pred, class Store>
  void mask_store(uint32_t n, Pred&& pred, Store&& store) const {
    const uint32_t nw = ((n + 63) / 64) * 2;
    for (uint32_t w = 0; w < nw; ++w) {
      uint32_t v = 0;
      for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t i = w * 32 + j;
        if (i < n && pred(i)) v |= 1u << j;
      }
      store(w, v);
    }
  }
  // Inclusive scan fused with a compaction: sel(i, incl) picks items given their inclusive
  // prefix, emit(i, k, incl) gets the rank k among picked items. Returns the number picked.
  template <class T, class Op, class In, class Sel, class Emit>
  uint32_t scan_compact(uint32_t n, T id, Op&& op, In&& in, Sel&& sel, Emit&& emit) const {
    T acc = id;
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; ++i) {
      acc = op(acc, in(i));
      if (sel(i, acc)) emit(i, k++, acc);
    }
    return k;
  }
  uint32_t reduce_or(uint32_t v) const { return v; }
  template <class T>
  T reduce_add(T v) const { return v; }
  // Chunked ballots (the WavePar loop, run sequentially): per chunk of 64 items, bits(i) gives up
  // to 4 predicate bits per item, m[k] = the chunk's 64-bit mask of bit k; sel(i, l, m) picks items,
  // emit(i, l, m, rank) runs for the picked ones in item order, then uni(base, m) once per chunk
  // (state carried between chunks). Returns the number picked.
  static constexpr bool kChunks = true;
  template <class Bits, class Sel, class Emit, class Uni>
  uint32_t chunks(uint32_t n, Bits&& bits, Sel&& sel, Emit&& emit, Uni&& uni) const {
    uint32_t k = 0;
    for (uint32_t base = 0; base < n; base += 64) {
      uint64_t m[4] = {0, 0, 0, 0};
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t i = base + l;
        const uint32_t b = i < n ? bits(i) : 0u;
        for (int q = 0; q < 4; ++q)
          if ((b >> q) & 1u) m[q] |= 1ull << l;
      }
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t i = base + l;
        if (i < n && sel(i, l, m)) emit(i, l, m, k++);
      }
      uni(base, m);
    }
    return k;
  }
  void sync() const {}
  static uint64_t clock() { return 0; }
  template <class F>
  void single(F&& f) const { f(); }
  bool leader() const { return true; }
  static uint64_t cas64(uint64_t* p, uint64_t cmp, uint64_t val) {
    uint64_t old = *p;
    if (old == cmp) *p = val;
    return old;
  }
  static uint32_t cas32(uint32_t* p, uint32_t cmp, uint32_t val) {
    uint32_t old = *p;
    if (old == cmp) *p = val;
    return old;
  }
  static void min32(uint32_t* p, uint32_t v) { if (v < *p) *p = v; }
  static void min64(uint64_t* p, uint64_t v) { if (v < *p) *p = v; }
  static void max32(uint32_t* p, uint32_t v) { if (v > *p) *p = v; }
  static uint32_t add32(uint32_t* p, uint32_t v) { uint32_t o = *p; *p += v; return o; }
  static void or32(uint32_t* p, uint32_t v) { *p |= v; }
  static uint32_t fetch_or32(uint32_t* p, uint32_t v) { const uint32_t o = *p; *p |= v; return o; }
  // Integer accumulation over items: f(i, part) adds item i's contribution into part[0..D)
  // (int32 partials); sums[d] receives the exact int64 total. tmp is unused on the host.
  template <int D, class F>
  void accum_rows(uint32_t n, F&& f, int32_t* tmp, int64_t* sums) const {
    (void)tmp;
    int64_t acc[D];
    int32_t part[D];
    for (int d = 0; d < D; ++d) acc[d] = 0;
    for (uint32_t i = 0; i < n; ++i) {
      for (int d = 0; d < D; ++d) part[d] = 0;
      f(i, part);
      for (int d = 0; d < D; ++d) acc[d] += part[d];
    }
    for (int d = 0; d < D; ++d) sums[d] = acc[d];
  }
};

#if defined(__HIPCC__)
namespace pardetail {
// Shuffle any POD element 32 bits at a time.
template <class T>
__device__ inline T shfl_up_t(T v, int o) {
  constexpr int N = (int)((sizeof(T) + 3) / 4);
  int w[N];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __shfl_up(w[k], o);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}
template <class T>
__device__ inline T shfl_t(T v, int src) {
  constexpr int N = (int)((sizeof(T) + 3) / 4);
  int w[N];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __shfl(w[k], src);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}
// Cross-lane moves by DPP (a VALU operand modifier: a few cycles, no LDS crossbar round trip
// like ds_bpermute), one 32-bit word at a time for any POD element.
template <int CTRL, class T>
__device__ __forceinline__ T dpp_mov_t(T v) {
  constexpr int N = (int)((sizeof(T) + 3) / 4);
  int w[N] = {};
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __builtin_amdgcn_mov_dpp(w[k], CTRL, 0xF, 0xF, false);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}
// Lane 63's value in every lane (scalar read-lane per word).
template <class T>
__device__ __forceinline__ T bcast63(T v) {
  constexpr int N = (int)((sizeof(T) + 3) / 4);
  int w[N] = {};
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __builtin_amdgcn_readlane(w[k], 63);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}
// Inclusive wave64 scan (op associative, not necessarily commutative): Hillis-Steele inside
// each row of 16 lanes with row_shr:1/2/4/8, then row_bcast:15 and row_bcast:31 carry the row
// totals across rows (the rocPRIM warp_scan_dpp schedule): 6 DPP moves instead of 6
// ds_bpermute round trips.
template <class T, class Op>
__device__ __forceinline__ T wave_incl_scan(T x, uint32_t lane, Op&& op) {
  const uint32_t rl = lane & 15u;
  { const T t = dpp_mov_t<0x111>(x); if (rl >= 1u) x = op(t, x); }
  { const T t = dpp_mov_t<0x112>(x); if (rl >= 2u) x = op(t, x); }
  { const T t = dpp_mov_t<0x114>(x); if (rl >= 4u) x = op(t, x); }
  { const T t = dpp_mov_t<0x118>(x); if (rl >= 8u) x = op(t, x); }
  { const T t = dpp_mov_t<0x142>(x); if ((lane & 31u) >= 16u) x = op(t, x); }
  { const T t = dpp_mov_t<0x143>(x); if (lane >= 32u) x = op(t, x); }
  return x;
}
}  // namespace pardetail

struct WavePar {
  static constexpr bool kPartTables = false;  // short documents: tables fit the slice (registers matter more)
  static constexpr uint32_t kWaves = 1;
  uint32_t lane;
  __device__ uint32_t wave_index() const { return 0; }
  __device__ WavePar() : lane(threadIdx.x & 63) {}

  template <class F>
  __device__ __forceinline__ void for_n(uint32_t n, F&& f) const {
    for (uint32_t i = lane; i < n; i += 64) f(i);
  }
  // The per-document passes are bound by memory latency (scratch arrays mostly miss L2), so
  // the pure parts of a pass (predicates, scan inputs, reduction terms) are evaluated for
  // kUnroll chunks of 64 items before any of them is consumed: each lane keeps kUnroll
  // independent loads in flight instead of one. Results are unchanged (chunk order is kept,
  // integer reductions are exact in any order).
  static constexpr uint32_t kU = TB_UNROLL;
  template <class S, class Pred, class Emit>
  __device__ __forceinline__ uint32_t compact(uint32_t n, Pred&& pred, Emit&& emit) const {
    uint32_t k = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t base = 0; base < n; base += 64 * kU) {
      S st[kU];
      bool p[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = base + 64 * u + lane;
        st[u] = S{};
        p[u] = i < n && pred(i, st[u]);
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = base + 64 * u + lane;
        const uint64_t m = __ballot(p[u]);
        if (p[u]) emit(i, k + (uint32_t)__popcll(m & lt), st[u]);
        k += (uint32_t)__popcll(m);
      }
    }
    return k;
  }
  template <class T>
  __device__ __forceinline__ T wave_sum(T v) const {
    return pardetail::bcast63(pardetail::wave_incl_scan(v, lane, [](T a, T b) { return a + b; }));
  }
  template <class T>
  __device__ __forceinline__ T wave_max(T v) const {
    return pardetail::bcast63(pardetail::wave_incl_scan(v, lane, [](T a, T b) { return a > b ? a : b; }));
  }
  template <class T>
  __device__ __forceinline__ T wave_min(T v) const {
    return pardetail::bcast63(pardetail::wave_incl_scan(v, lane, [](T a, T b) { return a < b ? a : b; }));
  }
  template <class T, class F>
  __device__ __forceinline__ T sum(uint32_t n, F&& f) const {
    T s[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) s[u] = 0;
    uint32_t i = lane;
    for (; i + 64 * (kU - 1) < n; i += 64 * kU) {
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) s[u] += f(i + 64 * u);
    }
    for (; i < n; i += 64) s[0] += f(i);
#pragma unroll
    for (uint32_t u = 1; u < kU; ++u) s[0] += s[u];
    return wave_sum(s[0]);
  }
  template <class T, class F>
  __device__ __forceinline__ T max(uint32_t n, T init, F&& f) const {
    T s[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) s[u] = init;
    uint32_t i = lane;
    for (; i + 64 * (kU - 1) < n; i += 64 * kU) {
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) { T v = f(i + 64 * u); if (v > s[u]) s[u] = v; }
    }
    for (; i < n; i += 64) { T v = f(i); if (v > s[0]) s[0] = v; }
#pragma unroll
    for (uint32_t u = 1; u < kU; ++u) if (s[u] > s[0]) s[0] = s[u];
    return wave_max(s[0]);
  }
  template <class T, class F>
  __device__ __forceinline__ T min(uint32_t n, T init, F&& f) const {
    T s[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) s[u] = init;
    uint32_t i = lane;
    for (; i + 64 * (kU - 1) < n; i += 64 * kU) {
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) { T v = f(i + 64 * u); if (v < s[u]) s[u] = v; }
    }
    for (; i < n; i += 64) { T v = f(i); if (v < s[0]) s[0] = v; }
#pragma unroll
    for (uint32_t u = 1; u < kU; ++u) if (s[u] < s[0]) s[0] = s[u];
    return wave_min(s[0]);
  }
  template <class T, class Op, class In, class Out>
  __device__ __forceinline__ T scan(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    T carry = id;
    for (uint32_t base0 = 0; base0 < n; base0 += 64 * kU) {
      T xs[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = base0 + 64 * u + lane;
        xs[u] = i < n ? in(i) : id;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t base = base0 + 64 * u;
        if (base >= n) break;
        const uint32_t i = base + lane;
        const T x = pardetail::wave_incl_scan(xs[u], lane, op);
        T excl = pardetail::shfl_up_t(x, 1);
        if (lane == 0) excl = id;
        if (i < n) out(i, op(carry, excl));
        carry = op(carry, pardetail::bcast63(x));
      }
    }
    return carry;
  }
  // Same contract as scan(), for expensive ops over long inputs: each lane folds K consecutive
  // items sequentially in registers, only the 64 block totals go through the cross-lane scan,
  // then each lane replays its block to emit the prefixes (op evaluated ~2x per item instead of
  // log2(64) = 6x, and K-fold fewer shuffles).
  template <int K, class T, class Op, class In, class Out>
  __device__ __forceinline__ T scan_blocked(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    T carry = id;
    for (uint32_t base = 0; base < n; base += 64u * K) {
      const uint32_t start = base + lane * K;
      T tot = id;
      for (int k = 0; k < K; ++k) {
        const uint32_t i = start + k;
        if (i < n) tot = op(tot, in(i));
      }
      const T x = pardetail::wave_incl_scan(tot, lane, op);
      T excl = pardetail::shfl_up_t(x, 1);
      if (lane == 0) excl = id;
      T run = op(carry, excl);
      for (int k = 0; k < K; ++k) {
        const uint32_t i = start + k;
        if (i < n) {
          const T v = in(i);
          out(i, run);
          run = op(run, v);
        }
      }
      carry = op(carry, pardetail::bcast63(x));
    }
    return carry;
  }
  __device__ __forceinline__ uint32_t reduce_or(uint32_t v) const {
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
    return v;
  }
  template <class T>
  __device__ __forceinline__ T reduce_add(T v) const { return wave_sum(v); }
  static constexpr bool kChunks = true;
  template <class Bits, class Sel, class Emit, class Uni>
  __device__ __forceinline__ uint32_t chunks(uint32_t n, Bits&& bits, Sel&& sel, Emit&& emit, Uni&& uni) const {
    uint32_t k = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + lane;
      const uint32_t b = i < n ? bits(i) : 0u;
      uint64_t m[4];
      m[0] = __ballot(b & 1u);
      m[1] = __ballot(b & 2u);
      m[2] = __ballot(b & 4u);
      m[3] = __ballot(b & 8u);
      const bool s = i < n && sel(i, lane, m);
      const uint64_t sm = __ballot(s);
      if (s) emit(i, lane, m, k + (uint32_t)__popcll(sm & lt));
      k += (uint32_t)__popcll(sm);
      uni(base, m);
    }
    return k;
  }
  template <class Pred>
  __device__ __forceinline__ void mask_bits(uint32_t n, Pred&& pred, uint32_t* bits) const {
    for (uint32_t base = 0; base < n; base += 64 * kU) {
      bool p[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = base + 64 * u + lane;
        p[u] = i < n && pred(i);
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t b0 = base + 64 * u;
        const uint64_t m = __ballot(p[u]);
        if (b0 < n && lane < 2) bits[(b0 >> 5) + lane] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
      }
    }
  }
  template <class Pred, class Store>
  __device__ __forceinline__ void mask_store(uint32_t n, Pred&& pred, Store&& store) const {
    for (uint32_t b0 = 0; b0 < n; b0 += 64) {
      const uint32_t i = b0 + lane;
      const uint64_t m = __ballot(i < n && pred(i));
      if (lane < 2) store((b0 >> 5) + lane, lane ? (uint32_t)(m >> 32) : (uint32_t)m);
    }
  }
  template <class T, class Op, class In, class Sel, class Emit>
  __device__ __forceinline__ uint32_t scan_compact(uint32_t n, T id, Op&& op, In&& in, Sel&& sel,
                                                   Emit&& emit) const {
    T carry = id;
    uint32_t k = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t base0 = 0; base0 < n; base0 += 64 * kU) {
      T xs[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t i = base0 + 64 * u + lane;
        xs[u] = i < n ? in(i) : id;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t base = base0 + 64 * u;
        if (base >= n) break;
        const uint32_t i = base + lane;
        const T x = pardetail::wave_incl_scan(xs[u], lane, op);
        const T incl = op(carry, x);
        const bool p = i < n && sel(i, incl);
        const uint64_t m = __ballot(p);
        if (p) emit(i, k + (uint32_t)__popcll(m & lt), incl);
        k += (uint32_t)__popcll(m);
        carry = op(carry, pardetail::bcast63(x));
      }
    }
    return k;
  }
  __device__ __forceinline__ void sync() const { __syncthreads(); }
  __device__ __forceinline__ static uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
  template <class F>
  __device__ __forceinline__ void single(F&& f) const { if (lane == 0) f(); }
  __device__ __forceinline__ bool leader() const { return lane == 0; }
  __device__ __forceinline__ static uint64_t cas64(uint64_t* p, uint64_t cmp, uint64_t val) {
    return atomicCAS((unsigned long long*)p, (unsigned long long)cmp, (unsigned long long)val);
  }
  __device__ __forceinline__ static uint32_t cas32(uint32_t* p, uint32_t cmp, uint32_t val) {
    return atomicCAS(p, cmp, val);
  }
  __device__ __forceinline__ static void min32(uint32_t* p, uint32_t v) { atomicMin(p, v); }
  __device__ __forceinline__ static void min64(uint64_t* p, uint64_t v) {
    atomicMin((unsigned long long*)p, (unsigned long long)v);
  }
  __device__ __forceinline__ static void max32(uint32_t* p, uint32_t v) { atomicMax(p, v); }
  __device__ __forceinline__ static uint32_t add32(uint32_t* p, uint32_t v) { return atomicAdd(p, v); }
  __device__ __forceinline__ static void or32(uint32_t* p, uint32_t v) { atomicOr(p, v); }
  __device__ __forceinline__ static uint32_t fetch_or32(uint32_t* p, uint32_t v) { return atomicOr(p, v); }

  // Each lane accumulates its items (i = lane, lane+64, ...) in D int32 registers, so the
  // item loads of one lane are independent of the other lanes' and of each other; the 64 x D
  // partials then go through `tmp` (64*D int32, LDS when available) and lane d sums column d
  // in int64. Callers bound the per-lane magnitude so int32 partials cannot overflow.
  template <int D, class F>
  __device__ __forceinline__ void accum_rows(uint32_t n, F&& f, int32_t* tmp, int64_t* sums) const {
    int32_t part[D];
#pragma unroll
    for (int d = 0; d < D; ++d) part[d] = 0;
    for (uint32_t i = lane; i < n; i += 64) f(i, part);
#pragma unroll
    for (int d = 0; d < D; ++d) tmp[lane * D + d] = part[d];
    __syncthreads();
    for (int d = (int)lane; d < D; d += 64) {
      int64_t s = 0;
      for (int r = 0; r < 64; ++r) s += tmp[r * D + d];
      sums[d] = s;
    }
    __syncthreads();
  }

};

// One workgroup of NT threads (NT/64 waves) per document, for long documents: the same
// contract as WavePar with block-wide results. Cross-wave exchange goes through `xs`, a small
// LDS buffer the kernel provides (>= 16 * NT/64 bytes). Every primitive ends with a barrier, so
// `xs` can be reused by the next call.
template <int NT>
struct BlockPar {
  static_assert(NT % 64 == 0 && NT >= 128 && NT <= 1024, "block of whole waves");
  static constexpr int NW = NT / 64;
  static constexpr bool kChunks = false;
#ifdef TB_NO_PART_TABLES
  static constexpr bool kPartTables = false;
#else
  static constexpr bool kPartTables = true;   // long documents: LDS-partitioned hash tables
#endif
  static constexpr uint32_t kWaves = NW;
  uint32_t tid, lane, wid;
  char* xs = nullptr;
  __device__ uint32_t wave_index() const { return wid; }
  __device__ BlockPar() : tid(threadIdx.x), lane(threadIdx.x & 63), wid(threadIdx.x >> 6) {}

  template <class F>
  __device__ __forceinline__ void for_n(uint32_t n, F&& f) const {
    for (uint32_t i = tid; i < n; i += NT) f(i);
  }
  template <class S, class Pred, class Emit>
  __device__ __forceinline__ uint32_t compact(uint32_t n, Pred&& pred, Emit&& emit) const {
    uint32_t k = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t* cnt = (uint32_t*)xs;
    for (uint32_t base = 0; base < n; base += NT) {
      const uint32_t i = base + tid;
      S st{};
      const bool p = i < n && pred(i, st);
      const uint64_t m = __ballot(p);
      if (lane == 0) cnt[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, tot = 0;
      for (int w = 0; w < NW; ++w) {
        const uint32_t c = cnt[w];
        if (w < (int)wid) before += c;
        tot += c;
      }
      if (p) emit(i, k + before + (uint32_t)__popcll(m & lt), st);
      k += tot;
      __syncthreads();
    }
    return k;
  }
  template <class T, class Op>
  __device__ __forceinline__ T block_reduce(T v, Op&& op) const {
    for (int o = 32; o > 0; o >>= 1) v = op(v, pardetail::shfl_t(v, (int)(lane ^ o)));
    T* t = (T*)xs;
    if (lane == 0) t[wid] = v;
    __syncthreads();
    T r = t[0];
    for (int w = 1; w < NW; ++w) r = op(r, t[w]);
    __syncthreads();
    return r;
  }
  template <class T, class F>
  __device__ __forceinline__ T sum(uint32_t n, F&& f) const {
    T s = 0;
    for (uint32_t i = tid; i < n; i += NT) s += f(i);
    return block_reduce(s, [](T a, T b) { return a + b; });
  }
  template <class T, class F>
  __device__ __forceinline__ T max(uint32_t n, T init, F&& f) const {
    T s = init;
    for (uint32_t i = tid; i < n; i += NT) { T v = f(i); if (v > s) s = v; }
    return block_reduce(s, [](T a, T b) { return a > b ? a : b; });
  }
  template <class T, class F>
  __device__ __forceinline__ T min(uint32_t n, T init, F&& f) const {
    T s = init;
    for (uint32_t i = tid; i < n; i += NT) { T v = f(i); if (v < s) s = v; }
    return block_reduce(s, [](T a, T b) { return a < b ? a : b; });
  }
  // Exclusive prefix of this wave's inclusive totals across waves (in wave order).
  template <class T, class Op>
  __device__ __forceinline__ void cross_wave(T wave_incl_last, T id, Op&& op, T& before, T& total) const {
    T* t = (T*)xs;
    if (lane == 63) t[wid] = wave_incl_last;
    __syncthreads();
    before = id;
    total = id;
    for (int w = 0; w < NW; ++w) {
      const T v = t[w];
      if (w < (int)wid) before = op(before, v);
      total = op(total, v);
    }
    __syncthreads();
  }
  template <class T, class Op, class In, class Out>
  __device__ __forceinline__ T scan(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    T carry = id;
    for (uint32_t base = 0; base < n; base += NT) {
      const uint32_t i = base + tid;
      T x = i < n ? in(i) : id;
      x = pardetail::wave_incl_scan(x, lane, op);
      T excl = pardetail::shfl_up_t(x, 1);
      if (lane == 0) excl = id;
      T before, total;
      cross_wave(pardetail::bcast63(x), id, op, before, total);
      if (i < n) out(i, op(carry, op(before, excl)));
      carry = op(carry, total);
    }
    return carry;
  }
  template <int K, class T, class Op, class In, class Out>
  __device__ __forceinline__ T scan_blocked(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    T carry = id;
    for (uint32_t base = 0; base < n; base += (uint32_t)NT * K) {
      const uint32_t start = base + tid * K;
      T tot = id;
      for (int k = 0; k < K; ++k) {
        const uint32_t i = start + k;
        if (i < n) tot = op(tot, in(i));
      }
      T x = pardetail::wave_incl_scan(tot, lane, op);
      T excl = pardetail::shfl_up_t(x, 1);
      if (lane == 0) excl = id;
      T before, total;
      cross_wave(pardetail::bcast63(x), id, op, before, total);
      T run = op(carry, op(before, excl));
      for (int k = 0; k < K; ++k) {
        const uint32_t i = start + k;
        if (i < n) {
          const T v = in(i);
          out(i, run);
          run = op(run, v);
        }
      }
      carry = op(carry, total);
    }
    return carry;
  }
  __device__ __forceinline__ uint32_t reduce_or(uint32_t v) const {
    return block_reduce(v, [](uint32_t a, uint32_t b) { return a | b; });
  }
  template <class T>
  __device__ __forceinline__ T reduce_add(T v) const {
    return block_reduce(v, [](T a, T b) { return a + b; });
  }
  template <class Pred>
  __device__ __forceinline__ void mask_bits(uint32_t n, Pred&& pred, uint32_t* bits) const {
    for (uint32_t base = wid * 64; base < n; base += NT) {
      const uint32_t i = base + lane;
      const uint64_t m = __ballot(i < n && pred(i));
      if (lane < 2) bits[(base >> 5) + lane] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
  }
  template <class Pred, class Store>
  __device__ __forceinline__ void mask_store(uint32_t n, Pred&& pred, Store&& store) const {
    for (uint32_t base = wid * 64; base < n; base += NT) {
      const uint32_t i = base + lane;
      const uint64_t m = __ballot(i < n && pred(i));
      if (lane < 2) store((base >> 5) + lane, lane ? (uint32_t)(m >> 32) : (uint32_t)m);
    }
  }
  template <class T, class Op, class In, class Sel, class Emit>
  __device__ __forceinline__ uint32_t scan_compact(uint32_t n, T id, Op&& op, In&& in, Sel&& sel,
                                                   Emit&& emit) const {
    T carry = id;
    uint32_t k = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t* cnt = (uint32_t*)(xs + 16 * NW);  // past cross_wave's slots (T <= 16 bytes); xs has 64 B slack
    for (uint32_t base = 0; base < n; base += NT) {
      const uint32_t i = base + tid;
      T x = i < n ? in(i) : id;
      x = pardetail::wave_incl_scan(x, lane, op);
      T before, total;
      cross_wave(pardetail::bcast63(x), id, op, before, total);
      const T incl = op(carry, op(before, x));
      const bool p = i < n && sel(i, incl);
      const uint64_t m = __ballot(p);
      if (lane == 0) cnt[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t pre = 0, tot = 0;
      for (int w = 0; w < NW; ++w) {
        const uint32_t c = cnt[w];
        if (w < (int)wid) pre += c;
        tot += c;
      }
      if (p) emit(i, k + pre + (uint32_t)__popcll(m & lt), incl);
      k += tot;
      carry = op(carry, total);
      __syncthreads();
    }
    return k;
  }
  __device__ __forceinline__ void sync() const { __syncthreads(); }
  __device__ __forceinline__ static uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
  template <class F>
  __device__ __forceinline__ void single(F&& f) const { if (tid == 0) f(); }
  __device__ __forceinline__ bool leader() const { return tid == 0; }
  __device__ __forceinline__ static uint64_t cas64(uint64_t* p, uint64_t cmp, uint64_t val) {
    return atomicCAS((unsigned long long*)p, (unsigned long long)cmp, (unsigned long long)val);
  }
  __device__ __forceinline__ static uint32_t cas32(uint32_t* p, uint32_t cmp, uint32_t val) {
    return atomicCAS(p, cmp, val);
  }
  __device__ __forceinline__ static void min32(uint32_t* p, uint32_t v) { atomicMin(p, v); }
  __device__ __forceinline__ static void min64(uint64_t* p, uint64_t v) {
    atomicMin((unsigned long long*)p, (unsigned long long)v);
  }
  __device__ __forceinline__ static void max32(uint32_t* p, uint32_t v) { atomicMax(p, v); }
  __device__ __forceinline__ static uint32_t add32(uint32_t* p, uint32_t v) { return atomicAdd(p, v); }
  __device__ __forceinline__ static void or32(uint32_t* p, uint32_t v) { atomicOr(p, v); }
  __device__ __forceinline__ static uint32_t fetch_or32(uint32_t* p, uint32_t v) { return atomicOr(p, v); }
};

// NT/64 waves on one document with few barriers: items [0, n) are cut into one contiguous
// segment per wave (whole 64-item chunks), every wave runs the WavePar loop over its own
// segment, and only the per-wave totals cross waves (through `xs`, double-buffered so one barrier
// per primitive suffices). Compactions and scans run in two passes over the segment (count /
// total first, then emit with the wave's offset): their predicates and inputs are evaluated
// twice, in exchange for one barrier per call instead of two per 64 x NW items (BlockPar).
// `xs` must hold >= 2 * 16 * NW bytes; the owner resets `gen` never (it only alternates halves).
template <int NT>
struct SegPar {
  static_assert(NT % 64 == 0 && NT >= 128 && NT <= 1024, "block of whole waves");
  static constexpr int NW = NT / 64;
  static constexpr bool kPartTables = false;
  static constexpr bool kChunks = false;
  static constexpr uint32_t kWaves = NW;
  uint32_t tid, lane, wid;
  char* xs = nullptr;
  mutable uint32_t gen = 0;
  __device__ uint32_t wave_index() const { return wid; }
  __device__ SegPar() : tid(threadIdx.x), lane(threadIdx.x & 63), wid(threadIdx.x >> 6) {}

  // this wave's item range [b, e)
  __device__ __forceinline__ void seg(uint32_t n, uint32_t& b, uint32_t& e) const {
    const uint32_t chunks = (n + 63) >> 6;
    const uint32_t per = (chunks + NW - 1) / NW;
    b = wid * per * 64;
    e = b + per * 64;
    if (b > n) b = n;
    if (e > n) e = n;
  }
  template <class T>
  __device__ __forceinline__ T* slot() const {
    return (T*)(xs + (gen & 1u) * 16 * NW);
  }
  // exclusive prefix (over waves before this one) and total of a per-wave value; one barrier
  template <class T, class Op>
  __device__ __forceinline__ void across(T mine, T id, Op&& op, T& before, T& total) const {
    T* t = slot<T>();
    if (lane == 0) t[wid] = mine;
    __syncthreads();
    before = id;
    total = id;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const T v = t[w];
      if (w < (int)wid) before = op(before, v);
      total = op(total, v);
    }
    ++gen;
  }
  template <class T, class Op>
  __device__ __forceinline__ T all(T mine, T id, Op&& op) const {
    T before, total;
    across(mine, id, op, before, total);
    return total;
  }

  template <class F>
  __device__ __forceinline__ void for_n(uint32_t n, F&& f) const {
    uint32_t b, e;
    seg(n, b, e);
    for (uint32_t i = b + lane; i < e; i += 64) f(i);
  }
  template <class S, class Pred, class Emit>
  __device__ __forceinline__ uint32_t compact(uint32_t n, Pred&& pred, Emit&& emit) const {
    uint32_t b, e;
    seg(n, b, e);
    uint32_t cnt = 0;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      S st{};
      cnt += (uint32_t)__popcll(__ballot(i < e && pred(i, st)));
    }
    uint32_t before, total;
    across(cnt, 0u, [](uint32_t a, uint32_t c) { return a + c; }, before, total);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t k = before;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      S st{};
      const bool p = i < e && pred(i, st);
      const uint64_t m = __ballot(p);
      if (p) emit(i, k + (uint32_t)__popcll(m & lt), st);
      k += (uint32_t)__popcll(m);
    }
    return total;
  }
  template <class T>
  __device__ __forceinline__ T wave_sum(T v) const {
    return pardetail::bcast63(pardetail::wave_incl_scan(v, lane, [](T a, T c) { return a + c; }));
  }
  template <class T, class F>
  __device__ __forceinline__ T sum(uint32_t n, F&& f) const {
    uint32_t b, e;
    seg(n, b, e);
    T s = 0;
    for (uint32_t i = b + lane; i < e; i += 64) s += f(i);
    return all(wave_sum(s), (T)0, [](T a, T c) { return a + c; });
  }
  template <class T, class F>
  __device__ __forceinline__ T max(uint32_t n, T init, F&& f) const {
    uint32_t b, e;
    seg(n, b, e);
    T s = init;
    for (uint32_t i = b + lane; i < e; i += 64) { T v = f(i); if (v > s) s = v; }
    s = pardetail::bcast63(pardetail::wave_incl_scan(s, lane, [](T a, T c) { return a > c ? a : c; }));
    return all(s, init, [](T a, T c) { return a > c ? a : c; });
  }
  template <class T, class F>
  __device__ __forceinline__ T min(uint32_t n, T init, F&& f) const {
    uint32_t b, e;
    seg(n, b, e);
    T s = init;
    for (uint32_t i = b + lane; i < e; i += 64) { T v = f(i); if (v < s) s = v; }
    s = pardetail::bcast63(pardetail::wave_incl_scan(s, lane, [](T a, T c) { return a < c ? a : c; }));
    return all(s, init, [](T a, T c) { return a < c ? a : c; });
  }
  template <class T, class Op, class In, class Out>
  __device__ __forceinline__ T scan(uint32_t n, T id, Op&& op, In&& in, Out&& out) const {
    uint32_t b, e;
    seg(n, b, e);
    T tot = id;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      const T x = pardetail::wave_incl_scan(i < e ? in(i) : id, lane, op);
      tot = op(tot, pardetail::bcast63(x));
    }
    T before, total;
    across(tot, id, op, before, total);
    T carry = before;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      const T v = i < e ? in(i) : id;
      const T x = pardetail::wave_incl_scan(v, lane, op);
      T excl = pardetail::shfl_up_t(x, 1);
      if (lane == 0) excl = id;
      if (i < e) out(i, op(carry, excl));
      carry = op(carry, pardetail::bcast63(x));
    }
    return total;
  }
  template <class T, class Op, class In, class Sel, class Emit>
  __device__ __forceinline__ uint32_t scan_compact(uint32_t n, T id, Op&& op, In&& in, Sel&& sel,
                                                   Emit&& emit) const {
    // pass 1: the segment's scan total (what carries into the next segment); its selected count
    // needs the incoming carry, so the two are exchanged in two steps
    uint32_t b, e;
    seg(n, b, e);
    T tot = id;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      const T x = pardetail::wave_incl_scan(i < e ? in(i) : id, lane, op);
      tot = op(tot, pardetail::bcast63(x));
    }
    T before, total;
    across(tot, id, op, before, total);
    uint32_t cnt = 0;
    {
      T carry = before;
      for (uint32_t base = b; base < e; base += 64) {
        const uint32_t i = base + lane;
        const T x = pardetail::wave_incl_scan(i < e ? in(i) : id, lane, op);
        const T incl = op(carry, x);
        cnt += (uint32_t)__popcll(__ballot(i < e && sel(i, incl)));
        carry = op(carry, pardetail::bcast63(x));
      }
    }
    uint32_t kbefore, ktotal;
    across(cnt, 0u, [](uint32_t a, uint32_t c) { return a + c; }, kbefore, ktotal);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    T carry = before;
    uint32_t k = kbefore;
    for (uint32_t base = b; base < e; base += 64) {
      const uint32_t i = base + lane;
      const T x = pardetail::wave_incl_scan(i < e ? in(i) : id, lane, op);
      const T incl = op(carry, x);
      const bool p = i < e && sel(i, incl);
      const uint64_t m = __ballot(p);
      if (p) emit(i, k + (uint32_t)__popcll(m & lt), incl);
      k += (uint32_t)__popcll(m);
      carry = op(carry, pardetail::bcast63(x));
    }
    return ktotal;
  }
  __device__ __forceinline__ uint32_t reduce_or(uint32_t v) const {
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
    return all(v, 0u, [](uint32_t a, uint32_t c) { return a | c; });
  }
  template <class T>
  __device__ __forceinline__ T reduce_add(T v) const {
    return all(wave_sum(v), (T)0, [](T a, T c) { return a + c; });
  }
  template <class Pred, class Store>
  __device__ __forceinline__ void mask_store(uint32_t n, Pred&& pred, Store&& store) const {
    uint32_t b, e;
    seg(n, b, e);
    for (uint32_t b0 = b; b0 < e; b0 += 64) {
      const uint32_t i = b0 + lane;
      const uint64_t m = __ballot(i < e && pred(i));
      if (lane < 2) store((b0 >> 5) + lane, lane ? (uint32_t)(m >> 32) : (uint32_t)m);
    }
  }
  __device__ __forceinline__ void sync() const { __syncthreads(); }
  __device__ __forceinline__ static uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
  template <class F>
  __device__ __forceinline__ void single(F&& f) const { if (tid == 0) f(); }
  __device__ __forceinline__ bool leader() const { return tid == 0; }
  __device__ __forceinline__ static void or32(uint32_t* p, uint32_t v) { atomicOr(p, v); }
  __device__ __forceinline__ static uint32_t fetch_or32(uint32_t* p, uint32_t v) { return atomicOr(p, v); }
};
#endif

}  // namespace tb
