// HIP kernels for gfx950 (MI355X). C ABI, launched on a caller-provided stream (the native HIP
// runtime layer's, csrc/hip/runtime.hip).
//
// Document kernels run one wavefront per document (block = 64 lanes = one wave64): the lanes
// cooperate through DPP shuffles and ballots (csrc/common/par.h WavePar), per-document working
// arrays live in a per-document slice of an HBM scratch arena (L2-resident while the wave
// works on it). Grid = number of documents, visited through a length-sorted permutation so the
// longest documents start first (tail-latency balance under the power-law length distribution).
//
//  tb_stage_analyze   : decode + UAX#29 words + lines + hashes -> Gopher/FineWeb records
//  tb_langid_mfma     : fastText int8 embedding bag + bf16 MFMA head (16 docs per tile) -> language records
//  tb_c4_pass_a       : C4 line filtering, citation removal, rewritten text into scratch
//  tb_c4_pass_b       : compaction of the rewritten texts into the next content version
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <string>

#include "../common/docproc.h"
#include "../common/gate.h"
#include "../common/badwords.h"

using namespace tb;

namespace {

constexpr uint32_t kMaxLdsPerDoc = 160 * 1024;
// Workgroup kernels also hold static LDS (g_block_xs) on top of the dynamic slice: a 160 KB
// slice fails at launch (HSA_STATUS_ERROR_INVALID_ALLOCATION, measured), so they take <= 128 KB.
constexpr uint32_t kMaxLdsPerBlk = 128 * 1024;

struct DevTables {
  const uint16_t* s1;
  const uint32_t* s2;
  const uint16_t* l1;
  const int32_t* l2;
};

// Dynamic LDS: each workgroup (= one wave = one document) gets `lds_bytes` of fast arena; the
// document's working arrays are carved from it first and spill to its HBM scratch slice.
extern __shared__ __attribute__((aligned(16))) char g_lds_arena[];

template <class P = WavePar>
__device__ __forceinline__ DocCtx<P> make_ctx(const DevTables& t, const uint64_t* pw, uint32_t pw_n,
                                             char* scratch, const int64_t* scratch_off, int doc, int k,
                                             uint32_t* flags, uint32_t lds_bytes, uint64_t* prof) {
  DocCtx<P> x;
  x.prof = prof ? prof + (size_t)doc * kPhaseSlots : nullptr;
  x.lds = lds_bytes ? (char*)g_lds_arena : nullptr;
  x.lcap = lds_bytes;
  x.lused = 0;
  x.ucd = UcdView{t.s1, t.s2, t.l1, t.l2};
  x.pw = pw;
  x.pw_n = pw_n;
  x.ipw = pw ? pw + pw_n + 1 : nullptr;
  // scratch slices are laid out in dispatch order (k = position in the launched permutation), so
  // the waves resident at the same time work in one contiguous window of the arena
  x.scr = scratch + scratch_off[k];
  x.cap = (uint64_t)(scratch_off[k + 1] - scratch_off[k]);
  x.used = 0;
  x.flag = flags + doc;
  return x;
}

// Per-wave LDS copies that turn the hottest global reads into LDS reads: the compact UCD properties
// of U+0000..U+00FF (every decode looks up ASCII and Latin-1 letters there instead of the two-level
// global table) and, for wave-path documents, the text
// itself (read by every pass: lead bytes, decoding, hashing, byte verification). The text copy
// moves whole dwords (the batch buffers are padded, so the up to 3 bytes read past a document's
// end stay inside the allocation).
template <class P>
__device__ __forceinline__ void lds_ascii_props(DocCtx<P>& x) {
  uint16_t* asc = x.template try_lds<uint16_t>(256);
  if (!asc) return;
  x.par.for_n(256, [&](uint32_t c) { asc[c] = compact_prop(x.ucd.props(c)); });
  x.par.sync();
  x.asc = asc;
}

template <class P>
__device__ __forceinline__ const uint8_t* lds_text(DocCtx<P>& x, const uint8_t* b, uint32_t n) {
  const uintptr_t a0 = (uintptr_t)b & ~(uintptr_t)3;
  const uint32_t head = (uint32_t)((uintptr_t)b - a0);
  const uint32_t nd = (head + n + 3) >> 2;
  uint32_t* d = x.template try_lds<uint32_t>(nd + 1);
  if (!d) return b;
  const uint32_t* src = (const uint32_t*)a0;
  x.par.for_n(nd, [&](uint32_t k) { d[k] = src[k]; });
  x.par.sync();
  return (const uint8_t*)d + head;
}

// C4 pass A leaves src[0] relative to the document's scratch slice (the convention the host
// emulation shares); pass B copies straight out of the arena, so the leader makes it absolute.
template <class P>
__device__ __forceinline__ void c4_src_absolute(DocCtx<P>& x, int64_t* src, int64_t slice_begin) {
  if (x.par.leader() && src[0] >= 0) src[0] += slice_begin;
}

// The stage kernel is register-bound (occupancy = waves/SIMD the VGPR budget allows). With the
// n-gram orders moved to k_gr_ngrams / k_gr_split_wave it is built for 8 waves/SIMD (64 VGPRs,
// the spills it adds sit outside the per-chunk loops) with a 5 KB LDS slice per wave: 4.55 vs
// 5.05 ms per launch at 6 waves / 6.5 KB, 7 waves no gain (profiles/r8_wpe/; 6 beat 4 and 5 before,
// profiles/r7_ngram/ab_occupancy.txt; before the move 4 waves won, round 2).
#define TB_STAGE_KERNEL(NAME, ATTR)                                                                   \
  __global__ __launch_bounds__(64) ATTR void NAME(                                                   \
      const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes, \
      const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t ndocs, char* scratch,        \
      const int64_t* __restrict__ scratch_off, const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs, \
      int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof,                               \
      const uint8_t* __restrict__ dead, uint32_t* line_stats, GrExport* gr_export, DictIn dict) {      \
    const int doc = perm ? perm[blockIdx.x] : (int)blockIdx.x;                                        \
    if (doc >= ndocs || (dead && dead[doc])) return;                                                  \
    DocCtx<WavePar> x = make_ctx(tabs, pw, pw_n, scratch, scratch_off, doc, (int)blockIdx.x, flags, lds_bytes, prof);   \
    const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);                                           \
    lds_ascii_props(x);                                                                               \
    const uint8_t* b = lds_text(x, bytes + off[doc], n);                                              \
    StageOut out{rec, (uint32_t)ndocs, (uint32_t)doc};                                                \
    if (line_stats) out.line_stats = line_stats + line_stats_base(off[doc], doc);                     \
    if (gr_export) { out.gr_export = gr_export + blockIdx.x; out.b_global = bytes + off[doc]; }       \
    out.dict = dict;                                                                                  \
    analyze_stage<WavePar, false>(x, *stage, *plan, LidTables{}, b, n, out); /* LD: own kernel */ \
  }

#ifndef TB_STAGE_WPE
#define TB_STAGE_WPE 8
#endif
TB_STAGE_KERNEL(k_stage_analyze_wave, __attribute__((amdgpu_waves_per_eu(TB_STAGE_WPE, 8))))

// Long documents: one workgroup of kBlockThreads (8 waves by default) per document (BlockPar), launched
// over the long prefix of the length-sorted permutation.
#ifndef TB_BLOCK_THREADS
#define TB_BLOCK_THREADS 512
#endif
constexpr int kBlockThreads = TB_BLOCK_THREADS;
// Register budget of the long-document stage kernel: 6 waves per SIMD (<= 80 VGPRs), so with the
// default 48 KB LDS slice three 512-thread workgroups (three documents) share a CU instead of one
// (174 VGPRs unconstrained). The kernel is latency-bound; config 5 (4096 x 50 KB documents,
// profiles/r2_c5/blk_variants.txt): 70.9K docs/s unconstrained/64 KB, 110.0K at 4 waves/64 KB,
// 113.7K at 6 waves/48 KB. TB_BLK_WPE=k builds another budget (0: none) for A/B runs.
// Re-measured with the round-5 kernels (profiles/r8_blk4): 4 waves (128 VGPRs, 93 spilled
// instead of 229) at 64 KB gives 139.9K vs 150.4K at 6 waves -- the spills stay cheaper than
// the lost occupancy.
#ifndef TB_BLK_WPE
#define TB_BLK_WPE 6
#endif
#if TB_BLK_WPE > 0
#define TB_BLK_ATTR __attribute__((amdgpu_waves_per_eu(TB_BLK_WPE, 8)))
#else
#define TB_BLK_ATTR
#endif
__shared__ __attribute__((aligned(16))) char g_block_xs[16 * (kBlockThreads / 64) + 64];

template <int NT, bool kPre = false>
__device__ __forceinline__ void stage_blk_body(
    const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes,
    const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t ndocs, char* scratch,
    const int64_t* __restrict__ scratch_off, const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs,
    int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof, const uint8_t* __restrict__ dead,
    GrExport* gr_export, int32_t n_split, uint32_t split_bytes, uint32_t* line_stats, const PreDoc* pre,
    int32_t n_pre, DictIn dict) {
  const int doc = perm[blockIdx.x];
  if (doc >= ndocs || (dead && dead[doc])) return;
  DocCtx<BlockPar<NT>> x =
      make_ctx<BlockPar<NT>>(tabs, pw, pw_n, scratch, scratch_off, doc, (int)blockIdx.x, flags, lds_bytes, prof);
  x.par.xs = g_block_xs;
  lds_ascii_props(x);
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  StageOut out{rec, (uint32_t)ndocs, (uint32_t)doc};
  out.dict = dict;
  if (line_stats) out.line_stats = line_stats + line_stats_base(off[doc], doc);
  if constexpr (kPre) {
    if (pre[blockIdx.x].n != n) return;  // (never: the host builds the descriptors from these lengths)
    out.pre = pre + blockIdx.x;
  }
  // split documents (the first n_split launch positions, longer than split_bytes) export their
  // word arrays; k_gr_dup_split finishes their duplicated n-gram orders
  if (gr_export && (int)blockIdx.x < n_split && n > split_bytes) out.gr_export = gr_export + blockIdx.x;
  analyze_stage<BlockPar<NT>, false, kPre>(x, *stage, *plan, LidTables{}, b, n, out);
}

#define TB_STAGE_BLK_KERNEL(NAME, NT, PRE)                                                             \
  __global__ __launch_bounds__(NT) TB_BLK_ATTR void NAME(                                            \
      const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes, \
      const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t ndocs, char* scratch,         \
      const int64_t* __restrict__ scratch_off, const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs,  \
      int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof, const uint8_t* __restrict__ dead,   \
      GrExport* gr_export, int32_t n_split, uint32_t split_bytes, uint32_t* line_stats,                \
      const PreDoc* pre, int32_t n_pre, DictIn dict) {                                                 \
    stage_blk_body<NT, PRE>(plan, stage, bytes, off, perm, ndocs, scratch, scratch_off, pw, pw_n, tabs, rec, flags, \
                       lds_bytes, prof, dead, gr_export, n_split, split_bytes, line_stats, pre, n_pre, dict); \
  }
TB_STAGE_BLK_KERNEL(k_stage_analyze_blk, kBlockThreads, false)
// documents with a pre-pass (tb_stage_analyze_blk with `pre`): every launch position has one
TB_STAGE_BLK_KERNEL(k_stage_analyze_blk_pre, kBlockThreads, true)

// SURVEY 5.7 intra-document split: one workgroup per (split document, task): n_tasks = the
// GopherRepetition step's duplicated n-gram orders, its top orders, then duplicated lines and
// duplicated paragraphs. Block k handles launch
// position k / n_tasks (perm order, the stage kernel's export slot) and task k % n_tasks; each
// task works in its own 1/n_tasks share of the document's unused scratch slice.
// Persistent (SURVEY 5.7 work queue): the grid is what the CUs hold at once; every workgroup
// takes the next (document, task) from an atomic cursor until the queue is empty, in launch order
// (documents longest first, their tasks together), so the heaviest tasks start first and a
// workgroup that finishes early takes more. Every workgroup exits once the cursor passes the end.
__global__ __launch_bounds__(kBlockThreads) TB_BLK_ATTR void k_gr_dup_split(
    const DevStage* __restrict__ stage, int32_t gr_step, const int32_t* __restrict__ perm, int32_t n_split,
    int32_t n_tasks, int32_t ndocs, const GrExport* __restrict__ ex, const uint64_t* __restrict__ pw, uint32_t pw_n,
    DevTables tabs, int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint32_t* cursor) {
  __shared__ int s_task;
  const int total = n_split * n_tasks;
  const DevStep& ds = stage->steps[gr_step];
  while (true) {
    if (threadIdx.x == 0) s_task = (int)atomicAdd(cursor, 1u);
    __syncthreads();
    const int task = s_task;
    __syncthreads();  // (s_task is rewritten by the next iteration's claim)
    if (task >= total) break;
    const int k = task / n_tasks, t = task % n_tasks;
    const int doc = perm[k];
    if (doc >= ndocs) continue;
    const GrExport e = ex[k];
    if (!e.valid) continue;  // not exported: skipped, returned early (flagged for the CPU path) or short
    DocCtx<BlockPar<kBlockThreads>> x;
    x.prof = nullptr;
    x.lds = lds_bytes ? (char*)g_lds_arena : nullptr;
    x.lcap = lds_bytes;
    x.lused = 0;
    x.ucd = UcdView{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
    x.pw = pw;
    x.pw_n = pw_n;
    x.ipw = pw ? pw + pw_n + 1 : nullptr;
    const uint64_t region = (e.free_cap / (uint64_t)n_tasks) & ~255ull;
    x.scr = e.free_base + (uint64_t)t * region;
    x.cap = region;
    x.used = 0;
    x.flag = flags + doc;
    x.par.xs = g_block_xs;
    int64_t* r = rec + (int64_t)ds.rec_prefix * ndocs + (int64_t)doc * ds.width;
    if (t < ds.n_dup) gr_dup_one_order(x, ds, t, e, r);
    else if (t < ds.n_dup + ds.n_top) gr_top_one_order(x, ds, t - ds.n_dup, e, r);
    else if (t < ds.n_dup + ds.n_top + 2) gr_lines_split(x, t - ds.n_dup - ds.n_top, e, r);
    if (x.overflow) x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW);
    __syncthreads();  // the task's LDS is the next task's
  }
}

// ---- n-gram orders of wave documents, one workgroup per document (k_gr_ngrams) ---------------
// The stage kernel exports each wave document's word arrays (GrExport: canonical word ids, byte
// prefix WL, concatenation hash prefixes K / PB). Here kNgWaves waves share one document: they
// stage its arrays into LDS once (coalesced), then each wave takes whole orders (duplicated, then
// top), one gram per lane at a time, and its table in the
// wave's own LDS region; every LDS array comes from __shared__ declarations (ds_* instructions).
// Records equal gr_dup_one_order / gr_top_one_order (the canonical id of a gram is the smallest
// index of an equal gram however the table is probed). The host launches it over the shorter
// wave documents of the length-sorted launch (the longer ones take one wave per (document, order),
// k_gr_split_wave, whose tables use a dynamic LDS slice); a document with more words than the
// workgroup's arrays hold (or byte prefixes past 16 bits) runs the generic per-order code
// (gr_dup_one_order / gr_top_one_order) over its HBM scratch instead.
constexpr int kNgWaves = 4;

// LDS of one document's workgroup for documents of at most MAXW words: the staged word arrays and
// one region per wave, the larger of the duplicated-order layout (u32 table, u16 canonical ids,
// candidate positions and slots, seen / repeat bitmaps) and the top-order layout (u32 table, u16
// candidate positions, u32 counts packed with slots). The table's space first holds the two
// candidate bitmaps of the order (ng_candidates).
template <uint32_t MAXW>
struct NgShared {
  static_assert(MAXW % 64 == 0, "whole waves of grams");
  static constexpr uint32_t kMaxW = MAXW;
  static constexpr uint32_t kCap = MAXW + MAXW / 2 + 4;  // table slots (1.5 G + 2, rounded)
  static constexpr uint32_t kSW = (MAXW + 31) / 32 + 1;
  // candidate bitmaps: two arrays of kBW words (a power of two, >= 16 bits per gram) in the table
  static constexpr uint32_t kBW = MAXW / 2;
  static_assert(2 * kBW <= kCap && (kBW & (kBW - 1)) == 0, "bitmaps fit the table space");
  static constexpr uint32_t kDupBytes = 4 * kCap + 3 * 2 * MAXW + 4 * 2 * ((kSW + 3) & ~3u);
  static constexpr uint32_t kTopBytes = 4 * kCap + 2 * MAXW + 4 * MAXW;
  static constexpr uint32_t kRegion = ((kDupBytes > kTopBytes ? kDupBytes : kTopBytes) + 15) & ~15u;
  uint64_t K[MAXW + 1];
  uint64_t PB[MAXW + 1];
  uint16_t wid[MAXW + 1];
  uint16_t WL[MAXW + 1];
  uint4 region[kNgWaves][kRegion / 16];
};

// the documents the LDS path of k_gr_ngrams<hi> takes: <= hi words, 16-bit word byte prefixes
__device__ __forceinline__ bool ng_fits(const GrExport& e, uint32_t hi) {
  return e.W <= hi && e.WL[e.W] <= 0xFFFFu;
}

__device__ __forceinline__ uint32_t ng_home(uint64_t k, uint32_t capn) {
  return (uint32_t)(((k & 0xFFFFFFFFull) * capn) >> 32);
}

// Repeat candidates of one order: a superset of the positions whose gram occurs more than once.
// Every gram sets bit h(key) of `once` (fetch-or); a gram that finds its bit already set sets it
// in `twice`. Equal grams have equal keys, so every repeated gram lands on a bit of `twice`; a
// gram whose bit no other gram set occurs once (it cannot repeat), and only the candidates go
// through the exact canonicalisation. With >= 16 bits per gram a unique gram is a false candidate
// with probability < 1/16. Both bitmaps (kBW words each) must be zero on entry. Candidate
// positions land in `list` in increasing order; returns their number (wave-uniform).
template <class NS, class KeyF>
__device__ __forceinline__ uint32_t ng_candidates(uint32_t G, uint32_t lane, uint32_t* once, uint32_t* twice,
                                                  uint16_t* hbuf, uint16_t* list, KeyF&& key) {
  constexpr uint32_t kMask = NS::kBW * 32u - 1u;
  static_assert(kMask <= 0xFFFFu, "bit index in 16 bits");
  // (each position's bit index goes through hbuf, not registers: the kernel is register-bound)
#pragma unroll 1
  for (uint32_t p = lane; p < G; p += 64) {
    const uint32_t h = (uint32_t)(key(p) >> 20) & kMask;
    hbuf[p] = (uint16_t)h;
    const uint32_t bit = 1u << (h & 31u);
    if (atomicOr(&once[h >> 5], bit) & bit) atomicOr(&twice[h >> 5], bit);
  }
  __builtin_amdgcn_wave_barrier();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t nc = 0;
#pragma unroll 1
  for (uint32_t base = 0; base < G; base += 64) {
    const uint32_t p = base + lane;
    bool c = false;
    if (p < G) {
      const uint32_t h = hbuf[p];
      c = (twice[h >> 5] >> (h & 31u)) & 1u;
    }
    const uint64_t m = __ballot(c);
    if (c) list[nc + (uint32_t)__popcll(m & lt)] = (uint16_t)p;
    nc += (uint32_t)__popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  return nc;
}

// gram equality of order n (DupGrams::eq over the staged arrays; the byte comparison of grams with
// different word sequences reads the exported HBM arrays)
// (out of line: the byte comparison of different word splits with equal hashes practically never
// runs, and inlined its seven array pointers stay live in registers through the whole order)
__device__ __attribute__((noinline)) bool ng_dup_eq_bytes(const GrExport* ep, uint32_t p, uint32_t q, uint32_t n) {
  const DupGrams dg{ep->wid, ep->WL, ep->K, ep->PB, ep->bs, ep->be, ep->b};
  return dg.eq(p, q, n);
}
template <class NS>
__device__ __forceinline__ bool ng_dup_eq(const NS& S, const GrExport* ep, uint32_t p, uint32_t q, uint32_t n) {
  if ((uint32_t)(S.WL[p + n] - S.WL[p]) != (uint32_t)(S.WL[q + n] - S.WL[q])) return false;
  uint32_t dw = 0;
  for (uint32_t k = 0; k < n; ++k) dw |= (uint32_t)(S.wid[p + k] ^ S.wid[q + k]);
  if (dw == 0) return true;
  return ng_dup_eq_bytes(ep, p, q, n);
}

template <class NS>
__device__ __forceinline__ int64_t ng_dup_order(NS& S, const GrExport* ep, uint32_t W, uint32_t n, uint32_t lane,
                                                uint4* region, bool prof, uint64_t& c_canon, uint64_t& c_walk) {
  const uint64_t t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t G = W - n + 1;
  const uint32_t SW = (G + 31) / 32 + 1;
  const uint32_t SWa = (SW + 3u) & ~3u;
  uint32_t* tab = (uint32_t*)region;
  uint16_t* gc = (uint16_t*)(tab + NS::kCap);   // per position: canonical candidate index
  uint16_t* list = gc + NS::kMaxW;              // candidate positions
  uint16_t* gsl = list + NS::kMaxW;             // per candidate: its table slot
  uint32_t* sn = (uint32_t*)(gsl + NS::kMaxW);
  uint32_t* R = sn + SWa;
  for (uint32_t i = lane; i < 2 * NS::kBW; i += 64) tab[i] = 0;
  for (uint32_t i = lane; i < 2 * SWa; i += 64) sn[i] = 0;
  __builtin_amdgcn_wave_barrier();
  auto key = [&](uint32_t p) {
    return dev_key(S.PB[p + n] * (S.K[p + n] - S.K[p]), (uint32_t)(S.WL[p + n] - S.WL[p]));
  };
  const uint32_t nc = ng_candidates<NS>(G, lane, tab, tab + NS::kBW, gc, list, key);
  if (nc < 2) {  // no gram occurs twice: nothing repeats, the walk counts nothing
    if (prof) c_canon += __builtin_amdgcn_s_memtime() - t0;
    return 0;
  }
  // exact canonicalisation of the candidates: slot value (fp << 16) | (candidate index + 1)
  const uint32_t capn = nc + (nc >> 1) + 2;
  for (uint32_t i = lane; i < capn; i += 64) tab[i] = 0;
  __builtin_amdgcn_wave_barrier();
#pragma unroll 1
  for (uint32_t c = lane; c < nc; c += 64) {
    const uint32_t p = list[c];
    const uint64_t k = key(p);
    const uint32_t fp = (uint32_t)(k >> 48);
    const uint32_t mine = (fp << 16) | (c + 1);
    uint32_t sl = ng_home(k, capn);
    while (true) {
      uint32_t cur = tab[sl];
      if (cur == 0) {
        cur = atomicCAS(&tab[sl], 0u, mine);
        if (cur == 0) break;
      }
      if ((cur >> 16) == fp && ng_dup_eq(S, ep, p, list[(cur & 0xFFFFu) - 1u], n)) {
        if ((cur & 0xFFFFu) > c + 1u) atomicMin(&tab[sl], mine);
        break;
      }
      if (++sl == capn) sl = 0;
    }
    gsl[c] = (uint16_t)sl;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll 1
  for (uint32_t c = lane; c < nc; c += 64) {
    const uint32_t g = (tab[gsl[c]] & 0xFFFFu) - 1u;
    const uint32_t p = list[c];
    gc[p] = (uint16_t)g;
    if (g != c) {
      const uint32_t q = list[g];
      atomicOr(&R[p >> 5], 1u << (p & 31));
      atomicOr(&R[q >> 5], 1u << (q & 31));
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint64_t t1 = prof ? __builtin_amdgcn_s_memtime() : 0;
  c_canon += t1 - t0;
  // greedy walk (reference find_all_duplicate, utils/text.rs:241-259; dup_walk_wave over LDS):
  // it only stops at repeated positions (candidates), whose gc holds the class id
  const uint32_t nw = (G + 31) >> 5;
  int64_t rep = 0;
  uint32_t idx = 0;
  while (idx < G) {
    uint32_t p0 = G;
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
    uint32_t g = 0xFFFFFFFFu, l = 0;
    if (act) {
      g = gc[p];
      l = (uint32_t)(S.WL[p + n] - S.WL[p]);
    }
    const bool seen0 = act && ((sn[g >> 5] >> (g & 31)) & 1u);
    uint64_t A = __ballot(act), Sm = __ballot(seen0), cnt = 0, fv = 0;
    uint32_t next = p0 + 64;
    while (A) {
      const uint32_t k = (uint32_t)__builtin_ctzll(A);
      if ((Sm >> k) & 1ull) {
        cnt |= 1ull << k;
        const uint32_t jj = k + n;
        A = jj >= 64 ? 0ull : (A & (~0ull << jj));
        if (p0 + jj > next) next = p0 + jj;
      } else {
        fv |= 1ull << k;
        Sm |= __ballot(g == (uint32_t)__builtin_amdgcn_readlane((int)g, (int)k));
        A &= A - 1;
      }
    }
    if ((fv >> lane) & 1ull) atomicOr(&sn[g >> 5], 1u << (g & 31));
    uint32_t add = ((cnt >> lane) & 1ull) ? l : 0u;
    for (int o = 32; o > 0; o >>= 1) add += (uint32_t)__shfl_xor((int)add, o);
    rep += add;
    __builtin_amdgcn_wave_barrier();
    idx = next;
  }
  if (prof) c_walk += __builtin_amdgcn_s_memtime() - t1;
  return rep;
}

// top n-gram order (reference find_top_duplicate, utils/text.rs:211-238): space-joined grams are
// equal iff their word sequences are, so grams are grouped by their canonical word-id tuples
// (fingerprint table, exact tuple comparison on a match) and counted per canonical gram. Only the
// repeat candidates (ng_candidates) are grouped: every other gram occurs once.
template <class NS>
__device__ __forceinline__ int64_t ng_top_order(NS& S, uint32_t W, uint32_t n, uint32_t lane, uint4* region) {
  const uint32_t G = W - n + 1;
  uint32_t* tab = (uint32_t*)region;
  uint16_t* list = (uint16_t*)(tab + NS::kCap);
  uint32_t* cnt = (uint32_t*)(list + NS::kMaxW);  // per candidate: slot << 16 | count
  for (uint32_t i = lane; i < 2 * NS::kBW; i += 64) tab[i] = 0;
  __builtin_amdgcn_wave_barrier();
  auto key = [&](uint32_t p) {
    uint64_t h = (uint64_t)n << 56;
    for (uint32_t k = 0; k < n; ++k) h = (h ^ S.wid[p + k]) * 0x9E3779B97F4A7C15ull + k;
    return mix64(h);
  };
  const uint32_t nc = ng_candidates<NS>(G, lane, tab, tab + NS::kBW, (uint16_t*)cnt, list, key);
  if (nc < 2) return 0;  // every gram occurs once
  const uint32_t capn = nc + (nc >> 1) + 2;
  for (uint32_t i = lane; i < capn; i += 64) tab[i] = 0;
  __builtin_amdgcn_wave_barrier();
#pragma unroll 1
  for (uint32_t c = lane; c < nc; c += 64) {
    const uint32_t p = list[c];
    const uint64_t k = key(p);
    const uint32_t fp = (uint32_t)(k >> 48);
    const uint32_t mine = (fp << 16) | (c + 1);
    uint32_t sl = ng_home(k, capn);
    while (true) {
      uint32_t cur = tab[sl];
      if (cur == 0) {
        cur = atomicCAS(&tab[sl], 0u, mine);
        if (cur == 0) break;
      }
      if ((cur >> 16) == fp) {
        const uint32_t qc = (cur & 0xFFFFu) - 1u;
        const uint32_t q = list[qc];
        uint32_t dw = 0;
        for (uint32_t k2 = 0; k2 < n; ++k2) dw |= (uint32_t)(S.wid[p + k2] ^ S.wid[q + k2]);
        if (dw == 0) {
          if (qc > c) atomicMin(&tab[sl], mine);
          break;
        }
      }
      if (++sl == capn) sl = 0;
    }
    cnt[c] = sl << 16;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll 1
  for (uint32_t c = lane; c < nc; c += 64) {
    const uint32_t g = (tab[cnt[c] >> 16] & 0xFFFFu) - 1u;
    atomicAdd(&cnt[g], 1u);  // low half: counts <= nc <= MAXW never carry into the slot
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t mx = 0;
  for (uint32_t c = lane; c < nc; c += 64) mx = (cnt[c] & 0xFFFFu) > mx ? (cnt[c] & 0xFFFFu) : mx;
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t v = (uint32_t)__shfl_xor((int)mx, o);
    mx = v > mx ? v : mx;
  }
  if (mx <= 1) return 0;
  uint32_t ml = 0;
  for (uint32_t c = lane; c < nc; c += 64) {
    if ((cnt[c] & 0xFFFFu) != mx) continue;
    const uint32_t p = list[c];
    const uint32_t len = (uint32_t)(S.WL[p + n] - S.WL[p]) + n - 1;
    ml = len > ml ? len : ml;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)ml, o);
    ml = w > ml ? w : ml;
  }
  return (int64_t)ml * (int64_t)mx;
}

#ifndef TB_NG_WPE
#define TB_NG_WPE 8  // 2.51 -> 2.29 ms/step vs 6 (profiles/r8_wpe/)
#endif
// Documents with more words than the workgroup's arrays hold (or byte prefixes past 16 bits) are
// not run here: their launch positions go to a list after the export array (NgRest), and
// k_gr_ngrams_rest runs their orders with the generic per-order code afterwards. Keeping that code
// out of this kernel keeps its registers (and the profiling counters, kProf) off the hot path.
struct NgRest {
  uint32_t count;   // documents in `pos`
  uint32_t cursor;  // k_gr_ngrams_rest's task cursor
  uint32_t pad[2];
  // followed by uint32_t pos[n_docs]
};
__host__ __device__ inline NgRest* ng_rest(const GrExport* ex, int32_t n_docs) {
  return (NgRest*)((char*)ex + (size_t)n_docs * sizeof(GrExport));
}

template <uint32_t MAXW, bool kProf>
__global__ __launch_bounds__(64 * kNgWaves) __attribute__((amdgpu_waves_per_eu(TB_NG_WPE, 8))) void k_gr_ngrams(
    const DevStage* __restrict__ stage, int32_t gr_step, const int32_t* __restrict__ perm, int32_t ndocs,
    const GrExport* __restrict__ ex, int32_t k0, NgRest* rest, int64_t* rec, uint64_t* prof) {
  __shared__ NgShared<MAXW> S;
  const int k = k0 + (int)blockIdx.x;
  const int doc = perm[k];
  if (doc >= ndocs) return;
  const GrExport& e = ex[k];
  if (!e.valid) return;  // dead, returned early (flagged for the CPU path) or no n-grams
  const uint32_t W = e.W;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (!ng_fits(e, MAXW)) {
    if (tid == 0) ((uint32_t*)(rest + 1))[atomicAdd(&rest->count, 1u)] = (uint32_t)k;
    return;
  }
  const DevStep& ds = stage->steps[gr_step];
  int64_t* r = rec + (int64_t)ds.rec_prefix * ndocs + (int64_t)doc * ds.width;
  const int nt = ds.n_dup + ds.n_top;
  uint64_t* pf = kProf ? prof + (size_t)doc * kPhaseSlots : nullptr;
  const uint64_t t0 = kProf ? __builtin_amdgcn_s_memtime() : 0;
  for (uint32_t i = tid; i <= W; i += 64 * kNgWaves) {
    S.K[i] = e.K[i];
    S.PB[i] = e.PB[i];
    S.WL[i] = (uint16_t)e.WL[i];
    S.wid[i] = i < W ? (uint16_t)e.wid[i] : (uint16_t)0;
  }
  __syncthreads();
  if (kProf && tid == 0) atomicAdd((unsigned long long*)&pf[PH_GR_DUP], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0));
  uint64_t c_canon = 0, c_walk = 0, c_top = 0;  // (profiling: this wave's cycles per phase)
  for (int t = (int)wv; t < nt; t += kNgWaves) {
    int64_t v = 0;
    if (t < ds.n_dup) {
      const uint32_t n = (uint32_t)ds.dup_n[t];
      if (n > 0 && W >= n) v = ng_dup_order(S, ex + k, W, n, lane, S.region[wv], kProf, c_canon, c_walk);
    } else {
      const uint32_t n = (uint32_t)ds.top_n[t - ds.n_dup];
      const uint64_t ts = kProf ? __builtin_amdgcn_s_memtime() : 0;
      if (n > 0 && W >= n) v = ng_top_order(S, W, n, lane, S.region[wv]);
      if (kProf) c_top += __builtin_amdgcn_s_memtime() - ts;
    }
    // record: the top orders first, then the duplicated orders
    if (lane == 0) r[rec_gr_fixed() + (t < ds.n_dup ? ds.n_top + t : t - ds.n_dup)] = v;
  }
  if (kProf && lane == 0) {
    atomicAdd((unsigned long long*)&pf[PH_GR_DUP_CANON], (unsigned long long)c_canon);
    atomicAdd((unsigned long long*)&pf[PH_GR_DUP_WALK], (unsigned long long)c_walk);
    atomicAdd((unsigned long long*)&pf[PH_GR_TOP_CANON], (unsigned long long)c_top);
  }
}

// The orders of the documents k_gr_ngrams listed in NgRest (more words than its arrays hold): one
// wave per (document, order) task from an atomic cursor, the generic per-order code over the
// document's HBM scratch (each order in its own share of the unused slice). Persistent: a fixed
// grid, every wave leaves once the cursor passes the last task.
__global__ __launch_bounds__(64) void k_gr_ngrams_rest(
    const DevStage* __restrict__ stage, int32_t gr_step, const int32_t* __restrict__ perm, int32_t ndocs,
    const GrExport* __restrict__ ex, NgRest* rest, const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs,
    int64_t* rec, uint32_t* flags) {
  const DevStep& ds = stage->steps[gr_step];
  const int nt = ds.n_dup + ds.n_top;
  const uint32_t total = __hip_atomic_load(&rest->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * (uint32_t)nt;
  const uint32_t* pos = (const uint32_t*)(rest + 1);
  while (true) {
    uint32_t task = 0;
    if (threadIdx.x == 0) task = atomicAdd(&rest->cursor, 1u);
    task = (uint32_t)__builtin_amdgcn_readfirstlane((int)task);
    if (task >= total) break;
    const int k = (int)pos[task / (uint32_t)nt], t = (int)(task % (uint32_t)nt);
    const int doc = perm[k];
    const GrExport e = ex[k];
    int64_t* r = rec + (int64_t)ds.rec_prefix * ndocs + (int64_t)doc * ds.width;
    DocCtx<WavePar> x;
    x.prof = nullptr;
    x.lds = nullptr;
    x.lcap = 0;
    x.lused = 0;
    x.ucd = UcdView{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
    x.pw = pw;
    x.pw_n = pw_n;
    x.ipw = pw ? pw + pw_n + 1 : nullptr;
    const uint64_t region = (e.free_cap / (uint64_t)nt) & ~255ull;
    x.scr = e.free_base + (uint64_t)t * region;
    x.cap = region;
    x.used = 0;
    x.flag = flags + doc;
    if (t < ds.n_dup) gr_dup_one_order(x, ds, t, e, r);
    else gr_top_one_order(x, ds, t - ds.n_dup, e, r);
    if (x.overflow) x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW);
  }
}

// The n-gram orders of wave documents (split mode of the wave stage kernel): one wave per
// (document, task), task = duplicated n-gram order t < n_dup, then top order t - n_dup. Block k
// handles launch position k / n_tasks of the wave launch (its export slot) and task k % n_tasks;
// every task works in its own share of the document's unused scratch slice (tables stay in the
// LDS slice for wave-sized documents). Same records as the in-stage path.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_gr_split_wave(
    const DevStage* __restrict__ stage, int32_t gr_step, const int32_t* __restrict__ perm, int32_t n_tasks,
    int32_t ndocs, const GrExport* __restrict__ ex, const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs,
    int64_t* rec, uint32_t* flags, uint32_t lds_bytes) {
  const int k = (int)blockIdx.x / n_tasks, t = (int)blockIdx.x % n_tasks;
  const int doc = perm[k];
  if (doc >= ndocs) return;
  const GrExport e = ex[k];
  if (!e.valid) return;  // not exported: dead, returned early (flagged for the CPU path) or no n-grams
  DocCtx<WavePar> x;
  x.prof = nullptr;
  x.lds = lds_bytes ? (char*)g_lds_arena : nullptr;
  x.lcap = lds_bytes;
  x.lused = 0;
  x.ucd = UcdView{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
  x.pw = pw;
  x.pw_n = pw_n;
  x.ipw = pw ? pw + pw_n + 1 : nullptr;
  const uint64_t region = (e.free_cap / (uint64_t)n_tasks) & ~255ull;
  x.scr = e.free_base + (uint64_t)t * region;
  x.cap = region;
  x.used = 0;
  x.flag = flags + doc;
  const DevStep& ds = stage->steps[gr_step];
  int64_t* r = rec + (int64_t)ds.rec_prefix * ndocs + (int64_t)doc * ds.width;
  if (t < ds.n_dup) gr_dup_one_order(x, ds, t, e, r);
  else if (t < ds.n_dup + ds.n_top) gr_top_one_order(x, ds, t - ds.n_dup, e, r);
  if (x.overflow) x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW);
}

// index of the highest set bit of m (m != 0)
__device__ __forceinline__ int lid_top(uint64_t m) { return 63 - __clzll((long long)m); }

// Language ID v3 (csrc/common/langid.h): two fastText bags + bf16 MFMA head, 16 documents per
// 256-thread workgroup: wave w gathers documents w, w + 4, w + 8, w + 12 of the tile one after
// another (launch positions blockIdx.x * 16 + ...; the length-sorted order keeps a tile's
// documents alike in size). Per 64-byte chunk every lane finds the n-grams ending at its code
// point (a chunked walk with the previous letters carried in registers; at most one gram per order
// n = 1..4, so each order has a fixed slot) and loads each gram's 16-byte embedding row with one
// dwordx4. Rows are added SWAR-style: the table holds E + 128 as
// unsigned bytes, even and odd bytes go to the two 16-bit halves of a register, the 1-/2-gram
// slots into one set of 8 packed registers (dims 0..15), the 3-/4-gram slots into another (dims
// 16..31) — no lane-dependent selects. Every 64 chunks (and at the end) a butterfly over the
// lanes (packed step first: two lanes' 64-chunk sums still fit 16 bits) folds the packed sums into
// one exact int32 dim per lane; minus 128 x #grams of its bag, that is the document's exact
// 32-dim sum, which the wave quantises with the document's block exponent (lid_block_exp /
// lid_quant: integers |a| <= 255, exact in bf16) into row r of the workgroup's 16 x 32 A tile in
// LDS. Wave 0 then runs the head as one v_mfma_f32_16x16x32_bf16 (A: 16 docs x 32 dims, B: the
// head transposed, 16 columns x 32 dims, integer bf16) and 16 lanes turn their row of the exact
// fp32 result into the record (lid_decide_v3). Same records as LangidModel on the host.
constexpr int kLidTile = 16;
constexpr int kLidWaves = 8;  // two documents per wave per tile
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Adds the 16-byte row of bucket g to one bag's packed sums: p[2q] holds dims 4q, 4q + 2 (even
// bytes of dword q), p[2q + 1] dims 4q + 1, 4q + 3.
__device__ __forceinline__ void lid_row_swar(const uint8_t* __restrict__ Eb, uint32_t g, uint32_t* p) {
  const uint4 w = *(const uint4*)(Eb + (size_t)g * kLidRowDim);
  const uint32_t v[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[2 * q] += v[q] & 0x00FF00FFu;
    p[2 * q + 1] += (v[q] >> 8) & 0x00FF00FFu;
  }
}

// Pair table of the 1-/2-gram bag (built once per model by k_lid_pairs, copied into every
// workgroup's LDS): over a 32-symbol alphabet — 0 = the word boundary / no letter, 1..26 = a-z
// (the ASCII letter & 0x1F), 27..31 = æ ø å ä ö — entry (x, y) holds, pre-split into the packed
// 16-bit layout of the bag's sums, every 1-/2-gram row a position with previous letter x and
// letter y adds: y != 0: E[1-gram y] + E[2-gram (x or boundary, y)]; y == 0, x != 0: E[2-gram
// (x, boundary)]; (0, 0): nothing. One position's orders 1 and 2 are then one LDS row (two
// ds_read_b128 + 8 adds) instead of two hashes, two 16-byte gathers and 32 unpack/add
// instructions. A position with a letter outside the alphabet takes the hashed gathers (rare in
// the model's languages). The table is followed by one zero row: the gather of an n-gram a
// position does not have points there, so the loop has no per-order branches.
constexpr int kLidSyms = 32;
constexpr int kLidPairs = kLidSyms * kLidSyms;
constexpr uint32_t kLidSymMiss = 32;
constexpr int kLidAuxBytes = kLidPairs * 32 + kLidRowDim;  // pair table + zero row

// the letter of alphabet symbol i (0: the word boundary)
__device__ __forceinline__ uint32_t lid_sym_letter(int i) {
  if (i == 0) return kLidBoundary;
  if (i <= 26) return 'a' + (uint32_t)(i - 1);
  return i == 27 ? 0xE6 : i == 28 ? 0xF8 : i == 29 ? 0xE5 : i == 30 ? 0xE4 : 0xF6;
}

// symbol of a non-ASCII lowercase letter: 27..31, or kLidSymMiss
__device__ __forceinline__ uint32_t lid_sym_latin(uint32_t l) {
  return l == 0xE6 ? 27u : l == 0xF8 ? 28u : l == 0xE5 ? 29u : l == 0xE4 ? 30u : l == 0xF6 ? 31u : kLidSymMiss;
}

__global__ __launch_bounds__(256) void k_lid_pairs(const uint8_t* __restrict__ Eb, uint32_t* __restrict__ aux) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < kLidPairs) {
    const int x = i / kLidSyms, y = i % kLidSyms;
    uint32_t d[kLidRowDim];
#pragma unroll
    for (int k = 0; k < kLidRowDim; ++k) d[k] = 0;
    auto add = [&](uint32_t g) {
      for (int k = 0; k < kLidRowDim; ++k) d[k] += Eb[(size_t)g * kLidRowDim + k];
    };
    if (y != 0) add(lid_hash(lid_sym_letter(y), 0, 0, 0, 1));
    if (x != 0 || y != 0) add(lid_hash(lid_sym_letter(x), lid_sym_letter(y), 0, 0, 2));
    // packed: dword 2q = dims 4q | 4q + 2 << 16, dword 2q + 1 = dims 4q + 1 | 4q + 3 << 16
    for (int q = 0; q < 4; ++q) {
      aux[i * 8 + 2 * q] = d[4 * q] | d[4 * q + 2] << 16;
      aux[i * 8 + 2 * q + 1] = d[4 * q + 1] | d[4 * q + 3] << 16;
    }
  }
  if (i < kLidRowDim / 4) aux[kLidPairs * 8 + i] = 0;  // the zero row
}

// the letter at lead byte `cur` = b[s] (< lim): ASCII and the Latin-1 block (lead byte 0xC3,
// U+00C0..U+00FF: letters except U+00D7 / U+00F7, upper case U+00C0..U+00DE lowered by 0x20 —
// the UCD's answers for that block) inline, the rest through the UCD tables (lid_letter)
__device__ __forceinline__ uint32_t lid_letter_dev(uint32_t cur, const uint8_t* b, uint32_t n, uint32_t s,
                                                   const UcdView& ucd) {
  if (cur < 0x80u) return (cur | 0x20u) - 'a' < 26u ? (cur | 0x20u) : 0u;
  if (cur == 0xC3u && s + 1 < n) {
    const uint32_t c = 0xC0u | (b[s + 1] & 0x3Fu);
    return (c == 0xD7u || c == 0xF7u) ? 0u : (c < 0xDFu ? c | 0x20u : c);
  }
  return lid_letter(ucd, b, n, s);
}

// Adds one 16-byte row (E + 128 bytes) to a bag's packed sums: p[2q] holds dims 4q, 4q + 2 (even
// bytes of dword q), p[2q + 1] dims 4q + 1, 4q + 3.
__device__ __forceinline__ void lid_add_u8(uint4 w, uint32_t* p) {
  const uint32_t v[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[2 * q] += v[q] & 0x00FF00FFu;
    p[2 * q + 1] += (v[q] >> 8) & 0x00FF00FFu;
  }
}

// Butterfly step: the lanes whose bit `m` is set keep the upper half of the n values, the others
// the lower half; each adds its partner's copy of the half it keeps.
template <int N>
__device__ __forceinline__ void lid_halve(const int32_t* in, int32_t* out, bool upper, int m) {
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    const int32_t keep = upper ? in[N / 2 + j] : in[j];
    const int32_t give = upper ? in[j] : in[N / 2 + j];
    out[j] = keep + __shfl_xor(give, m);
  }
}

// Folds both bags' packed sums (pa: dims 0..15, pb: dims 16..31; <= 64 chunks each) over the wave
// into `dsum` (lane l: dim 16 b5 + 4 (2 b4 + b3) + b2 + 2 b1 of lane l, lanes l and l ^ 1 alike) and
// clears them.
__device__ __forceinline__ void lid_fold(uint32_t* pa, uint32_t* pb, int lane, int32_t& dsum) {
  const bool up = (lane >> 5) & 1;
  uint32_t kept[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t keep = up ? pb[j] : pa[j];
    const uint32_t give = up ? pa[j] : pb[j];
    kept[j] = keep + (uint32_t)__shfl_xor((int)give, 32);  // two 64-chunk sums: < 2^16 per half
    pa[j] = pb[j] = 0;
  }
  int32_t u[16], v8[8], v4[4], v2[2], v1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // u[4q + 2e + h] = dim 4q + e + 2h of the kept bag
    u[2 * j] = (int32_t)(kept[j] & 0xFFFFu);
    u[2 * j + 1] = (int32_t)(kept[j] >> 16);
  }
  lid_halve<16>(u, v8, (lane >> 4) & 1, 16);
  lid_halve<8>(v8, v4, (lane >> 3) & 1, 8);
  lid_halve<4>(v4, v2, (lane >> 2) & 1, 4);
  lid_halve<2>(v2, &v1, (lane >> 1) & 1, 2);
  dsum += v1 + __shfl_xor(v1, 1);
}

// One document's quantised doc vector into A row `arow` (and its exponent / count). Per 64-byte
// chunk every lane handles the code point position at its byte: the letters of the previous
// three positions come from the wave's slot array in LDS (slot 3 + r holds the letter of the
// chunk's r-th position, slots 0..2 the last three of the previous chunks; the letter is stored
// with its alphabet symbol in bits 24..29), orders 1 + 2 are one pair-table row (pairs, LDS), orders
// 3 and 4 one hashed 16-byte gather each (an absent order gathers the zero row at `zero`).
__device__ __forceinline__ void lid_doc_vector(const uint8_t* __restrict__ b, uint32_t n, const UcdView& ucd,
                                               const uint8_t* __restrict__ Eb, const uint8_t* __restrict__ zero,
                                               const uint4* pairs, uint32_t* slot, int lane, uint16_t* arow,
                                               int32_t* e_out, int64_t* cnt_out) {
  // the cut: byte offset of code point kLidMaxCps (or n), by counting lead bytes per chunk
  uint32_t lim = n;
  if (n > (uint32_t)kLidMaxCps) {
    uint32_t seen = 0;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      const uint64_t m = __ballot(i < n && utf8_is_lead(b[i]));
      const uint32_t c = (uint32_t)__popcll(m);
      if (seen + c > (uint32_t)kLidMaxCps) {
        uint64_t mm = m;
        for (uint32_t k = seen; k < (uint32_t)kLidMaxCps; ++k) mm &= mm - 1;
        lim = base + (uint32_t)__builtin_ctzll(mm);
        break;
      }
      seen += c;
    }
  }
  uint32_t pa[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, pb[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  int32_t dsum = 0;
  uint32_t cnt_lo = 0, cnt_hi = 0, chunks = 0;  // grams of the 1-2-gram / 3-4-gram bags
  const uint32_t B = kLidBoundary;
  if (lane < 3) slot[lane] = 0;
  uint8_t cur = (uint32_t)lane < lim ? b[lane] : (uint8_t)0;
  for (uint32_t base = 0; base <= lim; base += 64) {
    const uint32_t s = base + (uint32_t)lane;
    const uint8_t nxt = s + 64 < lim ? b[s + 64] : (uint8_t)0;
    const bool lead = s < lim && utf8_is_lead(cur);
    const bool emit = lead || s == lim;  // position lim: the virtual non-letter after the cut
    uint32_t l0 = 0, y = 0;
    if (lead) {
      l0 = lid_letter_dev(cur, b, n, s, ucd);
      y = l0 < 0x80u ? (l0 & 0x1Fu) : lid_sym_latin(l0);
    }
    const uint64_t M = __ballot(lead);
    const uint64_t EM = __ballot(emit);
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(EM >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)EM, 0u));
    if (lead) slot[3 + r] = l0 | y << 24;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t e1 = slot[2 + r], e2 = slot[1 + r], e3 = slot[r];
    if (!emit) e1 = e2 = e3 = 0;
    const uint32_t lm1 = e1 & 0xFFFFFFu, lm2 = e2 & 0xFFFFFFu, lm3 = e3 & 0xFFFFFFu;
    const uint32_t x = e1 >> 24;  // symbol of the previous letter (0: none)
    // orders 1 + 2
    const bool miss = ((x | y) & kLidSymMiss) != 0;
    const uint4* pr = pairs + 2 * (miss ? 0u : (x << 5 | y));
    const uint4 t0 = pr[0], t1 = pr[1];
    pa[0] += t0.x; pa[1] += t0.y; pa[2] += t0.z; pa[3] += t0.w;
    pa[4] += t1.x; pa[5] += t1.y; pa[6] += t1.z; pa[7] += t1.w;
    cnt_lo += (l0 != 0u) + ((l0 | lm1) != 0u);
    if (__ballot(miss)) {
      if (miss) {
        if (l0) lid_add_u8(*(const uint4*)(Eb + (size_t)lid_hash(l0, 0, 0, 0, 1) * kLidRowDim), pa);
        if (l0 | lm1)
          lid_add_u8(*(const uint4*)(Eb + (size_t)lid_hash(lm1 ? lm1 : B, l0 ? l0 : B, 0, 0, 2) * kLidRowDim), pa);
      }
    }
    // orders 3 and 4
    const uint32_t x0 = l0 ? l0 : B;
    const bool v3 = lm1 != 0u, v4 = v3 && lm2 != 0u;
    const uint8_t* g3 = v3 ? Eb + (size_t)lid_hash(lm2 ? lm2 : B, lm1, x0, 0, 3) * kLidRowDim : zero;
    const uint8_t* g4 = v4 ? Eb + (size_t)lid_hash(lm3 ? lm3 : B, lm2, lm1, x0, 4) * kLidRowDim : zero;
    lid_add_u8(*(const uint4*)g3, pb);
    lid_add_u8(*(const uint4*)g4, pb);
    cnt_hi += (uint32_t)v3 + (uint32_t)v4;
    if ((++chunks & 63u) == 0) lid_fold(pa, pb, lane, dsum);
    // carry: the last three positions' letters to slots 0..2
    const uint32_t c = (uint32_t)__popcll(M);
    uint32_t keep = 0;
    if (lane < 3) keep = slot[c + lane];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < 3) slot[lane] = keep;
    cur = nxt;
  }
  lid_fold(pa, pb, lane, dsum);
  for (int o = 1; o < 64; o <<= 1) {
    cnt_lo += (uint32_t)__shfl_xor((int)cnt_lo, o);
    cnt_hi += (uint32_t)__shfl_xor((int)cnt_hi, o);
  }
  const uint32_t cnt = cnt_lo + cnt_hi;
  const bool up = ((lane >> 5) & 1) != 0;
  const int32_t S = dsum - 128 * (int32_t)(up ? cnt_hi : cnt_lo);
  const int dim = ((lane >> 5) & 1) * 16 + (2 * ((lane >> 4) & 1) + ((lane >> 3) & 1)) * 4 + ((lane >> 2) & 1) +
                  2 * ((lane >> 1) & 1);
  int32_t smax = S < 0 ? -S : S;
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t t = __shfl_xor(smax, o);
    smax = t > smax ? t : smax;
  }
  const int e = cnt ? lid_block_exp((int64_t)smax, (int64_t)cnt) : 0;
  if ((lane & 1) == 0) arow[dim] = cnt ? lid_bf16_bits((float)lid_quant((int64_t)S, e, (int64_t)cnt)) : (uint16_t)0;
  if (lane == 0) {
    *e_out = e;
    *cnt_out = (int64_t)cnt;
  }
  // (no dictionary-script flag: the language records are exact for every script; a document
  // with such code points goes to the CPU path only if it reaches a segmentation pass)
}

// Persistent: each workgroup copies the pair table into LDS once and then takes tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... (the grid is what the CUs hold at once: 4 workgroups of
// 8 waves per CU, 33 KB of pair table each).
__global__ __launch_bounds__(64 * kLidWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_langid_mfma(
    const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off, const int32_t* __restrict__ perm,
    int32_t ndocs, DevTables tabs, const uint8_t* __restrict__ Eb, const uint8_t* __restrict__ aux,
    const uint16_t* __restrict__ WT, double w_scale, const float* __restrict__ bias, int64_t* rec, int32_t width,
    uint64_t* prof) {
  __shared__ __attribute__((aligned(16))) uint16_t A[kLidTile][kLidDim];
  __shared__ float Cm[kLidTile][kLidHeadCols];
  __shared__ int32_t ex[kLidTile];
  __shared__ int64_t cn[kLidTile];
  __shared__ uint4 pairs[2 * kLidPairs];
  __shared__ uint32_t slots[kLidWaves][68];
  const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const UcdView ucd{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
  for (int i = (int)threadIdx.x; i < 2 * kLidPairs; i += 64 * kLidWaves) pairs[i] = ((const uint4*)aux)[i];
  const uint8_t* zero = aux + kLidPairs * 32;
  __syncthreads();
  const int ntiles = (ndocs + kLidTile - 1) / kLidTile;
  for (int tile = (int)blockIdx.x; tile < ntiles; tile += (int)gridDim.x) {
    for (int r = w; r < kLidTile; r += kLidWaves) {
      const int pos = tile * kLidTile + r;
      const int doc = pos < ndocs ? (perm ? perm[pos] : pos) : -1;
      if (doc < 0) {
        if (lane < kLidDim) A[r][lane] = 0;
        if (lane == 0) {
          ex[r] = 0;
          cn[r] = 0;
        }
        continue;
      }
      const uint64_t t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
      lid_doc_vector(bytes + off[doc], (uint32_t)(off[doc + 1] - off[doc]), ucd, Eb, zero, pairs, slots[w], lane,
                     A[r], &ex[r], &cn[r]);
      if (prof && lane == 0) prof[(size_t)doc * kPhaseSlots + PH_LID] += __builtin_amdgcn_s_memtime() - t0;
    }
    __syncthreads();
    if (w == 0) {
      // lane l: A[row l & 15][k 8 (l >> 4) .. +8), B[k 8 (l >> 4) .. +8][col l & 15] (= WT row)
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&A[lane & 15][8 * (lane >> 4)]);
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(WT + (lane & 15) * kLidDim + 8 * (lane >> 4));
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw, c, 0, 0, 0);
      // D[row (l >> 4) * 4 + r][col l & 15]
#pragma unroll
      for (int r = 0; r < 4; ++r) Cm[(lane >> 4) * 4 + r][lane & 15] = c[r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const int p2 = tile * kLidTile + lane;
      if (lane < kLidTile && p2 < ndocs) {
        const int d2 = perm ? perm[p2] : p2;
        double C[kLidLangs];
#pragma unroll
        for (int l = 0; l < kLidLangs; ++l) C[l] = (double)Cm[lane][l];
        lid_decide_v3(C, ex[lane], cn[lane], w_scale, bias, rec + (int64_t)d2 * width);
      }
    }
    __syncthreads();  // A / Cm / ex / cn are the next tile's
  }
}

// TB_C4_WPE: register budget of the C4 pass A wave kernel (0: none). 8 waves/SIMD = 64 VGPRs,
// one fewer than it takes unconstrained: 2.86 -> 2.42 ms/step (profiles/r8_c4w8/).
// 7 waves/SIMD (70 VGPRs, no spill): with the dictionary-script inputs the 8-wave build spills 9
// VGPRs, and that build rewrote a few documents wrongly on the GPU (test_badwords_device, C4 in
// front; the 6- and 7-wave builds and the host emulation of the same source are exact) -- unexplained,
// so the kernel stays spill-free
#ifndef TB_C4_WPE
#define TB_C4_WPE 7
#endif
#if TB_C4_WPE > 0
#define TB_C4_ATTR __attribute__((amdgpu_waves_per_eu(TB_C4_WPE, 8)))
#else
#define TB_C4_ATTR
#endif
__global__ __launch_bounds__(64) TB_C4_ATTR void k_c4_pass_a(
    const DevC4* __restrict__ c4, const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
    const int32_t* __restrict__ perm, int32_t ndocs, char* scratch, const int64_t* __restrict__ scratch_off,
    const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs, int64_t* rec, int64_t* src, uint32_t* flags,
    uint32_t lds_bytes, uint64_t* prof, const uint8_t* __restrict__ dead, const uint32_t* __restrict__ line_stats,
    uint32_t* c4_words, DictLines dict_lines) {
  const int doc = perm ? perm[blockIdx.x] : (int)blockIdx.x;
  if (doc >= ndocs || (dead && dead[doc])) return;  // skipped: record zeros, rewritten length 0
  DocCtx<WavePar> x = make_ctx(tabs, pw, pw_n, scratch, scratch_off, doc, (int)blockIdx.x, flags, lds_bytes, prof);
  lds_ascii_props(x);
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  c4_pass_a(x, *c4, b, n, rec + (int64_t)doc * 7, src + (int64_t)doc * 2,
            line_stats ? line_stats + line_stats_base(off[doc], doc) : nullptr, c4_words ? c4_words + doc : nullptr,
            dict_lines.at((uint32_t)doc));
  c4_src_absolute(x, src + (int64_t)doc * 2, scratch_off[blockIdx.x]);
}

__global__ __launch_bounds__(kBlockThreads) void k_c4_pass_a_blk(
    const DevC4* __restrict__ c4, const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
    const int32_t* __restrict__ perm, int32_t ndocs, char* scratch, const int64_t* __restrict__ scratch_off,
    const uint64_t* __restrict__ pw, uint32_t pw_n, DevTables tabs, int64_t* rec, int64_t* src, uint32_t* flags,
    uint32_t lds_bytes, uint64_t* prof, const uint8_t* __restrict__ dead, const uint32_t* __restrict__ line_stats,
    uint32_t* c4_words, DictLines dict_lines) {
  const int doc = perm[blockIdx.x];
  if (doc >= ndocs || (dead && dead[doc])) return;
  DocCtx<BlockPar<kBlockThreads>> x =
      make_ctx<BlockPar<kBlockThreads>>(tabs, pw, pw_n, scratch, scratch_off, doc, (int)blockIdx.x, flags, lds_bytes, prof);
  x.par.xs = g_block_xs;
  lds_ascii_props(x);
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  c4_pass_a(x, *c4, b, n, rec + (int64_t)doc * 7, src + (int64_t)doc * 2,
            line_stats ? line_stats + line_stats_base(off[doc], doc) : nullptr, c4_words ? c4_words + doc : nullptr,
            dict_lines.at((uint32_t)doc));
  c4_src_absolute(x, src + (int64_t)doc * 2, scratch_off[blockIdx.x]);
}

// C4 bad words (reference c4_filters.rs:431-441,463-551): does any list entry occur, case-folded,
// with \W (or text edge) on both sides (no boundary requirement for CJK lists)? One wave per
// document, four documents per workgroup; every code point position (UTF-8 lead byte) of a
// 64-byte chunk starts a walk of the hashed trie table (csrc/common/badwords.h) in parallel; the
// wave stops at the first chunk that contains a match. In the batch pipeline it reads the content
// version its step sees and skips the documents a pass before the step filtered
// (0 < dead <= dead_max); matched: -1 skipped / no list, 0 no match, 1 match.
constexpr int kBwWaves = 4;
// Work items: without a segment list, wave w takes document w and the start positions
// [0, seg_bytes) and writes its verdict; with one (seg_doc / seg_idx, launched afterwards on the
// same stream), wave w takes positions [seg_idx * seg_bytes, +seg_bytes) of document seg_doc[w] —
// the long documents' remaining segments, so no single wave walks a whole long document — skips
// documents already decided, and only ever writes a match.
__global__ __launch_bounds__(64 * kBwWaves) void k_badwords_match(
    const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off, int32_t nitems,
    const int32_t* __restrict__ root, const uint8_t* __restrict__ cjk, int32_t root0, int32_t cjk0,
    const uint8_t* __restrict__ dead, uint32_t dead_max, BwTable tab, DevTables tabs, BwFold fold,
    int8_t* __restrict__ matched, const int32_t* __restrict__ seg_doc, const int32_t* __restrict__ seg_idx,
    uint32_t seg_bytes) {
  __shared__ uint8_t asc[128];
  const UcdView ucd{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
  if (threadIdx.x < 128) asc[threadIdx.x] = bw_ascii_entry(ucd, fold, threadIdx.x);
  __syncthreads();
  const int item = (int)blockIdx.x * kBwWaves + (int)(threadIdx.x >> 6);
  if (item >= nitems) return;
  const int doc = seg_doc ? seg_doc[item] : item;
  const uint32_t lane = threadIdx.x & 63;
  const int32_t r0 = root ? root[doc] : root0;
  const uint32_t dd = dead ? dead[doc] : 0u;
  if (seg_doc) {
    if (matched[doc] != 0) return;  // decided (match, or skipped) by the first pass
  } else if (r0 < 0 || (dd != 0 && dd <= dead_max)) {
    if (lane == 0) matched[doc] = -1;
    return;
  }
  const uint8_t* b = bytes + off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
  const bool any_edge = (cjk ? cjk[doc] : (uint8_t)cjk0) != 0;
  const uint32_t p0 = seg_doc ? (uint32_t)seg_idx[item] * seg_bytes : 0u;
  const uint32_t p1 = p0 + seg_bytes < n ? p0 + seg_bytes : n;
  bool found = false;
  // 256 positions per iteration, 4 consecutive bytes per lane: the left-boundary test of a
  // position reads the previous byte from the lane's own bytes or its neighbour; only positions
  // that start a word walk the trie (the walk itself may run past the segment end)
  for (uint32_t base = p0; base < p1 && !found; base += 256) {
    const uint32_t s0 = base + 4 * lane;
    uint8_t c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = s0 + k < p1 ? b[s0 + k] : (uint8_t)0;
    const uint8_t before = s0 > 0 && s0 < p1 ? b[s0 - 1] : (uint8_t)' ';
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t s = s0 + k;
      if (s >= p1 || !utf8_is_lead(c[k])) continue;
      const uint8_t pb = k ? c[k - 1] : before;
      bool left = any_edge || s == 0 || (pb < 0x80 ? (asc[pb] & 0x80u) == 0 : bw_left_ok(b, n, s, ucd, asc));
      if (left && bw_walk_from(b, n, s, r0, any_edge, tab, ucd, fold, asc)) { found = true; break; }
    }
    found = __ballot(found) != 0;
  }
  if (lane == 0 && (found || !seg_doc)) matched[doc] = found ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_c4_pass_b(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
                                                   int32_t ndocs, const char* __restrict__ scratch,
                                                   const int64_t* __restrict__ scratch_off,
                                                   const int64_t* __restrict__ src, const int64_t* __restrict__ new_off,
                                                   uint8_t* __restrict__ out) {
  const int doc = blockIdx.x;
  if (doc >= ndocs) return;
  const int64_t len = new_off[doc + 1] - new_off[doc];
  const int64_t s = src[2 * doc];
  (void)scratch_off;  // src holds absolute arena offsets (c4_src_absolute)
  const uint8_t* from = s < 0 ? bytes + off[doc] : (const uint8_t*)scratch + s;
  uint8_t* to = out + new_off[doc];
  for (int64_t i = threadIdx.x; i < len; i += blockDim.x) to[i] = from[i];
}


// Step gate (csrc/common/gate.h): one thread per document. A live document that a step of the
// just-finished pass filters (or that a kernel flagged for the CPU path) gets `code`: later
// passes skip it. Codes are written once, so dead[doc] = the first pass the document skipped.
__global__ __launch_bounds__(256) void k_gate(const DevGate* __restrict__ gate, GateRecs recs, int32_t ndocs,
                                              const uint32_t* __restrict__ flags, uint8_t* dead, uint8_t code) {
  const int doc = blockIdx.x * blockDim.x + threadIdx.x;
  if (doc >= ndocs || dead[doc]) return;
  bool fail = flags[doc] != 0;
  const int ns = gate->n_steps;
  for (int s = 0; s < ns && !fail; ++s) {
    const DevGateStep& g = gate->steps[s];
    if (g.kind == GK_NONE) continue;
    const int64_t* r = recs.p[g.slot] + (int64_t)g.prefix * ndocs + (int64_t)doc * g.width;
    fail = gate_fails(g, r);
  }
  if (fail) dead[doc] = code;
}

// K16 resolve (csrc/common/gate.h resolve_doc): one thread per document. Writes the first failing
// step, the status, and the compaction inputs of the outputs: per document 4 int64 lanes
// {kept bytes, excluded bytes, kept count, excluded count} of its final content version, which four
// strided scans turn into output positions and byte offsets for k_compact.
struct VersionTab {
  const uint8_t* b[kMaxVersions];
  const int64_t* off[kMaxVersions];
};

__global__ __launch_bounds__(256) void k_resolve(const DevResolve* __restrict__ rp, GateRecs recs, int32_t ndocs,
                                                 const uint32_t* __restrict__ flags, VersionTab vt,
                                                 int32_t* __restrict__ fail, uint8_t* __restrict__ status,
                                                 uint8_t* __restrict__ fver, int64_t* __restrict__ lanes) {
  const int doc = blockIdx.x * blockDim.x + threadIdx.x;
  if (doc >= ndocs) return;
  int32_t f, v;
  uint8_t st;
  resolve_doc(*rp, recs.p, ndocs, doc, flags[doc], f, st, v);
  fail[doc] = f;
  status[doc] = st;
  fver[doc] = (uint8_t)v;
  const int64_t len = vt.off[v][doc + 1] - vt.off[v][doc];
  int64_t* l = lanes + 4 * (int64_t)doc;
  l[0] = st == kResolveKept ? len : 0;
  l[1] = st == kResolveFiltered ? len : 0;
  l[2] = st == kResolveKept ? 1 : 0;
  l[3] = st == kResolveFiltered ? 1 : 0;
}

// K16 compaction: one 256-thread workgroup per document copies its final content into the output
// buffer — kept documents first, then excluded ones, each group in document order (the order the
// host path produces) — and writes its output row and start offset. sc = the four inclusive scans
// [kept bytes | excluded bytes | kept count | excluded count], n entries each. The copy works in
// destination-aligned dwords: each thread loads the two source dwords that cover its destination
// dword and funnel-shifts them together (v_alignbyte), so interior bytes move 4 at a time whatever
// the relative alignment; only the partial first and last destination dwords go byte by byte.
// Source reads may run up to 3 bytes past a document (the batch and version buffers are padded).
constexpr int kCompactThreads = 256;  // LANES threads per document: 64 (four per workgroup) or 256

template <int kCompactLanes>
__global__ __launch_bounds__(kCompactThreads) void k_compact(const uint8_t* __restrict__ status,
                                                             const uint8_t* __restrict__ fver, VersionTab vt,
                                                             int32_t ndocs, const int64_t* __restrict__ sc,
                                                             uint8_t* __restrict__ out, int64_t cap,
                                                             int64_t* __restrict__ out_off, int32_t* __restrict__ rows,
                                                             int32_t* __restrict__ err) {
  const int doc = (int)blockIdx.x * (kCompactThreads / kCompactLanes) + (int)(threadIdx.x / kCompactLanes);
  const int t = (int)(threadIdx.x % kCompactLanes);
  if (doc >= ndocs) return;
  const int64_t n = ndocs;
  const int64_t nk = sc[3 * n - 1], nx = sc[4 * n - 1], kb = sc[n - 1], xb = sc[2 * n - 1];
  if (doc == 0 && t == 0) out_off[nk + nx] = kb + xb;
  const uint8_t st = status[doc];
  if (st != kResolveKept && st != kResolveFiltered) return;
  const int v = fver[doc];
  const int64_t s0 = vt.off[v][doc], len = vt.off[v][doc + 1] - s0;
  int64_t pos, boff;
  if (st == kResolveKept) {
    pos = sc[2 * n + doc] - 1;
    boff = sc[doc] - len;
  } else {
    pos = nk + sc[3 * n + doc] - 1;
    boff = kb + sc[n + doc] - len;
  }
  if (boff < 0 || len < 0 || boff + len > cap) {  // never with the C4 growth bound; checked anyway
    if (t == 0) *err = 1;
    return;
  }
  if (t == 0) {
    out_off[pos] = boff;
    rows[pos] = doc;
  }
  if (len == 0) return;
  const uint8_t* src = vt.b[v] + s0;
  uint8_t* dst = out + boff;
  // destination dwords fully inside [boff, boff + len): [a0, a1) in dword units of `out`
  const int64_t a0 = (boff + 3) >> 2, a1 = (boff + len) >> 2;
  if (a1 <= a0) {  // short: no whole destination dword
    for (int64_t i = t; i < len; i += kCompactLanes) dst[i] = src[i];
    return;
  }
  const int64_t head = a0 * 4 - boff, tail = boff + len - a1 * 4;  // bytes before / after
  if (t < head) dst[t] = src[t];
  if (t < tail) dst[len - tail + t] = src[len - tail + t];
  // destination dword w (absolute) takes source bytes from sp = src + (4w - boff)
  const uintptr_t sbase = (uintptr_t)src + (uintptr_t)head;  // source of the first whole dword
  const uint32_t sh = (uint32_t)(sbase & 3u);
  const uint32_t* s32 = (const uint32_t*)(sbase - sh);
  uint32_t* d32 = (uint32_t*)out + a0;
  const int64_t nw = a1 - a0;
  for (int64_t k = t; k < nw; k += kCompactLanes) {
    const uint32_t lo = s32[k];
    const uint32_t hi = sh ? s32[k + 1] : 0u;
    // little endian: bytes sh.. of lo, then the low bytes of hi
    d32[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  }
}

__global__ void k_pow_table(uint64_t* pw, uint32_t n) {
  // pw[i] = B^i and pw[n + 1 + i] = B^-i, computed independently per element (exact modular
  // arithmetic); the buffer holds 2n + 2 entries
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) {
    pw[i] = hpow(kHashBase, i);
    pw[n + 1 + i] = hpow(kHashBaseInv, i);
  }
}

// the code points and UAX#29 word-break marks of very long documents, spread over
// many workgroups before their stage workgroups run (StageOut::pre). Launch grids are
// (tile or chunk, document): k_pre_count counts the lead bytes of every 16 KB tile, k_pre_decode
// writes each tile's code points at the offset its earlier tiles give (the non-packed Cps layout
// decode() produces for documents of 64 KiB and more), k_pre_wb evaluates word_mark() for 64 code
// points per wave (the rules look across tile borders freely: the whole property array exists).
constexpr uint32_t kPreTile = 16384;
constexpr uint32_t kPreThreads = 256;  // 64 bytes per thread

__global__ __launch_bounds__(kPreThreads) void k_pre_count(const uint8_t* __restrict__ bytes,
                                                           const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ perm,
                                                           const uint8_t* __restrict__ dead,
                                                           const PreDoc* __restrict__ pre, uint32_t tiles_max,
                                                           int64_t* __restrict__ cnt) {
  __shared__ uint32_t red[kPreThreads / 64];
  const uint32_t j = blockIdx.x, s = blockIdx.y;
  const int doc = perm[s];
  const uint32_t n = pre[s].n;
  const uint32_t b0 = j * kPreTile;
  if (b0 >= n || (dead && dead[doc]) || off[doc + 1] - off[doc] != (int64_t)n) return;
  const uint8_t* b = bytes + off[doc];
  const uint32_t e = b0 + kPreTile < n ? b0 + kPreTile : n;
  // code points (low half) and runs of '\n' (high half)
  uint32_t c = 0;
  for (uint32_t i = b0 + threadIdx.x; i < e; i += kPreThreads) {
    const uint8_t v = b[i];
    c += utf8_is_lead(v) ? 1u : 0u;
    if (v == '\n' && (i == 0 || b[i - 1] != '\n')) c += 1u << 16;
  }
  for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kPreThreads / 64; ++w) t += red[w];
    cnt[(size_t)s * tiles_max + j] = t;  // both halves < 2^16: a tile is 16 KB
  }
}

__global__ __launch_bounds__(kPreThreads) void k_pre_decode(const uint8_t* __restrict__ bytes,
                                                            const int64_t* __restrict__ off,
                                                            const int32_t* __restrict__ perm,
                                                            const uint8_t* __restrict__ dead, PreDoc* pre,
                                                            uint32_t tiles_max, const int64_t* __restrict__ cnt,
                                                            DevTables tabs) {
  __shared__ uint32_t xs[kPreThreads + 1];
  __shared__ uint32_t ys[kPreThreads + 1];
  const uint32_t j = blockIdx.x, s = blockIdx.y;
  const int doc = perm[s];
  const PreDoc d = pre[s];
  const uint32_t n = d.n;
  const uint32_t b0 = j * kPreTile;
  if (b0 >= n || (dead && dead[doc]) || off[doc + 1] - off[doc] != (int64_t)n) return;
  const uint8_t* b = bytes + off[doc];
  const UcdView ucd{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
  // this thread's 64 bytes, loaded at once (16 independent loads): lead count, then the
  // block's exclusive scan of the counts
  const uint32_t t0 = b0 + 64 * threadIdx.x;
  const uint32_t t1 = t0 + 64 < n ? t0 + 64 : n;
  uint32_t v[16];
#pragma unroll
  for (uint32_t q = 0; q < 16; ++q) {
    uint32_t w = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t i = t0 + 4 * q + k;
      w |= (i < t1 ? (uint32_t)b[i] : 0u) << (8 * k);
    }
    v[q] = w;
  }
  auto byte_of = [&](uint32_t i) -> uint32_t { return (v[(i - t0) >> 2] >> (8 * ((i - t0) & 3))) & 0xFFu; };
  uint32_t prev = (t0 > 0 && t0 < n) ? (uint32_t)b[t0 - 1] : 0u;
  uint32_t c = 0, pv = prev;
  for (uint32_t i = t0; i < t1; ++i) {
    const uint32_t c0 = byte_of(i);
    c += utf8_is_lead((uint8_t)c0) ? 1u : 0u;
    if (c0 == '\n' && (i == 0 || pv != '\n')) c += 1u << 16;
    pv = c0;
  }
  xs[threadIdx.x] = c;  // code points | runs << 16 (< 2^16 each: 64 bytes)
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t bc = 0, br = 0;
    for (uint32_t q = 0; q < j; ++q) {
      const uint32_t t = (uint32_t)cnt[(size_t)s * tiles_max + q];
      bc += t & 0xFFFFu;
      br += t >> 16;
    }
    for (uint32_t q = 0; q < kPreThreads; ++q) {
      const uint32_t t = xs[q];
      xs[q] = bc;
      ys[q] = br;
      bc += t & 0xFFFFu;
      br += t >> 16;
    }
    xs[kPreThreads] = bc;  // code points and runs before the next tile
    ys[kPreThreads] = br;
  }
  __syncthreads();
  uint32_t k = xs[threadIdx.x], kr = ys[threadIdx.x];
  bool dict = false;
  uint32_t fs = 0xFFFFFFFFu, le = 0;  // first / one past the last non-whitespace code point
  pv = prev;
  for (uint32_t i = t0; i < t1; ++i) {
    const uint32_t c0 = byte_of(i);
    const uint32_t last = pv;
    pv = c0;
    if (!utf8_is_lead((uint8_t)c0)) continue;
    if (c0 == '\n' && (i == 0 || last != '\n')) {  // a run of '\n' starts at code point k
      uint32_t q = i + 1;
      while (q < n && b[q] == '\n') ++q;
      d.nl_pos[kr] = k;
      d.nl_len[kr] = q - i;
      ++kr;
    }
    int len;
    const uint32_t p = ucd.props(c0 < 0x80 ? c0 : utf8_decode(b, i, n, &len));
    d.off[k] = i;
    d.prop[k] = compact_prop(p);
    dict |= (p & P_DICT) != 0;
    if (!is_ws(compact_prop(p))) {
      fs = k < fs ? k : fs;
      le = k + 1;
    }
    ++k;
  }
  if (dict) atomicOr(&pre[s].dict, 1u);
  if (le) {
    atomicMin(&pre[s].tcs, fs);
    atomicMax(&pre[s].tce, le);
  }
  if (threadIdx.x == 0 && b0 + kPreTile >= n) {  // the last tile closes the arrays
    const uint32_t C = xs[kPreThreads];
    d.off[C] = n;
    d.prop[C] = 0;
    pre[s].C = C;
    pre[s].NL = ys[kPreThreads];
  }
}

__global__ __launch_bounds__(64) void k_pre_wb(const int32_t* __restrict__ perm, const uint8_t* __restrict__ dead,
                                               PreDoc* pre) {
  const uint32_t j = blockIdx.x, s = blockIdx.y;
  const PreDoc d = pre[s];
  const uint32_t C = d.C;
  if (64 * j > C || (dead && dead[perm[s]])) return;
  if (j == 0 && threadIdx.x == 0) {  // the runs of '\n' inside [tcs, tce) (gopher_rep_record)
    auto lower = [&](uint32_t v) {
      uint32_t lo = 0, hi = d.NL;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (d.nl_pos[mid] < v) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    pre[s].nl_a = lower(d.tcs);
    pre[s].nl_e = lower(d.tce);
  }
  const uint32_t i = 64 * j + threadIdx.x;
  const bool m = i <= C && word_mark(PropArr{nullptr, d.prop}, C, i);
  const uint64_t bits = __ballot(m);
  if (threadIdx.x < 2) d.wbm[2 * j + threadIdx.x] = threadIdx.x ? (uint32_t)(bits >> 32) : (uint32_t)bits;
}

// The pre-pass words (words() over the precomputed code points and marks), as a segmented scan
// spread over waves: MODE 0 writes every 64-code-point chunk's scan aggregate, k_pre_words_scan
// turns them into per-chunk carry-ins (one wave per document), MODE 1 counts the chunk's words,
// k_pre_words_scan (counts) gives each chunk its first word index, MODE 2 writes the words.
__device__ __forceinline__ WSeg pre_wseg_in(const PreDoc& d, uint32_t j) {
  const uint32_t p = d.prop[j];
  const bool ws = is_ws(p);
  const uint32_t bit = (d.wbm[j >> 5] >> (j & 31)) & 1u;
  return WSeg{bit | ((!(p & P_PUNCT) && !ws) ? 2u : 0u) | ((p & P_ALPHA) ? 4u : 0u), ws ? 0xFFFFFFFFu : j,
              ws ? 0u : j + 1};
}

template <int MODE>
__global__ __launch_bounds__(64) void k_pre_words(const int32_t* __restrict__ perm, const uint8_t* __restrict__ dead,
                                                  const PreDoc* __restrict__ pre) {
  const uint32_t c = blockIdx.x, s = blockIdx.y;
  const PreDoc d = pre[s];
  const uint32_t C = d.C;
  const uint32_t nch = (C + 63) / 64;
  if (c >= nch || (dead && dead[perm[s]])) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t j = 64 * c + lane;
  const WSeg id{0u, 0xFFFFFFFFu, 0u};
  const WSeg x = j < C ? pre_wseg_in(d, j) : id;
  const WSeg loc = pardetail::wave_incl_scan(x, lane, [](const WSeg& a, const WSeg& b) { return wseg_op(a, b); });
  if (MODE == 0) {
    if (lane == 63) {
      d.wtmp[3 * c] = loc.bits;
      d.wtmp[3 * c + 1] = loc.first;
      d.wtmp[3 * c + 2] = loc.last;
    }
    return;
  }
  const uint32_t* cin = d.wtmp + 3 * (size_t)nch;
  const WSeg carry{cin[3 * c], cin[3 * c + 1], cin[3 * c + 2]};
  const WSeg in = wseg_op(carry, loc);
  const bool sel = j < C && ((d.wbm[(j + 1) >> 5] >> ((j + 1) & 31)) & 1u) && (in.bits & 2u);
  const uint64_t m = __ballot(sel);
  uint32_t* wcnt = d.wtmp + 6 * (size_t)nch;
  if (MODE == 1) {
    if (lane == 0) wcnt[c] = (uint32_t)__popcll(m);
    return;
  }
  if (sel) {
    const uint32_t* wbase = wcnt + nch;
    const uint32_t k = wbase[c] + (uint32_t)__popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
    d.wcs[k] = in.first;
    d.wce[k] = in.last;
    d.wbs[k] = d.off[in.first];
    d.wbe[k] = d.off[in.last];
    d.wal[k] = (in.bits & 4u) ? 1 : 0;
  }
}

// One wave per document: MODE 0 scans the chunk aggregates into carry-ins (exclusive), MODE 1 the
// word counts into first word indices (and W).
template <int MODE>
__global__ __launch_bounds__(64) void k_pre_words_scan(const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ dead, PreDoc* pre) {
  const uint32_t s = blockIdx.x;
  const PreDoc d = pre[s];
  if (dead && dead[perm[s]]) return;
  const uint32_t nch = (d.C + 63) / 64;
  const uint32_t lane = threadIdx.x;
  if (MODE == 0) {
    const WSeg id{0u, 0xFFFFFFFFu, 0u};
    auto op = [](const WSeg& a, const WSeg& b) { return wseg_op(a, b); };
    WSeg carry = id;
    uint32_t* cin = d.wtmp + 3 * (size_t)nch;
    for (uint32_t b0 = 0; b0 < nch; b0 += 64) {
      const uint32_t q = b0 + lane;
      const WSeg v = q < nch ? WSeg{d.wtmp[3 * q], d.wtmp[3 * q + 1], d.wtmp[3 * q + 2]} : id;
      const WSeg incl = pardetail::wave_incl_scan(v, lane, op);
      WSeg excl = pardetail::shfl_up_t(incl, 1);
      if (lane == 0) excl = id;
      const WSeg e = op(carry, excl);
      if (q < nch) {
        cin[3 * q] = e.bits;
        cin[3 * q + 1] = e.first;
        cin[3 * q + 2] = e.last;
      }
      carry = op(carry, pardetail::bcast63(incl));
    }
  } else {
    uint32_t* wcnt = d.wtmp + 6 * (size_t)nch;
    uint32_t* wbase = wcnt + nch;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nch; b0 += 64) {
      const uint32_t q = b0 + lane;
      const uint32_t v = q < nch ? wcnt[q] : 0u;
      const uint32_t incl = pardetail::wave_incl_scan(v, lane, [](uint32_t a, uint32_t b) { return a + b; });
      if (q < nch) wbase[q] = carry + incl - v;
      carry += pardetail::bcast63(incl);
    }
    if (lane == 0) pre[s].W = carry;
  }
}

// SURVEY 5.7, GopherRepetition's word arrays of the pre-pass documents over many workgroups
// (gopher_rep_record computes the same in the document's own workgroup for the others): per
// chunk of 2048 words (256 threads, 8 consecutive words each)
//   MODE 0  zero the canonicalisation table (1.5 W + 2 slots of 64 bits)
//   MODE 1  word hash (the polynomial hash of its bytes = span_hash8), insert into the table
//           (fingerprint | smallest index + 1, CAS + atomic min: canonicalize()'s 64-bit path),
//           chunk sum of the word lengths
//   MODE 2  canonical id (verified byte-equal; a collision flags the document for the CPU path),
//           WL / PB from the chunk's length base, chunk sum of wh[k] B^-WL[k+1]
//   MODE 3  K from the chunk's base of those terms
// with k_pre_wsum (one wave per document) turning chunk sums into bases between the passes.
constexpr uint32_t kPreWChunk = 2048;
constexpr uint32_t kPreWThreads = 256;
constexpr uint32_t kPreWPer = kPreWChunk / kPreWThreads;
constexpr uint32_t kPreWTabChunk = 3072;  // table slots zeroed per workgroup (1.5 x a chunk)

__device__ __forceinline__ uint64_t pow_at(const uint64_t* pw, uint32_t pw_n, uint32_t k) {
  return k <= pw_n ? pw[k] : hpow(kHashBase, k);
}
__device__ __forceinline__ uint64_t ipow_at(const uint64_t* pw, uint32_t pw_n, uint32_t k) {
  return k <= pw_n ? pw[pw_n + 1 + k] : hpow(kHashBaseInv, k);
}

// exclusive block scan (kPreWThreads threads) of one value per thread; *tot = the block total
template <class T>
__device__ __forceinline__ T pre_block_scan(T v, T* sh, T* tot) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T incl = pardetail::wave_incl_scan(v, lane, [](T a, T b) { return a + b; });
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  T base = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < kPreWThreads / 64; ++q) {
    if (q < w) base += sh[q];
    all += sh[q];
  }
  __syncthreads();
  *tot = all;
  return base + incl - v;
}

template <int MODE>
__global__ __launch_bounds__(kPreWThreads) void k_pre_wcanon(const uint8_t* __restrict__ bytes,
                                                             const int64_t* __restrict__ off,
                                                             const int32_t* __restrict__ perm,
                                                             const uint8_t* __restrict__ dead,
                                                             const PreDoc* __restrict__ pre,
                                                             const uint64_t* __restrict__ pw, uint32_t pw_n,
                                                             uint32_t* flags) {
  __shared__ uint64_t sh[kPreWThreads / 64];
  const uint32_t c = blockIdx.x, s = blockIdx.y;
  const int doc = perm[s];
  if (dead && dead[doc]) return;
  const PreDoc d = pre[s];
  const uint32_t W = d.W;
  const uint32_t nch = (W + kPreWChunk - 1) / kPreWChunk;
  const uint32_t capn = W + (W >> 1) + 2;
  if (MODE == 0) {
    const uint32_t a = c * kPreWTabChunk;
    for (uint32_t i = a + threadIdx.x; i < capn && i < a + kPreWTabChunk; i += kPreWThreads) d.wtab[i] = 0;
    return;
  }
  if (c >= (nch ? nch : 1u)) return;  // (W == 0: chunk 0 writes the closing entries)
  const uint8_t* b = bytes + off[doc];
  const uint32_t t0 = c * kPreWChunk + threadIdx.x * kPreWPer;
  uint32_t len[kPreWPer];
  uint32_t lsum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPreWPer; ++j) {
    const uint32_t k = t0 + j;
    len[j] = k < W ? d.wbe[k] - d.wbs[k] : 0u;
    lsum += len[j];
  }
  if (MODE == 1) {
#pragma unroll
    for (uint32_t j = 0; j < kPreWPer; ++j) {
      const uint32_t k = t0 + j;
      if (k >= W) break;
      const uint32_t bs = d.wbs[k], be = d.wbe[k];
      uint64_t h = 0;
      for (uint32_t q = bs; q < be; ++q) h = hash_push(h, b[q]);
      d.wh[k] = h;
      const uint64_t key = dev_key(h, be - bs);
      const uint64_t fp = (key >> 32) | 1ull;
      const uint64_t mine = (fp << 32) | (uint64_t)(k + 1);
      uint32_t slot = (uint32_t)(((key & 0xFFFFFFFFull) * capn) >> 32);
      while (true) {
        unsigned long long cur = d.wtab[slot];
        if (cur == 0) {
          cur = atomicCAS((unsigned long long*)&d.wtab[slot], 0ull, (unsigned long long)mine);
          if (cur == 0) break;
        }
        if ((cur >> 32) == fp) {
          if ((cur & 0xFFFFFFFFull) > (uint64_t)k + 1u) atomicMin((unsigned long long*)&d.wtab[slot], mine);
          break;
        }
        if (++slot == capn) slot = 0;
      }
      d.wslot[k] = slot;
    }
    uint64_t tot;
    (void)pre_block_scan<uint64_t>(lsum, sh, &tot);
    if (threadIdx.x == 0) d.wcsum[c] = tot;
    return;
  }
  // MODE 2 / 3: this thread's first word's WL from the chunk base + the block scan
  uint64_t tot;
  const uint64_t lbase = (nch ? d.wcsum[nch + c] : 0ull) + pre_block_scan<uint64_t>(lsum, sh, &tot);
  if (MODE == 2) {
    uint32_t wl = (uint32_t)lbase;
    uint64_t tsum = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t j = 0; j < kPreWPer; ++j) {
      const uint32_t k = t0 + j;
      if (k >= W) break;
      d.wl[k] = wl;
      d.wpb[k] = pow_at(pw, pw_n, wl);
      uint32_t cc = (uint32_t)(d.wtab[d.wslot[k]] & 0xFFFFFFFFull) - 1u;
      if (cc != k && !bytes_eq<WavePar>(b, d.wbs[k], d.wbe[k], d.wbs[cc], d.wbe[cc])) {
        bad = true;
        cc = k;
      }
      d.wid[k] = cc;
      wl += len[j];
      tsum += d.wh[k] * ipow_at(pw, pw_n, wl);
    }
    if (bad) atomicOr(&flags[doc], DOC_NEEDS_CPU);
    uint64_t ttot;
    (void)pre_block_scan<uint64_t>(tsum, sh, &ttot);
    if (threadIdx.x == 0) {
      if (nch) d.wcsum[2 * nch + c] = ttot;
      if (c + 1 >= nch) {  // the closing entries
        const uint32_t total = (uint32_t)((nch ? d.wcsum[nch + c] : 0ull) + tot);
        d.wl[W] = total;
        d.wpb[W] = pow_at(pw, pw_n, total);
      }
    }
    return;
  }
  // MODE 3
  uint32_t wl = (uint32_t)lbase;
  uint64_t t[kPreWPer];
  uint64_t tsum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPreWPer; ++j) {
    const uint32_t k = t0 + j;
    wl += len[j];
    t[j] = k < W ? d.wh[k] * ipow_at(pw, pw_n, wl) : 0ull;
    tsum += t[j];
  }
  uint64_t ttot;
  uint64_t kb = (nch ? d.wcsum[3 * nch + c] : 0ull) + pre_block_scan<uint64_t>(tsum, sh, &ttot);
#pragma unroll
  for (uint32_t j = 0; j < kPreWPer; ++j) {
    const uint32_t k = t0 + j;
    if (k >= W) break;
    d.wk[k] = kb;
    kb += t[j];
  }
  if (threadIdx.x == 0 && c + 1 >= nch) d.wk[W] = (nch ? d.wcsum[3 * nch + c] : 0ull) + ttot;
}

// One wave per document: exclusive scans of the chunk sums (MODE 0: lengths [0, nch) -> [nch, 2 nch);
// MODE 1: K terms [2 nch, 3 nch) -> [3 nch, 4 nch)); MODE 1 also marks the arrays ready.
template <int MODE>
__global__ __launch_bounds__(64) void k_pre_wsum(const int32_t* __restrict__ perm, const uint8_t* __restrict__ dead,
                                                 PreDoc* pre) {
  const uint32_t s = blockIdx.x;
  if (dead && dead[perm[s]]) return;
  const PreDoc d = pre[s];
  const uint32_t nch = (d.W + kPreWChunk - 1) / kPreWChunk;
  const uint32_t lane = threadIdx.x;
  const uint64_t* in = d.wcsum + (MODE ? 2 * nch : 0);
  uint64_t* out = d.wcsum + (MODE ? 3 * nch : nch);
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < nch; b0 += 64) {
    const uint32_t q = b0 + lane;
    const uint64_t v = q < nch ? in[q] : 0ull;
    const uint64_t incl = pardetail::wave_incl_scan(v, lane, [](uint64_t a, uint64_t b) { return a + b; });
    if (q < nch) out[q] = carry + incl - v;
    carry += pardetail::bcast63(incl);
  }
  if (MODE == 1 && lane == 0) pre[s].wready = 1;
}

}  // namespace

// CUs of the current device (queried once; thread-safe static initialisation)
static int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

extern "C" {

int tb_scan_strided_i64(hipStream_t stream, const int64_t* src, int64_t stride, int64_t n, int64_t* out);  // runtime.hip

int tb_stage_analyze(hipStream_t stream, const void* plan, const void* stage, const uint8_t* bytes,
                     const int64_t* off, const int32_t* perm, int32_t ndocs, char* scratch,
                     const int64_t* scratch_off, const uint64_t* pw, uint32_t pw_n, const uint16_t* s1,
                     const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec, uint32_t* flags,
                     uint32_t lds_bytes, uint64_t* prof, int32_t waves, int32_t nblocks, const uint8_t* dead,
                     uint32_t* line_stats, void* gr_export, const int64_t* dict_moff, const uint32_t* dict_bits,
                     const uint32_t* dict_words) {
  if (ndocs <= 0) return 0;
  if (nblocks <= 0) nblocks = ndocs;  // grid: docs perm[0 .. nblocks)
  if (lds_bytes > kMaxLdsPerDoc) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  if (waves != TB_STAGE_WPE) return (int)hipErrorInvalidValue;  // the one build (see TB_STAGE_KERNEL)
  auto kern = k_stage_analyze_wave;
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  hipLaunchKernelGGL(kern, dim3(nblocks), dim3(64), lds_bytes, stream, (const DevPlan*)plan,
                     (const DevStage*)stage, bytes, off, perm, ndocs, scratch, scratch_off, pw, pw_n, t, rec, flags,
                     lds_bytes, prof, dead, line_stats, (GrExport*)gr_export, DictIn{dict_moff, dict_bits, dict_words});
  return (int)hipGetLastError();
}

// Wave documents in split mode (tb_stage_analyze with gr_export): n_docs export slots, n_tasks =
// the GopherRepetition step's duplicated + top n-gram orders. Launch positions (the host puts the
// longer documents first): [0, n_big) one wave per (document, order) (k_gr_split_wave), the rest
// with block != 0 one workgroup per document (k_gr_ngrams<256>); block == 0: k_gr_split_wave for
// all. Measured (profiles/r7_ngram): workgroups of the 512-word class lost to the per-order waves
// for documents over 1.2 KB (LDS-limited occupancy), all-waves lost to this split.
int tb_gr_split_wave(hipStream_t stream, const void* stage, int32_t gr_step, const int32_t* perm, int32_t n_docs,
                     int32_t n_tasks, int32_t ndocs, const void* gr_export, const uint64_t* pw, uint32_t pw_n,
                     const uint16_t* s1, const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec,
                     uint32_t* flags, uint32_t lds_bytes, int32_t block, uint64_t* prof, int32_t n_big) {
  if (n_docs <= 0 || n_tasks <= 0) return 0;
  if (!perm || !gr_export || gr_step < 0 || gr_step >= kMaxStageSteps || n_tasks > 2 * kMaxNgramEntries ||
      lds_bytes > kMaxLdsPerDoc || n_big < 0 || n_big > n_docs)
    return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  const GrExport* ex = (const GrExport*)gr_export;
  const int32_t n_wave = block ? n_big : n_docs;
  if (n_wave > 0) {
    if (lds_bytes > 65536)
      (void)hipFuncSetAttribute((const void*)k_gr_split_wave, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_bytes);
    hipLaunchKernelGGL(k_gr_split_wave, dim3((uint32_t)n_wave * (uint32_t)n_tasks), dim3(64), lds_bytes, stream,
                       (const DevStage*)stage, gr_step, perm, n_tasks, ndocs, ex, pw, pw_n, t, rec, flags, lds_bytes);
  }
  if (block && n_docs > n_big) {
    // (the export buffer carries NgRest + n_docs positions after the descriptors, zeroed)
    NgRest* rest = ng_rest(ex, n_docs);
    if (prof)
      hipLaunchKernelGGL((k_gr_ngrams<256, true>), dim3((uint32_t)(n_docs - n_big)), dim3(64 * kNgWaves), 0, stream,
                         (const DevStage*)stage, gr_step, perm, ndocs, ex, n_big, rest, rec, prof);
    else
      hipLaunchKernelGGL((k_gr_ngrams<256, false>), dim3((uint32_t)(n_docs - n_big)), dim3(64 * kNgWaves), 0,
                         stream, (const DevStage*)stage, gr_step, perm, ndocs, ex, n_big, rest, rec, nullptr);
    hipLaunchKernelGGL(k_gr_ngrams_rest, dim3(512), dim3(64), 0, stream, (const DevStage*)stage, gr_step, perm,
                       ndocs, ex, rest, pw, pw_n, t, rec, flags);
  }
  return (int)hipGetLastError();
}

// Long-document variants: `perm` must point at the long prefix of the length-sorted
// permutation, `nblocks` documents, one workgroup each.
int tb_stage_analyze_blk(hipStream_t stream, const void* plan, const void* stage, const uint8_t* bytes,
                         const int64_t* off, const int32_t* perm, int32_t nblocks, int32_t ndocs, char* scratch,
                         const int64_t* scratch_off, const uint64_t* pw, uint32_t pw_n, const uint16_t* s1,
                         const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec, uint32_t* flags,
                         uint32_t lds_bytes, uint64_t* prof, const uint8_t* dead, void* gr_export, int32_t n_split,
                         uint32_t split_bytes, int32_t threads, uint32_t* line_stats, const void* pre,
                         int32_t n_pre, const int64_t* dict_moff, const uint32_t* dict_bits, const uint32_t* dict_words) {
  if (nblocks <= 0) return 0;
  if (!perm || lds_bytes > kMaxLdsPerBlk || n_split < 0 || n_split > nblocks) return (int)hipErrorInvalidValue;
  if (threads != kBlockThreads) return (int)hipErrorInvalidValue;
  if (pre && (threads != kBlockThreads || n_pre != nblocks)) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  auto kern = pre ? k_stage_analyze_blk_pre : k_stage_analyze_blk;
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  hipLaunchKernelGGL(kern, dim3(nblocks), dim3(threads), lds_bytes, stream,
                     (const DevPlan*)plan, (const DevStage*)stage, bytes, off, perm, ndocs, scratch, scratch_off, pw,
                     pw_n, t, rec, flags, lds_bytes, prof, dead, (GrExport*)gr_export, n_split,
                     split_bytes, line_stats, (const PreDoc*)pre, n_pre, DictIn{dict_moff, dict_bits, dict_words});
  return (int)hipGetLastError();
}

// gr_export: n_split descriptors written by tb_stage_analyze_blk (zeroed by the caller first);
// gr_step: index of the GopherRepetition step in the stage, n_tasks its duplicated + top n-gram
// orders.
int tb_gr_dup_split(hipStream_t stream, const void* stage, int32_t gr_step, const int32_t* perm, int32_t n_split,
                    int32_t n_tasks, int32_t ndocs, const void* gr_export, const uint64_t* pw, uint32_t pw_n,
                    const uint16_t* s1, const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec,
                    uint32_t* flags, uint32_t lds_bytes, uint32_t* cursor) {
  if (n_split <= 0 || n_tasks <= 0) return 0;
  if (!perm || !gr_export || gr_step < 0 || gr_step >= kMaxStageSteps || n_tasks > 2 * kMaxNgramEntries + 2 ||
      lds_bytes > kMaxLdsPerBlk)
    return (int)hipErrorInvalidValue;
  if (!cursor) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)k_gr_dup_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  // the persistent grid: resident workgroups per CU (registers, LDS) x CUs, at most one per task
  const int cus = device_cus();
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_gr_dup_split, kBlockThreads, lds_bytes) !=
          hipSuccess || per_cu <= 0)
    per_cu = 1;
  const int64_t total = (int64_t)n_split * n_tasks;
  // persistent: one resident wave of workgroups pulls tasks from the cursor (one workgroup per
  // task, ordered by the hardware dispatcher instead, measured slower: profiles/r8_c5/)
  const int grid = (int)std::min<int64_t>(total, (int64_t)cus * per_cu);
  (void)hipMemsetAsync(cursor, 0, sizeof(uint32_t), stream);
  hipLaunchKernelGGL(k_gr_dup_split, dim3((uint32_t)grid), dim3(kBlockThreads), lds_bytes, stream,
                     (const DevStage*)stage, gr_step, perm, n_split, n_tasks, ndocs, (const GrExport*)gr_export, pw,
                     pw_n, t, rec, flags, lds_bytes, cursor);
  return (int)hipGetLastError();
}

// GopherRepetition word arrays of the npre pre-pass documents (after tb_pre_decode; the
// descriptors' wh / wtab / wk / wpb / wcsum / wslot / wid / wl hold [W + 1]-sized buffers,
// wtab [1.5 W + 2], wcsum [4 chunks]; chunks_max >= ceil(max W / 2048)).
int tb_pre_wcanon(hipStream_t stream, const uint8_t* bytes, const int64_t* off, const int32_t* perm, int32_t npre,
                  const uint8_t* dead, void* pre, uint32_t chunks_max, const uint64_t* pw, uint32_t pw_n,
                  uint32_t* flags) {
  if (npre <= 0) return 0;
  if (!perm || !pre || !pw || !flags || chunks_max == 0 || npre > 65535) return (int)hipErrorInvalidValue;
  const PreDoc* p = (const PreDoc*)pre;
  const dim3 gz(chunks_max + 1, (uint32_t)npre), g(chunks_max, (uint32_t)npre);
  hipLaunchKernelGGL(k_pre_wcanon<0>, gz, dim3(kPreWThreads), 0, stream, bytes, off, perm, dead, p, pw, pw_n, flags);
  hipLaunchKernelGGL(k_pre_wcanon<1>, g, dim3(kPreWThreads), 0, stream, bytes, off, perm, dead, p, pw, pw_n, flags);
  hipLaunchKernelGGL(k_pre_wsum<0>, dim3((uint32_t)npre), dim3(64), 0, stream, perm, dead, (PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_wcanon<2>, g, dim3(kPreWThreads), 0, stream, bytes, off, perm, dead, p, pw, pw_n, flags);
  hipLaunchKernelGGL(k_pre_wsum<1>, dim3((uint32_t)npre), dim3(64), 0, stream, perm, dead, (PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_wcanon<3>, g, dim3(kPreWThreads), 0, stream, bytes, off, perm, dead, p, pw, pw_n, flags);
  return (int)hipGetLastError();
}

size_t tb_sizeof_gr_export() { return sizeof(GrExport); }
size_t tb_sizeof_pre_doc() { return sizeof(PreDoc); }

// Decode + word-break marks of the first npre launch positions of the long-document launch
// (`pre`: npre descriptors with n / off / prop / wbm set, C and dict zeroed; cnt: int64
// [npre * tiles_max], tiles_max >= ceil(max n / 16 KB)).
int tb_pre_decode(hipStream_t stream, const uint8_t* bytes, const int64_t* off, const int32_t* perm, int32_t npre,
                  const uint8_t* dead, void* pre, uint32_t tiles_max, int64_t* cnt, const uint16_t* s1,
                  const uint32_t* s2, const uint16_t* l1, const int32_t* l2) {
  if (npre <= 0) return 0;
  if (!perm || !pre || !cnt || tiles_max == 0 || npre > 65535) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  const dim3 g(tiles_max, (uint32_t)npre);
  hipLaunchKernelGGL(k_pre_count, g, dim3(kPreThreads), 0, stream, bytes, off, perm, dead, (const PreDoc*)pre,
                     tiles_max, cnt);
  hipLaunchKernelGGL(k_pre_decode, g, dim3(kPreThreads), 0, stream, bytes, off, perm, dead, (PreDoc*)pre, tiles_max,
                     (const int64_t*)cnt, t);
  // chunks of 64 code points: C + 1 <= n + 1 positions
  const uint32_t chunks = tiles_max * (kPreTile / 64) + 1;
  hipLaunchKernelGGL(k_pre_wb, dim3(chunks, (uint32_t)npre), dim3(64), 0, stream, perm, dead, (PreDoc*)pre);
  const dim3 gw(chunks, (uint32_t)npre);
  hipLaunchKernelGGL(k_pre_words<0>, gw, dim3(64), 0, stream, perm, dead, (const PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_words_scan<0>, dim3((uint32_t)npre), dim3(64), 0, stream, perm, dead, (PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_words<1>, gw, dim3(64), 0, stream, perm, dead, (const PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_words_scan<1>, dim3((uint32_t)npre), dim3(64), 0, stream, perm, dead, (PreDoc*)pre);
  hipLaunchKernelGGL(k_pre_words<2>, gw, dim3(64), 0, stream, perm, dead, (const PreDoc*)pre);
  return (int)hipGetLastError();
}

int tb_c4_pass_a_blk(hipStream_t stream, const void* c4, const uint8_t* bytes, const int64_t* off,
                     const int32_t* perm, int32_t nblocks, int32_t ndocs, char* scratch, const int64_t* scratch_off,
                     const uint64_t* pw, uint32_t pw_n, const uint16_t* s1, const uint32_t* s2, const uint16_t* l1,
                     const int32_t* l2, int64_t* rec, int64_t* src, uint32_t* flags, uint32_t lds_bytes,
                     uint64_t* prof, const uint8_t* dead, const uint32_t* line_stats, uint32_t* c4_words,
                     const int64_t* dict_loff, const uint32_t* dict_ldata) {
  if (nblocks <= 0) return 0;
  if (!perm || lds_bytes > kMaxLdsPerBlk) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)k_c4_pass_a_blk, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_bytes);
  hipLaunchKernelGGL(k_c4_pass_a_blk, dim3(nblocks), dim3(kBlockThreads), lds_bytes, stream, (const DevC4*)c4,
                     bytes, off, perm, ndocs, scratch, scratch_off, pw, pw_n, t, rec, src, flags, lds_bytes, prof, dead,
                     line_stats, c4_words, DictLines{dict_loff, dict_ldata});
  return (int)hipGetLastError();
}

int tb_block_threads() { return kBlockThreads; }

int tb_badwords_match(hipStream_t stream, const uint8_t* bytes, const int64_t* off, int32_t nitems, const int32_t* root,
                      const uint8_t* cjk, int32_t root0, int32_t cjk0, const uint8_t* dead, uint32_t dead_max,
                      const uint32_t* table, uint32_t table_mask, const uint16_t* s1, const uint32_t* s2,
                      const uint16_t* l1, const int32_t* l2, const uint16_t* f1, const int32_t* f2, int8_t* matched,
                      const int32_t* seg_doc, const int32_t* seg_idx, uint32_t seg_bytes) {
  if (nitems <= 0) return 0;
  if (!table || ((table_mask + 1) & table_mask) != 0 || seg_bytes < 256 || (seg_bytes & 255) || (!seg_doc != !seg_idx))
    return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  const BwTable bt{table, table_mask};
  const BwFold fold{f1, f2};
  hipLaunchKernelGGL(k_badwords_match, dim3((nitems + kBwWaves - 1) / kBwWaves), dim3(64 * kBwWaves), 0, stream, bytes,
                     off, nitems, root, cjk, root0, cjk0, dead, dead_max, bt, t, fold, matched, seg_doc, seg_idx,
                     seg_bytes);
  return (int)hipGetLastError();
}

// The pair table of k_langid_mfma (+ its zero row) from the embedding table, into aux
// [tb_langid_aux_bytes()]: once per model.
int tb_langid_aux_bytes() { return kLidAuxBytes; }
int tb_langid_prepare(hipStream_t stream, const uint8_t* E, uint8_t* aux) {
  if (!E || !aux) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_lid_pairs, dim3((kLidPairs + 255) / 256), dim3(256), 0, stream, E, (uint32_t*)aux);
  return (int)hipGetLastError();
}

// k_langid_mfma: records of every document (perm order, 16 per tile); Eb = E + 128 as uint8
// [buckets * 16] (the biased block-sparse embedding table), aux its pair table
// (tb_langid_prepare), WT bf16 bits [16 * 32] (the head transposed, columns >= 5 zero), bias float [8].
int tb_langid_mfma(hipStream_t stream, const uint8_t* bytes, const int64_t* off, const int32_t* perm, int32_t ndocs,
                   const uint16_t* s1, const uint32_t* s2, const uint16_t* l1, const int32_t* l2, const uint8_t* E,
                   const uint8_t* aux, const uint16_t* WT, double w_scale, const float* bias, int64_t* rec,
                   int32_t width, uint64_t* prof) {
  if (ndocs <= 0) return 0;
  if (!E || !aux || !WT || !bias || !rec || width < 2 || !(w_scale > 0)) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  const int ntiles = (ndocs + kLidTile - 1) / kLidTile;
  const int cus = device_cus();
  const int grid = ntiles < 4 * cus ? ntiles : 4 * cus;
  hipLaunchKernelGGL(k_langid_mfma, dim3(grid), dim3(64 * kLidWaves), 0, stream, bytes, off, perm, ndocs, t, E, aux,
                     WT, w_scale, bias, rec, width, prof);
  return (int)hipGetLastError();
}

int tb_c4_pass_a(hipStream_t stream, const void* c4, const uint8_t* bytes, const int64_t* off, const int32_t* perm,
                 int32_t ndocs, char* scratch, const int64_t* scratch_off, const uint64_t* pw, uint32_t pw_n,
                 const uint16_t* s1, const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec,
                 int64_t* src, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof, int32_t nblocks,
                 const uint8_t* dead, const uint32_t* line_stats, uint32_t* c4_words, const int64_t* dict_loff,
                 const uint32_t* dict_ldata) {
  if (ndocs <= 0) return 0;
  if (nblocks <= 0) nblocks = ndocs;
  if (lds_bytes > kMaxLdsPerDoc) return (int)hipErrorInvalidValue;
  DevTables t{s1, s2, l1, l2};
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)k_c4_pass_a, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  hipLaunchKernelGGL(k_c4_pass_a, dim3(nblocks), dim3(64), lds_bytes, stream, (const DevC4*)c4, bytes, off, perm, ndocs,
                     scratch, scratch_off, pw, pw_n, t, rec, src, flags, lds_bytes, prof, dead, line_stats, c4_words,
                     DictLines{dict_loff, dict_ldata});
  return (int)hipGetLastError();
}

int tb_c4_pass_b(hipStream_t stream, const uint8_t* bytes, const int64_t* off, int32_t ndocs, const char* scratch,
                 const int64_t* scratch_off, const int64_t* src, const int64_t* new_off, uint8_t* out) {
  if (ndocs <= 0) return 0;
  hipLaunchKernelGGL(k_c4_pass_b, dim3(ndocs), dim3(256), 0, stream, bytes, off, ndocs, scratch, scratch_off, src,
                     new_off, out);
  return (int)hipGetLastError();
}


int tb_gate(hipStream_t stream, const void* gate, const int64_t* const* recs, int32_t nrecs, int32_t ndocs,
            const uint32_t* flags, uint8_t* dead, int32_t code) {
  if (ndocs <= 0) return 0;
  if (nrecs < 0 || nrecs > kMaxGateSteps || code <= 0 || code > 255) return (int)hipErrorInvalidValue;
  GateRecs r{};
  for (int i = 0; i < nrecs; ++i) r.p[i] = recs[i];
  hipLaunchKernelGGL(k_gate, dim3((ndocs + 255) / 256), dim3(256), 0, stream, (const DevGate*)gate, r, ndocs, flags,
                     dead, (uint8_t)code);
  return (int)hipGetLastError();
}

size_t tb_sizeof_gate() { return sizeof(DevGate); }

// K16: resolve + four scans + compaction, all on `stream`. vb/vo: content versions 0..nver-1;
// lanes: 4*ndocs int64 scratch, sc: 4*ndocs int64 scan output; out must hold the final contents
// (cap bytes: the caller bounds it by version 0 plus the C4 growth; a document that would pass
// the end sets *err and is not written), out_off ndocs+1, rows ndocs.
int tb_resolve(hipStream_t stream, const void* rp, const int64_t* const* recs, int32_t nrecs, int32_t ndocs,
               const uint32_t* flags, const uint8_t* const* vb, const int64_t* const* vo, int32_t nver,
               int32_t* fail, uint8_t* status, uint8_t* fver, int64_t* lanes, int64_t* sc, uint8_t* out,
               int64_t cap, int64_t* out_off, int32_t* rows, int32_t* err) {
  if (ndocs <= 0) return 0;
  if (nrecs < 0 || nrecs > kMaxGateSteps || nver < 1 || nver > kMaxVersions) return (int)hipErrorInvalidValue;
  GateRecs r{};
  for (int i = 0; i < nrecs; ++i) r.p[i] = recs[i];
  VersionTab vt{};
  for (int i = 0; i < nver; ++i) {
    vt.b[i] = vb[i];
    vt.off[i] = vo[i];
  }
  hipLaunchKernelGGL(k_resolve, dim3((ndocs + 255) / 256), dim3(256), 0, stream, (const DevResolve*)rp, r, ndocs,
                     flags, vt, fail, status, fver, lanes);
  for (int j = 0; j < 4; ++j) {
    const int rc = tb_scan_strided_i64(stream, lanes + j, 4, ndocs, sc + (int64_t)j * ndocs);
    if (rc) return rc;
  }
  // one wave per document (short documents, the common case), a whole workgroup per document once
  // they average over 8 KB (the output holds every document, so cap / ndocs is about their length)
  if (cap / (ndocs > 0 ? ndocs : 1) > 8192)
    hipLaunchKernelGGL(k_compact<256>, dim3(ndocs), dim3(kCompactThreads), 0, stream, status, fver, vt, ndocs, sc, out, cap, out_off, rows,
                     err);
  else
    hipLaunchKernelGGL(k_compact<64>, dim3((ndocs + 3) / 4), dim3(kCompactThreads), 0, stream, status, fver, vt, ndocs, sc, out, cap, out_off, rows,
                     err);
  return (int)hipGetLastError();
}

size_t tb_sizeof_resolve() { return sizeof(DevResolve); }


int tb_pow_table(hipStream_t stream, uint64_t* pw, uint32_t n) {
  hipLaunchKernelGGL(k_pow_table, dim3((n + 256) / 256), dim3(256), 0, stream, pw, n);
  return (int)hipGetLastError();
}

int tb_phase_slots() { return kPhaseSlots; }
int tb_stage_waves() { return TB_STAGE_WPE; }  // waves per SIMD the wave stage kernel is built for

int tb_abi_version() { return 24; }
size_t tb_sizeof_plan() { return sizeof(DevPlan); }
size_t tb_sizeof_stage() { return sizeof(DevStage); }
size_t tb_sizeof_c4() { return sizeof(DevC4); }

}  // extern "C"
