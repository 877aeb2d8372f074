// LDS-resident stage kernel for short documents (csrc/common/lds_stage.h): one wave64 per
// document, every working array in the wave's dynamic LDS slice (ds_* instructions only, no
// HBM scratch). The host launches it once per length bucket of the longest-first permutation, the
// slice sized for the bucket's longest document, so the number of resident waves per CU follows
// from the documents' footprint (160 KiB / slice). A document whose arrays do not fit is appended
// to a retry list; k_stage_retry then recomputes the listed documents with the generic algorithm
// (docproc.h analyze_stage over an HBM scratch slice per retry workgroup).
#include <hip/hip_runtime.h>

#include "../common/lds_stage.h"

using namespace tb;

namespace {

struct LdsTables {
  const uint16_t* s1;
  const uint32_t* s2;
  const uint16_t* l1;
  const int32_t* l2;
};

extern __shared__ __attribute__((aligned(16))) char g_lds_stage[];

// Stage of one content version for launch positions [pos0, pos0 + gridDim.x) of `perm`: one
// document per workgroup, P = WavePar (one wave) or BlockPar<NT> (NT/64 waves sharing the slice).
template <class P>
__device__ __forceinline__ void stage_lds_body(P par, const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage,
                                                  const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
                                                  const int32_t* __restrict__ perm, int32_t pos0, int32_t ndocs,
                                                  LdsTables tabs, int64_t* rec, uint32_t* flags, uint32_t lds_bytes,
                                                  uint64_t* prof, const uint8_t* __restrict__ dead,
                                                  uint32_t* __restrict__ retry_cnt, int32_t* __restrict__ retry_pos) {
  const int k = pos0 + (int)blockIdx.x;
  const int doc = perm[k];
  if (doc >= ndocs || (dead && dead[doc])) return;
  const int64_t o0 = off[doc];
  const uint32_t n = (uint32_t)(off[doc + 1] - o0);
  LCtx<P> x;
  x.par = par;
  x.a.base = (TB_LDS char*)g_lds_stage;
  x.a.cap = lds_bytes & ~7u;
  x.ucd = UcdView{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
  x.flag = flags + doc;
  x.prof = prof ? prof + (size_t)doc * kPhaseSlots : nullptr;
  TB_LDS uint16_t* asc = x.a.template get<uint16_t>(128);
  TB_LDS uint8_t* tx = x.a.template get<uint8_t>(n + 16);
  bool fail = x.a.ovf || n > kLdsMaxDoc;
  if (!fail) {
    x.par.for_n(128, [&](uint32_t c) { asc[c] = compact_prop(x.ucd.props(c)); });
    // the text, 4-aligned in LDS: destination dword q = source bytes [4q, 4q + 4) (two aligned
    // global dwords funnel-shifted; the batch buffers are padded past the last document), then
    // two zero dwords of padding for the 4-byte-wide readers
    const uint8_t* src = bytes + o0;
    const uint32_t sh = (uint32_t)((uintptr_t)src & 3u);
    const uint32_t* s32 = (const uint32_t*)(src - sh);
    TB_LDS uint32_t* d32 = (TB_LDS uint32_t*)tx;
    const uint32_t nd = (n + 3) >> 2;
    x.par.for_n(nd + 2, [&](uint32_t q) {
      uint32_t v = 0;
      if (q < nd) {
        const uint32_t lo = s32[q];
        v = sh ? __builtin_amdgcn_alignbyte(s32[q + 1], lo, sh) : lo;
        const uint32_t rem = n - 4 * q;
        if (rem < 4) v &= 0xFFFFFFFFu >> (32 - 8 * rem);
      }
      d32[q] = v;
    });
    x.par.sync();
    x.asc = asc;
    fail = lds_analyze_stage(x, *stage, *plan, tx, n, rec, (uint32_t)ndocs, (uint32_t)doc) != LDS_OK;
  }
  if (fail && x.par.leader()) {
    const uint32_t i = atomicAdd(retry_cnt, 1u);
    retry_pos[i] = k;
  }
}

// Register budgets: unconstrained (no spills, 2 waves/SIMD) for slices that allow few waves per CU
// anyway, 4 and 8 waves/SIMD (some spilling) for the small slices of short documents; the host
// picks per length bucket (tb_stage_lds `waves`).
#define TB_STAGE_LDS_KERNEL(NAME, ATTR)                                                                         \
  __global__ __launch_bounds__(64) ATTR void NAME(                                                             \
      const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes,  \
      const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t pos0, int32_t ndocs,           \
      LdsTables tabs, int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof,                       \
      const uint8_t* __restrict__ dead, uint32_t* __restrict__ retry_cnt, int32_t* __restrict__ retry_pos) {   \
    stage_lds_body(WavePar(), plan, stage, bytes, off, perm, pos0, ndocs, tabs, rec, flags, lds_bytes, prof,     \
                   dead, retry_cnt, retry_pos);                                                                \
  }
TB_STAGE_LDS_KERNEL(k_stage_lds, )
TB_STAGE_LDS_KERNEL(k_stage_lds_w4, __attribute__((amdgpu_waves_per_eu(4, 8))))
TB_STAGE_LDS_KERNEL(k_stage_lds_w8, __attribute__((amdgpu_waves_per_eu(8, 8))))

// Multi-wave workgroups for the longer short documents: NT/64 waves cooperate on one document in
// one slice (SegPar: each wave scans a contiguous segment of every pass, one barrier per
// primitive), so a 2-4 KB document's ~40 KB slice keeps several waves busy instead of one.
template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_stage_lds_seg(
    const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes,
    const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t pos0, int32_t ndocs, LdsTables tabs,
    int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof, const uint8_t* __restrict__ dead,
    uint32_t* __restrict__ retry_cnt, int32_t* __restrict__ retry_pos) {
  __shared__ __attribute__((aligned(16))) char xs[2 * 16 * (NT / 64) + 64];
  SegPar<NT> par;
  par.xs = xs;
  stage_lds_body(par, plan, stage, bytes, off, perm, pos0, ndocs, tabs, rec, flags, lds_bytes, prof, dead, retry_cnt,
                 retry_pos);
}
template __global__ void k_stage_lds_seg<128>(const DevPlan*, const DevStage*, const uint8_t*, const int64_t*,
                                              const int32_t*, int32_t, int32_t, LdsTables, int64_t*, uint32_t*,
                                              uint32_t, uint64_t*, const uint8_t*, uint32_t*, int32_t*);
template __global__ void k_stage_lds_seg<256>(const DevPlan*, const DevStage*, const uint8_t*, const int64_t*,
                                              const int32_t*, int32_t, int32_t, LdsTables, int64_t*, uint32_t*,
                                              uint32_t, uint64_t*, const uint8_t*, uint32_t*, int32_t*);

// Generic recomputation of the documents k_stage_lds could not fit: workgroup b handles list
// entries b, b + gridDim.x, ... in its own HBM scratch slice (slice_bytes each) and the usual
// per-wave LDS arena of the generic kernel. Every wave leaves once the list is exhausted.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_stage_retry(
    const DevPlan* __restrict__ plan, const DevStage* __restrict__ stage, const uint8_t* __restrict__ bytes,
    const int64_t* __restrict__ off, const int32_t* __restrict__ perm, int32_t ndocs, char* scratch,
    uint64_t slice_bytes, const uint64_t* __restrict__ pw, uint32_t pw_n, LdsTables tabs, int64_t* rec,
    uint32_t* flags, uint32_t lds_bytes, uint64_t* prof, const uint32_t* __restrict__ retry_cnt,
    const int32_t* __restrict__ retry_pos) {
  const uint32_t cnt = *retry_cnt;
  for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const int doc = perm[retry_pos[i]];
    DocCtx<WavePar> x;
    x.prof = prof ? prof + (size_t)doc * kPhaseSlots : nullptr;
    x.lds = lds_bytes ? (char*)g_lds_stage : nullptr;
    x.lcap = lds_bytes;
    x.lused = 0;
    x.ucd = UcdView{tabs.s1, tabs.s2, tabs.l1, tabs.l2};
    x.pw = pw;
    x.pw_n = pw_n;
    x.ipw = pw ? pw + pw_n + 1 : nullptr;
    x.scr = scratch + (uint64_t)blockIdx.x * slice_bytes;
    x.cap = slice_bytes;
    x.used = 0;
    x.flag = flags + doc;
    const uint8_t* b = bytes + off[doc];
    const uint32_t n = (uint32_t)(off[doc + 1] - off[doc]);
    if (scratch_bytes_for_dev(n) > slice_bytes) {  // never for documents the host put on the LDS path
      x.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW);
      continue;
    }
    uint32_t* asc = x.template try_lds<uint32_t>(128);
    if (asc) {
      x.par.for_n(128, [&](uint32_t c) { asc[c] = x.ucd.props(c); });
      x.par.sync();
      x.asc = asc;
    }
    StageOut out{rec, (uint32_t)ndocs, (uint32_t)doc};
    analyze_stage<WavePar, false>(x, *stage, *plan, LidTables{nullptr, nullptr}, b, n, out);
    x.par.sync();
  }
}

}  // namespace

extern "C" {

// One length bucket: launch positions [pos0, pos0 + nblocks) of perm, lds_bytes per wave.
int tb_stage_lds(hipStream_t stream, const void* plan, const void* stage, const uint8_t* bytes, const int64_t* off,
                 const int32_t* perm, int32_t pos0, int32_t nblocks, int32_t ndocs, const uint16_t* s1,
                 const uint32_t* s2, const uint16_t* l1, const int32_t* l2, int64_t* rec, uint32_t* flags,
                 uint32_t lds_bytes, uint64_t* prof, const uint8_t* dead, uint32_t* retry_cnt, int32_t* retry_pos,
                 int32_t waves, int32_t threads) {
  if (nblocks <= 0) return 0;
  if (!perm || !retry_cnt || !retry_pos || pos0 < 0 || lds_bytes < 512 || lds_bytes > 159 * 1024)
    return (int)hipErrorInvalidValue;
  LdsTables t{s1, s2, l1, l2};
  // threads > 64: one multi-wave workgroup per document (k_stage_lds_seg)
  auto kern = threads == 256 ? k_stage_lds_seg<256> : threads == 128 ? k_stage_lds_seg<128>
              : waves == 8   ? k_stage_lds_w8       : waves == 4      ? k_stage_lds_w4 : k_stage_lds;
  if (threads != 64 && threads != 128 && threads != 256) return (int)hipErrorInvalidValue;
  if (lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  hipLaunchKernelGGL(kern, dim3((uint32_t)nblocks), dim3((uint32_t)threads), lds_bytes, stream, (const DevPlan*)plan,
                     (const DevStage*)stage, bytes, off, perm, pos0, ndocs, t, rec, flags, lds_bytes, prof, dead,
                     retry_cnt, retry_pos);
  return (int)hipGetLastError();
}

int tb_stage_retry(hipStream_t stream, const void* plan, const void* stage, const uint8_t* bytes, const int64_t* off,
                   const int32_t* perm, int32_t ndocs, char* scratch, uint64_t slice_bytes, int32_t grid,
                   const uint64_t* pw, uint32_t pw_n, const uint16_t* s1, const uint32_t* s2, const uint16_t* l1,
                   const int32_t* l2, int64_t* rec, uint32_t* flags, uint32_t lds_bytes, uint64_t* prof,
                   const uint32_t* retry_cnt, const int32_t* retry_pos) {
  if (grid <= 0) return 0;
  if (!perm || !retry_cnt || !retry_pos || !scratch || lds_bytes > 65536) return (int)hipErrorInvalidValue;
  LdsTables t{s1, s2, l1, l2};
  hipLaunchKernelGGL(k_stage_retry, dim3((uint32_t)grid), dim3(64), lds_bytes, stream, (const DevPlan*)plan,
                     (const DevStage*)stage, bytes, off, perm, ndocs, scratch, slice_bytes, pw, pw_n, t, rec, flags,
                     lds_bytes, prof, retry_cnt, retry_pos);
  return (int)hipGetLastError();
}

}  // extern "C"
