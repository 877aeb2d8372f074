// Device-side step gating: which documents are already filtered before a device pass runs.
//
// The reference executor stops a document at its first failing step; later steps never run on it
// (reference executor.rs:30-57). The batched device path runs passes (stages / C4 rewrites) over
// whole batches, so after each pass a gate kernel evaluates the pass/fail branch of every step
// the pass produced records for and marks failing documents dead; later passes skip them. On
// CommonCrawl-shaped input the Gopher steps alone filter ~75 % of documents, so the C4 rewrite
// and the FineWeb stage only do a quarter of the work.
//
// gate_fails() mirrors the pass/fail branches of the host decision code (csrc/host/filters.cpp
// decide_t, which follows the reference filters) with the same double-precision expressions. It
// is only an optimisation: the host resolver re-derives every decision from the records and
// recomputes on the CPU path any document it finds alive that the device skipped, so a
// disagreement can cost time but never change an output.
#pragma once
#include "tb_common.h"

namespace tb {

constexpr int kMaxGateSteps = 8;
constexpr int kMaxGateNgrams = 16;

enum GateKind : int32_t {
  GK_NONE = 0,
  GK_GOPHER_QUALITY = 1,
  GK_GOPHER_REP = 2,
  GK_FINEWEB = 3,
  GK_LANGID = 4,
  GK_C4 = 5,
};

// GopherQuality optional thresholds (bit i of `has` set = configured)
enum : int32_t {
  GQ_T_MIN_WORDS = 0, GQ_T_MAX_WORDS, GQ_T_MIN_AVG, GQ_T_MAX_AVG, GQ_T_SYMBOL, GQ_T_BULLET, GQ_T_ELL_LINES,
  GQ_T_ALPHA, GQ_T_MIN_STOP,
};
// GopherRepetition optional fractions
enum : int32_t { GR_T_PARA = 0, GR_T_PARA_CHAR, GR_T_LINE, GR_T_LINE_CHAR };

struct DevGateStep {
  int32_t kind;
  int32_t slot;      // which record buffer (GateRecs::p[slot])
  int32_t prefix;    // element offset of this step's records = prefix * ndocs
  int32_t width;     // int64 fields per document
  uint32_t has;      // optional-threshold bits
  int32_t n_top, n_dup;
  int32_t flag;      // FineWeb: line_punct_exclude_zero
  int64_t i[4];      // integer thresholds
  double d[8];       // real thresholds
  int64_t top_n[kMaxGateNgrams];
  double top_thr[kMaxGateNgrams];
  int64_t dup_n[kMaxGateNgrams];
  double dup_thr[kMaxGateNgrams];
};

struct DevGate {
  int32_t n_steps;
  int32_t pad;
  DevGateStep steps[kMaxGateSteps];
};

struct GateRecs {
  const int64_t* p[kMaxGateSteps];
};

TB_HD int64_t gate_max1(int64_t v) { return v > 1 ? v : 1; }

// True when the step's decision for record `r` is "filtered" (or an error): the document does
// not reach any later step.
TB_HD bool gate_fails(const DevGateStep& g, const int64_t* r) {
  switch (g.kind) {
    case GK_GOPHER_QUALITY: {  // decide_t GopherQuality (reference gopher_quality.rs:198-317)
      const int64_t n = r[0];
      const double ncalc = (double)gate_max1(n);
      const double avg = n > 0 ? (double)r[1] / (double)n : 0.0;
      const double hash_ratio = (double)r[2] / ncalc;
      const double ell_ratio = (double)r[3] / ncalc;
      const double lcalc = (double)gate_max1(r[4]);
      const double bullet = (double)r[5] / lcalc;
      const double ell_lines = (double)r[6] / lcalc;
      const double alpha = (double)r[7] / ncalc;
      const uint32_t h = g.has;
      if ((h >> GQ_T_MIN_WORDS & 1) && n < g.i[0]) return true;
      if ((h >> GQ_T_MAX_WORDS & 1) && n > g.i[1]) return true;
      if ((h >> GQ_T_MIN_AVG & 1) && avg < g.d[0]) return true;
      if ((h >> GQ_T_MAX_AVG & 1) && n > 0 && avg > g.d[1]) return true;
      if ((h >> GQ_T_SYMBOL & 1) && (hash_ratio > g.d[2] || ell_ratio > g.d[2])) return true;
      if ((h >> GQ_T_BULLET & 1) && bullet > g.d[3]) return true;
      if ((h >> GQ_T_ELL_LINES & 1) && ell_lines > g.d[4]) return true;
      if ((h >> GQ_T_ALPHA & 1) && alpha < g.d[5]) return true;
      if ((h >> GQ_T_MIN_STOP & 1) && g.i[2] > 0 && r[8] < g.i[2]) return true;
      return false;
    }
    case GK_GOPHER_REP: {  // decide_t GopherRepetition (reference gopher_rep.rs:52-220)
      if (r[0] < 0) return true;
      const double C = (double)gate_max1(r[0]);
      const double para_len = (double)gate_max1(r[1]);
      const double line_len = (double)gate_max1(r[4]);
      const uint32_t h = g.has;
      if ((h >> GR_T_PARA & 1) && (double)r[2] / para_len > g.d[0]) return true;
      if ((h >> GR_T_PARA_CHAR & 1) && (double)r[3] / C > g.d[1]) return true;
      if ((h >> GR_T_LINE & 1) && (double)r[5] / line_len > g.d[2]) return true;
      if ((h >> GR_T_LINE_CHAR & 1) && (double)r[6] / C > g.d[3]) return true;
      int k = 7;
      for (int t = 0; t < g.n_top; ++t, ++k)
        if (g.top_n[t] > 0 && (double)r[k] / C > g.top_thr[t]) return true;
      for (int t = 0; t < g.n_dup; ++t, ++k)
        if (g.dup_n[t] > 0 && (double)r[k] / C > g.dup_thr[t]) return true;
      return false;
    }
    case GK_FINEWEB: {  // decide_t FineWeb (reference fineweb_quality.rs:71-226)
      const int64_t nl = r[0];
      if (nl == 0) return true;
      double ratio = (double)r[1] / (double)nl;
      if (ratio < g.d[0] && !(ratio == 0.0 && g.flag)) return true;
      ratio = (double)r[2] / (double)nl;
      if (ratio > g.d[1]) return true;
      const int64_t tot = r[4];
      ratio = tot > 0 ? (double)r[3] / (double)tot : 0.0;
      if (ratio > g.d[2]) return true;
      const int64_t w = r[6], nls = r[5];
      if (w == 0) return nls > 0;
      return (double)nls / (double)w > g.d[3];
    }
    case GK_LANGID: {  // decide_t LanguageDetection (reference language_filter.rs:35-93)
      const int64_t lang = r[0];
      if (lang < 0 || lang >= 32) return true;
      if (!((g.has >> lang) & 1u)) return true;
      union { int64_t i; double d; } u;
      u.i = r[1];
      return u.d < g.d[0];
    }
    case GK_C4: {  // decide_t C4Quality (reference c4_filters.rs:147-295)
      if (r[0] || r[1]) return true;
      return g.i[0] > 0 && r[5] < g.i[0];
    }
    default:
      return false;
  }
}

// ---- K16 resolve: the executor's first-failure chain over the whole pipeline ----------------
// (reference executor.rs:32-46 + producer_logic.rs:148-167). Valid only when every pipeline step
// runs on the device and has a gate kind (build_resolve refuses otherwise): then the per-document
// outcome — first failing step, kept / filtered, final content version — is a pure function of
// the device records and needs no host decision. The host still re-derives every decision from
// the same records (decide_t) and compares; a disagreement falls back to host assembly.

// status codes (as BatchState::status_): 0 kept, 1 filtered, 3 delegated to the CPU path
constexpr uint8_t kResolveKept = 0, kResolveFiltered = 1, kResolveDelegated = 3;
constexpr int32_t kResolveDelegatedStep = 1 << 30;
constexpr int kMaxVersions = 8;  // content versions the resolve kernel can read (C4 rewrites + 1)

struct DevResolve {
  DevGate gate;                          // every pipeline step in pipeline order
  int32_t step_index[kMaxGateSteps];     // pipeline index of gate.steps[k]
  int32_t c4_version[kMaxGateSteps];     // C4 rewrite step: content version it produces, else -1
};

// One document: fail = first failing pipeline step (-1 none, kResolveDelegatedStep when flagged),
// status, ver = content version the outputs carry (C4 rewrites apply to every document that reaches
// the step unless its lorem-ipsum / curly-bracket branch fired: BatchState::apply_records).
TB_HD void resolve_doc(const DevResolve& rp, const int64_t* const* recs, int64_t ndocs, int64_t doc, uint32_t flags,
                       int32_t& fail, uint8_t& status, int32_t& ver) {
  fail = -1;
  status = kResolveKept;
  ver = 0;
  if (flags) {
    fail = kResolveDelegatedStep;
    status = kResolveDelegated;
    return;
  }
  for (int s = 0; s < rp.gate.n_steps; ++s) {
    const DevGateStep& g = rp.gate.steps[s];
    const int64_t* r = recs[g.slot] + (int64_t)g.prefix * ndocs + doc * g.width;
    if (rp.c4_version[s] >= 0 && !r[0] && !r[1]) ver = rp.c4_version[s];
    if (gate_fails(g, r)) {
      fail = rp.step_index[s];
      status = kResolveFiltered;
      return;
    }
  }
}

}  // namespace tb
