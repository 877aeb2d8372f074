// Builds the POD device plan (csrc/common/devplan.h) from step configs, and runs the device
// document algorithms (csrc/common/docproc.h) on the host with the sequential policy.
#include "devplan_build.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../common/docproc.h"

namespace tb {

int dev_kind_of(const StepCfg& c) {
  switch (c.kind) {
    case StepKind::GopherQuality: return DK_GOPHER_QUALITY;
    case StepKind::GopherRepetition: return DK_GOPHER_REP;
    case StepKind::FineWebQuality: return DK_FINEWEB;
    case StepKind::LanguageDetection: return DK_LANGID;
    default: return DK_NONE;
  }
}

bool device_supported(const StepCfg& c, std::string* why) {
  if (c.kind == StepKind::GopherRepetition) {
    if (c.top_n_grams.size() > (size_t)kMaxNgramEntries || c.dup_n_grams.size() > (size_t)kMaxNgramEntries) {
      if (why) *why = "more than 16 n-gram entries";
      return false;
    }
    for (auto& e : c.top_n_grams) if (e.first > (1 << 20)) { if (why) *why = "n too large"; return false; }
    for (auto& e : c.dup_n_grams) if (e.first > (1 << 20)) { if (why) *why = "n too large"; return false; }
  }
  if (c.kind == StepKind::FineWebQuality && c.stop_chars.size() > (size_t)kMaxStopChars) {
    if (why) *why = "more than 16 stop_chars";
    return false;
  }
  if (c.kind == StepKind::GopherQuality) {
    size_t bytes = 0;
    for (auto& w : c.stop_words) bytes += w.size();
    if (c.stop_words.size() > (size_t)kMaxStopWords || bytes > (size_t)kStopBlobBytes) {
      if (why) *why = "stop word list too large for the device table";
      return false;
    }
  }
  return true;
}

static int add_stop_set(DevPlan& plan, const std::vector<std::string>& words) {
  if (plan.n_stop_sets >= kMaxStopSets) throw std::runtime_error("too many distinct stop-word sets");
  DevStopSet& ss = plan.stops[plan.n_stop_sets];
  std::memset(&ss, 0, sizeof(ss));
  std::vector<std::string> uniq;
  for (auto& w : words)
    if (std::find(uniq.begin(), uniq.end(), w) == uniq.end()) uniq.push_back(w);
  int32_t pos = 0;
  for (size_t i = 0; i < uniq.size(); ++i) {
    const std::string& w = uniq[i];
    ss.off[i] = pos;
    std::memcpy(ss.blob + pos, w.data(), w.size());
    pos += (int32_t)w.size();
    const uint64_t key = dev_key(hash_bytes((const uint8_t*)w.data(), (uint32_t)w.size()), (uint32_t)w.size());
    uint32_t slot = (uint32_t)(key >> 17) & (kStopTableSize - 1);
    while (ss.keys[slot] != 0) slot = (slot + 1) & (kStopTableSize - 1);
    ss.keys[slot] = key;
    ss.idx[slot] = (int32_t)i;
  }
  ss.off[uniq.size()] = pos;
  ss.n = (int32_t)uniq.size();
  for (auto& w : uniq) ss.max_len = std::max<int32_t>(ss.max_len, (int32_t)w.size());
  if (ss.n <= kStopLiteMaxWords && pos <= kStopLiteMaxBlob) {
    uint32_t ns = 16;
    while (ns < 4u * (uint32_t)ss.n) ns <<= 1;
    ss.lite_nslots = (int32_t)ns;
    ss.all_ascii7 = 1;
    for (size_t i = 0; i < uniq.size(); ++i) {
      uint32_t h = kStopLiteHash0;
      for (unsigned char c : uniq[i]) h = stop_lite_hash_push(h, c);
      uint32_t slot = stop_lite_slot(h, ns);
      while (ss.lite_slots[slot] != 0) slot = (slot + 1) & (ns - 1);
      ss.lite_slots[slot] = (h & 0xFFFF0000u) | (uint32_t)(i + 1);
      const std::string& w = uniq[i];
      bool ascii = !w.empty() && w.size() <= 7;
      for (unsigned char c : w) ascii = ascii && c < 0x80;
      if (!ascii) ss.all_ascii7 = 0;
      if (ascii) {
        uint64_t key = (uint64_t)w.size() << 56;
        for (size_t k = 0; k < w.size(); ++k) key |= (uint64_t)(unsigned char)w[k] << (8 * k);
        uint32_t fs = stop_fast_slot(key, ns);
        while (ss.fast_keys[fs] != 0) fs = (fs + 1) & (ns - 1);
        ss.fast_keys[fs] = key;
      }
    }
  }
  return plan.n_stop_sets++;
}

DevStage build_stage(const std::vector<StepCfg>& steps, const std::vector<int>& idx, DevPlan& plan) {
  DevStage st;
  std::memset(&st, 0, sizeof(st));
  if (idx.size() > (size_t)kMaxStageSteps) throw std::runtime_error("too many steps in one device stage");
  int prefix = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    const StepCfg& c = steps[idx[i]];
    DevStep& d = st.steps[i];
    d.kind = dev_kind_of(c);
    if (d.kind == DK_NONE) throw std::runtime_error("step " + c.name + " has no device stage form");
    d.width = record_width(c);
    d.rec_prefix = prefix;
    prefix += d.width;
    if (c.kind == StepKind::GopherQuality) d.stop_set = add_stop_set(plan, c.stop_words);
    if (c.kind == StepKind::GopherRepetition) {
      d.n_top = (int32_t)c.top_n_grams.size();
      d.n_dup = (int32_t)c.dup_n_grams.size();
      for (int k = 0; k < d.n_top; ++k) d.top_n[k] = (int32_t)c.top_n_grams[k].first;
      for (int k = 0; k < d.n_dup; ++k) d.dup_n[k] = (int32_t)c.dup_n_grams[k].first;
    }
    if (c.kind == StepKind::FineWebQuality) {
      d.n_stop_chars = (int32_t)c.stop_chars.size();
      for (int k = 0; k < d.n_stop_chars; ++k) d.stop_chars[k] = c.stop_chars[k];
      d.short_line_length = c.short_line_length;
    }
  }
  st.n_steps = (int32_t)idx.size();
  st.width_total = prefix;
  return st;
}

DevC4 build_c4(const StepCfg& c) {
  DevC4 d;
  std::memset(&d, 0, sizeof(d));
  d.split_paragraph = c.split_paragraph;
  d.remove_citations = c.remove_citations;
  d.filter_no_terminal_punct = c.filter_no_terminal_punct;
  d.filter_lorem_ipsum = c.filter_lorem_ipsum;
  d.filter_javascript = c.filter_javascript;
  d.filter_curly_bracket = c.filter_curly_bracket;
  d.filter_policy = c.filter_policy;
  d.min_words_per_line = c.min_words_per_line;
  d.max_word_length = c.max_word_length;
  d.min_num_sentences = c.min_num_sentences > 0 ? c.min_num_sentences : 0;
  return d;
}

DevGateStep build_gate_step(const StepCfg& c, int slot, int prefix) {
  DevGateStep g;
  std::memset(&g, 0, sizeof(g));
  g.slot = slot;
  g.prefix = prefix;
  g.width = record_width(c);
  auto opt_d = [&](const std::optional<double>& v, int bit, int k) {
    if (v) { g.has |= 1u << bit; g.d[k] = *v; }
  };
  auto opt_i = [&](const std::optional<int64_t>& v, int bit, int k) {
    if (v) { g.has |= 1u << bit; g.i[k] = *v; }
  };
  switch (c.kind) {
    case StepKind::GopherQuality:
      g.kind = GK_GOPHER_QUALITY;
      opt_i(c.min_doc_words, GQ_T_MIN_WORDS, 0);
      opt_i(c.max_doc_words, GQ_T_MAX_WORDS, 1);
      opt_d(c.min_avg_word_length, GQ_T_MIN_AVG, 0);
      opt_d(c.max_avg_word_length, GQ_T_MAX_AVG, 1);
      opt_d(c.max_symbol_word_ratio, GQ_T_SYMBOL, 2);
      opt_d(c.max_bullet_lines_ratio, GQ_T_BULLET, 3);
      opt_d(c.max_ellipsis_lines_ratio, GQ_T_ELL_LINES, 4);
      opt_d(c.max_non_alpha_words_ratio, GQ_T_ALPHA, 5);
      opt_i(c.min_stop_words, GQ_T_MIN_STOP, 2);
      break;
    case StepKind::GopherRepetition:
      if (c.top_n_grams.size() > (size_t)kMaxGateNgrams || c.dup_n_grams.size() > (size_t)kMaxGateNgrams)
        return DevGateStep{};  // GK_NONE: never gates
      g.kind = GK_GOPHER_REP;
      opt_d(c.dup_para_frac, GR_T_PARA, 0);
      opt_d(c.dup_para_char_frac, GR_T_PARA_CHAR, 1);
      opt_d(c.dup_line_frac, GR_T_LINE, 2);
      opt_d(c.dup_line_char_frac, GR_T_LINE_CHAR, 3);
      g.n_top = (int32_t)c.top_n_grams.size();
      g.n_dup = (int32_t)c.dup_n_grams.size();
      for (int k = 0; k < g.n_top; ++k) { g.top_n[k] = c.top_n_grams[k].first; g.top_thr[k] = c.top_n_grams[k].second; }
      for (int k = 0; k < g.n_dup; ++k) { g.dup_n[k] = c.dup_n_grams[k].first; g.dup_thr[k] = c.dup_n_grams[k].second; }
      break;
    case StepKind::FineWebQuality:
      g.kind = GK_FINEWEB;
      g.d[0] = c.line_punct_thr;
      g.d[1] = c.short_line_thr;
      g.d[2] = c.char_duplicates_ratio;
      g.d[3] = c.new_line_ratio;
      g.flag = c.line_punct_exclude_zero ? 1 : 0;
      break;
    case StepKind::LanguageDetection:
      g.kind = GK_LANGID;
      for (int l : c.allowed_langs)
        if (l >= 0 && l < 32) g.has |= 1u << l;
      g.d[0] = c.min_confidence;
      break;
    case StepKind::C4Quality:
      g.kind = GK_C4;
      g.i[0] = c.min_num_sentences;
      break;
    default:
      g.kind = GK_NONE;  // host-only steps are never evaluated on the device
      break;
  }
  return g;
}

DevGate build_gate(const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries) {
  DevGate gate;
  std::memset(&gate, 0, sizeof(gate));
  if (entries.size() > (size_t)kMaxGateSteps) throw std::runtime_error("too many steps in one device gate");
  for (size_t k = 0; k < entries.size(); ++k) {
    const auto& e = entries[k];
    if (e[0] < 0 || e[0] >= (int)steps.size() || e[1] < 0 || e[1] >= kMaxGateSteps)
      throw std::runtime_error("device gate entry out of range");
    gate.steps[k] = build_gate_step(steps[e[0]], e[1], e[2]);
  }
  gate.n_steps = (int32_t)entries.size();
  return gate;
}

void gate_host(const DevGate& g, const std::vector<const int64_t*>& recs, int64_t ndocs, const uint32_t* flags,
               uint8_t* dead, uint8_t code) {
  for (int s = 0; s < g.n_steps; ++s)
    if (g.steps[s].kind != GK_NONE && (g.steps[s].slot < 0 || g.steps[s].slot >= (int)recs.size()))
      throw std::runtime_error("gate record slot out of range");
  for (int64_t doc = 0; doc < ndocs; ++doc) {  // same loop body as k_gate
    if (dead[doc]) continue;
    bool fail = flags && flags[doc] != 0;
    for (int s = 0; s < g.n_steps && !fail; ++s) {
      const DevGateStep& st = g.steps[s];
      if (st.kind == GK_NONE) continue;
      fail = gate_fails(st, recs[st.slot] + (int64_t)st.prefix * ndocs + doc * st.width);
    }
    if (fail) dead[doc] = code;
  }
}

DevResolve build_resolve(const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries,
                         const std::vector<int>& c4_version) {
  if (entries.size() != c4_version.size()) throw std::invalid_argument("resolve: entries / versions length");
  // every step needs an entry, except trailing TokenCounter steps (they never filter; their
  // counts are added after the resolve) and C4BadWords steps (resolved as passing: the host
  // draws their keep fractions and moves the documents they filter, Engine._device_resolve_agrees)
  size_t n_need = steps.size();
  while (n_need > 0 && steps[n_need - 1].kind == StepKind::TokenCounter) --n_need;
  size_t n_bw = 0;
  for (size_t s = 0; s < n_need; ++s) n_bw += steps[s].kind == StepKind::C4BadWords;
  if (entries.size() + n_bw < n_need || entries.size() > steps.size())
    throw std::invalid_argument("resolve: every pipeline step needs an entry");
  for (size_t k = 0; k < entries.size(); ++k)
    if (entries[k][0] >= 0 && entries[k][0] < (int)steps.size() && steps[entries[k][0]].kind == StepKind::C4BadWords)
      throw std::invalid_argument("resolve: C4BadWords has no device decision");
  for (size_t k = 0; k < entries.size(); ++k)
    if (entries[k][0] < 0 || entries[k][0] >= (int)n_need)
      throw std::invalid_argument("resolve: every pipeline step needs an entry");
  DevResolve rp;
  std::memset(&rp, 0, sizeof(rp));
  rp.gate = build_gate(steps, entries);  // range checks, <= kMaxGateSteps
  for (size_t k = 0; k < entries.size(); ++k) {
    if (rp.gate.steps[k].kind == GK_NONE)
      throw std::invalid_argument("resolve: step " + std::to_string(entries[k][0]) + " has no device decision");
    if (k > 0 && entries[k][0] <= entries[k - 1][0]) throw std::invalid_argument("resolve: steps out of order");
    if (c4_version[k] >= kMaxVersions || (c4_version[k] >= 0 && rp.gate.steps[k].kind != GK_C4))
      throw std::invalid_argument("resolve: content version out of range");
    rp.step_index[k] = entries[k][0];
    rp.c4_version[k] = c4_version[k];
  }
  return rp;
}

void resolve_host(const DevResolve& rp, const std::vector<const int64_t*>& recs, int64_t ndocs,
                  const uint32_t* flags, const std::vector<const char*>& vdata,
                  const std::vector<const int64_t*>& voff, std::vector<int32_t>& fail, std::vector<uint8_t>& status,
                  std::string& out, std::vector<int64_t>& out_off, std::vector<int32_t>& rows) {
  for (int s = 0; s < rp.gate.n_steps; ++s) {
    if (rp.gate.steps[s].slot < 0 || rp.gate.steps[s].slot >= (int)recs.size())
      throw std::runtime_error("resolve record slot out of range");
    if (rp.c4_version[s] >= (int)voff.size()) throw std::runtime_error("resolve version out of range");
  }
  fail.assign(ndocs, -1);
  status.assign(ndocs, 0);
  std::vector<int32_t> ver(ndocs, 0);
  for (int64_t doc = 0; doc < ndocs; ++doc)  // k_resolve
    resolve_doc(rp, recs.data(), ndocs, doc, flags ? flags[doc] : 0u, fail[doc], status[doc], ver[doc]);
  out.clear();
  out_off.assign(ndocs + 1, 0);
  rows.assign(ndocs, 0);
  int64_t pos = 0;
  for (uint8_t want : {kResolveKept, kResolveFiltered})  // k_compact: kept, then excluded, doc order
    for (int64_t doc = 0; doc < ndocs; ++doc) {
      if (status[doc] != want) continue;
      const int v = ver[doc];
      out_off[pos] = (int64_t)out.size();
      rows[pos++] = (int32_t)doc;
      out.append(vdata[v] + voff[v][doc], (size_t)(voff[v][doc + 1] - voff[v][doc]));
    }
  out_off[pos] = (int64_t)out.size();
}

std::vector<uint64_t> pow_table(uint32_t n) {
  // [0, n]: B^i, then [n + 1, 2n + 1]: B^-i (the layout tb_pow_table writes on the device)
  std::vector<uint64_t> pw(2 * (size_t)n + 2);
  pw[0] = 1;
  pw[n + 1] = 1;
  for (uint32_t i = 1; i <= n; ++i) {
    pw[i] = hmul(pw[i - 1], kHashBase);
    pw[n + 1 + i] = hmul(pw[n + i], kHashBaseInv);
  }
  return pw;
}

uint64_t scratch_bytes_for(uint32_t doc_len, bool split) { return scratch_bytes_for_dev(doc_len, split); }

// Largest per-byte arena need the emulators have seen: max over documents of
// (peak - 4096) / (len + 64), kept in milli-bytes so one atomic max covers it.
static std::atomic<uint64_t> g_scratch_need_milli{0};
static std::atomic<uint64_t> g_scratch_need_len{0};
static void note_scratch(uint64_t peak, uint32_t n) {
  const uint64_t over = peak > 4096 ? peak - 4096 : 0;
  const uint64_t m = over * 1000 / ((uint64_t)n + 64);
  uint64_t cur = g_scratch_need_milli.load(std::memory_order_relaxed);
  while (m > cur && !g_scratch_need_milli.compare_exchange_weak(cur, m)) {}
  if (m >= cur) g_scratch_need_len.store(n, std::memory_order_relaxed);
}
// probe mode: the emulators give every document 1 KB of arena per byte, so no document
// overflows and the high-water marks are the true needs
static std::atomic<bool> g_scratch_probe{false};
void set_scratch_probe(bool on) { g_scratch_probe = on; }
static uint64_t emu_cap(uint32_t n, bool split) {
  return g_scratch_probe ? 1024 * ((uint64_t)n + 64) + 4096 : scratch_bytes_for(n, split);
}
std::pair<double, uint32_t> scratch_need(bool reset) {
  const std::pair<double, uint32_t> r{g_scratch_need_milli.load() / 1000.0, (uint32_t)g_scratch_need_len.load()};
  if (reset) { g_scratch_need_milli = 0; g_scratch_need_len = 0; }
  return r;
}

uint64_t line_stats_buffer_words(const int64_t* off, int64_t ndocs) { return line_stats_words(off, ndocs); }

void emulate_stage(const std::vector<StepCfg>& steps, const std::vector<int>& idx, int64_t ndocs,
                   const char* data, const int64_t* off, int nthreads, const LangidModel* lid,
                   std::vector<int64_t>& rec, std::vector<uint32_t>& flags, uint32_t lds_bytes, const uint8_t* dead,
                   bool weak_keys, uint32_t* line_stats, int split_tasks, DictIn dict) {
  DevPlan* plan = new DevPlan();
  std::memset(plan, 0, sizeof(DevPlan));
  DevStage st = build_stage(steps, idx, *plan);
  int gr_pos = -1;
  for (int s = 0; s < st.n_steps; ++s)
    if (st.steps[s].kind == DK_GOPHER_REP) gr_pos = s;
  bool has_lid = false;
  for (int s = 0; s < st.n_steps; ++s) has_lid |= st.steps[s].kind == DK_LANGID;
  if (has_lid && !lid) { delete plan; throw std::runtime_error("language model required"); }
  rec.assign((size_t)st.width_total * ndocs, 0);
  flags.assign(ndocs, 0);
  uint32_t maxlen = 0;
  for (int64_t i = 0; i < ndocs; ++i) maxlen = std::max<uint32_t>(maxlen, (uint32_t)(off[i + 1] - off[i]));
  std::vector<uint64_t> pw = pow_table(maxlen + 16);
  const UcdView ucd = host_ucd();
  parallel_for(ndocs, nthreads, [&](int64_t a, int64_t b) {
    std::vector<char> scratch;
    std::vector<char> lds(lds_bytes + 16);  // stands in for the wave's LDS slice
    for (int64_t i = a; i < b; ++i) {
      if (dead && dead[i]) continue;  // skipped by the device gate: record stays zero
      const uint32_t n = (uint32_t)(off[i + 1] - off[i]);
      const uint64_t need = emu_cap(n, split_tasks > 0 && gr_pos >= 0);
      if (scratch.size() < need) scratch.resize(need);
      DocCtx<SeqPar> x;
      x.ucd = ucd;
      x.pw = pw.data();
      x.pw_n = (uint32_t)(pw.size() / 2 - 1);
      x.ipw = pw.data() + x.pw_n + 1;
      x.scr = scratch.data();
      x.cap = need;
      x.lds = lds_bytes ? lds.data() : nullptr;
      x.lcap = lds_bytes;
      x.flag = &flags[i];
      x.weak_keys = weak_keys;
      StageOut out{rec.data(), (uint32_t)ndocs, (uint32_t)i};
      out.dict = dict;
      if (line_stats) out.line_stats = line_stats + line_stats_base(off[i], i);
      GrExport ex{};
      if (split_tasks > 0 && gr_pos >= 0) out.gr_export = &ex;
      analyze_stage(x, st, *plan, lid ? lid->tables() : LidTables{}, (const uint8_t*)data + off[i], n, out);
      if (x.overflow) continue;
      if (!out.gr_export || !ex.valid) {
        note_scratch(x.peak, n);
        continue;
      }
      // k_gr_dup_split, one task after another: task t works in slice t of the exported rest
      const DevStep& ds = st.steps[gr_pos];
      int64_t* r = rec.data() + (int64_t)ds.rec_prefix * ndocs + i * ds.width;
      const uint64_t region = (ex.free_cap / (uint64_t)split_tasks) & ~255ull;
      uint64_t task_peak = 0;
      bool over = false;
      for (int t = 0; t < split_tasks; ++t) {
        DocCtx<SeqPar> y;
        y.ucd = ucd;
        y.pw = pw.data();
        y.pw_n = x.pw_n;
        y.ipw = x.ipw;
        y.scr = ex.free_base + (uint64_t)t * region;
        y.cap = region;
        y.lds = lds_bytes ? lds.data() : nullptr;
        y.lcap = lds_bytes;
        y.flag = &flags[i];
        if (t < ds.n_dup) gr_dup_one_order(y, ds, t, ex, r);
        else if (t < ds.n_dup + ds.n_top) gr_top_one_order(y, ds, t - ds.n_dup, ex, r);
        else if (t < ds.n_dup + ds.n_top + 2) gr_lines_split(y, t - ds.n_dup - ds.n_top, ex, r);
        if (y.overflow) { y.set_flag(DOC_NEEDS_CPU | DOC_OVERFLOW); over = true; }
        task_peak = std::max<uint64_t>(task_peak, (y.peak + 255) & ~255ull);
      }
      // the slices are equal, so the document needs (export end) + tasks x (largest task)
      if (!over) note_scratch((uint64_t)(ex.free_base - scratch.data()) + (uint64_t)split_tasks * task_peak, n);
    }
  });
  delete plan;
}


void emulate_c4(const StepCfg& step, int64_t ndocs, const char* data, const int64_t* off, int nthreads,
                std::vector<int64_t>& rec, std::string& new_data, std::vector<int64_t>& new_off,
                std::vector<uint32_t>& flags, uint32_t lds_bytes, const uint8_t* dead, const uint32_t* line_stats,
                uint32_t* c4_words, DictLines dict_lines) {
  DevC4 c4 = build_c4(step);
  rec.assign((size_t)rec::C4_WIDTH * ndocs, 0);
  flags.assign(ndocs, 0);
  std::vector<std::string> outs(ndocs);
  uint32_t maxlen = 0;
  for (int64_t i = 0; i < ndocs; ++i) maxlen = std::max<uint32_t>(maxlen, (uint32_t)(off[i + 1] - off[i]));
  std::vector<uint64_t> pw = pow_table(maxlen + 16);
  const UcdView ucd = host_ucd();
  parallel_for(ndocs, nthreads, [&](int64_t a, int64_t b) {
    std::vector<char> scratch;
    std::vector<char> lds(lds_bytes + 16);  // stands in for the wave's LDS slice
    for (int64_t i = a; i < b; ++i) {
      if (dead && dead[i]) continue;  // skipped: record zeros, empty rewrite
      const uint32_t n = (uint32_t)(off[i + 1] - off[i]);
      const uint64_t need = emu_cap(n, false);
      if (scratch.size() < need) scratch.resize(need);
      DocCtx<SeqPar> x;
      x.ucd = ucd;
      x.pw = pw.data();
      x.pw_n = (uint32_t)(pw.size() / 2 - 1);
      x.ipw = pw.data() + x.pw_n + 1;
      x.scr = scratch.data();
      x.cap = need;
      x.lds = lds_bytes ? lds.data() : nullptr;
      x.lcap = lds_bytes;
      x.flag = &flags[i];
      int64_t src[2] = {-1, 0};
      const uint8_t* b = (const uint8_t*)data + off[i];
      c4_pass_a(x, c4, b, n, rec.data() + i * rec::C4_WIDTH, src,
                line_stats ? line_stats + line_stats_base(off[i], i) : nullptr, c4_words ? c4_words + i : nullptr,
                dict_lines.at((uint32_t)i));
      if (!x.overflow) note_scratch(x.peak, n);
      if (flags[i] & DOC_NEEDS_CPU) continue;
      if (src[0] < 0) outs[i].assign((const char*)b, n);
      else outs[i].assign(scratch.data() + src[0], (size_t)src[1]);
    }
  });
  new_off.assign(ndocs + 1, 0);
  size_t tot = 0;
  for (auto& s : outs) tot += s.size();
  new_data.clear();
  new_data.reserve(tot);
  for (int64_t i = 0; i < ndocs; ++i) {
    new_data += outs[i];
    new_off[i + 1] = (int64_t)new_data.size();
  }
}

}  // namespace tb
