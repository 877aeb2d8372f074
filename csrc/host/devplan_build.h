#pragma once
#include <array>
#include <string>
#include <vector>

#include "../common/devplan.h"
#include "../common/gate.h"
#include "filters.h"
#include "pipeline.h"

namespace tb {

// Per-document device scratch (devplan.h scratch_bytes_for_dev).
uint64_t scratch_bytes_for(uint32_t doc_len, bool split = false);
// Largest (peak - 4096) / (len + 64) arena bytes per text byte used by an emulated document
// since the last reset, and that document's length.
std::pair<double, uint32_t> scratch_need(bool reset);
void set_scratch_probe(bool on);  // emulators: unbounded arenas (measure needs, never overflow)

int dev_kind_of(const StepCfg& c);
bool device_supported(const StepCfg& c, std::string* why);
DevStage build_stage(const std::vector<StepCfg>& steps, const std::vector<int>& idx, DevPlan& plan);
DevC4 build_c4(const StepCfg& c);
// Gate (csrc/common/gate.h) over steps: entries = (step index, record slot, record prefix).
DevGateStep build_gate_step(const StepCfg& c, int slot, int prefix);
DevGate build_gate(const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries);
// K16 resolve plan over the whole pipeline: entries = (step index, record slot, record prefix) of
// every step in pipeline order, c4_version[k] = content version step k produces (-1: none).
// Throws std::invalid_argument when the pipeline cannot be resolved on the device (a host-only
// step, a step without a gate kind, too many steps or versions).
DevResolve build_resolve(const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries,
                         const std::vector<int>& c4_version);
// Host run of k_resolve + k_compact (same per-document function, same output layout).
void resolve_host(const DevResolve& rp, const std::vector<const int64_t*>& recs, int64_t ndocs,
                  const uint32_t* flags, const std::vector<const char*>& vdata,
                  const std::vector<const int64_t*>& voff, std::vector<int32_t>& fail, std::vector<uint8_t>& status,
                  std::string& out, std::vector<int64_t>& out_off, std::vector<int32_t>& rows);
std::vector<uint64_t> pow_table(uint32_t n);  // B^0..B^n followed by B^-0..B^-n

void emulate_stage(const std::vector<StepCfg>& steps, const std::vector<int>& idx, int64_t ndocs,
                   const char* data, const int64_t* off, int nthreads, const LangidModel* lid,
                   std::vector<int64_t>& rec, std::vector<uint32_t>& flags, uint32_t lds_bytes = 0,
                   const uint8_t* dead = nullptr, bool weak_keys = false, uint32_t* line_stats = nullptr,
                   int split_tasks = 0, DictIn dict = DictIn{});
// split_tasks > 0: every document runs the intra-document split of its GopherRepetition step
// (stage export, then the k_gr_dup_split tasks in turn, each in its slice of the arena rest)
uint64_t line_stats_buffer_words(const int64_t* off, int64_t ndocs);  // u32 size of a batch's line export
// line_stats: the C4 line export of the batch (docproc.h line_stats_base layout), written by
// emulate_stage and read by emulate_c4 of the same content version, as on the device
void emulate_c4(const StepCfg& step, int64_t ndocs, const char* data, const int64_t* off, int nthreads,
                std::vector<int64_t>& rec, std::string& new_data, std::vector<int64_t>& new_off,
                std::vector<uint32_t>& flags, uint32_t lds_bytes = 0, const uint8_t* dead = nullptr,
                const uint32_t* line_stats = nullptr, uint32_t* c4_words = nullptr, DictLines dict_lines = DictLines{});
// Host run of k_gate (same loop body): dead[doc] = code for live docs that a gated step filters.
void gate_host(const DevGate& g, const std::vector<const int64_t*>& recs, int64_t ndocs, const uint32_t* flags,
               uint8_t* dead, uint8_t code);

}  // namespace tb
