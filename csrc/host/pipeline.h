// Batch execution state shared by the CPU path and the GPU path.
//
// A batch holds the documents of one Parquet read batch as packed UTF-8 (data + int64 offsets).
// Steps are applied in pipeline order; per document the first failing step wins and later
// steps do not run (reference executor.rs:30-57). Metadata written by executed steps is kept in
// insertion order and merged over the input metadata when the outputs are assembled.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../common/langid.h"
#include "filters.h"
#include "json.h"

namespace tb {

// fn(begin, end) over [0, n) in chunks on the process-wide worker pool (nthreads incl. the caller).
void parallel_for(int64_t n, int nthreads, const std::function<void(int64_t, int64_t)>& fn);
// fn(task) for task in [0, ntasks) on the worker pool, at most nthreads at a time.
void parallel_tasks(int64_t ntasks, int nthreads, const std::function<void(int64_t)>& fn);

// CPU-time attribution of the pool: the jobs a thread submits while a PoolTag is alive are
// charged to its name (thread CPU time of the caller and of every worker inside the job);
// untagged jobs go to "other". Names must be string literals.
struct PoolTag {
  explicit PoolTag(const char* name);
  ~PoolTag();
  const char* prev;
};
// (name, CPU seconds) of every tag so far
std::vector<std::pair<std::string, double>> pool_cpu_stats();

struct LangidModel {
  int version = 3;         // int8 embeddings + MFMA head (csrc/common/langid.h)
  std::vector<float> b;    // [kLidRow]
  std::vector<int8_t> E;   // [kLidBuckets * kLidRowDim] embedding rows (block-sparse halves)
  std::vector<int16_t> W;  // [kLidDim * kLidLangs] integer head
  double w_scale = 0;
  // Detect the language of `text`: returns lang index or -1, confidence in *conf.
  int detect(std::string_view text, double* conf) const;
  // Exact sums of the text's n-gram rows (out[sum_width()]: embedding dims); returns the
  // n-gram count.
  int64_t sums(std::string_view text, int64_t* out) const;
  int sum_width() const { return kLidDim; }
  // The language record (r[0] language or -1, r[1] confidence bits) from sums() output.
  void record(const int64_t* s, int64_t cnt, int64_t* r) const;
  LidTables tables() const {
    LidTables t;
    t.bias = b.data();
    t.E = E.data();
    t.W = W.data();
    t.w_scale = w_scale;
    return t;
  }
};

// C4 bad-words matcher for one language (reference c4_filters.rs:298-551).
struct BadWordsLang {
  bool cjk = false;
  struct Node { std::unordered_map<uint32_t, int> next; bool term = false; };
  std::vector<Node> trie;
  bool match(std::string_view text) const;
};

// rand 0.8 `StdRng` (ChaCha12, key from `seed_from_u64` via PCG32) and `gen::<f32>()`, so a
// seeded C4BadWordsFilter draws the same keep/drop sequence as the reference
// (c4_filters.rs:303-309, :520).
struct StdRng {
  uint32_t key[8];
  uint64_t counter = 0;
  uint32_t buf[16];
  int pos = 16;
  explicit StdRng(uint64_t seed);
  uint32_t next_u32();
  float gen_f32() { return (float)(next_u32() >> 8) * (1.0f / 16777216.0f); }
};

// All loaded bad-words tries flattened for the device matcher (k_badwords_match): per node a
// sorted edge list (folded code point -> node) and a terminal flag; per language a root node.
struct BadWordsAutomaton {
  std::vector<int32_t> first_edge;  // [nodes + 1]
  std::vector<uint32_t> edge_cp;    // [edges], sorted per node
  std::vector<int32_t> edge_to;     // [edges]
  std::vector<uint8_t> term;        // [nodes]
  std::unordered_map<std::string, int32_t> root;
  std::unordered_map<std::string, bool> cjk;
};

struct BadWordsModule {
  std::string cache_dir;
  BadWordsAutomaton flatten() const;
  std::unique_ptr<StdRng> rng;  // shared by every document, drawn in document order
  std::unordered_map<std::string, std::shared_ptr<BadWordsLang>> langs;  // nullptr = no list
  std::shared_ptr<BadWordsLang> get(const std::string& lang, bool* supported);
};

struct Version {
  const char* data = nullptr;
  const int64_t* off = nullptr;
  std::string own_data;
  std::vector<int64_t> own_off;
};

// Output column buffer handed to Python without a copy. Large buffers come from a small
// recycling pool (released by the numpy owner), so steady-state batches reuse already-faulted
// pages instead of paying mmap + first-touch faults + munmap for ~100 MB per batch.
struct RawBuf {
  char* p = nullptr;
  size_t n = 0;
  size_t cap = 0;
  void alloc(size_t bytes);
  static void release(char* p, size_t cap);
};

// Per-batch resolver. Hot-path design (one batch = up to ~1e5 documents):
//   * applying a step only derives each alive document's status from its record
//     (decide_status: no strings), records stay where they were produced (device D2H buffers
//     or owned CPU-path arrays);
//   * reasons and metadata are formatted once, at output assembly, by re-running the shared
//     decision code over the records of the steps each document executed;
//   * no per-document heap objects survive a step, so building and dropping a batch is cheap.
class BatchState {
 public:
  BatchState(int64_t n, const char* data, const int64_t* off, const char* meta_data,
             const int64_t* meta_off, const uint8_t* meta_valid, int nthreads);

  int64_t size() const { return n_; }
  int nthreads() const { return nthreads_; }
  std::string_view content(int64_t i) const;
  int add_version(const char* data, const int64_t* off);  // borrowed buffers
  int add_owned_version(std::string&& data, std::vector<int64_t>&& off);

  // Apply a step whose per-document records were computed elsewhere (GPU, host tokenizer).
  // `rec` is borrowed and must outlive the batch. For C4 steps `rewrite_version` is the
  // version holding the rewritten contents.
  void apply_records(const StepCfg& cfg, int step_index, const int64_t* rec, int width,
                     int rewrite_version);
  // CPU path: compute records for alive docs and apply them for steps [begin, end).
  void run_cpu(const std::vector<StepCfg>& steps, int begin, int end, SegBackend be,
               const LangidModel* lid, BadWordsModule* bw);
  void apply_badwords(const StepCfg& cfg, int step_index, BadWordsModule& mod);
  // Device path of the bad-words step: languages per alive document (lists loaded), then the
  // decisions from externally computed matches (-1 n/a, 0, 1), drawing the keep-fraction RNG
  // in document order exactly like apply_badwords.
  std::vector<std::string> badwords_languages(const StepCfg& cfg, BadWordsModule& mod) const;
  // per alive document an index into names (names[0] = the step's default language), lists loaded
  void badwords_lang_codes(const StepCfg& cfg, BadWordsModule& mod, std::vector<int32_t>& code,
                           std::vector<std::string>& names) const;
  void apply_badwords_codes(const StepCfg& cfg, int step_index, BadWordsModule& mod, const int8_t* matched,
                            const std::vector<int32_t>& code, const std::vector<std::string>& names);
  void apply_badwords_matched(const StepCfg& cfg, int step_index, BadWordsModule& mod, const int8_t* matched,
                              const std::vector<std::string>& lang);
  // Current contents of documents idx, packed (for device steps that run after the resolve).
  void gather(const std::vector<int64_t>& idx, RawBuf& data, std::vector<int64_t>& off) const;

  // Remove documents from this batch (they are processed elsewhere, e.g. the CPU oracle path).
  void delegate(const int64_t* idx, int64_t n);
  std::vector<int64_t> alive_indices() const;
  const std::vector<int32_t>& fail_step() const { return fail_step_; }
  const std::vector<uint8_t>& status() const { return status_; }  // 0 ok, 1 filtered, 2 error, 3 delegated
  const std::vector<int32_t>& cur_version() const { return cur_version_; }
  std::string reason(int64_t i) const;

  // Output assembly for a subset of documents (indices): contents and metadata JSON.
  void assemble(const std::vector<int64_t>& idx, RawBuf& text_data, std::vector<int64_t>& text_off,
                RawBuf& meta_data, std::vector<int64_t>& meta_off, std::vector<uint8_t>& meta_valid,
                bool with_text = true) const;
  int64_t meta_parse_failures() const { return meta_fail_.load(); }

 private:
  struct StepRec {
    std::unique_ptr<StepCfg> cfg;  // own copy: callers may pass temporaries
    const int64_t* rec = nullptr;
    int width = 0;
    std::vector<int64_t> own;
  };
  // C4BadWordsFilter outcome per document (decided with the shared RNG stream in doc order).
  struct BwOut {
    std::vector<int8_t> code;           // BwStatus or -1 (not executed)
    std::vector<std::string> lang;      // only for BW_MISSING_LANG_FAIL reasons
  };
  StepRec& step_slot(int step_index);
  void set_status(int64_t doc, int step_index, uint8_t st);
  bool input_meta(int64_t i, FlatMeta& out) const;
  void step_meta(int64_t doc, int s, Decision& d) const;  // metadata of step s for doc
  void step_meta_json(int64_t doc, int s, CharBuf& out, bool& first) const;  // same, as JSON members
  int step_kind(int s) const;  // StepKind of applied step s, -1 if none

  int64_t n_;
  int nthreads_;
  int n_applied_ = 0;  // steps [0, n_applied_) have been applied (in order)
  std::vector<Version> versions_;
  std::vector<int32_t> cur_version_;
  std::vector<int32_t> fail_step_;
  std::vector<uint8_t> status_;
  const char* meta_data_ = nullptr;
  const int64_t* meta_off_ = nullptr;
  const uint8_t* meta_valid_ = nullptr;
  std::vector<StepRec> recs_;                 // by step index
  std::vector<std::unique_ptr<BwOut>> bw_;    // by step index (nullptr unless bad-words step)
  std::vector<std::string> own_content_;      // CPU path rewritten contents (cur_version == -1)
  mutable std::atomic<int64_t> meta_fail_{0};
};

}  // namespace tb
