#include <unordered_map>
#include "pipeline.h"

#include <unicode/uchar.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <ctime>
#include <fstream>
#include <condition_variable>
#include <mutex>
#include <pthread.h>
#include <random>
#include <sstream>

#include "../common/langid.h"

namespace tb {

// Persistent worker pool shared by every parallel_for of the process (resolve, assembly,
// staging copies, emulation, HTML decoding). Several Python threads submit jobs concurrently;
// each job is a chunk counter that its caller and up to nthreads-1 pool workers drain. The
// caller always works on its own job, so a job completes even when every worker is busy
// elsewhere. Workers live for the whole process (no per-call thread creation).
namespace {
thread_local const char* tl_pool_tag = nullptr;

struct TagStats {
  std::mutex mu;
  std::vector<std::pair<const char*, std::atomic<uint64_t>*>> ns;  // tag -> CPU nanoseconds
  std::atomic<uint64_t>* slot(const char* tag) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : ns)
      if (e.first == tag) return e.second;
    ns.emplace_back(tag, new std::atomic<uint64_t>(0));
    return ns.back().second;
  }
};
TagStats& tag_stats() {
  static TagStats* t = new TagStats();  // leaked on purpose: pool workers outlive statics
  return *t;
}
uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

struct PoolJob {
  const std::function<void(int64_t)>* fn;
  int64_t nchunks;
  int max_helpers;
  std::atomic<uint64_t>* cpu = nullptr;  // the submitter's tag counter
  std::atomic<int64_t> next{0};
  std::atomic<int64_t> done{0};
  int helpers = 0;   // workers that took the job (guarded by the pool mutex)
  int active = 0;    // workers still inside work() (guarded by the pool mutex)
  void work() {
    const uint64_t t0 = thread_cpu_ns();
    int64_t c;
    while ((c = next.fetch_add(1, std::memory_order_relaxed)) < nchunks) {
      (*fn)(c);
      done.fetch_add(1, std::memory_order_release);
    }
    cpu->fetch_add(thread_cpu_ns() - t0, std::memory_order_relaxed);
  }
};

class WorkerPool {
 public:
  static WorkerPool& get() {
    static WorkerPool* p = new WorkerPool();  // leaked on purpose: workers outlive statics
    return *p;
  }
  void run(int64_t nchunks, int nthreads, const std::function<void(int64_t)>& fn) {
    PoolJob job;
    job.fn = &fn;
    job.nchunks = nchunks;
    job.cpu = tag_stats().slot(tl_pool_tag ? tl_pool_tag : "other");
    job.max_helpers = std::max(0, nthreads - 1);
    {
      std::unique_lock<std::mutex> g(mu_);
      while ((int)workers_.size() < job.max_helpers)
        workers_.emplace_back([this] {
          pthread_setname_np(pthread_self(), "tb-pool");  // attributable in per-thread CPU profiles
          loop();
        });
      jobs_.push_back(&job);
    }
    cv_.notify_all();
    job.work();
    std::unique_lock<std::mutex> g(mu_);
    for (size_t i = 0; i < jobs_.size(); ++i)
      if (jobs_[i] == &job) { jobs_.erase(jobs_.begin() + (long)i); break; }
    // chunks taken by workers may still be running; the job lives on this stack frame
    done_cv_.wait(g, [&] { return job.active == 0 && job.done.load(std::memory_order_acquire) == nchunks; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(mu_);
    while (true) {
      PoolJob* j = nullptr;
      cv_.wait(g, [&] {
        for (PoolJob* c : jobs_)
          if (c->helpers < c->max_helpers && c->next.load(std::memory_order_relaxed) < c->nchunks) { j = c; return true; }
        return false;
      });
      ++j->helpers;
      ++j->active;
      g.unlock();
      j->work();
      g.lock();
      --j->active;
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<PoolJob*> jobs_;
  std::vector<std::thread> workers_;
};
}  // namespace

PoolTag::PoolTag(const char* name) : prev(tl_pool_tag) { tl_pool_tag = name; }
PoolTag::~PoolTag() { tl_pool_tag = prev; }

std::vector<std::pair<std::string, double>> pool_cpu_stats() {
  TagStats& t = tag_stats();
  std::lock_guard<std::mutex> g(t.mu);
  std::vector<std::pair<std::string, double>> out;
  for (auto& e : t.ns) out.emplace_back(e.first, 1e-9 * (double)e.second->load(std::memory_order_relaxed));
  return out;
}

void parallel_tasks(int64_t ntasks, int nthreads, const std::function<void(int64_t)>& fn) {
  if (ntasks <= 0) return;
  if (nthreads <= 1 || ntasks == 1) {
    // on the caller alone: charged to its tag too
    const uint64_t t0 = thread_cpu_ns();
    for (int64_t c = 0; c < ntasks; ++c) fn(c);
    tag_stats().slot(tl_pool_tag ? tl_pool_tag : "other")->fetch_add(thread_cpu_ns() - t0, std::memory_order_relaxed);
    return;
  }
  WorkerPool::get().run(ntasks, (int)std::min<int64_t>(nthreads, ntasks), fn);
}

void parallel_for(int64_t n, int nthreads, const std::function<void(int64_t, int64_t)>& fn) {
  if (n <= 0) return;
  if (nthreads <= 1 || n < 256) {
    parallel_tasks(1, 1, [&](int64_t) { fn(0, n); });
    return;
  }
  const int64_t chunks = std::min<int64_t>((int64_t)nthreads * 8, (n + 63) / 64);
  parallel_tasks(chunks, nthreads, [&](int64_t c) { fn(n * c / chunks, n * (c + 1) / chunks); });
}

// ------------------------------------------------------------------------------------------
// Language identification (CPU inference with the same arithmetic as the device path).
int64_t LangidModel::sums(std::string_view text, int64_t* out) const {
  const uint8_t* b8 = (const uint8_t*)text.data();
  const uint32_t n = (uint32_t)text.size();
  const UcdView& u = host_ucd();
  const int D = sum_width();
  int32_t part[kLidDim] = {0};
  for (int l = 0; l < D; ++l) out[l] = 0;
  int64_t cnt = 0;
  uint32_t lm3 = 0, lm2 = 0, lm1 = 0;
  int ncp = 0;
  auto emit = [&](uint32_t g, int order) {
    lid_add_emb(E.data(), g, order, part);
    for (int l = 0; l < D; ++l) { out[l] += part[l]; part[l] = 0; }
  };
  uint32_t i = 0;
  for (; i < n && ncp < kLidMaxCps; ++ncp) {
    const uint32_t l0 = lid_letter(u, b8, n, i);
    int len;
    (void)utf8_decode(b8, i, n, &len);
    i += len;
    cnt += lid_grams_n(lm3, lm2, lm1, l0, emit);
    lm3 = lm2;
    lm2 = lm1;
    lm1 = l0;
  }
  // virtual non-letter at the cut / end of text
  cnt += lid_grams_n(lm3, lm2, lm1, 0, emit);
  return cnt;
}

void LangidModel::record(const int64_t* s, int64_t cnt, int64_t* r) const {
  lid_record_v3(s, cnt, tables(), r);
}

int LangidModel::detect(std::string_view text, double* conf) const {
  int64_t s[kLidDim];
  const int64_t cnt = sums(text, s);
  int64_t r[2];
  record(s, cnt, r);
  std::memcpy(conf, &r[1], sizeof(double));
  return (int)r[0];
}

// ------------------------------------------------------------------------------------------
// C4 bad words.
static const char* const kBadwordsLangs[] = {
    "ar", "cs", "da", "de", "en", "eo", "es", "fa", "fi", "fil", "fr", "fr-CA-u-sd-caqc", "hi", "hu",
    "it", "ja", "kab", "ko", "nl", "no", "pl", "pt", "ru", "sv", "th", "tlh", "tr", "zh"};

static std::vector<uint32_t> fold_cps(std::string_view s) {
  std::vector<uint32_t> out;
  const uint8_t* b = (const uint8_t*)s.data();
  uint32_t n = (uint32_t)s.size();
  for (uint32_t i = 0; i < n;) {
    int len;
    uint32_t c = utf8_decode(b, i, n, &len);
    out.push_back((uint32_t)u_foldCase((UChar32)c, U_FOLD_CASE_DEFAULT));
    i += len;
  }
  return out;
}

bool BadWordsLang::match(std::string_view text) const {
  CpView v;
  v.build(text);
  std::vector<uint32_t> f(v.n());
  for (int i = 0; i < v.n(); ++i) f[i] = (uint32_t)u_foldCase((UChar32)v.cp[i], U_FOLD_CASE_DEFAULT);
  auto is_w = [&](int i) { return (v.prop[i] & P_WORDCHAR) != 0; };
  for (int i = 0; i < v.n(); ++i) {
    if (!cjk && i > 0 && is_w(i - 1)) continue;  // (?:\W|^)
    int node = 0;
    for (int j = i; j < v.n(); ++j) {
      auto it = trie[node].next.find(f[j]);
      if (it == trie[node].next.end()) break;
      node = it->second;
      if (trie[node].term && (cjk || j + 1 == v.n() || !is_w(j + 1))) return true;  // (?:\W|$)
    }
  }
  return false;
}

std::shared_ptr<BadWordsLang> BadWordsModule::get(const std::string& lang, bool* supported) {
  bool sup = false;
  for (auto l : kBadwordsLangs) if (lang == l) sup = true;
  *supported = sup;
  if (!sup) return nullptr;
  auto it = langs.find(lang);
  if (it != langs.end()) return it->second;
  std::string path = cache_dir + "/" + lang;
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("badwords list for '" + lang + "' not found in cache dir '" +
                                   cache_dir + "' (no network: place the LDNOOBW list at " + path + ")");
  std::stringstream ss;
  ss << f.rdbuf();
  std::string content = ss.str();
  auto bl = std::make_shared<BadWordsLang>();
  bl->cjk = (lang == "ja" || lang == "th" || lang == "zh");
  bl->trie.emplace_back();
  int nwords = 0;
  std::string_view cv(content);
  size_t p = 0;
  while (p <= cv.size()) {
    size_t q = cv.find('\n', p);
    if (q == std::string_view::npos) q = cv.size();
    std::string_view line = trim(cv.substr(p, q - p));
    if (!line.empty()) {
      auto cps = fold_cps(line);
      int node = 0;
      for (uint32_t c : cps) {
        auto it = bl->trie[node].next.find(c);
        if (it == bl->trie[node].next.end()) {
          bl->trie.emplace_back();
          int nn = (int)bl->trie.size() - 1;
          bl->trie[node].next[c] = nn;
          node = nn;
        } else {
          node = it->second;
        }
      }
      bl->trie[node].term = true;
      ++nwords;
    }
    p = q + 1;
  }
  std::shared_ptr<BadWordsLang> res = nwords ? bl : nullptr;
  langs[lang] = res;
  return res;
}

BadWordsAutomaton BadWordsModule::flatten() const {
  BadWordsAutomaton a;
  a.first_edge.push_back(0);
  std::vector<std::string> names;
  for (auto& kv : langs) names.push_back(kv.first);
  std::sort(names.begin(), names.end());
  for (const auto& name : names) {
    const auto& bl = langs.at(name);
    if (!bl) continue;
    const int32_t base = (int32_t)a.term.size();
    a.root[name] = base;
    a.cjk[name] = bl->cjk;
    for (const auto& node : bl->trie) {
      std::vector<std::pair<uint32_t, int>> edges(node.next.begin(), node.next.end());
      std::sort(edges.begin(), edges.end());
      for (auto& e : edges) {
        a.edge_cp.push_back(e.first);
        a.edge_to.push_back(base + e.second);
      }
      a.first_edge.push_back((int32_t)a.edge_cp.size());
      a.term.push_back(node.term ? 1 : 0);
    }
  }
  return a;
}

void BatchState::gather(const std::vector<int64_t>& idx, RawBuf& data, std::vector<int64_t>& off) const {
  PoolTag pool_tag("gather");
  const int64_t m = (int64_t)idx.size();
  off.assign(m + 1, 0);
  for (int64_t k = 0; k < m; ++k) off[k + 1] = off[k] + (int64_t)content(idx[k]).size();
  data.alloc((size_t)off[m]);
  parallel_for(m, nthreads_, [&](int64_t a, int64_t b) {
    for (int64_t k = a; k < b; ++k) {
      std::string_view t = content(idx[k]);
      if (!t.empty()) std::memcpy(data.p + off[k], t.data(), t.size());
    }
  });
}

StdRng::StdRng(uint64_t state) {
  for (int i = 0; i < 8; ++i) {  // rand_core SeedableRng::seed_from_u64
    state = state * 6364136223846793005ull + 11634580027462260723ull;
    const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
    const uint32_t rot = (uint32_t)(state >> 59);
    key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
  }
}

static inline uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

uint32_t StdRng::next_u32() {
  if (pos >= 16) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                       key[4], key[5], key[6], key[7], (uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u};
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = st[i];
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 6; ++r) {  // 12 rounds
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) buf[i] = x[i] + st[i];
    ++counter;
    pos = 0;
  }
  return buf[pos++];
}

// ------------------------------------------------------------------------------------------
namespace {
struct BufPool {
  std::mutex mu;
  std::vector<std::pair<char*, size_t>> free;  // (ptr, capacity)
  static constexpr size_t kMin = 1 << 20;
  static constexpr size_t kMaxFree = 8;
};
BufPool& buf_pool() {
  static BufPool* p = new BufPool();  // leaked on purpose: numpy owners may outlive statics
  return *p;
}
}  // namespace

void RawBuf::alloc(size_t bytes) {
  n = bytes;
  if (bytes >= BufPool::kMin) {
    BufPool& bp = buf_pool();
    std::lock_guard<std::mutex> g(bp.mu);
    int best = -1;
    for (int i = 0; i < (int)bp.free.size(); ++i)
      if (bp.free[i].second >= bytes && (best < 0 || bp.free[i].second < bp.free[best].second)) best = i;
    if (best >= 0) {
      p = bp.free[best].first;
      cap = bp.free[best].second;
      bp.free.erase(bp.free.begin() + best);
      return;
    }
  }
  cap = bytes < BufPool::kMin ? std::max<size_t>(bytes, 1) : bytes + bytes / 8;  // headroom for reuse
  p = new char[cap];
}

void RawBuf::release(char* p, size_t cap) {
  if (!p) return;
  if (cap >= BufPool::kMin) {
    BufPool& bp = buf_pool();
    std::lock_guard<std::mutex> g(bp.mu);
    if (bp.free.size() < BufPool::kMaxFree) {
      bp.free.emplace_back(p, cap);
      return;
    }
    // pool full: drop the smallest buffer (keep large ones: they serve every batch size)
    int small = 0;
    for (int i = 1; i < (int)bp.free.size(); ++i)
      if (bp.free[i].second < bp.free[small].second) small = i;
    if (bp.free[small].second < cap) std::swap(bp.free[small].first, p), std::swap(bp.free[small].second, cap);
  }
  delete[] p;
}

BatchState::BatchState(int64_t n, const char* data, const int64_t* off, const char* meta_data,
                       const int64_t* meta_off, const uint8_t* meta_valid, int nthreads)
    : n_(n), nthreads_(std::max(1, nthreads)) {
  versions_.emplace_back();
  versions_[0].data = data;
  versions_[0].off = off;
  cur_version_.assign(n, 0);
  fail_step_.assign(n, -1);
  status_.assign(n, 0);
  if (meta_data && meta_off) {
    meta_data_ = meta_data;
    meta_off_ = meta_off;
    meta_valid_ = meta_valid;
  }
}

std::string_view BatchState::content(int64_t i) const {
  int v = cur_version_[i];
  if (v < 0) return own_content_[i];
  const Version& ver = versions_[v];
  return std::string_view(ver.data + ver.off[i], (size_t)(ver.off[i + 1] - ver.off[i]));
}

int BatchState::add_version(const char* data, const int64_t* off) {
  versions_.emplace_back();
  versions_.back().data = data;
  versions_.back().off = off;
  return (int)versions_.size() - 1;
}

int BatchState::add_owned_version(std::string&& data, std::vector<int64_t>&& off) {
  versions_.emplace_back();
  Version& v = versions_.back();
  v.own_data = std::move(data);
  v.own_off = std::move(off);
  v.data = v.own_data.data();
  v.off = v.own_off.data();
  return (int)versions_.size() - 1;
}

BatchState::StepRec& BatchState::step_slot(int step_index) {
  if ((int)recs_.size() <= step_index) recs_.resize(step_index + 1);
  if ((int)bw_.size() <= step_index) bw_.resize(step_index + 1);
  n_applied_ = std::max(n_applied_, step_index + 1);
  return recs_[step_index];
}

void BatchState::set_status(int64_t doc, int step_index, uint8_t st) {
  if (st) {
    fail_step_[doc] = step_index;
    status_[doc] = st;
  }
}

bool BatchState::input_meta(int64_t i, FlatMeta& out) const {
  out.clear();
  if (!meta_data_ || (meta_valid_ && !meta_valid_[i])) return false;
  std::string_view js(meta_data_ + meta_off_[i], (size_t)(meta_off_[i + 1] - meta_off_[i]));
  return parse_meta_json(js, out);
}

void BatchState::apply_records(const StepCfg& cfg, int step_index, const int64_t* rec, int width,
                               int rewrite_version) {
  PoolTag pool_tag("apply_records");
  StepRec& sr = step_slot(step_index);
  sr.cfg = std::make_unique<StepCfg>(cfg);
  sr.rec = rec;
  sr.width = width;
  const bool c4_rewrite = cfg.kind == StepKind::C4Quality && rewrite_version >= 0;
  parallel_for(n_, nthreads_, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      if (fail_step_[i] >= 0) continue;
      const int64_t* r = rec + i * width;
      if (c4_rewrite && !r[rec::C4_LOREM] && !r[rec::C4_CURLY]) cur_version_[i] = rewrite_version;
      set_status(i, step_index, decide_status(cfg, r));
    }
  });
}

void BatchState::badwords_lang_codes(const StepCfg& cfg, BadWordsModule& mod, std::vector<int32_t>& code,
                                     std::vector<std::string>& names) const {
  PoolTag pool_tag("badwords");
  // The document language: metadata "language" (no step writes that key, so only the input
  // metadata can hold it), else the configured default (reference c4_filters.rs:464-468); as an
  // index into `names` (names[0] = the default), -1 for documents already filtered.
  code.assign((size_t)n_, -1);
  names.assign(1, cfg.default_language);
  std::vector<std::string> val;
  std::vector<uint8_t> has;
  if (meta_data_) {
    val.resize((size_t)n_);
    has.assign((size_t)n_, 0);
    parallel_for(n_, nthreads_, [&](int64_t a, int64_t b) {
      FlatMeta fm;
      for (int64_t i = a; i < b; ++i)
        if (fail_step_[i] < 0 && input_meta(i, fm) && fm.has("language")) {
          val[(size_t)i] = std::string(fm.get("language"));
          has[(size_t)i] = 1;
        }
    });
  }
  std::unordered_map<std::string, int32_t> idx;
  idx.emplace(cfg.default_language, 0);
  std::vector<uint8_t> used(1, 0);
  for (int64_t i = 0; i < n_; ++i) {
    if (fail_step_[i] >= 0) continue;
    int32_t c = 0;
    if (!has.empty() && has[(size_t)i]) {
      auto it = idx.find(val[(size_t)i]);
      if (it == idx.end()) {
        it = idx.emplace(val[(size_t)i], (int32_t)names.size()).first;
        names.push_back(val[(size_t)i]);
        used.push_back(0);
      }
      c = it->second;
    }
    code[(size_t)i] = c;
    used[(size_t)c] = 1;
  }
  // word lists load lazily, on this thread, once per language some document uses
  for (size_t k = 0; k < names.size(); ++k) {
    if (!used[k]) continue;
    bool sup;
    mod.get(names[k], &sup);
  }
}

std::vector<std::string> BatchState::badwords_languages(const StepCfg& cfg, BadWordsModule& mod) const {
  std::vector<int32_t> code;
  std::vector<std::string> names;
  badwords_lang_codes(cfg, mod, code, names);
  std::vector<std::string> lang((size_t)n_);
  for (int64_t i = 0; i < n_; ++i) if (code[(size_t)i] >= 0) lang[(size_t)i] = names[(size_t)code[(size_t)i]];
  return lang;
}

void BatchState::apply_badwords(const StepCfg& cfg, int step_index, BadWordsModule& mod) {
  std::vector<int32_t> code;
  std::vector<std::string> names;
  badwords_lang_codes(cfg, mod, code, names);
  std::vector<std::shared_ptr<BadWordsLang>> lists(names.size());
  for (size_t k = 0; k < names.size(); ++k) {
    auto it = mod.langs.find(names[k]);
    if (it != mod.langs.end()) lists[k] = it->second;
  }
  std::vector<int8_t> matched(n_, -1);  // -1 n/a, 0 no match, 1 match
  parallel_for(n_, nthreads_, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      if (code[(size_t)i] < 0) continue;
      const auto& l = lists[(size_t)code[(size_t)i]];
      if (l) matched[i] = l->match(content(i)) ? 1 : 0;
    }
  });
  apply_badwords_codes(cfg, step_index, mod, matched.data(), code, names);
}

void BatchState::apply_badwords_matched(const StepCfg& cfg, int step_index, BadWordsModule& mod,
                                        const int8_t* matched, const std::vector<std::string>& lang) {
  std::vector<int32_t> code((size_t)n_, -1);
  std::vector<std::string> names;
  std::unordered_map<std::string, int32_t> idx;
  for (int64_t i = 0; i < n_; ++i) {
    if (fail_step_[i] >= 0) continue;
    auto it = idx.find(lang[(size_t)i]);
    if (it == idx.end()) {
      it = idx.emplace(lang[(size_t)i], (int32_t)names.size()).first;
      names.push_back(lang[(size_t)i]);
    }
    code[(size_t)i] = it->second;
  }
  apply_badwords_codes(cfg, step_index, mod, matched, code, names);
}

void BatchState::apply_badwords_codes(const StepCfg& cfg, int step_index, BadWordsModule& mod, const int8_t* matched,
                                      const std::vector<int32_t>& code, const std::vector<std::string>& names) {
  step_slot(step_index);
  auto out = std::make_unique<BwOut>();
  out->code.assign(n_, -1);
  out->lang.resize(n_);
  if (!mod.rng) {
    uint64_t seed = cfg.seed ? *cfg.seed : (((uint64_t)std::random_device{}() << 32) ^ std::random_device{}());
    mod.rng = std::make_unique<StdRng>(seed);
  }
  std::vector<uint8_t> sup(names.size(), 0);
  for (size_t k = 0; k < names.size(); ++k)
    for (auto l : kBadwordsLangs) if (names[k] == l) sup[k] = 1;
  // keep-fraction draws from the shared stream, in document order
  for (int64_t i = 0; i < n_; ++i) {
    if (fail_step_[i] >= 0 || code[(size_t)i] < 0) continue;
    const size_t c = (size_t)code[(size_t)i];
    int8_t st;
    if (!sup[c]) {
      st = cfg.fail_on_missing_language ? BW_MISSING_LANG_FAIL : BW_NO_REGEX;
      if (st == BW_MISSING_LANG_FAIL) out->lang[i] = names[c];
    } else if (matched[i] < 0) {
      st = BW_NO_REGEX;
    } else if (matched[i] == 1) {
      st = (cfg.keep_fraction > 0.0 && mod.rng->gen_f32() < (float)cfg.keep_fraction) ? BW_KEPT_BY_FRACTION
                                                                                      : BW_FILTERED;
    } else {
      st = BW_PASSED;
    }
    out->code[i] = st;
    set_status(i, step_index, (st == BW_FILTERED || st == BW_MISSING_LANG_FAIL) ? 1 : 0);
  }
  bw_[step_index] = std::move(out);
}

void BatchState::run_cpu(const std::vector<StepCfg>& steps, int begin, int end, SegBackend be,
                         const LangidModel* lid, BadWordsModule* bw) {
  PoolTag pool_tag("cpu_steps");
  for (int s = begin; s < end; ++s) {
    const StepCfg& cfg = steps[s];
    if (cfg.kind == StepKind::C4BadWords) {
      if (!bw) throw std::runtime_error("C4BadWordsFilter requires a badwords module");
      apply_badwords(cfg, s, *bw);
      continue;
    }
    if (cfg.kind == StepKind::TokenCounter)
      throw std::runtime_error("TokenCounter records must be supplied by the host tokenizer");
    if (cfg.kind == StepKind::LanguageDetection && !lid)
      throw std::runtime_error("LanguageDetectionFilter requires a language-id model");
    const int width = record_width(cfg);
    StepRec& sr = step_slot(s);
    sr.cfg = std::make_unique<StepCfg>(cfg);
    sr.width = width;
    sr.own.assign((size_t)n_ * width, 0);
    sr.rec = sr.own.data();
    if (cfg.kind == StepKind::C4Quality && own_content_.empty()) own_content_.resize(n_);
    parallel_for(n_, nthreads_, [&](int64_t a, int64_t b) {
      std::string nc;
      for (int64_t i = a; i < b; ++i) {
        if (fail_step_[i] >= 0) continue;
        std::string_view text = content(i);
        int64_t* r = sr.own.data() + i * width;
        if (cfg.kind == StepKind::LanguageDetection) {
          double conf = 0;
          r[rec::LD_LANG] = lid->detect(text, &conf);
          std::memcpy(&r[rec::LD_CONF_BITS], &conf, sizeof(double));
        } else {
          compute_record(cfg, text, be, r, &nc);
        }
        if (cfg.kind == StepKind::C4Quality && !r[rec::C4_LOREM] && !r[rec::C4_CURLY]) {
          own_content_[i] = std::move(nc);
          cur_version_[i] = -1;
        }
        set_status(i, s, decide_status(cfg, r));
      }
    });
  }
}

void BatchState::delegate(const int64_t* idx, int64_t n) {
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = idx[k];
    if (i < 0 || i >= n_) continue;
    fail_step_[i] = 1 << 30;
    status_[i] = 3;
  }
}

std::vector<int64_t> BatchState::alive_indices() const {
  std::vector<int64_t> out;
  for (int64_t i = 0; i < n_; ++i) if (fail_step_[i] < 0) out.push_back(i);
  return out;
}

void BatchState::step_meta(int64_t doc, int s, Decision& d) const {
  d.pass = true;
  d.error = false;
  d.reason.clear();
  d.meta.clear();
  if (s < (int)bw_.size() && bw_[s]) {
    const BwOut& b = *bw_[s];
    switch (b.code[doc]) {
      case BW_PASSED: d.meta.emplace_back("c4_badwords_filter_status", "passed"); break;
      case BW_NO_REGEX: d.meta.emplace_back("c4_badwords_filter_status", "passed_no_regex"); break;
      case BW_KEPT_BY_FRACTION: d.meta.emplace_back("c4_badwords_filter_status", "passed_kept_by_fraction"); break;
      case BW_FILTERED:
        d.pass = false;
        d.reason = "document_removed_with_badwords";
        d.meta.emplace_back("c4_badwords_filter_status", "filtered");
        d.meta.emplace_back("c4_badwords_filter_reason", d.reason);
        break;
      case BW_MISSING_LANG_FAIL:
        d.pass = false;
        d.reason = "There is no badwords list available for '" + b.lang[doc] +
                   "'. Set fail_on_missing_language=False to continue anyway.";
        d.meta.emplace_back("c4_badwords_filter_status", "filtered");
        d.meta.emplace_back("c4_badwords_filter_reason", d.reason);
        break;
      default: break;
    }
    return;
  }
  if (s >= (int)recs_.size() || !recs_[s].cfg) return;
  const StepRec& sr = recs_[s];
  decide(*sr.cfg, sr.rec + doc * sr.width, d);
}

int BatchState::step_kind(int s) const {
  if (s < (int)bw_.size() && bw_[s]) return (int)StepKind::C4BadWords;
  if (s < (int)recs_.size() && recs_[s].cfg) return (int)recs_[s].cfg->kind;
  return -1;
}

static void json_member(CharBuf& out, bool& first, std::string_view k, std::string_view v) {
  if (!first) out.push_back(',');
  first = false;
  json_escape_append(out, k);
  out.push_back(':');
  json_escape_append(out, v);
}

void BatchState::step_meta_json(int64_t doc, int s, CharBuf& out, bool& first) const {
  if (s < (int)bw_.size() && bw_[s]) {
    const BwOut& b = *bw_[s];
    switch (b.code[doc]) {
      case BW_PASSED: json_member(out, first, "c4_badwords_filter_status", "passed"); break;
      case BW_NO_REGEX: json_member(out, first, "c4_badwords_filter_status", "passed_no_regex"); break;
      case BW_KEPT_BY_FRACTION: json_member(out, first, "c4_badwords_filter_status", "passed_kept_by_fraction"); break;
      case BW_FILTERED:
        json_member(out, first, "c4_badwords_filter_status", "filtered");
        json_member(out, first, "c4_badwords_filter_reason", "document_removed_with_badwords");
        break;
      case BW_MISSING_LANG_FAIL: {
        Decision d;
        step_meta(doc, s, d);
        for (auto& kv : d.meta) json_member(out, first, kv.first, kv.second);
        break;
      }
      default: break;
    }
    return;
  }
  if (s >= (int)recs_.size() || !recs_[s].cfg) return;
  const StepRec& sr = recs_[s];
  const int fs = fail_step_[doc];
  if (fs < 0 || s < fs) {
    // the step passed: its members are constants for these kinds (filters.cpp decide_t's pass
    // branches), no need to re-run the decision
    auto lit = [&](std::string_view member) {
      if (!first) out.push_back(',');
      first = false;
      out.append(member.data(), member.size());
    };
    switch (sr.cfg->kind) {
      case StepKind::GopherQuality: lit("\"gopher_quality_filter_status\":\"passed\""); return;
      case StepKind::GopherRepetition: lit("\"gopher_repetition_filter_status\":\"passed\""); return;
      case StepKind::C4Quality: lit("\"c4_filter_status\":\"passed\""); return;
      case StepKind::FineWebQuality: return;
      default: break;
    }
  }
  decide_meta_json(*sr.cfg, sr.rec + doc * sr.width, out, first);
}

std::string BatchState::reason(int64_t i) const {
  const int s = fail_step_[i];
  if (s < 0 || s >= n_applied_) return std::string();
  Decision d;
  step_meta(i, s, d);
  return d.reason;
}

namespace {
std::mutex g_charbuf_mu;
std::vector<std::unique_ptr<CharBuf>>* g_charbufs = new std::vector<std::unique_ptr<CharBuf>>();
}  // namespace

// Every metadata key a step decision can write (filters.cpp decide_t, step_meta): an input key
// outside this list cannot be overwritten by a step.
static bool is_step_key(std::string_view k) {
  static const std::string_view kStepKeys[] = {
      "gopher_quality_filter_status", "gopher_quality_filter_reasons", "gopher_repetition_filter_status",
      "gopher_repetition_filter_reasons", "gopher_repetition_filter_reason", "c4_filter_status",
      "c4_filter_reasons", "line-filter-too_long_word", "line-filter-no_terminal_punc",
      "line-filter-too_few_words", "fineweb_filter_status", "fineweb_filter_reason", "Detected language",
      "Detected language confidence", "token_count", "c4_badwords_filter_status", "c4_badwords_filter_reason"};
  for (const auto& sk : kStepKeys)
    if (k == sk) return true;
  return false;
}

static bool meta_collides(const FlatMeta& fm) {
  for (const auto& e : fm.e)
    if (is_step_key(fm.key(e))) return true;
  return false;
}

// Is `s` an input metadata object whose text is already its own canonical serialization: no
// whitespace, only string members, no byte that json_escape_append would escape (no '\\', no
// control character), at most 16 members with distinct keys none of which a step writes? Then
// parse_meta_json + append_json would reproduce `s` byte for byte, and the output metadata is
// `s` without its closing brace followed by the steps' members. `inner` = the members' text.
static bool canonical_meta(std::string_view s, std::string_view& inner) {
  const size_t n = s.size();
  if (n < 2 || s[0] != '{' || s[n - 1] != '}') return false;
  inner = s.substr(1, n - 2);
  if (n == 2) return true;
  std::string_view keys[16];
  int nk = 0;
  size_t i = 1;
  // one quoted string without escapes at s[i]; returns its contents
  auto str = [&](std::string_view& out) -> bool {
    if (i >= n || s[i] != '"') return false;
    const size_t a = ++i;
    while (i < n) {
      const unsigned char c = (unsigned char)s[i];
      if (c == '"') break;
      if (c < 0x20 || c == '\\') return false;
      ++i;
    }
    if (i >= n) return false;
    out = s.substr(a, i - a);
    ++i;
    return true;
  };
  while (true) {
    std::string_view k, v;
    if (!str(k) || i >= n || s[i] != ':') return false;
    ++i;
    if (!str(v) || nk == 16 || is_step_key(k)) return false;
    for (int j = 0; j < nk; ++j)
      if (keys[j] == k) return false;
    keys[nk++] = k;
    if (i == n - 1) return true;  // the closing brace
    if (s[i] != ',') return false;
    ++i;
  }
}

static std::unique_ptr<CharBuf> take_charbuf() {
  std::lock_guard<std::mutex> g(g_charbuf_mu);
  if (g_charbufs->empty()) return std::make_unique<CharBuf>();
  auto p = std::move(g_charbufs->back());
  g_charbufs->pop_back();
  p->clear();
  return p;
}

static void give_charbuf(std::unique_ptr<CharBuf> p) {
  std::lock_guard<std::mutex> g(g_charbuf_mu);
  if (g_charbufs->size() < 512) g_charbufs->push_back(std::move(p));
}

void BatchState::assemble(const std::vector<int64_t>& idx, RawBuf& text_data, std::vector<int64_t>& text_off,
                          RawBuf& meta_data, std::vector<int64_t>& meta_off,
                          std::vector<uint8_t>& meta_valid, bool with_text) const {
  PoolTag pool_tag("assemble");
  const int64_t m = (int64_t)idx.size();
  // text: sizes are known up front -> offsets, then one parallel gather into the final buffer
  // (with_text=false: the device compacted the texts already, only the metadata is built here)
  text_off.assign(with_text ? m + 1 : 0, 0);
  for (int64_t k = 0; k < m && with_text; ++k) {
    const int64_t i = idx[k];
    int64_t len;
    const int v = cur_version_[i];
    if (v < 0) len = (int64_t)own_content_[i].size();
    else len = versions_[v].off[i + 1] - versions_[v].off[i];
    text_off[k + 1] = text_off[k] + len;
  }
  if (with_text) text_data.alloc((size_t)text_off[m]);
  // metadata: formatted per chunk (sizes unknown), then concatenated
  const int nchunks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)nthreads_ * 4, m / 256));
  // per-chunk metadata buffers come from a process-wide free list: their pages stay mapped and
  // warm from batch to batch
  std::vector<std::unique_ptr<CharBuf>> mparts(nchunks);
  for (auto& p : mparts) p = take_charbuf();
  meta_off.assign(m + 1, 0);
  meta_valid.assign(m, 0);
  // Steps of distinct kinds never write the same metadata key (each kind has its own keys), so
  // per-document metadata is then a plain concatenation in step order.
  bool fast_meta = std::getenv("TB_META_FAST") == nullptr || std::string(std::getenv("TB_META_FAST")) != "0";
  for (int a = 0; a < n_applied_ && fast_meta; ++a)
    for (int b = a + 1; b < n_applied_ && fast_meta; ++b)
      if (step_kind(a) >= 0 && step_kind(a) == step_kind(b)) fast_meta = false;
  auto worker = [&](int64_t c) {
    thread_local FlatMeta fm;
    thread_local Decision d;
    {
      const int64_t a = m * c / nchunks, b = m * (c + 1) / nchunks;
      CharBuf& md = *mparts[c];
      md.reserve((size_t)(b - a) * 192);
      for (int64_t k = a; k < b; ++k) {
        const int64_t i = idx[k];
        if (with_text) {
          std::string_view t = content(i);
          if (!t.empty()) std::memcpy(text_data.p + text_off[k], t.data(), t.size());
        }
        const bool has_input = meta_data_ && (!meta_valid_ || meta_valid_[i]);
        const int last = status_[i] == 0 ? n_applied_ - 1 : std::min(fail_step_[i], n_applied_ - 1);
        if (!has_input && fast_meta) {
          // no input metadata and no key written by two steps: the steps' members go straight
          // into the column buffer in step order (what the map below would produce)
          const size_t before = md.size();
          md.push_back('{');
          bool first = true;
          for (int s = 0; s <= last; ++s) step_meta_json(i, s, md, first);
          if (first) {
            md.resize(before);
            meta_off[k + 1] = 0;
          } else {
            md.push_back('}');
            meta_off[k + 1] = (int64_t)(md.size() - before);
            meta_valid[k] = 1;
          }
          continue;
        }
        if (has_input && fast_meta) {
          std::string_view inner;
          const std::string_view raw(meta_data_ + meta_off_[i], (size_t)(meta_off_[i + 1] - meta_off_[i]));
          if (canonical_meta(raw, inner)) {
            // the input members as they are (their text is canonical), then the steps' members
            const size_t before = md.size();
            md.push_back('{');
            md.append(inner.data(), inner.size());
            bool first = inner.empty();
            for (int s = 0; s <= last; ++s) step_meta_json(i, s, md, first);
            if (first) {
              md.resize(before);
              meta_off[k + 1] = 0;
            } else {
              md.push_back('}');
              meta_off[k + 1] = (int64_t)(md.size() - before);
              meta_valid[k] = 1;
            }
            continue;
          }
        }
        if (has_input) {
          if (!input_meta(i, fm)) meta_fail_.fetch_add(1, std::memory_order_relaxed);
        } else {
          fm.clear();
        }
        if (fast_meta && !meta_collides(fm)) {
          // the input members (in input order), then the steps' members: what the map below
          // produces when no step key is among the input keys (set() then only appends)
          const size_t before = md.size();
          md.push_back('{');
          bool first = true;
          for (const auto& e : fm.e) {
            if (!first) md.push_back(',');
            first = false;
            json_escape_append(md, fm.key(e));
            md.push_back(':');
            json_escape_append(md, fm.value(e));
          }
          for (int s = 0; s <= last; ++s) step_meta_json(i, s, md, first);
          if (first) {
            md.resize(before);
            meta_off[k + 1] = 0;
          } else {
            md.push_back('}');
            meta_off[k + 1] = (int64_t)(md.size() - before);
            meta_valid[k] = 1;
          }
          continue;
        }
        for (int s = 0; s <= last; ++s) {
          step_meta(i, s, d);
          for (auto& kv : d.meta) fm.set(kv.first, kv.second);
        }
        if (fm.empty()) {
          meta_off[k + 1] = 0;  // length; prefix-summed below
        } else {
          const size_t before = md.size();
          thread_local std::string js;
          js.clear();
          fm.append_json(js);
          md.append(js.data(), js.size());
          meta_off[k + 1] = (int64_t)(md.size() - before);
          meta_valid[k] = 1;
        }
      }
    }
  };
  parallel_tasks(nchunks, nthreads_, worker);
  for (int64_t k = 0; k < m; ++k) meta_off[k + 1] += meta_off[k];
  meta_data.alloc((size_t)meta_off[m]);
  std::vector<size_t> base(nchunks + 1, 0);
  for (int c = 0; c < nchunks; ++c) base[c + 1] = base[c] + mparts[c]->size();
  parallel_tasks(nchunks, nthreads_, [&](int64_t c) {
    if (mparts[c]->size()) std::memcpy(meta_data.p + base[c], mparts[c]->data(), mparts[c]->size());
  });
  for (auto& p : mparts) give_charbuf(std::move(p));
}

}  // namespace tb
