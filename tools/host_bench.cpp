// Host output-assembly micro-benchmark (single thread): records of a synthetic corpus through the
// device-emulation path, then BatchState::assemble of the kept and excluded rows, timed. Build
// with -pg for a gprof profile:  tools/host_bench.sh [ndocs] [reps]
#include <chrono>
#include <sys/resource.h>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../csrc/host/devplan_build.h"
#include "../csrc/host/filters.h"
#include "../csrc/host/pipeline.h"

using namespace tb;

static std::string doc(std::mt19937_64& rng) {
  static const char* words[] = {"the", "and", "of", "data", "filter", "model", "window", "house", "garden", "river",
                                "people", "cookie", "hund", "kat", "smörgås", "naïve", "with", "that", "have", "be"};
  static const char* seps[] = {" ", " ", " ", " ", " ", ", ", ". ", ".\n", "! ", "? ", "\n\n", "... "};
  std::string s;
  const int n = 40 + (int)(rng() % 300);
  for (int i = 0; i < n; ++i) {
    s += words[rng() % (sizeof(words) / sizeof(*words))];
    s += seps[rng() % (sizeof(seps) / sizeof(*seps))];
  }
  return s;
}

int main(int argc, char** argv) {
  const int ndocs = argc > 1 ? std::atoi(argv[1]) : 20000;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const int nthreads = argc > 3 ? std::atoi(argv[3]) : 1;
  std::mt19937_64 rng(7);
  std::string data;
  std::vector<int64_t> off{0};
  for (int i = 0; i < ndocs; ++i) {
    data += doc(rng);
    off.push_back((int64_t)data.size());
  }
  std::vector<StepCfg> st(3);
  st[0].kind = StepKind::GopherRepetition;
  st[0].name = "GopherRepetitionFilter";
  st[0].dup_line_frac = 0.3;
  st[0].dup_para_frac = 0.3;
  st[0].dup_line_char_frac = 0.2;
  st[0].dup_para_char_frac = 0.2;
  st[0].top_n_grams = {{2, 0.2}, {3, 0.18}, {4, 0.16}};
  st[0].dup_n_grams = {{5, 0.15}, {6, 0.14}, {7, 0.13}, {8, 0.12}, {9, 0.11}, {10, 0.10}};
  st[1].kind = StepKind::GopherQuality;
  st[1].name = "GopherQualityFilter";
  st[1].min_doc_words = 50;
  st[1].max_doc_words = 100000;
  st[1].min_avg_word_length = 3.0;
  st[1].max_avg_word_length = 10.0;
  st[1].max_symbol_word_ratio = 0.1;
  st[1].max_bullet_lines_ratio = 0.9;
  st[1].max_ellipsis_lines_ratio = 0.3;
  st[1].max_non_alpha_words_ratio = 0.8;
  st[1].min_stop_words = 2;
  st[1].stop_words = {"the", "be", "to", "of", "and", "that", "have", "with"};
  st[2].kind = StepKind::FineWebQuality;
  st[2].name = "FineWebQualityFilter";
  st[2].line_punct_thr = 0.12;
  st[2].short_line_thr = 0.67;
  st[2].short_line_length = 30;
  st[2].char_duplicates_ratio = 0.01;
  st[2].new_line_ratio = 0.3;
  st[2].stop_chars = {'.', '!', '?', '"', '\'', 0x201D};
  std::vector<int64_t> rec;
  std::vector<uint32_t> flags;
  emulate_stage(st, {0, 1, 2}, ndocs, data.data(), off.data(), 8, nullptr, rec, flags, 0);
  double best = 1e9;
  size_t meta_bytes = 0;
  int64_t kept = 0, excl = 0;
  // argv[4] = 1: every document carries input metadata (the CLI path's {"url": ...} column)
  const bool with_meta = argc > 4 && std::atoi(argv[4]) != 0;
  std::string meta;
  std::vector<int64_t> moff{0};
  for (int i = 0; i < ndocs && with_meta; ++i) {
    meta += "{\"url\":\"https://example.com/" + std::to_string(i) + "\"}";
    moff.push_back((int64_t)meta.size());
  }
  BatchState bs(ndocs, data.data(), off.data(), with_meta ? meta.data() : nullptr, with_meta ? moff.data() : nullptr,
                nullptr, nthreads);
  // argv[5] = 1: a LanguageDetection step first (synthetic records: language i % 5, confidence
  // 0.60 .. 0.99), as in the bench pipeline
  if (argc > 5 && std::atoi(argv[5]) != 0) {
    StepCfg ld;
    ld.kind = StepKind::LanguageDetection;
    ld.name = "LanguageDetectionFilter";
    ld.min_confidence = 0.65;
    ld.allowed_langs = {0, 1, 2, 3, 4};
    ld.allowed_codes = {"eng", "dan", "swe", "nno", "nob"};
    static std::vector<int64_t> lrec;
    lrec.assign((size_t)2 * ndocs, 0);
    for (int i = 0; i < ndocs; ++i) {
      const double conf = 0.60 + 0.39 * (double)((i * 7919) % 1000) / 1000.0;
      lrec[2 * i] = i % 5;
      std::memcpy(&lrec[2 * i + 1], &conf, sizeof(double));
    }
    bs.apply_records(ld, 0, lrec.data(), 2, -1);
  }
  const int s0 = (argc > 5 && std::atoi(argv[5]) != 0) ? 1 : 0;
  int prefix = 0;
  for (int s = 0; s < 3; ++s) {
    bs.apply_records(st[s], s0 + s, rec.data() + (int64_t)prefix * ndocs, record_width(st[s]), -1);
    prefix += record_width(st[s]);
  }
  std::vector<int64_t> k, e;
  for (int64_t i = 0; i < ndocs; ++i) (bs.status()[i] == 0 ? k : e).push_back(i);
  rusage ru0, ru1;
  getrusage(RUSAGE_SELF, &ru0);
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    RawBuf td, md;
    std::vector<int64_t> to, mo;
    std::vector<uint8_t> mv;
    bs.assemble(k, td, to, md, mo, mv);
    meta_bytes = (size_t)mo.back();
    bs.assemble(e, td, to, md, mo, mv);
    meta_bytes += (size_t)mo.back();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = dt < best ? dt : best;
    kept = (int64_t)k.size();
    excl = (int64_t)e.size();
    RawBuf::release(td.p, td.cap);
    RawBuf::release(md.p, md.cap);
  }
  getrusage(RUSAGE_SELF, &ru1);
  auto sec = [](const timeval& a, const timeval& b) { return (double)(b.tv_sec - a.tv_sec) + 1e-6 * (double)(b.tv_usec - a.tv_usec); };
  std::printf("assemble loop: user %.3f s, sys %.3f s over %d reps (minor faults %ld)\n", sec(ru0.ru_utime, ru1.ru_utime),
              sec(ru0.ru_stime, ru1.ru_stime), reps, ru1.ru_minflt - ru0.ru_minflt);
  {  // text-only reference: the same gathers without metadata
    double bt = 1e9;
    for (int r = 0; r < reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (auto* rows : {&k, &e}) {
        RawBuf td;
        std::vector<int64_t> to;
        bs.gather(*rows, td, to);
        RawBuf::release(td.p, td.cap);
      }
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      bt = dt < bt ? dt : bt;
    }
    std::printf("text-only gather %.2f ms\n", bt * 1e3);
  }
  std::printf("docs %d kept %lld excluded %lld meta %zu B: assemble %.2f ms (%.3f us/doc, %d threads)\n", ndocs,
              (long long)kept, (long long)excl, meta_bytes, best * 1e3, best * 1e6 / ndocs, nthreads);
  return 0;
}
