// Standalone self-test of the C++ host runtime, built with sanitizers (AddressSanitizer +
// UndefinedBehaviorSanitizer, or ThreadSanitizer) by tests/test_host_sanitizers.py:
//
//   * randomized documents (words, punctuation, newlines, citations, multi-byte text, entities)
//   * CPU records with both segmenters (ICU4C oracle and the UAX#29 rule engine) vs. the host
//     emulation of the device algorithms (SeqPar, with and without an LDS stand-in arena)
//   * multi-threaded BatchState: apply steps, output assembly, reasons
//   * JSON metadata parse/serialize round trips and HTML entity decoding on random input
//
// Exits non-zero on any mismatch; sanitizer reports abort the run.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../csrc/host/devplan_build.h"
#include "../csrc/host/filters.h"
#include "../csrc/host/html.h"
#include "../csrc/host/json.h"
#include "../csrc/host/pipeline.h"
#include "../csrc/host/text.h"
#include "../csrc/common/uax29.h"

using namespace tb;

static int g_fail = 0;
#define CHECK(c, ...)                                 \
  do {                                                \
    if (!(c)) {                                       \
      std::fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);              \
      std::fprintf(stderr, "\n");                     \
      ++g_fail;                                       \
    }                                                 \
  } while (0)

static std::string random_doc(std::mt19937_64& rng) {
  static const char* words[] = {"the", "and", "of", "data", "filter", "Lorem", "javascript", "policy", "cookie",
                                "hund", "kat", "smörgås", "ÆØÅ", "naïve", "Straße", "ΣΑΣ", "İstanbul", "co-op",
                                "3.14", "U.S.A.", "e-mail", "#tag", "…", "—", "“quote”"};
  static const char* seps[] = {" ", " ", " ", ", ", ". ", "! ", "? ", "\n", "\n\n", " [1] ", " [2, 3] ", "... ",
                               "\r\n", "\t", " - ", " • ", " &amp; ", " {x} "};
  std::string s;
  const int n = (int)(rng() % 200);
  for (int i = 0; i < n; ++i) {
    s += words[rng() % (sizeof(words) / sizeof(*words))];
    s += seps[rng() % (sizeof(seps) / sizeof(*seps))];
  }
  if (rng() % 5 == 0) {  // repetition for the Gopher statistics (cut at a code point boundary:
    size_t h = s.size() / 2;  // inputs are valid UTF-8, as Arrow strings are)
    while (h > 0 && ((unsigned char)s[h] & 0xC0) == 0x80) --h;
    s += s.substr(0, h);
  }
  return s;
}

static std::vector<StepCfg> steps() {
  std::vector<StepCfg> v;
  StepCfg gr{};
  gr.kind = StepKind::GopherRepetition;
  gr.name = "GopherRepetitionFilter";
  gr.dup_line_frac = 0.3;
  gr.dup_para_frac = 0.3;
  gr.dup_line_char_frac = 0.2;
  gr.dup_para_char_frac = 0.2;
  gr.top_n_grams = {{2, 0.2}, {3, 0.18}, {4, 0.16}};
  gr.dup_n_grams = {{5, 0.15}, {6, 0.14}, {7, 0.13}, {8, 0.12}, {9, 0.11}, {10, 0.10}};
  v.push_back(gr);
  StepCfg gq{};
  gq.kind = StepKind::GopherQuality;
  gq.name = "GopherQualityFilter";
  gq.min_doc_words = 5;
  gq.max_doc_words = 100000;
  gq.min_avg_word_length = 2.0;
  gq.max_avg_word_length = 10.0;
  gq.max_symbol_word_ratio = 0.1;
  gq.max_bullet_lines_ratio = 0.9;
  gq.max_ellipsis_lines_ratio = 0.3;
  gq.max_non_alpha_words_ratio = 0.8;
  gq.min_stop_words = 2;
  gq.stop_words = {"the", "be", "to", "of", "and", "that", "have", "with"};
  v.push_back(gq);
  StepCfg c4{};
  c4.kind = StepKind::C4Quality;
  c4.name = "C4QualityFilter";
  c4.split_paragraph = true;
  c4.remove_citations = true;
  c4.filter_no_terminal_punct = true;
  c4.min_num_sentences = 3;
  c4.min_words_per_line = 3;
  c4.max_word_length = 1000;
  c4.filter_lorem_ipsum = c4.filter_javascript = c4.filter_curly_bracket = c4.filter_policy = true;
  v.push_back(c4);
  StepCfg fw{};
  fw.kind = StepKind::FineWebQuality;
  fw.name = "FineWebQualityFilter";
  fw.line_punct_thr = 0.12;
  fw.short_line_thr = 0.67;
  fw.short_line_length = 30;
  fw.char_duplicates_ratio = 0.01;
  fw.new_line_ratio = 0.3;
  fw.stop_chars = {'.', '!', '?', '"', '\'', 0x201D};
  v.push_back(fw);
  return v;
}

// Every window (i-2, i-1, i, i+1) of word-break classes, i-2 / i+1 possibly absent: the pair-table
// rule (uax29.h wb_break_ctx_tab, the wave kernels' form) decides like the rule chain it was built
// from wherever that decides, and like the general walk (wb_break over the window as a text)
// wherever it decides without the walk.
struct WinAcc {
  const uint32_t* v;
  uint32_t p(int i) const { return v[i]; }
};
static void check_wb_pair_table() {
  int decided = 0;
  for (uint32_t a = 0; a <= (uint32_t)kWbClasses; ++a)
    for (uint32_t b = 0; b < (uint32_t)kWbClasses; ++b)
      for (uint32_t c = 0; c < (uint32_t)kWbClasses; ++c)
        for (uint32_t d = 0; d <= (uint32_t)kWbClasses; ++d) {
          const uint32_t pm2 = a == (uint32_t)kWbClasses ? 0xFFFFFFFFu : a;
          const uint32_t pp1 = d == (uint32_t)kWbClasses ? 0xFFFFFFFFu : d;
          const int x = wb_break_ctx(pm2, b, c, pp1), y = wb_break_ctx_tab(pm2, b, c, pp1);
          if (y == 2) continue;
          ++decided;
          uint32_t v[4];
          int n = 0;
          if (pm2 != 0xFFFFFFFFu) v[n++] = pm2;
          const int i = n + 1;
          v[n++] = b;
          v[n++] = c;
          if (pp1 != 0xFFFFFFFFu) v[n++] = pp1;
          CHECK(x == 2 || x == y, "wb pair table vs rules: %u %u %u %u", a, b, c, d);
          CHECK((int)wb_break(WinAcc{v}, n, i) == y, "wb pair table vs walk: %u %u %u %u", a, b, c, d);
        }
  CHECK(decided > 60000, "wb pair table decided %d windows", decided);
}

int main(int argc, char** argv) {
  check_wb_pair_table();
  const int ndocs = argc > 1 ? std::atoi(argv[1]) : 400;
  std::mt19937_64 rng(12345);
  std::vector<std::string> docs;
  for (int i = 0; i < ndocs; ++i) docs.push_back(random_doc(rng));
  std::string data;
  std::vector<int64_t> off{0};
  for (auto& d : docs) {
    data += d;
    off.push_back((int64_t)data.size());
  }
  const auto cfg = steps();

  // 1. records: ICU oracle vs rules vs device emulation (stage steps on the input version)
  for (SegBackend be : {SegBackend::Icu, SegBackend::Rules}) {
    for (int s : {0, 1, 3}) {
      std::vector<int64_t> emu;
      std::vector<uint32_t> flags;
      for (uint32_t lds : {0u, 4096u}) {
        emulate_stage(cfg, {s}, ndocs, data.data(), off.data(), 4, nullptr, emu, flags, lds);
        const int w = record_width(cfg[s]);
        for (int i = 0; i < ndocs; ++i) {
          if (flags[i]) continue;  // delegated (dictionary script / collision): not comparable
          std::vector<int64_t> r(w);
          std::string nc;
          compute_record(cfg[s], docs[i], be, r.data(), &nc);
          for (int k = 0; k < w; ++k)
            CHECK(r[k] == emu[(size_t)i * w + k], "step %d doc %d field %d: cpu %lld emu %lld", s, i, k,
                  (long long)r[k], (long long)emu[(size_t)i * w + k]);
        }
      }
    }
  }
  // C4 rewrite vs emulation
  {
    std::vector<int64_t> rec, no;
    std::vector<uint32_t> flags;
    std::string nd;
    emulate_c4(cfg[2], ndocs, data.data(), off.data(), 4, rec, nd, no, flags, 2048);
    for (int i = 0; i < ndocs; ++i) {
      if (flags[i]) continue;
      int64_t r[rec::C4_WIDTH];
      std::string nc;
      compute_record(cfg[2], docs[i], SegBackend::Icu, r, &nc);
      for (int k = 0; k < rec::C4_WIDTH; ++k) CHECK(r[k] == rec[(size_t)i * rec::C4_WIDTH + k], "c4 doc %d field %d", i, k);
      if (!r[rec::C4_LOREM] && !r[rec::C4_CURLY])
        CHECK(nc == nd.substr((size_t)no[i], (size_t)(no[i + 1] - no[i])), "c4 rewrite doc %d", i);
    }
  }
  // 2. multi-threaded batch resolution + assembly
  {
    std::string meta_data;
    std::vector<int64_t> meta_off{0};
    std::vector<uint8_t> meta_valid;
    for (int i = 0; i < ndocs; ++i) {
      if (i % 3 == 0) meta_data += "{\"language\":\"en\",\"k\":\"v" + std::to_string(i) + "\"}";
      if (i % 7 == 0) meta_data += "not json";
      meta_off.push_back((int64_t)meta_data.size());
      meta_valid.push_back(i % 5 != 0);
    }
    BatchState bs(ndocs, data.data(), off.data(), meta_data.data(), meta_off.data(), meta_valid.data(), 6);
    bs.run_cpu(cfg, 0, (int)cfg.size(), SegBackend::Rules, nullptr, nullptr);
    std::vector<int64_t> kept, excl;
    for (int i = 0; i < ndocs; ++i) (bs.status()[i] == 0 ? kept : excl).push_back(i);
    for (auto* idx : {&kept, &excl}) {
      RawBuf td, md;
      std::vector<int64_t> to, mo;
      std::vector<uint8_t> mv;
      bs.assemble(*idx, td, to, md, mo, mv);
      CHECK(to.size() == idx->size() + 1 && mo.size() == idx->size() + 1, "assemble sizes");
      for (size_t k = 0; k < idx->size(); ++k) {
        std::string_view js(md.p + mo[k], (size_t)(mo[k + 1] - mo[k]));
        MetaMap m;
        CHECK(!mv[k] || parse_meta_json(js, m), "metadata JSON does not parse: %.*s", (int)js.size(), js.data());
      }
      RawBuf::release(td.p, td.cap);
      RawBuf::release(md.p, md.cap);
    }
    for (int64_t i : excl) CHECK(!bs.reason(i).empty(), "empty reason for filtered doc %lld", (long long)i);
  }
  // 3. JSON / HTML on random bytes
  for (int t = 0; t < 2000; ++t) {
    std::string s;
    const int n = (int)(rng() % 40);
    static const char alphabet[] = "{}\":,\\u0041nrt &#;x3Cltamp\xC3\xA9\xE2\x80\x9D";
    for (int i = 0; i < n; ++i) s += alphabet[rng() % (sizeof(alphabet) - 1)];
    MetaMap m;
    if (parse_meta_json(s, m)) {
      std::string out;
      serialize_meta_json(m, out);
      MetaMap m2;
      CHECK(parse_meta_json(out, m2) && m2 == m, "JSON round trip");
    }
    std::string dec;
    html_decode(s, dec);
  }
  std::printf("host selftest: %d docs, %d failures\n", ndocs, g_fail);
  return g_fail ? 1 : 0;
}
