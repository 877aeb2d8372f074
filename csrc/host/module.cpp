// pybind11 bindings for the host runtime (_tbhost): text primitives, the CPU pipeline, the
// batch resolver used by the GPU path, HTML decoding and output assembly.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <optional>
#include <thread>
#include <unordered_map>

#include "../common/badwords.h"
#include "../common/bpe.h"
#include "../common/bpe_classes.inc"
#include "../common/langid.h"
#include "../common/ucd_tables.inc"
#include "filters.h"
#include "html.h"
#include "html_entities.inc"
#include "json.h"
#include "pipeline.h"
#include "devplan_build.h"
#include "rustfmt.h"
#include "text.h"

namespace py = pybind11;
using namespace tb;

template <class T>
static py::array_t<T> to_numpy(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}
static py::array_t<uint8_t> str_to_numpy(std::string&& s) {
  auto* heap = new std::string(std::move(s));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::string*>(p); });
  return py::array_t<uint8_t>({(py::ssize_t)heap->size()}, {(py::ssize_t)1},
                              (const uint8_t*)heap->data(), owner);
}

static py::array_t<uint8_t> raw_to_numpy(RawBuf& b) {
  auto* hold = new RawBuf(b);
  b.p = nullptr;
  py::capsule owner(hold, [](void* q) {
    auto* r = reinterpret_cast<RawBuf*>(q);
    RawBuf::release(r->p, r->cap);
    delete r;
  });
  return py::array_t<uint8_t>({(py::ssize_t)hold->n}, {(py::ssize_t)1}, (const uint8_t*)hold->p, owner);
}

static SegBackend be_of(const std::string& s) {
  if (s == "icu") return SegBackend::Icu;
  if (s == "rules") return SegBackend::Rules;
  throw std::invalid_argument("segmentation backend must be 'icu' or 'rules'");
}

template <class T>
static std::optional<T> opt(const py::dict& d, const char* k) {
  if (!d.contains(k) || d[k].is_none()) return std::nullopt;
  return d[k].cast<T>();
}

static StepCfg make_step(const py::dict& d) {
  StepCfg c;
  std::string t = d["type"].cast<std::string>();
  c.name = t;
  if (t == "C4QualityFilter") {
    c.kind = StepKind::C4Quality;
    c.split_paragraph = d["split_paragraph"].cast<bool>();
    c.remove_citations = d["remove_citations"].cast<bool>();
    c.filter_no_terminal_punct = d["filter_no_terminal_punct"].cast<bool>();
    c.min_num_sentences = d["min_num_sentences"].cast<int64_t>();
    c.min_words_per_line = d["min_words_per_line"].cast<int64_t>();
    c.max_word_length = d["max_word_length"].cast<int64_t>();
    c.filter_lorem_ipsum = d["filter_lorem_ipsum"].cast<bool>();
    c.filter_javascript = d["filter_javascript"].cast<bool>();
    c.filter_curly_bracket = d["filter_curly_bracket"].cast<bool>();
    c.filter_policy = d["filter_policy"].cast<bool>();
  } else if (t == "GopherRepetitionFilter") {
    c.kind = StepKind::GopherRepetition;
    c.dup_line_frac = opt<double>(d, "dup_line_frac");
    c.dup_para_frac = opt<double>(d, "dup_para_frac");
    c.dup_line_char_frac = opt<double>(d, "dup_line_char_frac");
    c.dup_para_char_frac = opt<double>(d, "dup_para_char_frac");
    if (d.contains("top_n_grams")) c.top_n_grams = d["top_n_grams"].cast<std::vector<std::pair<int64_t, double>>>();
    if (d.contains("dup_n_grams")) c.dup_n_grams = d["dup_n_grams"].cast<std::vector<std::pair<int64_t, double>>>();
  } else if (t == "GopherQualityFilter") {
    c.kind = StepKind::GopherQuality;
    c.min_doc_words = opt<int64_t>(d, "min_doc_words");
    c.max_doc_words = opt<int64_t>(d, "max_doc_words");
    c.min_avg_word_length = opt<double>(d, "min_avg_word_length");
    c.max_avg_word_length = opt<double>(d, "max_avg_word_length");
    c.max_symbol_word_ratio = opt<double>(d, "max_symbol_word_ratio");
    c.max_bullet_lines_ratio = opt<double>(d, "max_bullet_lines_ratio");
    c.max_ellipsis_lines_ratio = opt<double>(d, "max_ellipsis_lines_ratio");
    c.max_non_alpha_words_ratio = opt<double>(d, "max_non_alpha_words_ratio");
    c.min_stop_words = opt<int64_t>(d, "min_stop_words");
    c.stop_words = d["stop_words"].cast<std::vector<std::string>>();
  } else if (t == "FineWebQualityFilter") {
    c.kind = StepKind::FineWebQuality;
    c.line_punct_thr = d["line_punct_thr"].cast<double>();
    c.line_punct_exclude_zero = d["line_punct_exclude_zero"].cast<bool>();
    c.short_line_thr = d["short_line_thr"].cast<double>();
    c.short_line_length = d["short_line_length"].cast<int64_t>();
    c.char_duplicates_ratio = d["char_duplicates_ratio"].cast<double>();
    c.new_line_ratio = d["new_line_ratio"].cast<double>();
    c.stop_chars = d["stop_chars"].cast<std::vector<uint32_t>>();
  } else if (t == "LanguageDetectionFilter") {
    c.kind = StepKind::LanguageDetection;
    c.min_confidence = d["min_confidence"].cast<double>();
    c.allowed_langs = d["allowed_langs"].cast<std::vector<int>>();
    c.allowed_codes = d["allowed_codes"].cast<std::vector<std::string>>();
  } else if (t == "C4BadWordsFilter") {
    c.kind = StepKind::C4BadWords;
    c.keep_fraction = d["keep_fraction"].cast<double>();
    c.fail_on_missing_language = d["fail_on_missing_language"].cast<bool>();
    c.seed = opt<uint64_t>(d, "seed");
    c.default_language = d["default_language"].cast<std::string>();
  } else if (t == "TokenCounter") {
    c.kind = StepKind::TokenCounter;
    c.tokenizer_name = d["tokenizer_name"].cast<std::string>();
  } else {
    throw std::invalid_argument("unknown step type " + t);
  }
  return c;
}

// Holds the numpy buffers a BatchState borrows so they outlive it.
struct __attribute__((visibility("hidden"))) PyBatch {
  std::unique_ptr<BatchState> st;
  std::vector<py::object> keep;
};

static const char* buf_ptr(const py::array& a) { return (const char*)a.data(); }

PYBIND11_MODULE(_tbhost, m) {
  m.doc() = "textblaster_amd host runtime";

  py::enum_<StepKind>(m, "StepKind")
      .value("C4Quality", StepKind::C4Quality)
      .value("GopherRepetition", StepKind::GopherRepetition)
      .value("GopherQuality", StepKind::GopherQuality)
      .value("C4BadWords", StepKind::C4BadWords)
      .value("LanguageDetection", StepKind::LanguageDetection)
      .value("FineWebQuality", StepKind::FineWebQuality)
      .value("TokenCounter", StepKind::TokenCounter);

  py::class_<StepCfg>(m, "StepCfg")
      .def_readonly("kind", &StepCfg::kind)
      .def_property_readonly("n_dup", [](const StepCfg& c) { return (int)c.dup_n_grams.size(); })
      .def_property_readonly("n_top", [](const StepCfg& c) { return (int)c.top_n_grams.size(); })
      .def_readonly("name", &StepCfg::name)
      .def_readonly("remove_citations", &StepCfg::remove_citations)
      .def("record_width", [](const StepCfg& c) { return record_width(c); });
  m.def("make_step", &make_step);

  // ---- text primitives (reference utils/text.rs) ----
  m.def("split_into_words", [](const std::string& s, const std::string& be) {
    std::vector<std::string> out;
    for (auto w : split_into_words(s, be_of(be))) out.emplace_back(w);
    return out;
  }, py::arg("text"), py::arg("backend") = "rules");
  m.def("split_into_sentences", [](const std::string& s, const std::string& be) {
    std::vector<std::string> out;
    for (auto w : split_into_sentences(s, be_of(be))) out.emplace_back(w);
    return out;
  }, py::arg("text"), py::arg("backend") = "rules");
  m.def("word_breaks", [](const std::string& s, const std::string& be) { return word_breaks(s, be_of(be)); },
        py::arg("text"), py::arg("backend") = "rules");
  m.def("sentence_breaks", [](const std::string& s, const std::string& be) { return sentence_breaks(s, be_of(be)); },
        py::arg("text"), py::arg("backend") = "rules");
  m.def("find_duplicates", [](const std::vector<std::string>& items) {
    std::vector<std::string_view> v(items.begin(), items.end());
    return find_duplicates(v);
  });
  m.def("find_top_duplicate", [](const std::vector<std::string>& words, size_t n) {
    std::vector<std::string_view> v(words.begin(), words.end());
    return find_top_duplicate_ngrams(v, n);
  });
  m.def("find_all_duplicate", [](const std::vector<std::string>& words, size_t n) {
    std::vector<std::string_view> v(words.begin(), words.end());
    return find_all_duplicate(v, n);
  });
  m.def("remove_citations", [](const std::string& s) { return remove_citations(s); });
  m.def("rust_lowercase", [](const std::string& s) { return rust_lowercase(s); });
  m.def("rust_lines", [](const std::string& s) {
    std::vector<std::string> out;
    for (auto l : rust_lines(s)) out.emplace_back(l);
    return out;
  });
  m.def("trim", [](const std::string& s) { return std::string(trim(s)); });
  m.def("props", [](uint32_t cp) { return host_ucd().props(cp); });
  m.def("has_dict_script", [](const std::string& s) { return has_dict_script(s); });
  m.def("dict_word_marks", [](py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                              int nthreads) {
    std::vector<int64_t> moff;
    std::vector<uint32_t> bits;
    const int64_t nd = (int64_t)off.size() - 1;
    {
      py::gil_scoped_release nogil;
      dict_word_marks(data.data(), off.data(), nd, nthreads, moff, bits);
    }
    return py::make_tuple(to_numpy(std::move(moff)), to_numpy(std::move(bits)));
  }, py::arg("data"), py::arg("offsets"), py::arg("nthreads") = 8,
     "ICU word-break marks of the dictionary-script documents (text.h dict_word_marks)");
  m.def("dict_c4_lines", [](py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                            py::array_t<int64_t, py::array::c_style> moff, bool citations, int nthreads) {
    std::vector<int64_t> loff;
    std::vector<uint32_t> out;
    const int64_t nd = (int64_t)off.size() - 1;
    if ((int64_t)moff.size() < nd) throw std::runtime_error("dict_c4_lines: operand shapes");
    {
      py::gil_scoped_release nogil;
      dict_c4_lines(data.data(), off.data(), nd, moff.data(), citations, nthreads, loff, out);
    }
    return py::make_tuple(to_numpy(std::move(loff)), to_numpy(std::move(out)));
  }, py::arg("data"), py::arg("offsets"), py::arg("moff"), py::arg("citations"), py::arg("nthreads") = 8,
     "C4 per-line ICU word statistics of the dictionary-script documents (text.h dict_c4_lines)");
  m.def("ucd_fold_tables", []() {
    std::vector<uint16_t> f1(TB_UCD_FOLD_STAGE1, TB_UCD_FOLD_STAGE1 + sizeof(TB_UCD_FOLD_STAGE1) / 2);
    std::vector<int32_t> f2(TB_UCD_FOLD_STAGE2, TB_UCD_FOLD_STAGE2 + sizeof(TB_UCD_FOLD_STAGE2) / 4);
    return py::make_tuple(to_numpy(std::move(f1)), to_numpy(std::move(f2)));
  });
  m.def("ucd_tables", []() {
    std::vector<uint16_t> s1(TB_UCD_PROPS_STAGE1, TB_UCD_PROPS_STAGE1 + sizeof(TB_UCD_PROPS_STAGE1) / 2);
    std::vector<uint32_t> s2((const uint32_t*)TB_UCD_PROPS_STAGE2,
                             (const uint32_t*)TB_UCD_PROPS_STAGE2 + sizeof(TB_UCD_PROPS_STAGE2) / 4);
    std::vector<uint16_t> l1(TB_UCD_LOWER_STAGE1, TB_UCD_LOWER_STAGE1 + sizeof(TB_UCD_LOWER_STAGE1) / 2);
    std::vector<int32_t> l2(TB_UCD_LOWER_STAGE2, TB_UCD_LOWER_STAGE2 + sizeof(TB_UCD_LOWER_STAGE2) / 4);
    return py::make_tuple(to_numpy(std::move(s1)), to_numpy(std::move(s2)), to_numpy(std::move(l1)),
                          to_numpy(std::move(l2)));
  });
  // ---- C4 bad words: hashed trie table + host twin of k_badwords_match (csrc/common/badwords.h) ----
  m.def("bw_build_table", [](py::array_t<int32_t, py::array::c_style> fe, py::array_t<uint32_t, py::array::c_style> ec,
                             py::array_t<int32_t, py::array::c_style> et, py::array_t<uint8_t, py::array::c_style> term) {
    const int64_t nodes = (int64_t)term.size();
    if ((int64_t)fe.size() != nodes + 1 || ec.size() != et.size() || (nodes && fe.data()[nodes] != (int32_t)ec.size()))
      throw std::invalid_argument("bad-words automaton is malformed");
    return to_numpy(bw_build_table(fe.data(), nodes, ec.data(), et.data(), (int64_t)ec.size(), term.data()));
  });
  // Per document the input metadata's "language" value (the only source of that key: reference
  // c4_filters.rs:464-468) as an index into the returned name list, -1 when absent.
  m.def("meta_languages", [](py::array_t<uint8_t, py::array::c_style> md, py::array_t<int64_t, py::array::c_style> mo,
                             py::object mv, int nthreads) {
    PoolTag pool_tag("meta_languages");
    const int64_t n = (int64_t)mo.size() - 1;
    const uint8_t* valid = nullptr;
    py::array_t<uint8_t, py::array::c_style> va;
    if (!mv.is_none()) {
      va = mv.cast<py::array_t<uint8_t, py::array::c_style>>();
      if (va.size() < n) throw std::invalid_argument("meta_languages: validity shorter than the batch");
      valid = va.data();
    }
    if (n < 0 || (n > 0 && mo.data()[n] > (int64_t)md.size())) throw std::invalid_argument("meta_languages: offsets");
    std::vector<std::string> val((size_t)std::max<int64_t>(n, 0));
    std::vector<uint8_t> has((size_t)std::max<int64_t>(n, 0), 0);
    const char* d = (const char*)md.data();
    const int64_t* o = mo.data();
    {
      py::gil_scoped_release nogil;
      parallel_for(n, nthreads, [&](int64_t a, int64_t b) {
        FlatMeta fm;
        for (int64_t i = a; i < b; ++i) {
          if (valid && !valid[i]) continue;
          fm.clear();
          if (parse_meta_json(std::string_view(d + o[i], (size_t)(o[i + 1] - o[i])), fm) && fm.has("language")) {
            val[(size_t)i] = std::string(fm.get("language"));
            has[(size_t)i] = 1;
          }
        }
      });
    }
    std::vector<int32_t> code((size_t)std::max<int64_t>(n, 0), -1);
    std::vector<std::string> names;
    std::unordered_map<std::string, int32_t> idx;
    for (int64_t i = 0; i < n; ++i) {
      if (!has[(size_t)i]) continue;
      auto it = idx.find(val[(size_t)i]);
      if (it == idx.end()) {
        it = idx.emplace(val[(size_t)i], (int32_t)names.size()).first;
        names.push_back(val[(size_t)i]);
      }
      code[(size_t)i] = it->second;
    }
    return py::make_tuple(to_numpy(std::move(code)), names);
  }, py::arg("meta_data"), py::arg("meta_off"), py::arg("meta_valid") = py::none(), py::arg("nthreads") = 8);
  m.def("bw_match_batch", [](py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                             py::array_t<uint32_t, py::array::c_style> table, py::object roots, py::object cjk,
                             int32_t root0, int32_t cjk0, py::object dead, uint32_t dead_max, int nthreads) {
    PoolTag pool_tag("badwords");
    const int64_t n = (int64_t)off.size() - 1;
    const uint64_t slots = (uint64_t)table.size() / 4;
    if (n < 0 || slots == 0 || (slots & (slots - 1))) throw std::invalid_argument("bw_match_batch: shapes");
    const int32_t* rp = nullptr;
    const uint8_t* cp = nullptr;
    const uint8_t* dp = nullptr;
    py::array_t<int32_t, py::array::c_style> ra;
    py::array_t<uint8_t, py::array::c_style> ca, da;
    if (!roots.is_none()) { ra = roots.cast<py::array_t<int32_t, py::array::c_style>>(); rp = ra.data(); }
    if (!cjk.is_none()) { ca = cjk.cast<py::array_t<uint8_t, py::array::c_style>>(); cp = ca.data(); }
    if (!dead.is_none()) { da = dead.cast<py::array_t<uint8_t, py::array::c_style>>(); dp = da.data(); }
    if ((rp && ra.size() < n) || (cp && ca.size() < n) || (dp && da.size() < n))
      throw std::invalid_argument("bw_match_batch: per-document array shorter than the batch");
    std::vector<int8_t> out((size_t)n, -1);
    const BwTable bt{table.data(), (uint32_t)(slots - 1)};
    static const std::vector<uint16_t> f1(TB_UCD_FOLD_STAGE1, TB_UCD_FOLD_STAGE1 + sizeof(TB_UCD_FOLD_STAGE1) / 2);
    static const std::vector<int32_t> f2(TB_UCD_FOLD_STAGE2, TB_UCD_FOLD_STAGE2 + sizeof(TB_UCD_FOLD_STAGE2) / 4);
    const BwFold fold{f1.data(), f2.data()};
    const UcdView& ucd = host_ucd();
    uint8_t asc[128];
    for (uint32_t c = 0; c < 128; ++c) asc[c] = bw_ascii_entry(ucd, fold, c);
    const uint8_t* b = data.data();
    const int64_t* o = off.data();
    {
      py::gil_scoped_release nogil;
      parallel_for(n, nthreads, [&](int64_t a, int64_t e) {
        for (int64_t i = a; i < e; ++i) {
          const int32_t r = rp ? rp[i] : root0;
          const uint32_t d = dp ? dp[i] : 0u;
          if (r < 0 || (d != 0 && d <= dead_max)) continue;
          out[(size_t)i] = bw_match_doc(b + o[i], (uint32_t)(o[i + 1] - o[i]), r, (cp ? cp[i] : cjk0) != 0, bt, ucd,
                                        fold, asc) ? 1 : 0;
        }
      });
    }
    return to_numpy(std::move(out));
  }, py::arg("data"), py::arg("off"), py::arg("table"), py::arg("roots") = py::none(), py::arg("cjk") = py::none(),
     py::arg("root0") = -1, py::arg("cjk0") = 0, py::arg("dead") = py::none(), py::arg("dead_max") = 0,
     py::arg("nthreads") = 8);
  // ---- byte-level BPE token counting (csrc/common/bpe.h; device kernel csrc/hip/bpe.hip) ----
  m.def("bpe_classes", []() {
    std::vector<uint16_t> c1(TB_BPE_CLS_STAGE1, TB_BPE_CLS_STAGE1 + sizeof(TB_BPE_CLS_STAGE1) / 2);
    std::vector<uint32_t> c2(TB_BPE_CLS_STAGE2, TB_BPE_CLS_STAGE2 + sizeof(TB_BPE_CLS_STAGE2) / 4);
    return py::make_tuple(to_numpy(std::move(c1)), to_numpy(std::move(c2)));
  });
  m.def("bpe_build_table", [](py::array_t<uint32_t, py::array::c_style> a, py::array_t<uint32_t, py::array::c_style> b,
                              py::array_t<uint32_t, py::array::c_style> rank, py::array_t<uint32_t, py::array::c_style> nid) {
    // open addressing, load <= 1/2; a pair listed twice keeps its last rank (HashMap collect)
    const size_t n = (size_t)a.size();
    if ((size_t)b.size() != n || (size_t)rank.size() != n || (size_t)nid.size() != n)
      throw std::invalid_argument("bpe_build_table: operand shapes");
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    std::vector<uint64_t> keys(cap, kBpeEmpty), vals(cap, ~0ull);
    const uint64_t mask = cap - 1;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t key = ((uint64_t)a.data()[i] << 32) | b.data()[i];
      if (key == kBpeEmpty) throw std::invalid_argument("bpe_build_table: reserved pair");
      uint64_t h = bpe_hash(key) & mask;
      while (keys[h] != kBpeEmpty && keys[h] != key) h = (h + 1) & mask;
      keys[h] = key;
      vals[h] = ((uint64_t)rank.data()[i] << 32) | nid.data()[i];
    }
    return py::make_tuple(to_numpy(std::move(keys)), to_numpy(std::move(vals)), (uint32_t)mask);
  });
  m.def("bpe_count", [](py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                        py::array_t<uint32_t, py::array::c_style> byte_id, py::array_t<uint64_t, py::array::c_style> keys,
                        py::array_t<uint64_t, py::array::c_style> vals, uint32_t mask,
                        py::array_t<uint8_t, py::array::c_style> added, std::vector<int32_t> added_off, int32_t post_add,
                        int nthreads, int64_t chunk) {
    // host emulation of k_bpe_count: per document the token count, or kBpeHost. chunk > 0: the
    // wave split — the pre-tokens starting in each chunk-byte range counted independently
    // (bpe_count_range), as the kernel's lanes do
    if (byte_id.size() != 256 || (size_t)keys.size() != (size_t)mask + 1 || vals.size() != keys.size() ||
        added_off.size() > kBpeMaxAdded + 1 || (added_off.size() && added_off.back() > added.size()))
      throw std::invalid_argument("bpe_count: operand shapes");
    const int64_t nd = off.size() - 1;
    std::vector<int32_t> out(nd > 0 ? nd : 0);
    DevBpe T{};
    T.byte_id = byte_id.data();
    T.keys = keys.data();
    T.vals = vals.data();
    T.cls1 = TB_BPE_CLS_STAGE1;
    T.cls2 = TB_BPE_CLS_STAGE2;
    T.added = added.data();
    T.mask = mask;
    T.n_added = added_off.empty() ? 0 : (int32_t)added_off.size() - 1;
    for (size_t i = 0; i < added_off.size(); ++i) T.added_off[i] = added_off[i];
    T.post_add = post_add;
    const uint8_t* d = data.data();
    const int64_t* o = off.data();
    {
      py::gil_scoped_release nogil;
      const int nt = std::max(1, std::min<int>(nthreads, (int)(nd / 256) + 1));
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
          uint32_t cbuf[kBpeMaxWord], rbuf[kBpeMaxWord];
          std::vector<uint32_t> lc(kBpeMaxLong);
          std::vector<uint64_t> lv(kBpeMaxLong);
          std::vector<int32_t> lnx(kBpeMaxLong), lpv(kBpeMaxLong);
          const uint8_t* b = nullptr;
          // pre-tokens over kBpeMaxWord bytes: merged over arrays of their own length (as
          // k_bpe_long does), up to kBpeMaxLong bytes
          auto on_long = [&](int64_t s, int64_t e) -> int64_t {
            if (e - s > kBpeMaxLong) return -1;
            return bpe_word_long(T, b + s, (int)(e - s), lc.data(), lv.data(), lnx.data(), lpv.data());
          };
          for (int64_t k = t; k < nd; k += nt) {
            b = d + o[k];
            const int64_t n = o[k + 1] - o[k];
            if (chunk <= 0) {
              out[k] = bpe_count_doc(T, b, n, BpeArr{cbuf, 1}, BpeArr{rbuf, 1}, on_long);
              continue;
            }
            int64_t tot = T.post_add;
            bool bad = T.n_added && bpe_has_added(T, b, n);
            for (int64_t s0 = 0; s0 < n && !bad; s0 += chunk) {
              const int64_t x = bpe_count_range<true>(T, b, n, s0, std::min(n, s0 + chunk), BpeArr{cbuf, 1},
                                                      BpeArr{rbuf, 1}, on_long);
              if (x < 0) bad = true;
              tot += x;
            }
            out[k] = (bad || tot > 0x7FFFFFFF) ? kBpeHost : (int32_t)tot;
          }
        });
      for (auto& x : th) x.join();
    }
    return to_numpy(std::move(out));
  }, py::arg("data"), py::arg("off"), py::arg("byte_id"), py::arg("keys"), py::arg("vals"), py::arg("mask"),
        py::arg("added"), py::arg("added_off"), py::arg("post_add"), py::arg("nthreads") = 8, py::arg("chunk") = 0);
  m.def("fmt_f64", [](double x) { return fmt_f64(x); });
  m.def("fmt_fixed", [](double x, int prec) { return fmt_fixed(x, prec); });
  m.def("contains_byte", [](py::array_t<uint8_t, py::array::c_style> a, int v) {
    const void* p = a.data();
    const size_t n = (size_t)a.size();
    py::gil_scoped_release nogil;
    return n > 0 && std::memchr(p, v, n) != nullptr;
  });

  // ---- per-step records and decisions ----
  m.def("compute_record", [](const StepCfg& c, const std::string& text, const std::string& be) {
    std::vector<int64_t> r(record_width(c), 0);
    std::string nc;
    compute_record(c, text, be_of(be), r.data(), &nc);
    return py::make_tuple(r, py::bytes(nc));
  }, py::arg("step"), py::arg("text"), py::arg("backend") = "rules");
  m.def("decide", [](const StepCfg& c, const std::vector<int64_t>& r) {
    Decision d;
    decide(c, r.data(), d);
    return py::make_tuple(d.pass, d.error, d.reason, d.meta);
  });

  // ---- metadata JSON ----
  m.def("parse_meta_json", [](const std::string& s) -> py::object {
    MetaMap mm;
    if (!parse_meta_json(s, mm)) return py::none();
    return py::cast(mm);
  });
  m.def("serialize_meta_json", [](const MetaMap& mm) {
    std::string out;
    serialize_meta_json(mm, out);
    return out;
  });

  // ---- HTML entity decoding over a packed batch ----
  m.def("html_decode", [](const std::string& s) {
    std::string out;
    if (!html_decode(s, out)) return s;
    return out;
  });
  m.def("html_entity_table", []() {
    // The named-reference table (sorted bytewise) packed for the device decoder (csrc/hip/html.hip):
    // (names, name offsets, UTF-8 values, value offsets).
    std::string names, vals;
    std::vector<int32_t> no{0}, vo{0};
    for (int k = 0; k < kHtmlEntityCount; ++k) {
      names += kHtmlEntities[k].name;
      vals += kHtmlEntities[k].utf8;
      no.push_back((int32_t)names.size());
      vo.push_back((int32_t)vals.size());
    }
    return py::make_tuple(py::bytes(names), no, py::bytes(vals), vo);
  });
  m.def("html_decode_batch", [](py::array_t<uint8_t, py::array::c_style> data,
                                py::array_t<int64_t, py::array::c_style> off, int nthreads) -> py::object {
    PoolTag pool_tag("html_decode");
    const int64_t n = (int64_t)off.size() - 1;
    const char* d = (const char*)data.data();
    const int64_t* o = off.data();
    std::vector<std::string> dec(n);
    std::vector<uint8_t> changed(n, 0);
    {
      py::gil_scoped_release nogil;
      parallel_for(n, nthreads, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i)
          changed[i] = html_decode(std::string_view(d + o[i], (size_t)(o[i + 1] - o[i])), dec[i]);
      });
    }
    bool any = false;
    for (auto c : changed) any |= c != 0;
    if (!any) return py::none();
    std::string out;
    std::vector<int64_t> no(n + 1, 0);
    {
      py::gil_scoped_release nogil;
      size_t tot = 0;
      for (int64_t i = 0; i < n; ++i) tot += changed[i] ? dec[i].size() : (size_t)(o[i + 1] - o[i]);
      out.reserve(tot);
      for (int64_t i = 0; i < n; ++i) {
        if (changed[i]) out += dec[i];
        else out.append(d + o[i], (size_t)(o[i + 1] - o[i]));
        no[i + 1] = (int64_t)out.size();
      }
    }
    return py::make_tuple(str_to_numpy(std::move(out)), to_numpy(std::move(no)));
  });

  // ---- language id (CPU) ----
  py::class_<LangidModel, std::shared_ptr<LangidModel>>(m, "LangidModel")
      .def(py::init([](py::array_t<int8_t, py::array::c_style> E, py::array_t<int16_t, py::array::c_style> W,
                       double w_scale, py::array_t<float, py::array::c_style> b) {
        // int8 embedding rows + integer head (the MFMA tile's operands)
        auto mdl = std::make_shared<LangidModel>();
        if ((size_t)E.size() != (size_t)kLidBuckets * kLidRowDim) throw std::invalid_argument("E shape");
        if ((size_t)W.size() != (size_t)kLidDim * kLidLangs) throw std::invalid_argument("W shape");
        if ((size_t)b.size() != (size_t)kLidRow) throw std::invalid_argument("b shape");
        for (py::ssize_t i = 0; i < W.size(); ++i)
          if (W.data()[i] > kLidQMax || W.data()[i] < -kLidQMax) throw std::invalid_argument("W out of range");
        if (!(w_scale > 0)) throw std::invalid_argument("w_scale must be > 0");
        mdl->E.assign(E.data(), E.data() + E.size());
        mdl->W.assign(W.data(), W.data() + W.size());
        mdl->w_scale = w_scale;
        mdl->b.assign(b.data(), b.data() + b.size());
        return mdl;
      }))
      .def_readonly("version", &LangidModel::version)
      .def("detect", [](const LangidModel& mdl, const std::string& s) {
        double conf = 0;
        int l = mdl.detect(s, &conf);
        return py::make_tuple(l, conf);
      })
      .def("sums", [](const LangidModel& mdl, const std::string& s) {
        std::vector<int64_t> v(mdl.sum_width(), 0);
        const int64_t c = mdl.sums(s, v.data());
        return py::make_tuple(c, v);
      })
      .def("record", [](const LangidModel& mdl, const std::vector<int64_t>& sums, int64_t cnt) {
        if ((int)sums.size() != mdl.sum_width()) throw std::invalid_argument("sums width");
        int64_t r[2];
        mdl.record(sums.data(), cnt, r);
        double conf;
        std::memcpy(&conf, &r[1], sizeof(double));
        return py::make_tuple(r[0], conf);
      });
  m.def("lid_exp", [](double x) { return lid_exp(x); });
  m.def("langid_buckets", [](const std::string& s, bool with_order) -> py::object {
    // The hashed n-gram bucket ids of `s` (training-time featurizer, identical to the model's),
    // and with_order: their n-gram orders too.
    std::vector<uint32_t> out;
    std::vector<uint8_t> ord;
    const uint8_t* b = (const uint8_t*)s.data();
    const uint32_t n = (uint32_t)s.size();
    const UcdView& u = host_ucd();
    uint32_t lm3 = 0, lm2 = 0, lm1 = 0;
    int ncp = 0;
    auto emit = [&](uint32_t k, int order) { out.push_back(k); ord.push_back((uint8_t)order); };
    for (uint32_t i = 0; i < n && ncp < kLidMaxCps; ++ncp) {
      const uint32_t l0 = lid_letter(u, b, n, i);
      int len;
      (void)utf8_decode(b, i, n, &len);
      i += len;
      lid_grams_n(lm3, lm2, lm1, l0, emit);
      lm3 = lm2;
      lm2 = lm1;
      lm1 = l0;
    }
    lid_grams_n(lm3, lm2, lm1, 0, emit);
    if (with_order) return py::make_tuple(out, ord);
    return py::cast(out);
  }, py::arg("s"), py::arg("with_order") = false);
  m.attr("LID_ROW") = kLidRow;
  m.attr("LID_LANGS") = kLidLangs;
  m.attr("LID_BUCKETS") = kLidBuckets;
  m.attr("LID_DIM") = kLidDim;
  m.attr("LID_ROW_DIM") = kLidRowDim;
  m.attr("LID_QMAX") = kLidQMax;

  py::class_<StdRng>(m, "StdRng")
      .def(py::init<uint64_t>())
      .def("next_u32", &StdRng::next_u32)
      .def("gen_f32", &StdRng::gen_f32);

  py::class_<BadWordsModule, std::shared_ptr<BadWordsModule>>(m, "BadWordsModule")
      .def(py::init([](const std::string& dir) {
        auto b = std::make_shared<BadWordsModule>();
        b->cache_dir = dir;
        return b;
      }))
      .def("matches", [](BadWordsModule& b, const std::string& lang, const std::string& text) {
        bool sup;
        auto l = b.get(lang, &sup);
        if (!l) return false;
        return l->match(text);
      })
      .def("flatten", [](BadWordsModule& b) {
        BadWordsAutomaton a = b.flatten();
        py::dict roots, cjk;
        for (auto& kv : a.root) roots[py::str(kv.first)] = kv.second;
        for (auto& kv : a.cjk) cjk[py::str(kv.first)] = kv.second;
        return py::make_tuple(to_numpy(std::move(a.first_edge)), to_numpy(std::move(a.edge_cp)),
                              to_numpy(std::move(a.edge_to)), to_numpy(std::move(a.term)), roots, cjk);
      })
      .def("lookup", [](BadWordsModule& b, const std::string& lang) {
        // (supported language?, has a non-empty list?)
        bool sup;
        auto l = b.get(lang, &sup);
        return py::make_tuple(sup, (bool)l);
      });

  // Spans idx[k] of a packed (text, off) column gathered into a new packed column (multithreaded).
  m.def("gather_spans", [](py::array_t<uint8_t, py::array::c_style> text, py::array_t<int64_t, py::array::c_style> off,
                           py::array_t<int64_t, py::array::c_style> idx, int nthreads) {
    PoolTag pool_tag("gather_spans");
    const int64_t n = (int64_t)off.size() - 1, m = (int64_t)idx.size();
    const int64_t* o = off.data();
    const int64_t* ix = idx.data();
    std::vector<int64_t> no((size_t)m + 1, 0);
    for (int64_t k = 0; k < m; ++k) {
      if (ix[k] < 0 || ix[k] >= n) throw std::invalid_argument("gather_spans: index out of range");
      if (o[ix[k]] < 0 || o[ix[k] + 1] < o[ix[k]] || o[ix[k] + 1] > (int64_t)text.size())
        throw std::invalid_argument("gather_spans: offsets out of range");
      no[(size_t)k + 1] = no[(size_t)k] + (o[ix[k] + 1] - o[ix[k]]);
    }
    py::array_t<uint8_t> out((py::ssize_t)std::max<int64_t>(no[(size_t)m], 1));
    uint8_t* d = out.mutable_data();
    const uint8_t* t = text.data();
    {
      py::gil_scoped_release nogil;
      parallel_for(m, no[(size_t)m] >= (4 << 20) ? nthreads : 1, [&](int64_t a, int64_t b) {
        for (int64_t k = a; k < b; ++k)
          std::memcpy(d + no[(size_t)k], t + o[ix[k]], (size_t)(no[(size_t)k + 1] - no[(size_t)k]));
      });
    }
    const py::ssize_t total = (py::ssize_t)no[(size_t)m];
    py::object view = out[py::slice(0, total, 1)];
    return py::make_tuple(view, to_numpy(std::move(no)));
  }, py::arg("text"), py::arg("off"), py::arg("idx"), py::arg("nthreads") = 8);

  // Multi-threaded memcpy into a (pinned) staging buffer: dst[dst_off : dst_off + src.nbytes] = src.
  // CPU seconds of the native worker pool per job tag (PoolTag), since process start
  m.def("pool_cpu_stats", []() {
    py::dict d;
    for (auto& kv : pool_cpu_stats()) d[py::str(kv.first)] = kv.second;
    return d;
  });
  m.def("parallel_copy", [](py::array dst, int64_t dst_off, py::array src, int nthreads) {
    PoolTag pool_tag("stage_copy");
    if (!(dst.flags() & py::array::c_style) || !(src.flags() & py::array::c_style))
      throw std::invalid_argument("parallel_copy needs contiguous arrays");
    const int64_t nb = (int64_t)src.nbytes();
    if (dst_off < 0 || dst_off + nb > (int64_t)dst.nbytes()) throw std::invalid_argument("parallel_copy out of range");
    char* d = (char*)dst.mutable_data() + dst_off;
    const char* sp = (const char*)src.data();
    py::gil_scoped_release nogil;
    const int64_t chunk = 1 << 20;
    parallel_for((nb + chunk - 1) / chunk, nb >= (8 << 20) ? nthreads : 1, [&](int64_t a, int64_t b) {
      for (int64_t c = a; c < b; ++c) {
        const int64_t o = c * chunk, len = std::min<int64_t>(chunk, nb - o);
        std::memcpy(d + o, sp + o, (size_t)len);
      }
    });
  }, py::arg("dst"), py::arg("dst_off"), py::arg("src"), py::arg("nthreads") = 8);

  // ---- batch state ----
  py::class_<PyBatch>(m, "BatchState")
      .def(py::init([](py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                       py::object meta_data, py::object meta_off, py::object meta_valid, int nthreads) {
        auto pb = new PyBatch();
        pb->keep = {data, off, meta_data, meta_off, meta_valid};
        const char* md = nullptr;
        const int64_t* mo = nullptr;
        const uint8_t* mv = nullptr;
        if (!meta_data.is_none()) {
          md = buf_ptr(meta_data.cast<py::array>());
          mo = (const int64_t*)meta_off.cast<py::array>().data();
          if (!meta_valid.is_none()) mv = (const uint8_t*)meta_valid.cast<py::array>().data();
        }
        py::gil_scoped_release nogil;
        pb->st = std::make_unique<BatchState>((int64_t)off.size() - 1, (const char*)data.data(), off.data(),
                                              md, mo, mv, nthreads);
        return pb;
      }), py::arg("data"), py::arg("offsets"), py::arg("meta_data") = py::none(),
          py::arg("meta_offsets") = py::none(), py::arg("meta_valid") = py::none(), py::arg("nthreads") = 8)
      .def_property_readonly("size", [](PyBatch& b) { return b.st->size(); })
      .def_property_readonly("meta_parse_failures", [](PyBatch& b) { return b.st->meta_parse_failures(); })
      .def("add_version", [](PyBatch& b, py::array_t<uint8_t, py::array::c_style> data,
                             py::array_t<int64_t, py::array::c_style> off) {
        if ((int64_t)off.size() != b.st->size() + 1) throw std::invalid_argument("offsets length");
        b.keep.push_back(data);
        b.keep.push_back(off);
        return b.st->add_version((const char*)data.data(), off.data());
      })
      .def("run_cpu", [](PyBatch& b, const std::vector<StepCfg>& steps, int begin, int end, const std::string& be,
                         std::shared_ptr<LangidModel> lid, std::shared_ptr<BadWordsModule> bw) {
        py::gil_scoped_release nogil;
        b.st->run_cpu(steps, begin, end, be_of(be), lid.get(), bw.get());
      }, py::arg("steps"), py::arg("begin"), py::arg("end"), py::arg("backend") = "rules",
         py::arg("lid") = nullptr, py::arg("badwords") = nullptr)
      .def("apply_records", [](PyBatch& b, const StepCfg& c, int step_index,
                               py::array_t<int64_t, py::array::c_style> rec, int rewrite_version) {
        const int w = record_width(c);
        if ((int64_t)rec.size() != b.st->size() * w) throw std::invalid_argument("record array size");
        b.keep.push_back(rec);  // records are read again at output assembly
        py::gil_scoped_release nogil;
        b.st->apply_records(c, step_index, rec.data(), w, rewrite_version);
      }, py::arg("step"), py::arg("step_index"), py::arg("records"), py::arg("rewrite_version") = -1)
      .def("apply_badwords", [](PyBatch& b, const StepCfg& c, int step_index, std::shared_ptr<BadWordsModule> bw) {
        py::gil_scoped_release nogil;
        b.st->apply_badwords(c, step_index, *bw);
      })
      .def("badwords_languages", [](PyBatch& b, const StepCfg& c, std::shared_ptr<BadWordsModule> bw) {
        std::vector<std::string> out;
        {
          py::gil_scoped_release nogil;
          out = b.st->badwords_languages(c, *bw);
        }
        return out;
      })
      .def("apply_badwords_matched", [](PyBatch& b, const StepCfg& c, int step_index, std::shared_ptr<BadWordsModule> bw,
                                        py::array_t<int8_t, py::array::c_style> matched,
                                        const std::vector<std::string>& langs) {
        if ((int64_t)matched.size() != b.st->size() || (int64_t)langs.size() != b.st->size())
          throw std::invalid_argument("matched/langs length");
        py::gil_scoped_release nogil;
        b.st->apply_badwords_matched(c, step_index, *bw, matched.data(), langs);
      })
      .def("apply_badwords_device", [](PyBatch& b, const StepCfg& c, int step_index, std::shared_ptr<BadWordsModule> bw,
                                       py::array_t<int8_t, py::array::c_style> matched) {
        // the device matched the documents (k_badwords_match); languages and the keep-fraction
        // draws (document order) are decided here, as apply_badwords does
        if ((int64_t)matched.size() != b.st->size()) throw std::invalid_argument("matched length");
        py::gil_scoped_release nogil;
        std::vector<int32_t> code;
        std::vector<std::string> names;
        b.st->badwords_lang_codes(c, *bw, code, names);
        b.st->apply_badwords_codes(c, step_index, *bw, matched.data(), code, names);
      })
      .def("gather", [](PyBatch& b, py::array_t<int64_t, py::array::c_style> idx) {
        std::vector<int64_t> iv(idx.data(), idx.data() + idx.size());
        RawBuf d;
        std::vector<int64_t> o;
        {
          py::gil_scoped_release nogil;
          b.st->gather(iv, d, o);
        }
        return py::make_tuple(raw_to_numpy(d), to_numpy(std::move(o)));
      })
      .def("delegate", [](PyBatch& b, py::array_t<int64_t, py::array::c_style> idx) {
        b.st->delegate(idx.data(), (int64_t)idx.size());
      })
      .def("alive_indices", [](PyBatch& b) { return to_numpy(b.st->alive_indices()); })
      .def("fail_step", [](PyBatch& b) { return to_numpy(std::vector<int32_t>(b.st->fail_step())); })
      .def("status", [](PyBatch& b) { return to_numpy(std::vector<uint8_t>(b.st->status())); })
      .def("cur_version", [](PyBatch& b) { return to_numpy(std::vector<int32_t>(b.st->cur_version())); })
      .def("reasons", [](PyBatch& b, py::array_t<int64_t, py::array::c_style> idx) {
        std::vector<std::string> out;
        for (py::ssize_t k = 0; k < idx.size(); ++k) out.push_back(b.st->reason(idx.data()[k]));
        return out;
      })
      .def("contents", [](PyBatch& b, py::array_t<int64_t, py::array::c_style> idx) {
        py::list out;
        for (py::ssize_t k = 0; k < idx.size(); ++k) {
          auto s = b.st->content(idx.data()[k]);
          out.append(py::str(s.data(), s.size()));
        }
        return out;
      })
      .def("assemble", [](PyBatch& b, py::array_t<int64_t, py::array::c_style> idx, bool with_text) -> py::tuple {
        std::vector<int64_t> iv(idx.data(), idx.data() + idx.size());
        RawBuf td, md;
        std::vector<int64_t> to, mo;
        std::vector<uint8_t> mv;
        {
          py::gil_scoped_release nogil;
          b.st->assemble(iv, td, to, md, mo, mv, with_text);
        }
        if (!with_text) return py::make_tuple(py::none(), py::none(), raw_to_numpy(md), to_numpy(std::move(mo)),
                                              to_numpy(std::move(mv)));
        return py::make_tuple(raw_to_numpy(td), to_numpy(std::move(to)), raw_to_numpy(md),
                              to_numpy(std::move(mo)), to_numpy(std::move(mv)));
      }, py::arg("idx"), py::arg("with_text") = true);

  // ---- device plan building + host emulation of the device algorithms ----
  m.def("device_supported", [](const StepCfg& c) {
    std::string why;
    bool ok = device_supported(c, &why);
    return py::make_tuple(ok, why);
  });
  m.def("build_device_plan", [](const std::vector<StepCfg>& steps, const std::vector<std::vector<int>>& stages) {
    auto plan = std::make_unique<DevPlan>();
    std::memset(plan.get(), 0, sizeof(DevPlan));
    py::list st;
    for (auto& idx : stages) {
      DevStage d = build_stage(steps, idx, *plan);
      st.append(py::bytes((const char*)&d, sizeof(d)));
    }
    return py::make_tuple(py::bytes((const char*)plan.get(), sizeof(DevPlan)), st);
  });
  m.def("build_c4", [](const StepCfg& c) {
    DevC4 d = build_c4(c);
    return py::bytes((const char*)&d, sizeof(d));
  });
  m.def("build_gate", [](const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries) {
    DevGate g = build_gate(steps, entries);
    return py::bytes((const char*)&g, sizeof(g));
  });
  // Device gate decision on one record (host evaluation of the same TB_HD code; tests compare it
  // with decide_status over the step's whole decision space).
  m.def("gate_fails", [](const StepCfg& c, const std::vector<int64_t>& r) {
    if ((int)r.size() < record_width(c)) throw std::runtime_error("record too short");
    DevGateStep g = build_gate_step(c, 0, 0);
    return gate_fails(g, r.data());
  });
  m.def("decide_status", [](const StepCfg& c, const std::vector<int64_t>& r) {
    if ((int)r.size() < record_width(c)) throw std::runtime_error("record too short");
    return (int)decide_status(c, r.data());
  });
  m.attr("SIZEOF_DEV_GATE") = sizeof(DevGate);
  m.attr("SIZEOF_DEV_RESOLVE") = sizeof(DevResolve);
  m.attr("MAX_VERSIONS") = kMaxVersions;
  m.def("build_resolve", [](const std::vector<StepCfg>& steps, const std::vector<std::array<int, 3>>& entries,
                            const std::vector<int>& c4_version) {
    DevResolve rp = build_resolve(steps, entries, c4_version);
    return py::bytes((const char*)&rp, sizeof(rp));
  });
  m.def("resolve_host", [](const py::bytes& blob, const std::vector<py::array_t<int64_t, py::array::c_style>>& recs,
                           int64_t ndocs, py::array_t<uint32_t, py::array::c_style> flags,
                           const std::vector<py::array_t<uint8_t, py::array::c_style>>& vdata,
                           const std::vector<py::array_t<int64_t, py::array::c_style>>& voff) {
    std::string bs = blob;
    if (bs.size() != sizeof(DevResolve)) throw std::runtime_error("bad resolve blob");
    DevResolve rp;
    std::memcpy(&rp, bs.data(), sizeof(rp));
    if ((int64_t)flags.size() < ndocs || vdata.size() != voff.size()) throw std::runtime_error("resolve: operand shapes");
    for (int s = 0; s < rp.gate.n_steps; ++s) {
      const DevGateStep& st = rp.gate.steps[s];
      if (st.slot < 0 || st.slot >= (int)recs.size() ||
          (int64_t)recs[st.slot].size() < ((int64_t)st.prefix + st.width) * ndocs)
        throw std::runtime_error("resolve record buffer too short");
    }
    std::vector<const int64_t*> rp_ptrs;
    for (auto& r : recs) rp_ptrs.push_back(r.data());
    std::vector<const char*> vd;
    std::vector<const int64_t*> vo;
    for (size_t v = 0; v < vdata.size(); ++v) {
      if ((int64_t)voff[v].size() != ndocs + 1) throw std::runtime_error("resolve: version offsets length");
      vd.push_back((const char*)vdata[v].data());
      vo.push_back(voff[v].data());
    }
    std::vector<int32_t> fail, rows;
    std::vector<uint8_t> status;
    std::string out;
    std::vector<int64_t> out_off;
    {
      py::gil_scoped_release nogil;
      resolve_host(rp, rp_ptrs, ndocs, flags.data(), vd, vo, fail, status, out, out_off, rows);
    }
    return py::make_tuple(to_numpy(std::move(fail)), to_numpy(std::move(status)), str_to_numpy(std::move(out)),
                          to_numpy(std::move(out_off)), to_numpy(std::move(rows)));
  });
  m.def("stage_layout", [](const py::bytes& b) {
    std::string s = b;
    DevStage d;
    std::memcpy(&d, s.data(), sizeof(d));
    py::list out;
    for (int i = 0; i < d.n_steps; ++i) out.append(py::make_tuple(d.steps[i].kind, d.steps[i].width, d.steps[i].rec_prefix));
    return py::make_tuple(d.width_total, out);
  });
  m.def("pow_table", [](uint32_t n) { return to_numpy(pow_table(n)); });
  m.def("scratch_bytes_for", [](uint32_t n, bool split) { return scratch_bytes_for(n, split); }, py::arg("n"),
        py::arg("split") = false);
  m.def("scratch_need", [](bool reset) { return scratch_need(reset); }, py::arg("reset") = false);
  m.def("set_scratch_probe", &set_scratch_probe);
  m.attr("SCRATCH_PER_BYTE") = kScratchPerByte;
  m.attr("SCRATCH_PER_BYTE_SPLIT") = kScratchPerByteSplit;
  m.attr("C4_MAX_GROWTH") = kC4MaxGrowth;
  m.attr("SIZEOF_DEV_PLAN") = sizeof(DevPlan);
  m.attr("SIZEOF_DEV_STAGE") = sizeof(DevStage);
  m.attr("SIZEOF_DEV_C4") = sizeof(DevC4);
  m.attr("OFFSETOF_REC_BASE") = offsetof(DevStep, rec_base);
  m.attr("SIZEOF_DEV_STEP") = sizeof(DevStep);
  m.attr("OFFSETOF_STEPS") = offsetof(DevStage, steps);
  m.def("emulate_stage", [](const std::vector<StepCfg>& steps, const std::vector<int>& idx,
                            py::array_t<uint8_t, py::array::c_style> data, py::array_t<int64_t, py::array::c_style> off,
                            int nthreads, std::shared_ptr<LangidModel> lid, uint32_t lds_bytes,
                            std::optional<py::array_t<uint8_t, py::array::c_style>> dead, bool weak_keys,
                            std::optional<py::array_t<uint32_t, py::array::c_style>> line_stats, int split_tasks,
                            std::optional<py::array_t<int64_t, py::array::c_style>> dict_moff,
                            std::optional<py::array_t<uint32_t, py::array::c_style>> dict_bits,
                            std::optional<py::array_t<uint32_t, py::array::c_style>> dict_words) {
    std::vector<int64_t> rec;
    std::vector<uint32_t> flags;
    const int64_t nd = (int64_t)off.size() - 1;
    if (dead && (int64_t)dead->size() < nd) throw std::runtime_error("dead mask too short");
    const uint8_t* dp = dead ? dead->data() : nullptr;
    uint32_t* lp = nullptr;
    if (line_stats) {
      if ((uint64_t)line_stats->size() < line_stats_buffer_words(off.data(), nd)) throw std::runtime_error("line_stats too short");
      lp = line_stats->mutable_data();
    }
    DictIn dict;
    if (dict_moff) {
      if ((int64_t)dict_moff->size() < nd || !dict_bits) throw std::runtime_error("dict marks: operand shapes");
      const int64_t* mo = dict_moff->data();
      for (int64_t d = 0; d < nd; ++d) {  // every bitmap inside `bits` (the kernels trust the offsets)
        if (mo[d] < 0) continue;
        uint32_t C = 0;
        for (int64_t i = off.data()[d]; i < off.data()[d + 1]; ++i) C += (data.data()[i] & 0xC0) != 0x80;
        if (mo[d] + (int64_t)(2 * (((C + 1 + 63) / 64) * 2)) > (int64_t)dict_bits->size())
          throw std::runtime_error("dict marks: bitmap out of range");
      }
      dict.moff = mo;
      dict.bits = dict_bits->data();
    }
    if (dict_words) {
      if ((int64_t)dict_words->size() < nd) throw std::runtime_error("dict words: operand shapes");
      dict.words = dict_words->data();
    }
    {
      py::gil_scoped_release nogil;
      emulate_stage(steps, idx, nd, (const char*)data.data(), off.data(), nthreads, lid.get(), rec, flags, lds_bytes,
                    dp, weak_keys, lp, split_tasks, dict);
    }
    return py::make_tuple(to_numpy(std::move(rec)), to_numpy(std::move(flags)));
  }, py::arg("steps"), py::arg("idx"), py::arg("data"), py::arg("offsets"), py::arg("nthreads") = 8,
     py::arg("lid") = nullptr, py::arg("lds_bytes") = 0, py::arg("dead") = py::none(),
     py::arg("weak_keys") = false, py::arg("line_stats") = py::none(), py::arg("split_tasks") = 0,
     py::arg("dict_moff") = py::none(), py::arg("dict_bits") = py::none(), py::arg("dict_words") = py::none());
  m.def("line_stats_words", [](py::array_t<int64_t, py::array::c_style> off) {
    return line_stats_buffer_words(off.data(), (int64_t)off.size() - 1);
  }, "u32 words of a batch's C4 line export buffer (docproc.h line_stats_base)");
  m.def("gate_host", [](const py::bytes& gate, const std::vector<py::array_t<int64_t, py::array::c_style>>& recs,
                        int64_t ndocs, py::array_t<uint32_t, py::array::c_style> flags,
                        py::array_t<uint8_t, py::array::c_style> dead, int code) {
    std::string gs = gate;
    if (gs.size() != sizeof(DevGate)) throw std::runtime_error("bad gate blob");
    if (code <= 0 || code > 255) throw std::runtime_error("gate code out of range");
    if ((int64_t)dead.size() < ndocs || (int64_t)flags.size() < ndocs) throw std::runtime_error("gate: operand shapes");
    DevGate g;
    std::memcpy(&g, gs.data(), sizeof(g));
    std::vector<const int64_t*> rp;
    for (int s = 0; s < g.n_steps; ++s) {
      const DevGateStep& st = g.steps[s];
      if (st.kind == GK_NONE) continue;
      if (st.slot < 0 || st.slot >= (int)recs.size()) throw std::runtime_error("gate slot out of range");
      if ((int64_t)recs[st.slot].size() < ((int64_t)st.prefix + st.width) * ndocs)
        throw std::runtime_error("gate record buffer too short");
    }
    for (auto& r : recs) rp.push_back(r.data());
    gate_host(g, rp, ndocs, flags.data(), dead.mutable_data(), (uint8_t)code);
  });
  m.def("emulate_c4", [](const StepCfg& step, py::array_t<uint8_t, py::array::c_style> data,
                         py::array_t<int64_t, py::array::c_style> off, int nthreads, uint32_t lds_bytes,
                         std::optional<py::array_t<uint8_t, py::array::c_style>> dead,
                         std::optional<py::array_t<uint32_t, py::array::c_style>> line_stats,
                         std::optional<py::array_t<uint32_t, py::array::c_style>> c4_words,
                         std::optional<py::array_t<int64_t, py::array::c_style>> dict_loff,
                         std::optional<py::array_t<uint32_t, py::array::c_style>> dict_ldata) {
    std::vector<int64_t> rec, no;
    std::vector<uint32_t> flags;
    std::string nd;
    const int64_t n = (int64_t)off.size() - 1;
    if (dead && (int64_t)dead->size() < n) throw std::runtime_error("dead mask too short");
    const uint8_t* dp = dead ? dead->data() : nullptr;
    const uint32_t* lp = nullptr;
    if (line_stats) {
      if ((uint64_t)line_stats->size() < line_stats_buffer_words(off.data(), n)) throw std::runtime_error("line_stats too short");
      lp = line_stats->data();
    }
    uint32_t* wp = nullptr;
    if (c4_words) {
      if ((int64_t)c4_words->size() < n) throw std::runtime_error("c4_words too short");
      wp = c4_words->mutable_data();
    }
    DictLines dl;
    if (dict_loff) {
      if ((int64_t)dict_loff->size() < n || !dict_ldata) throw std::runtime_error("dict lines: operand shapes");
      for (int64_t d = 0; d < n; ++d) {
        const int64_t o = dict_loff->data()[d];
        if (o >= 0 && (o >= (int64_t)dict_ldata->size() ||
                       o + 1 + 2 * (int64_t)dict_ldata->data()[o] > (int64_t)dict_ldata->size()))
          throw std::runtime_error("dict lines: record out of range");
      }
      dl.off = dict_loff->data();
      dl.data = dict_ldata->data();
    }
    {
      py::gil_scoped_release nogil;
      emulate_c4(step, n, (const char*)data.data(), off.data(), nthreads, rec, nd, no, flags, lds_bytes, dp, lp, wp, dl);
    }
    return py::make_tuple(to_numpy(std::move(rec)), str_to_numpy(std::move(nd)), to_numpy(std::move(no)),
                          to_numpy(std::move(flags)));
  }, py::arg("step"), py::arg("data"), py::arg("offsets"), py::arg("nthreads") = 8, py::arg("lds_bytes") = 0,
     py::arg("dead") = py::none(), py::arg("line_stats") = py::none(), py::arg("c4_words") = py::none(),
     py::arg("dict_loff") = py::none(), py::arg("dict_ldata") = py::none());
}
