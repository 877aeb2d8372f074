"""C4 pass A's citation path from the stage's line export (docproc.h c4_pass_a_cite_export): the
host emulation of the device algorithms against the CPU ICU oracle on documents dense in
citation shapes (reference CITATION_REGEX, c4_filters.rs:33): multi-number lists, spaces inside
the brackets, citations glued to words, a trailing comma, a line feed inside a list, Arabic-Indic
digits (the non-ASCII fallback to the general path), empty brackets, and phrases joined across a
removed citation."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from textblaster_amd.config import load_pipeline_config_str  # noqa: E402
from textblaster_amd.pipeline.engine import Engine  # noqa: E402
from textblaster_amd.utils import synth  # noqa: E402

from test_emulated_device_path import outputs  # noqa: E402

CFG = """pipeline:
  - type: GopherQualityFilter
    min_doc_words: 1
    max_doc_words: 100000
    min_avg_word_length: 0.01
    max_avg_word_length: 100.0
    max_symbol_word_ratio: 100.0
    max_bullet_lines_ratio: 1.0
    max_ellipsis_lines_ratio: 1.0
    max_non_alpha_words_ratio: 0.01
    min_stop_words: 0
  - type: C4QualityFilter
    split_paragraph: true
    remove_citations: true
    filter_no_terminal_punct: true
    min_num_sentences: 2
    min_words_per_line: 3
    max_word_length: 1000
    filter_lorem_ipsum: true
    filter_javascript: true
    filter_curly_bracket: true
    filter_policy: true
  - type: FineWebQualityFilter
    line_punct_thr: 0.12
    line_punct_exclude_zero: false
    short_line_thr: 0.67
    short_line_length: 30
    char_duplicates_ratio: 0.01
    new_line_ratio: 0.3
"""
CITES = ["[1]", "[12]", "[1, 2]", "[1,2,3]", "[1,]", "[ 1]", "[1 ]", "[1][2]", "[١]", "[1, 2]",
         "[1,\n2]", "[a]", "[]", "[99999999]", "[1,  23]", "[1,\t2]"]
WORDS = ["alpha", "beta", "the", "and", "of", "gamma", "Delta", "x", "yy", "zzz", "javascript", "privacy",
         "policy", "été", "sø", "java", "script"]


def cite_corpus(n, seed):
    rng = np.random.default_rng(seed)
    texts = []
    for _ in range(n):
        lines = []
        for _ in range(int(rng.integers(1, 12))):
            toks = [CITES[int(rng.integers(0, len(CITES)))] if rng.random() < 0.12
                    else WORDS[int(rng.integers(0, len(WORDS)))] for _ in range(int(rng.integers(0, 14)))]
            s = " ".join(toks)
            if rng.random() < 0.2:
                s = s.replace(" [", "[")
            s += str(rng.choice([".", "", "!", "...", "?", " [3]", "[4].", "java[5]script."]))
            if rng.random() < 0.1:
                s = "  " + s + "  "
            lines.append(s)
        texts.append("\n".join(lines))
    return texts


def test_cite_export_path_equals_cpu_oracle():
    cfg = load_pipeline_config_str(CFG, "c4_cite.yaml")
    texts = cite_corpus(3000, 7) + synth.make_corpus(400, 900, seed=5)
    data, off = synth.pack(texts)
    a = Engine(cfg, backend="emulate", keep_reasons=True).process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", keep_reasons=True).process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    oa, ob = outputs(a), outputs(b)
    bad = [k for k in oa if oa[k] != ob[k]]
    assert not bad, [(k, texts[k][:120]) for k in bad[:3]]
    # the corpus exercises the path: most documents pass GopherQuality and reach C4
    assert np.count_nonzero((b.fail_step != 0) | (b.status == 0)) > 2500
