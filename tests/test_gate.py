"""Device step gating (csrc/common/gate.h): the gate's pass/fail branch must agree with the host
decision code on every record, and gating (including a deliberately wrong gate) must never
change an output: later passes only skip documents the resolver already finds filtered, and a
document the gate wrongly skipped is recomputed on the CPU path."""
import numpy as np
import pytest

from textblaster_amd.config import load_pipeline_config
from textblaster_amd.config.pipeline import load_pipeline_config_str
from textblaster_amd.pipeline.engine import Engine
from textblaster_amd.utils import synth

from test_emulated_device_path import EDGE, outputs

GATE_CFG = """
pipeline:
  - type: LanguageDetectionFilter
    min_confidence: 0.5
    allowed_languages: [eng, dan]
  - type: GopherRepetitionFilter
    dup_line_frac: 0.3
    dup_para_frac: 0.3
    dup_line_char_frac: 0.2
    dup_para_char_frac: 0.2
    top_n_grams: [[2, 0.2], [3, 0.18], [4, 0.16]]
    dup_n_grams: [[5, 0.15], [6, 0.14], [7, 0.1], [8, 0.12]]
  - type: GopherQualityFilter
    min_doc_words: 50
    max_doc_words: 100000
    min_avg_word_length: 3.0
    max_avg_word_length: 10.0
    max_symbol_word_ratio: 0.1
    max_bullet_lines_ratio: 0.9
    max_ellipsis_lines_ratio: 0.3
    max_non_alpha_words_ratio: 0.8
    min_stop_words: 2
  - type: C4QualityFilter
    split_paragraph: true
    remove_citations: true
    filter_no_terminal_punct: true
    min_num_sentences: 3
    min_words_per_line: 3
    max_word_length: 1000
    filter_lorem_ipsum: true
    filter_javascript: true
    filter_curly_bracket: true
    filter_policy: true
  - type: FineWebQualityFilter
    line_punct_thr: 0.12
    line_punct_exclude_zero: true
    short_line_thr: 0.67
    short_line_length: 30
    char_duplicates_ratio: 0.01
    new_line_ratio: 0.3
"""


def _steps(host, text):
    cfg = load_pipeline_config_str(text)
    return cfg, [host.make_step(s.native_dict()) for s in cfg.pipeline]


def _random_records(rng, width, n):
    r = rng.integers(-2, 60, size=(n, width)).astype(np.int64)
    # shrink some denominators / numerators to hit the boundaries (0, equal, max(1, x))
    r[rng.random((n, width)) < 0.15] = 0
    r[rng.random((n, width)) < 0.05] = 1
    return r


def test_gate_agrees_with_host_decision(host):
    cfg, steps = _steps(host, GATE_CFG)
    rng = np.random.default_rng(5)
    for st, sc in zip(steps, cfg.pipeline):
        w = st.record_width()
        recs = _random_records(rng, w, 4000)
        if sc.type == "LanguageDetectionFilter":
            recs[:, 0] = rng.integers(-1, 5, size=len(recs))
            conf = rng.choice([0.0, 0.49, 0.5, 0.51, 1.0], size=len(recs))
            recs[:, 1] = conf.view(np.int64)
        if sc.type == "GopherRepetitionFilter":
            recs[:, 0] = rng.integers(-1, 400, size=len(recs))
            recs[:, 7:] = rng.integers(0, 120, size=(len(recs), w - 7))
        if sc.type == "C4QualityFilter":
            recs[:, :2] = rng.integers(0, 2, size=(len(recs), 2)) * (rng.random((len(recs), 2)) < 0.2)
        mism = []
        for r in recs:
            r = r.tolist()
            if host.gate_fails(st, r) != (host.decide_status(st, r) != 0):
                mism.append(r)
        assert not mism, (sc.type, mism[:3])


@pytest.mark.parametrize("cfg_path", ["config/bench_pipeline.yaml", "config/pipeline_config.yaml", None])
def test_gated_emulation_equals_ungated(cfg_path, tmp_path):
    if cfg_path is None:
        p = tmp_path / "gate.yaml"
        p.write_text(GATE_CFG)
        cfg_path = str(p)
    cfg = load_pipeline_config(cfg_path)
    if any(s.type in ("TokenCounter", "C4BadWordsFilter") for s in cfg.pipeline):
        cfg.pipeline = [s for s in cfg.pipeline if s.type not in ("TokenCounter", "C4BadWordsFilter")]
    texts = synth.make_corpus(800, 900, seed=29) + EDGE
    data, off = synth.pack(texts)
    a = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True)
    assert a.device_runner.gates, "the pipeline has several device passes: gates expected"
    b = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True)
    b.device_runner.gates = {}
    ra, rb = a.process(data, off), b.process(data, off)
    assert outputs(ra) == outputs(rb)
    assert ra.reasons == rb.reasons
    # the gates did skip work
    res = a.device_runner.run(data, off)
    assert res.dead is not None and int(np.count_nonzero(res.dead)) > 0


def test_wrong_gate_is_caught_and_recomputed():
    from textblaster_amd.utils import metrics

    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    texts = synth.make_corpus(600, 900, seed=31) + EDGE
    data, off = synth.pack(texts)
    ref = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True).process(data, off)
    eng = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True)
    eng.device_runner.gate_corrupt = 5  # marks every 5th document dead after the first pass
    before = metrics.GATE_MISMATCH_DOCS_TOTAL._value.get()
    got = eng.process(data, off)
    assert metrics.GATE_MISMATCH_DOCS_TOTAL._value.get() > before
    assert got.n_delegated > 0
    assert outputs(got) == outputs(ref)
    assert got.reasons == ref.reasons
    np.testing.assert_array_equal(got.fail_step, ref.fail_step)
