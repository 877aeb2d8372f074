"""TokenCounter's byte-level BPE counter (csrc/common/bpe.h; device kernel k_bpe_count).

CPU: the native counter (the kernel's algorithm compiled for the host) must give exactly the
`tokenizers` library's ``len(encode(text, add_special_tokens=True).tokens)`` — the reference's
TokenCounter (src/pipeline/token/token_counter.rs:31-42) — on the checked-in gpt2-format fixture
and on tokenizers trained here (GPT-2 layout, a TemplateProcessing post-processor), over fuzz
text built from the regex's corner cases, the adversarial pool and the synthetic corpora. The
device pipeline's token counts (emulated, then on the GPU) must equal the CPU path's.
"""
import json
import os
import random
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from adversarial import adversarial_corpus  # noqa: E402

from textblaster_amd import native  # noqa: E402
from textblaster_amd.config import load_pipeline_config_str  # noqa: E402
from textblaster_amd.models.tokenizer import TokenCounterModel, build_bpe_spec, train_synthetic_bpe  # noqa: E402
from textblaster_amd.utils import synth  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPT2_FIXTURE = os.path.join(REPO, "tests", "fixtures", "tokenizers", "gpt2", "tokenizer.json")

POOL = ["a", "b", "'", "s", "t", "re", "ve", "ll", "m", "d", " ", "  ", "\n", "\t", "\r\n", "　", " ",
        "1", "42", "²", "Ⅻ", "é", "é", "日本", "\U0001F600", "!", "?", "...", "don't",
        "IT'S", "we're", "ß", "Σ", " 's", "\x1c", "\u0085", "​", "ﬁ", "٣", "x'llama", "''s"]


def fuzz(n, seed):
    rng = random.Random(seed)
    return ["".join(rng.choice(POOL) for _ in range(rng.randint(0, 40))) for _ in range(n)]


def corpus():
    return (synth.make_corpus(1500, 1024, seed=3) + synth.make_corpus(400, 1024, seed=4, vocab="zipf")
            + adversarial_corpus() + fuzz(3000, 5) + ["", " ", "'", "a" * 63, "a" * 64, "a" * 65, "x" * 200,
                                                       "<|endoftext|>", "a<|endoftext|>b", " \n "])


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    d = tmp_path_factory.mktemp("tok")
    return train_synthetic_bpe(str(d / "bpe4k.json"), vocab_size=4000, n_docs=1500, seed=2)


def native_counts(model, texts):
    data, off = synth.pack(texts)
    sp = model.bpe_spec()
    assert sp is not None
    raw = native.host().bpe_count(data, off, sp.byte_id, sp.keys, sp.vals, sp.mask, sp.added, sp.added_off,
                                  sp.post_add, 4)
    return raw, model.count_native(data, off, 4)


def check_equal(model, texts, max_host_frac=0.2):
    raw, full = native_counts(model, texts)
    ref = np.array(model.count(texts))
    ok = raw >= 0
    bad = np.nonzero(ok & (raw != ref))[0]
    assert not len(bad), [(texts[k][:60], int(raw[k]), int(ref[k])) for k in bad[:5]]
    np.testing.assert_array_equal(full, ref)  # host fallback fills the rest exactly
    assert (~ok).mean() <= max_host_frac
    return raw


def test_ascii_fast_path_matches_class_table():
    c1, c2 = native.host().bpe_classes()

    def table(c):
        return (int(c2[int(c1[c >> 7]) * 8 + ((c & 127) >> 4)]) >> (2 * (c & 15))) & 3

    def fast(c):
        ch = chr(c)
        if ch.isascii() and ch.isalpha():
            return 1
        if ch.isdigit():
            return 2
        if c == 32 or 9 <= c <= 13:
            return 3
        return 0

    assert [table(c) for c in range(128)] == [fast(c) for c in range(128)]
    # non-ASCII spot checks (letter, number, whitespace, other; U+1C89 is newer than this box's ICU)
    assert [table(c) for c in (0xE9, 0x0663, 0x3000, 0x2014, 0x1C89, 0x0301)] == [1, 2, 3, 0, 1, 0]


def test_gpt2_fixture_counts_equal_tokenizers():
    raw = check_equal(TokenCounterModel(GPT2_FIXTURE), corpus())
    assert raw[-4] >= 0  # a 200-byte pre-token: merged natively (bpe_word_long)
    assert raw[-3] == -2 and raw[-2] == -2  # added-token text goes to the tokenizer


def test_trained_bpe_counts_equal_tokenizers(trained):
    m = TokenCounterModel(trained)
    assert m.bpe_spec().mask + 1 >= 2 * 3000
    check_equal(m, corpus())


def test_long_pretokens_are_counted_natively(trained):
    """Pre-tokens over the 64-byte lane arrays (URLs, base64, indentation and dash runs, long letter
    runs) are merged by bpe_word_long, not sent to the host tokenizer: every document up to the
    2048-byte pre-token limit gets the tokenizers count."""
    m = TokenCounterModel(trained)
    rng = np.random.default_rng(21)
    texts = synth.inject_long_tokens(synth.make_corpus(600, 700, seed=22), 0.5, seed=1)
    texts += [synth.long_tokens(rng) for _ in range(300)]
    texts += ["a" * 2048, "b" * 2049, " " * 3000 + "x", "x" + "-" * 700 + "y", "ab" * 1500]
    raw = check_equal(m, texts, max_host_frac=0.01)
    long_ok = [t for t in texts if max(map(len, t.split()), default=0) <= 2048 and "b" * 2049 not in t
               and " " * 2049 not in t and "ab" * 1100 not in t]
    assert (raw[[texts.index(t) for t in long_ok]] >= 0).all()
    assert raw[texts.index("b" * 2049)] == -2  # over the device limit: the host tokenizer


def test_template_post_processor_adds_its_tokens(trained, tmp_path):
    tj = json.load(open(trained))
    tj["post_processor"] = {
        "type": "TemplateProcessing",
        "single": [{"SpecialToken": {"id": "<|endoftext|>", "type_id": 0}}, {"Sequence": {"id": "A", "type_id": 0}},
                   {"SpecialToken": {"id": "<|endoftext|>", "type_id": 0}}],
        "pair": [{"Sequence": {"id": "A", "type_id": 0}}, {"Sequence": {"id": "B", "type_id": 1}}],
        "special_tokens": {"<|endoftext|>": {"id": "<|endoftext|>", "ids": [0], "tokens": ["<|endoftext|>"]}}}
    p = tmp_path / "tpl.json"
    p.write_text(json.dumps(tj))
    m = TokenCounterModel(str(p))
    assert m.bpe_spec().post_add == 2
    check_equal(m, synth.make_corpus(300, 600, seed=8) + fuzz(300, 9) + [""])


def test_unsupported_tokenizers_have_no_spec():
    bert = os.path.join(REPO, "tests", "fixtures", "tokenizers", "bert-base-uncased", "tokenizer.json")
    assert TokenCounterModel(bert).bpe_spec() is None  # WordPiece: host tokenizer
    tj = json.load(open(GPT2_FIXTURE))
    for k, v in (("normalizer", {"type": "Lowercase"}), ("truncation", {"max_length": 8})):
        assert build_bpe_spec(dict(tj, **{k: v})) is None
    pt = dict(tj["pre_tokenizer"], add_prefix_space=True)
    assert build_bpe_spec(dict(tj, pre_tokenizer=pt)) is None


def _cfg():
    return load_pipeline_config_str(
        "pipeline:\n"
        "  - {type: C4QualityFilter, split_paragraph: true, remove_citations: true, filter_no_terminal_punct: false,"
        " min_num_sentences: 1, min_words_per_line: 1, max_word_length: 1000, filter_lorem_ipsum: true,"
        " filter_javascript: true, filter_curly_bracket: true, filter_policy: true}\n"
        "  - {type: GopherQualityFilter, min_doc_words: 20, max_doc_words: 100000, min_avg_word_length: 2.0,"
        " max_avg_word_length: 12.0, max_symbol_word_ratio: 0.2, max_bullet_lines_ratio: 0.9,"
        " max_ellipsis_lines_ratio: 0.5, max_non_alpha_words_ratio: 0.9, min_stop_words: 0, stop_words: []}\n"
        "  - {type: TokenCounter, tokenizer_name: gpt2}\n")


def test_emulated_device_token_counts_equal_cpu(trained):
    """Engine(emulate): K16 stays on with the trailing TokenCounter and the counts come from the
    kernel's algorithm over the kept outputs; outputs (token_count metadata included) equal the CPU
    path's."""
    from test_emulated_device_path import outputs

    from textblaster_amd.pipeline.engine import Engine

    texts = synth.make_corpus(2500, 900, seed=12) + fuzz(200, 13) + ["<|endoftext|> is here and so are we all."]
    data, off = synth.pack(texts)
    eng = Engine(_cfg(), backend="emulate", nthreads=4, keep_reasons=True, tokenizer_file=trained)
    assert eng.device_runner.resolve_blob is not None and eng.device_runner.bpe
    res = eng.submit(data, off)
    assert res.dev.resolved is not None and res.dev.resolved.tokens
    from textblaster_amd.utils import metrics

    h0, d0 = metrics.BPE_HOST_DOCS_TOTAL._value.get(), metrics.BPE_DEVICE_DOCS_TOTAL._value.get()
    a = eng.finish(res)
    # the fallback rate is observable: every kept document is counted once, on the host (added-token
    # text, a pre-token over 64 bytes) or from the device path
    nh = metrics.BPE_HOST_DOCS_TOTAL._value.get() - h0
    nd = metrics.BPE_DEVICE_DOCS_TOTAL._value.get() - d0
    assert nd > 0 and nh + nd == a.n_kept
    b = Engine(_cfg(), backend="cpu", nthreads=4, keep_reasons=True, tokenizer_file=trained,
               segmentation="icu").process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    oa, ob = outputs(a), outputs(b)
    assert oa == ob
    kept_meta = [m for k, t, m in oa.values() if k == "kept"]
    assert kept_meta and all(b'"token_count"' in m for m in kept_meta)


@pytest.mark.gpu
def test_device_token_counts_equal_cpu(trained):
    from test_emulated_device_path import outputs

    from textblaster_amd.ops import hiprt
    from textblaster_amd.pipeline.engine import Engine

    assert hiprt.device_count() > 0
    texts = synth.make_corpus(6000, 1000, seed=14) + fuzz(400, 15) + ["<|endoftext|> is here and so are we all."]
    data, off = synth.pack(texts)
    eng = Engine(_cfg(), backend="cuda", keep_reasons=True, tokenizer_file=trained)
    assert eng.device_runner.resolve_t is not None and eng.device_runner.bpe
    a = eng.process(data, off)
    b = Engine(_cfg(), backend="cpu", nthreads=8, keep_reasons=True, tokenizer_file=trained,
               segmentation="icu").process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    assert outputs(a) == outputs(b)


@pytest.mark.gpu
def test_bpe_kernel_equals_host(trained):
    """k_bpe_count directly on packed documents (no K16 count pointer) vs the host emulation."""
    from textblaster_amd.ops import hiprt
    from textblaster_amd.ops.kernels import Kernels

    m = TokenCounterModel(trained)
    texts = corpus()
    data, off = synth.pack(texts)
    raw, _ = native_counts(m, texts)
    k = Kernels(0)
    tabs = k.bpe_tables(m.bpe_spec())
    d_text = hiprt.to_device(np.concatenate([data, np.zeros(16, np.uint8)]))
    d_off = hiprt.to_device(off)
    out = hiprt.zeros(len(texts), np.int32)
    k.bpe_count(tabs, d_text, d_off, None, len(texts), out)
    np.testing.assert_array_equal(out.to_host(), raw)
