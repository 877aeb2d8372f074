"""The GPU backend's resolve path (records -> statuses -> lazily formatted metadata), driven by
the host port of the device kernels (``backend="emulate"``), must produce exactly the CPU ICU
oracle's outputs. Runs without a GPU."""
import numpy as np
import pytest

from textblaster_amd.config import load_pipeline_config
from textblaster_amd.pipeline.engine import Engine
from textblaster_amd.utils import synth

EDGE = ["", "   ", "\n\n", "a", "a\r\nb\r\n", "Hello.\n\n\nHello.\n\nHello.", "x [1] y [2, 3]. z",
        "ΣΑΣ ΣΑΣ.", "İstanbul THE the", "cooKie policy is here.", "lorem IPSUM dolor", "{ curly }",
        "日本語のテキストです。", "mixed 日本 text. Another sentence here.", "- bullet\n- bullet\n• x...",
        "Hi?There!Again.Yes" * 3,
        "Use of coo\u212Aies here, for all.\nJavaScript is needed. Yes it is.\n[1] [2,3] [4, 5, 6] text [a] [12\n"
        "Terms of USE apply to all lines here.\nA normal line that is fine. Another one.\nPRIVACY policy.",
        "Line one [1, 2 ,3] cites [99].\n\n  Indented line with words in it.  \nEnds with ellipsis...\nok.",
        "text with LOREM IPSUM inside"]


def outputs(res):
    out = {}
    for kind, parts in (("kept", res.kept), ("excluded", res.excluded)):
        for p in parts:
            for k, r in enumerate(p.rows):
                t = bytes(p.text_data[p.text_off[k]:p.text_off[k + 1]])
                m = bytes(p.meta_data[p.meta_off[k]:p.meta_off[k + 1]]) if p.meta_valid[k] else None
                out[int(r)] = (kind, t, m)
    return out


@pytest.mark.parametrize("cfg_path", ["config/bench_pipeline.yaml", "tests/config/test_pipeline_config.yaml"])
def test_emulated_device_path_equals_cpu_oracle(cfg_path):
    cfg = load_pipeline_config(cfg_path)
    texts = synth.make_corpus(1500, 900, seed=17) + EDGE
    data, off = synth.pack(texts)
    meta = [b'{"src":"x"}' if i % 3 == 0 else b"" for i in range(len(texts))]
    md = np.frombuffer(b"".join(meta), np.uint8).copy()
    mo = np.zeros(len(meta) + 1, np.int64)
    np.cumsum([len(m) for m in meta], out=mo[1:])
    mv = np.array([1 if m else 0 for m in meta], np.uint8)
    a = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True).process(data, off, (md, mo, mv))
    b = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True).process(data, off, (md, mo, mv))
    assert (a.n_kept, a.n_excluded) == (b.n_kept, b.n_excluded)
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    oa, ob = outputs(a), outputs(b)
    assert oa.keys() == ob.keys()
    diff = [k for k in oa if oa[k] != ob[k]]
    assert not diff, (diff[:3], [oa[k] for k in diff[:1]], [ob[k] for k in diff[:1]])


def test_pipelined_equals_sequential():
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    eng = Engine(cfg, backend="emulate", nthreads=4)
    batches = [synth.pack(synth.make_corpus(300, 700, seed=s)) for s in range(4)]
    seq = [outputs(eng.process(d, o)) for d, o in batches]
    pip = [outputs(r) for r in eng.process_many(batches)]
    assert seq == pip


@pytest.mark.parametrize("lds", [256, 4096, 16384])
def test_lds_arena_does_not_change_results(host, lds):
    """Device working arrays are carved from a per-wave LDS slice first and spill to HBM scratch;
    the host emulation runs the same allocator over a stand-in buffer: records, flags and
    rewritten texts must not depend on the slice size."""
    from textblaster_amd.models.langid import load_default
    from textblaster_amd.pipeline.plan import build_plan

    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    lid = load_default().native()
    texts = synth.make_corpus(400, 1200, seed=23) + EDGE
    data, off = synth.pack(texts)
    for idx in plan.stages:
        r0, f0 = host.emulate_stage(steps, idx, data, off, 4, lid, 0)
        r1, f1 = host.emulate_stage(steps, idx, data, off, 4, lid, lds)
        np.testing.assert_array_equal(r0, r1)
        np.testing.assert_array_equal(f0, f1)
    for i in plan.c4_steps:
        a = host.emulate_c4(steps[i], data, off, 4, 0)
        b = host.emulate_c4(steps[i], data, off, 4, lds)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("spec", ["kernel@2", "oom@1"])
def test_failed_batch_is_recovered(spec):
    """A failing device batch is re-run in halves (then on the CPU path) and the run continues
    with identical outputs (fault injection, emulated device backend)."""
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    batches = [synth.pack(synth.make_corpus(200, 600, seed=s)) for s in range(3)]
    ref = [outputs(r) for r in Engine(cfg, backend="emulate", nthreads=2).process_many(batches)]
    eng = Engine(cfg, backend="emulate", nthreads=2, fault_inject=spec)
    got = [outputs(r) for r in eng.process_many(batches, on_error="recover")]
    assert got == ref
    with pytest.raises(Exception, match="injected"):
        list(Engine(cfg, backend="emulate", nthreads=2, fault_inject=spec).process_many(batches))


def test_byte_budget_split_batches():
    """Batches above the device byte budget run as sub-batches; results are merged back in order."""
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    batches = [synth.pack(synth.make_corpus(300, 700, seed=s)) for s in range(2)]
    ref = [outputs(r) for r in Engine(cfg, backend="emulate", nthreads=2).process_many(batches)]
    eng = Engine(cfg, backend="emulate", nthreads=2)
    eng.max_batch_bytes = 20000
    res = list(eng.process_many(batches))
    assert [outputs(r) for r in res] == ref
    assert [r.n_docs for r in res] == [300, 300]


def test_gopher_repetition_records_equal_oracle_on_repetitive_text(host):
    """Device GopherRepetition records (host port of the kernel: canonical n-grams, repeated-
    position bitmaps, greedy duplicate walk) equal the ICU oracle's records field by field, on
    text with many repeated n-grams (different word splits of equal text included)."""
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    gi = [i for i, s in enumerate(cfg.pipeline) if s.type == "GopherRepetitionFilter"][0]
    rng = np.random.default_rng(3)
    texts = synth.make_corpus(300, 900, seed=41)
    words = "the cat sat on the mat and the dog ran".split()
    for _ in range(200):
        k = int(rng.integers(2, 10))
        texts.append(" ".join(rng.choice(words[:k], size=int(rng.integers(20, 400)))))
    texts += ["ab c a bc ab c a bc " * 20, "a b a b a b a b a b a b a b a b", "x y z\n\nx y z\nx y z"] + EDGE
    data, off = synth.pack(texts)
    rec, fl = host.emulate_stage(steps, [gi], data, off, 4, None, 0)
    w = steps[gi].record_width()
    rec = rec.reshape(len(texts), w)
    with_dups = 0
    for i, t in enumerate(texts):
        if fl[i]:
            continue
        ref = list(host.compute_record(steps[gi], t, "icu")[0])
        with_dups += any(ref[7 + 3:])
        assert ref == list(rec[i]), (i, t[:80], ref, list(rec[i]))
    assert with_dups > 100


def test_mixed_script_delegation_is_overlapped_and_exact(monkeypatch):
    """Dictionary-script documents (5 % with a CJK / Thai snippet, 1 % CJK) without host word marks
    (TB_TUNE dict_marks=0): process_many recomputes the delegated ones on the engine's delegation thread
    while later batches are resolved; the merged results equal the CPU oracle batch for batch, and
    documents the language gate already filtered (the CJK ones) are not delegated."""
    monkeypatch.setenv("TB_TUNE", "dict_marks=0")
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    batches = [synth.pack(synth.make_corpus(600, 800, seed=40 + s, mixed_script=True)) for s in range(3)]
    emu = Engine(cfg, backend="emulate", nthreads=4)
    cpu = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4)
    got = list(emu.process_many(batches))
    assert len(got) == 3
    n_dict = 0
    for (d, o), r in zip(batches, got):
        assert r.deferred is None
        ref = cpu.process(d, o)
        np.testing.assert_array_equal(r.fail_step, ref.fail_step)
        np.testing.assert_array_equal(r.status, ref.status)
        assert outputs(r) == outputs(ref)
        texts = [bytes(d[o[i]:o[i + 1]]).decode() for i in range(len(o) - 1)]

        def dict_script(ch):
            return "\u0e00" <= ch <= "\u0e7f" or "\u3040" <= ch <= "\u30ff" or "\u4e00" <= ch <= "\u9fff"

        dict_docs = [t for t in texts if any(dict_script(ch) for ch in t)]
        cjk_docs = [t for t in dict_docs if sum(ch.isascii() for ch in t) < len(t) // 2]
        n_dict += len(cjk_docs)
        # the CJK documents fail the language gate on the device: not delegated
        assert 0 < r.n_delegated <= len(dict_docs) - len(cjk_docs), (r.n_delegated, len(dict_docs), len(cjk_docs))
    assert n_dict > 0


def test_split_tasks_equal_one_pass_and_fit_the_reservation(host):
    """The intra-document n-gram split (stage export, then one k_gr_dup_split task per order and
    for duplicated lines / paragraphs, each in its slice of the document's arena) gives the same
    records as the one-pass stage, and neither path outgrows the devplan.h reservation
    (kScratchPerByte / kScratchPerByteSplit, sized by tools/scratch_need.py)."""
    from textblaster_amd.models.langid import load_default
    from textblaster_amd.pipeline.plan import build_plan

    lid = load_default().native()
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    gr = [steps[i] for i, s in enumerate(cfg.pipeline) if s.type == "GopherRepetitionFilter"][0]
    tasks = gr.n_dup + gr.n_top + 2
    texts = synth.make_corpus(120, 3000, seed=43) + EDGE + ["a " * 3000, "a\n" * 3000, "A b. " * 1200,
                                                             "x [1] " * 900, "a b.\n\n" * 900]
    data, off = synth.pack(texts)
    host.set_scratch_probe(True)
    try:
        for idx in plan.stages:
            host.scratch_need(True)
            r0, f0 = host.emulate_stage(steps, idx, data, off, 4, lid, 0)
            one, _ = host.scratch_need(True)
            r1, f1 = host.emulate_stage(steps, idx, data, off, 4, lid, 0, split_tasks=tasks)
            split, _ = host.scratch_need(True)
            np.testing.assert_array_equal(f0, f1)
            np.testing.assert_array_equal(r0, r1)
            assert one <= host.SCRATCH_PER_BYTE and split <= host.SCRATCH_PER_BYTE_SPLIT, (one, split)
    finally:
        host.set_scratch_probe(False)
    # under the real reservation nothing overflows (DOC_OVERFLOW = 2, docproc.h -> CPU path)
    for idx in plan.stages:
        _, f = host.emulate_stage(steps, idx, data, off, 4, lid, 0, split_tasks=tasks)
        assert not (f & 2).any()


def test_language_id_after_c4_is_recomputed_for_delegated_documents(tmp_path, monkeypatch):
    """A LanguageDetectionFilter placed after C4QualityFilter reads the rewritten text. For a
    delegated (dictionary-script) document the device's rewritten text is not the CPU path's, so
    its language-ID record must not be reused: the outputs equal the CPU oracle on a mixed-script
    corpus (the presets are limited to stages that read content version 0)."""
    cfg_text = open("config/bench_pipeline.yaml").read()
    lid = "  - {type: LanguageDetectionFilter, min_confidence: 0.65, allowed_languages: [dan, eng, swe, nob, nno]}\n"
    assert lid in cfg_text
    # (no stop-word minimum, so delegated documents get past GopherQuality and C4 to the last step)
    cfg_text = cfg_text.replace(lid, "").replace("min_stop_words: 2", "min_stop_words: 0") + \
        "  - {type: LanguageDetectionFilter, min_confidence: 0.5, allowed_languages: [dan, eng, swe, nob, nno]}\n"
    p = tmp_path / "lid_after_c4.yaml"
    p.write_text(cfg_text)
    monkeypatch.setenv("TB_TUNE", "dict_marks=0")  # dictionary-script documents go to the CPU path
    cfg = load_pipeline_config(str(p))
    assert [s.type for s in cfg.pipeline][-1] == "LanguageDetectionFilter"
    texts = synth.make_corpus(900, 800, seed=77, mixed_script=True)
    data, off = synth.pack(texts)
    emu = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True)
    cpu = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True)
    for got in (emu.process(data, off), next(iter(emu.process_many([(data, off)])))):
        ref = cpu.process(data, off)
        assert got.n_delegated > 0
        assert (ref.fail_step[np.nonzero(ref.status == 0)[0]] == -1).all()
        np.testing.assert_array_equal(got.fail_step, ref.fail_step)
        np.testing.assert_array_equal(got.status, ref.status)
        assert got.reasons == ref.reasons
        assert outputs(got) == outputs(ref)


@pytest.mark.parametrize("cfg_path", ["config/bench_pipeline.yaml", "config/pipeline_config.yaml",
                                      "config/bench_pipeline_survivor.yaml"])
def test_dictionary_scripts_stay_on_device_and_equal_oracle(cfg_path):
    """Dictionary-script documents (CJK / Thai snippets and CJK documents) keep their analysis on the
    device: the host supplies ICU word marks of the original text (stage kernels), ICU per-line word
    statistics for documents with citations (C4 pass A) and the rewrite's word count comes from C4
    (FineWeb after C4). No document is delegated, and records, statuses, reasons and outputs equal
    the CPU ICU oracle."""
    import yaml

    cfg = load_pipeline_config(cfg_path)
    if any(s.type == "TokenCounter" for s in cfg.pipeline):
        raw = yaml.safe_load(open(cfg_path))
        raw["pipeline"] = [s for s in raw["pipeline"] if s.get("type") != "TokenCounter"]
        from textblaster_amd.config.pipeline import parse_pipeline_config

        cfg = parse_pipeline_config(raw)
    texts = synth.make_corpus(2500, 900, seed=314, mixed_script=True)
    rng = np.random.default_rng(5)
    # cited dictionary-script lines, Thai, kana / han runs next to citations and line edges
    texts += ["日本語のテキストです[1]。東京は日本の首都です。\nこれは二行目です [2, 3]。",
              "ภาษาไทย [4] สวัสดีครับ.\n\nประเทศไทย is a country [5].",
              "Mixed 中文分词测试 text [6] with more words here. " * 8]
    data, off = synth.pack(texts)
    emu = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True)
    cpu = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True)
    a, b = emu.process(data, off), cpu.process(data, off)
    n_dict = sum(1 for t in texts if emu.h.has_dict_script(t))
    assert n_dict > 100
    assert a.n_delegated == 0
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    assert outputs(a) == outputs(b)
