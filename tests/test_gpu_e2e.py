"""End-to-end on the MI355X: Parquet -> device pipeline -> Parquet must equal the CPU ICU-oracle
run byte for byte (kept/excluded rows, rewritten text, metadata JSON including the language
confidence: the MFMA head's integers are exact and both sides share one explicit-fma exp).
Needs an MI355X."""
import os

import pyarrow.parquet as pq
import pytest

from textblaster_amd.data_model import TextDocument
from textblaster_amd.io.parquet import ParquetWriter
from textblaster_amd.runner import RunConfig, run
from textblaster_amd.utils import synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(REPO, "config", "bench_pipeline.yaml")


def test_device_run_equals_cpu_oracle(tmp_path):
    from textblaster_amd.ops import hiprt

    assert hiprt.device_count() > 0
    texts = synth.make_corpus(6000, 1024, seed=21) + ["", "日本語のテキストです。", "&amp; entity &lt;b&gt; text."]
    docs = [TextDocument(f"g{i}", t, "gpu", metadata={"n": str(i)} if i % 5 == 0 else {}) for i, t in enumerate(texts)]
    inp = str(tmp_path / "in.parquet")
    w = ParquetWriter(inp)
    w.write_batch(docs)
    w.close()
    outs = {}
    for backend in ("cuda", "cpu"):
        o, e = str(tmp_path / f"{backend}.o.parquet"), str(tmp_path / f"{backend}.e.parquet")
        st = run(RunConfig(inp, o, e, CFG, backend=backend, segmentation="icu", unit_rows=2048))
        outs[backend] = (st, pq.read_table(o), pq.read_table(e))
    (sg, og, eg), (sc, oc, ec) = outs["cuda"], outs["cpu"]
    assert (sg.docs, sg.kept, sg.excluded, sg.errors) == (sc.docs, sc.kept, sc.excluded, sc.errors)
    assert sg.step_filtered == sc.step_filtered
    assert og.column("id").equals(oc.column("id")) and og.column("text").equals(oc.column("text"))
    assert eg.column("id").equals(ec.column("id")) and eg.column("text").equals(ec.column("text"))
    # metadata (with the language confidence) identical, key order aside
    import json

    for a, b in zip(og.column("metadata").to_pylist() + eg.column("metadata").to_pylist(),
                    oc.column("metadata").to_pylist() + ec.column("metadata").to_pylist()):
        assert json.loads(a) == json.loads(b)


def test_device_fault_recovery(tmp_path):
    """An injected device failure on the 2nd batch is recovered (halves, then CPU) and the run's
    outputs are unchanged."""
    texts = synth.make_corpus(3000, 800, seed=5)
    inp = str(tmp_path / "in.parquet")
    w = ParquetWriter(inp)
    w.write_batch([TextDocument(f"f{i}", t, "gpu") for i, t in enumerate(texts)])
    w.close()
    res = {}
    for tag, fault in (("ok", None), ("fault", "kernel@2")):
        o, e = str(tmp_path / f"{tag}.o.parquet"), str(tmp_path / f"{tag}.e.parquet")
        st = run(RunConfig(inp, o, e, CFG, backend="cuda", unit_rows=1000, fault_inject=fault))
        res[tag] = (st.kept, st.excluded, pq.read_table(o).column("id"), pq.read_table(e).column("id"))
    assert res["ok"][:2] == res["fault"][:2]
    assert res["ok"][2].equals(res["fault"][2]) and res["ok"][3].equals(res["fault"][3])


def test_device_resolve_fast_path_equals_host_assembly(monkeypatch):
    """K16 on the GPU: k_resolve + scans + k_compact outputs are used (no fallback) and equal the
    host-assembled outputs of the same records."""
    import numpy as np

    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine
    from textblaster_amd.utils import metrics

    from test_emulated_device_path import EDGE, outputs

    cfg = load_pipeline_config(CFG)
    data, off = synth.pack(synth.make_corpus(20000, 1024, seed=33) + EDGE)
    before = metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get()
    eng = Engine(cfg, backend="cuda")
    assert eng.device_runner.resolve_t is not None
    a = eng.process(data, off)
    assert metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get() == before
    monkeypatch.setenv("TB_TUNE", "device_resolve=0")
    b = Engine(cfg, backend="cuda").process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert outputs(a) == outputs(b)


def _hard_corpus():
    """The adversarial pool (UAX#29 fuzz, chunk-boundary constructs), 4.5-90 KB documents in five
    languages and C4-heavy long documents (citations, policy / javascript lines, ellipses)."""
    import sys

    import numpy as np

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from adversarial import adversarial_corpus
    from test_emulated_device_path import EDGE

    rng = np.random.default_rng(19)
    langs = ["eng", "dan", "swe", "nob", "nno"]
    texts = synth.make_corpus(1500, 1024, seed=23) + EDGE + adversarial_corpus()
    texts += [synth.make_doc(rng, langs[k % 5], int(s)) for k, s in enumerate(np.geomspace(4500, 90000, 20))]
    texts += [synth.make_doc(rng, langs[k % 5], int(s), vocab_kind="zipf") for k, s in enumerate(np.geomspace(3000, 70000, 10))]
    c4ish = ("A line with a citation [1] and another [2, 3] here. Read our privacy policy today.\n"
             "JavaScript must be enabled. Short one...\nThe quick brown fox jumps over the lazy dog.\n"
             "Terms of use {apply} here and lorem ipsum is not.\n\n")
    texts += [c4ish * 150, (c4ish * 150).replace("\n", " "), c4ish * 600]
    return texts


@pytest.mark.parametrize("mode", ["default", "split", "pre"])
def test_device_equals_icu_oracle_on_hard_corpus(monkeypatch, mode):
    """Independent net for the device kernels: the GPU engine against the CPU ICU oracle (not the
    host emulation of the same source) on adversarial, long, split and C4-heavy documents; with
    the GopherRepetition dup orders of every >4.5 KB document split across workgroups ("split")
    and with every >=64 KB document decoded and word-segmented by the multi-workgroup pre-pass,
    the ones over 20 KB also split ("pre")."""
    import json

    import numpy as np

    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine

    from test_emulated_device_path import outputs

    if mode == "split":
        monkeypatch.setenv("TB_TUNE", "split_doc_bytes=4096")
    if mode == "pre":
        monkeypatch.setenv("TB_TUNE", "pre_doc_bytes=65536,split_doc_bytes=20000")
    cfg = load_pipeline_config(CFG)
    texts = _hard_corpus()
    data, off = synth.pack(texts)
    eng = Engine(cfg, backend="cuda", keep_reasons=True)
    if mode == "split":
        assert eng.device_runner.gr_split and eng.device_runner.split_doc_bytes <= 4608
    a = eng.process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", keep_reasons=True).process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons.keys() == b.reasons.keys()
    assert a.reasons == b.reasons  # confidences included (same exp bits on both sides)
    oa, ob = outputs(a), outputs(b)
    assert oa.keys() == ob.keys()
    bad = []
    for k in oa:
        (ka, ta, ma), (kb, tb, mb) = oa[k], ob[k]
        if ka != kb or ta != tb or (ma is None) != (mb is None):
            bad.append(k)
            continue
        if ma is not None and json.loads(ma) != json.loads(mb):
            bad.append(k)
    assert not bad, [(k, texts[k][:80]) for k in bad[:5]]
    lens = np.diff(off)
    assert np.count_nonzero(lens > 4500) >= 30


@pytest.mark.parametrize("cfg_name", ["bench_pipeline.yaml", "bench_pipeline_survivor.yaml"])
def test_device_dictionary_scripts_equal_oracle(cfg_name):
    """Mixed-script slice of the GPU-vs-ICU differential: CJK / Thai snippets,
    CJK documents, dictionary-script lines with citations, long documents (workgroup kernels) with
    snippets. The device keeps every one of them (host ICU word marks for the stage kernels, ICU line
    statistics for C4 pass A, the rewrite's word count for FineWeb): nothing is delegated, and the
    results equal the CPU ICU oracle byte for byte."""
    import numpy as np

    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine

    from test_emulated_device_path import outputs

    cfg = load_pipeline_config(os.path.join(REPO, "config", cfg_name))
    texts = synth.make_corpus(4000, 1024, seed=2718, mixed_script=True)
    rng = np.random.default_rng(11)
    for k, s in enumerate(np.geomspace(5000, 60000, 12)):
        t = synth.make_doc(rng, ["eng", "dan", "swe", "nob", "nno"][k % 5], int(s))
        cut = len(t) // 2
        texts.append(t[:cut] + " " + synth.CJK_SNIPPETS[k % len(synth.CJK_SNIPPETS)] + " [3] " + t[cut:])
    texts += ["日本語のテキストです[1]。東京は日本の首都です。\nこれは二行目です [2, 3]。",
              "ภาษาไทย [4] สวัสดีครับ.\n\nประเทศไทย is a country [5].",
              "Mixed 中文分词测试 text [6] with more words here. " * 8]
    data, off = synth.pack(texts)
    eng = Engine(cfg, backend="cuda", keep_reasons=True)
    a = eng.process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", keep_reasons=True).process(data, off)
    assert sum(1 for t in texts if eng.h.has_dict_script(t)) > 200
    assert a.n_delegated == 0
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    assert outputs(a) == outputs(b)


def test_device_equals_icu_oracle_on_megabyte_documents(monkeypatch, tmp_path):
    """The long-document bench shape (~1 MB documents: multi-workgroup pre-pass, split n-gram
    orders in the persistent k_gr_dup_split) against the CPU ICU oracle: two documents of 1-2 MB
    (one with a 60,000-type Zipf vocabulary, so the n-gram tables are large) among short ones.
    The word cap and the lorem / curly gates are lifted so that both pass GopherRepetition and
    GopherQuality, get rewritten by C4 and fail FineWeb with a ratio in the reason (an exact check
    of the device's FineWeb record of the 1-2 MB rewrites). Same decisions, rewritten text and
    metadata byte for byte."""
    import json

    import numpy as np

    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine

    from test_emulated_device_path import outputs

    monkeypatch.setenv("TB_TUNE", "pre_doc_bytes=65536,split_doc_bytes=32768")
    rng = np.random.default_rng(29)
    texts = [synth.make_doc(rng, "dan", 1_100_000), synth.make_doc(rng, "eng", 1_900_000, vocab_kind="zipf")]
    texts += synth.make_corpus(64, 1024, seed=31)
    data, off = synth.pack(texts)
    assert np.count_nonzero(np.diff(off) >= 1_000_000) == 2
    yml = open(CFG).read().replace("max_doc_words: 100000", "max_doc_words: 10000000")
    yml = yml.replace("filter_lorem_ipsum: true", "filter_lorem_ipsum: false")
    yml = yml.replace("filter_curly_bracket: true", "filter_curly_bracket: false")
    (tmp_path / "mb.yaml").write_text(yml)
    cfg = load_pipeline_config(str(tmp_path / "mb.yaml"))
    eng = Engine(cfg, backend="cuda", keep_reasons=True)
    assert eng.device_runner.pre_doc_bytes == 65536
    a = eng.process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", keep_reasons=True).process(data, off)
    assert a.n_delegated == 0
    assert list(b.fail_step[:2]) == [4, 4]  # both reach FineWeb (step 4) on the oracle
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    oa, ob = outputs(a), outputs(b)
    assert oa.keys() == ob.keys()
    for k in oa:
        (ka, ta, ma), (kb, tb, mb) = oa[k], ob[k]
        assert (ka, ta) == (kb, tb), (k, len(texts[k]))
        assert (ma is None) == (mb is None) and (ma is None or json.loads(ma) == json.loads(mb)), k
