"""Language-ID model (csrc/common/langid.h): the stage emulation's record (langid_record, the
device algorithm run on the host) equals the host model's decision for every document, the
featurizer emits the documented 1..4-grams, and the model file is validated on load."""
import numpy as np
import pytest

from textblaster_amd import native
from textblaster_amd.config import load_pipeline_config_str
from textblaster_amd.models.langid import LANGS, load, load_default
from textblaster_amd.pipeline.plan import build_plan
from textblaster_amd.utils import synth

EDGE = ["", "1234 !!!", "a", "ab", "abc", "Å", "ø ø øø øøø øøøø", "x" * 5000, ("ø" * 4095) + "abc def",
        "blåbærgrød og æblegrød", "The quick brown fox.", "Hvorfor kjem du ikkje?", "ΣΑΣ ΣΑΣ."]


def test_stage_emulation_record_equals_host_model():
    h = native.host()
    lid = load_default()
    cfg = load_pipeline_config_str(
        "pipeline:\n  - {type: LanguageDetectionFilter, min_confidence: 0.65, allowed_languages: [dan]}\n")
    steps = [h.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    texts = synth.make_corpus(400, 900, seed=3) + EDGE
    data, off = synth.pack(texts)
    rec, flags = h.emulate_stage(steps, plan.stages[0], data, off, 4, lid.native())
    rec = rec.reshape(len(texts), -1)
    m = lid.native()
    for i, t in enumerate(texts):
        lang, conf = m.detect(t)
        assert int(rec[i, 0]) == lang, (i, t[:40])
        if lang >= 0:
            assert rec[i, 1:2].view(np.float64)[0] == conf


def test_featurizer_gram_counts():
    h = native.host()
    # "ab": <a ab b> a> -> 1-grams a, b; 2-grams <a, ab; 3-grams <ab; end: b>, ab>, <ab> (4-gram)
    assert len(h.langid_buckets("ab")) == 2 + 2 + 1 + 3
    assert len(h.langid_buckets("")) == 0 and len(h.langid_buckets("123 !!")) == 0
    # 4-grams appear from the third letter on
    assert len(h.langid_buckets("abcd")) == 4 * 1 + 4 * 1 + 3 * 1 + 2 * 1 + 3
    assert all(0 <= b < h.LID_BUCKETS for b in h.langid_buckets("Blåbærgrød Øresund"))


def test_model_file_validation(tmp_path):
    h = native.host()
    good = load_default()
    p = tmp_path / "bad.npz"
    np.savez(p, P=good.P, b=good.b[:3])
    with pytest.raises(ValueError):
        load(str(p))
    P = good.P.copy().reshape(-1, h.LID_ROW)
    P[5, h.LID_LANGS] = 1  # padding column must stay zero
    np.savez(p, P=P.reshape(-1), b=good.b)
    with pytest.raises(ValueError):
        load(str(p))
    np.savez(p, emb=np.zeros(4, np.uint16), w=np.zeros(4, np.uint16), b=good.b)  # the round-2 format
    with pytest.raises(ValueError):
        load(str(p))
    assert len(LANGS) == h.LID_LANGS
