"""Language-ID models (csrc/common/langid.h): the stage emulation's record (langid_record, the
device algorithm run on the host) equals the host model's decision for every document (v3
fastText + MFMA head), the v3 integer head agrees with a plain fp32/f64
reference of the same model, the deterministic exp matches libm, the featurizer emits the
documented 1..4-grams, and model files are validated on load."""
import math

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
    assert lid.version == 3
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


def _float_reference(lid, text):
    """Plain fp64 fastText inference of the v3 model (no doc-vector quantisation):
    (language, confidence, logits)."""
    logits = lid.float_logits(text)
    if logits is None:
        return -1, 0.0, None
    p = np.exp(logits - logits.max())
    p /= p.sum()
    return int(np.argmax(logits)), float(p.max()), logits


def test_v3_mfma_head_matches_float_reference():
    """The integer head (block-exponent bf16 doc vector x integer bf16 weights: what the MFMA tile
    computes) vs. fp64 inference of the same model: same language unless the top two logits are
    within the doc vector's quantisation error, confidence within 0.015."""
    lid = load_default()
    assert lid.version == 3
    m = lid.native()
    texts = synth.make_corpus(300, 700, seed=11) + EDGE
    near = 0
    for t in texts:
        lang, conf = m.detect(t)
        ref_lang, ref_conf, logits = _float_reference(lid, t)
        if logits is None:
            assert lang == -1
            continue
        top2 = np.sort(logits)[-2:]
        if lang != ref_lang:
            assert top2[1] - top2[0] < 0.05, (t[:40], lang, ref_lang, logits)
            near += 1
            continue
        assert abs(conf - ref_conf) < 0.015, (t[:40], conf, ref_conf)
    assert near <= 2


def test_v3_integer_head_reproduced_in_numpy():
    """The v3 record from first principles: exact embedding sums, the block exponent and the
    half-even quantisation in Python integers, the integer head, softmax in f64."""
    h = native.host()
    lid = load_default()
    m = lid.native()
    E = lid.E.reshape(h.LID_BUCKETS, h.LID_ROW_DIM).astype(np.int64)
    W = lid.W.reshape(h.LID_DIM, h.LID_LANGS).astype(np.int64)
    for t in synth.make_corpus(120, 600, seed=5) + EDGE:
        g, order = h.langid_buckets(t, True)
        g, hi = np.asarray(g, dtype=np.int64), np.asarray(order) >= 3
        cnt, sums = m.sums(t)
        assert cnt == len(g)
        if cnt == 0:
            assert m.detect(t)[0] == -1
            continue
        S = np.concatenate([E[g[~hi]].sum(0), E[g[hi]].sum(0)])  # 1-2-gram bag | 3-4-gram bag
        assert list(S) == list(sums)
        smax = int(np.abs(S).max())
        e = 0
        while e < 30 and (smax << (e + 1)) <= 255 * cnt:
            e += 1
        a = []
        for v in S.tolist():
            num = abs(v) << e
            q, r = divmod(num, cnt)
            if 2 * r > cnt or (2 * r == cnt and q & 1):
                q += 1
            a.append(-q if v < 0 else q)
        assert max(abs(x) for x in a) <= 255
        C = np.asarray(a, dtype=np.int64) @ W
        assert np.abs(C).max() < 2 ** 24  # exact in the MFMA's fp32 accumulator
        logits = C.astype(np.float64) * math.ldexp(lid.w_scale, -e) + lid.b[:h.LID_LANGS].astype(np.float64)
        p = np.exp(logits - logits.max())
        lang, conf = m.detect(t)
        assert lang == int(np.argmax(logits))
        assert abs(conf - 1.0 / p.sum()) < 1e-12


def test_lid_exp_matches_libm():
    h = native.host()
    xs = np.concatenate([-np.geomspace(1e-12, 740, 4000), [0.0, -0.5, -1.0, -math.log(2) / 2]])
    for x in xs:
        ref = math.exp(x)
        got = h.lid_exp(float(x))
        assert abs(got - ref) <= 4e-16 * ref + 1e-310, (x, got, ref)
    assert h.lid_exp(-800.0) == 0.0


def test_model_file_validation(tmp_path):
    h = native.host()
    good = load_default()
    p = tmp_path / "bad.npz"
    np.savez(p, E=good.E, W=good.W, w_scale=good.w_scale, b=good.b[:3])
    with pytest.raises(ValueError):
        load(str(p))
    np.savez(p, P=np.zeros(8 << 16, np.int16), b=good.b)  # the removed v2 (folded table) format
    with pytest.raises(ValueError):
        load(str(p))
    np.savez(p, emb=np.zeros(4, np.uint16), w=np.zeros(4, np.uint16), b=good.b)  # the round-2 format
    with pytest.raises(ValueError):
        load(str(p))
    assert len(LANGS) == h.LID_LANGS


def test_v3_model_file_validation(tmp_path):
    h = native.host()
    good = load_default()
    p = tmp_path / "v3.npz"
    np.savez(p, E=good.E, W=good.W, w_scale=good.w_scale, b=good.b)
    assert load(str(p)).version == 3
    W = good.W.copy()
    W[3] = 300  # outside the bf16-exact integer range
    np.savez(p, E=good.E, W=W, w_scale=good.w_scale, b=good.b)
    with pytest.raises(ValueError):
        load(str(p))
    np.savez(p, E=good.E[:100], W=good.W, w_scale=good.w_scale, b=good.b)
    with pytest.raises(ValueError):
        load(str(p))
    np.savez(p, E=good.E, W=good.W, w_scale=0.0, b=good.b)
    with pytest.raises(ValueError):
        load(str(p))
    assert good.head_bf16_t().shape == (16, h.LID_DIM)
