"""C4BadWordsFilter on the device path (k_badwords_match).

CPU part: the data the kernel consumes — the flattened tries (`BadWordsModule.flatten`), the
case-fold table (`ucd_fold_tables`) and the property table — driven by a Python transcription of
the kernel's walk must reproduce the host matcher (ICU `u_foldCase`, `\\W` boundaries) on
randomized documents. GPU part: the device engine with a bad-words step equals the CPU oracle."""
import random

import numpy as np
import pytest

from textblaster_amd import native
from textblaster_amd.config import load_pipeline_config_str as parse_pipeline_config
from textblaster_amd.pipeline.engine import Engine
from textblaster_amd.utils import synth

LISTS = {
    "en": ["dummybadword", "exact phrase", "straße", "ΣΑΣ", "naïve", "co-op", "x"],
    "da": ["grimt", "æøå"],
    "ja": ["悪い", "ばか"],
}
WORDS = ["the", "Dummybadword", "DUMMYBADWORD", "dummybadwords", "xdummybadword", "exact", "phrase",
         "EXACT PHRASE", "exact  phrase", "STRASSE", "Straße", "STRAẞE", "σας", "ΣΑΣ", "NAÏVE", "co-op", "CO-OP",
         "x", "X", "xx", "grimt", "GRIMT", "ÆØÅ", "悪い", "ばか", "とても悪いです", "word", "İstanbul", "K"]
SEPS = [" ", " ", ", ", ". ", "\n", "-", "_", "'", "", "!", "\t"]


def write_lists(d):
    for lang, words in LISTS.items():
        (d / lang).write_text("\n".join(words) + "\n", encoding="utf-8")


def corpus(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(0, 12)
        out.append("".join(rng.choice(WORDS) + rng.choice(SEPS) for _ in range(k)))
    return out


def cfg_yaml(d, default_language, keep_fraction=0.0, with_c4=False):
    c4 = ("  - {type: C4QualityFilter, split_paragraph: true, remove_citations: true, filter_no_terminal_punct: "
          "false, min_num_sentences: 1, min_words_per_line: 1, max_word_length: 1000, filter_lorem_ipsum: true, "
          "filter_javascript: true, filter_curly_bracket: true, filter_policy: true}\n") if with_c4 else ""
    return (f"pipeline:\n{c4}  - {{type: C4BadWordsFilter, keep_fraction: {keep_fraction}, fail_on_missing_language: "
            f"false, default_language: {default_language}, seed: 7}}\n")


def kernel_walk(text: str, root: int, cjk: bool, auto, props, fold) -> bool:
    """Python transcription of k_badwords_match for one document."""
    fe, ec, et, term = auto
    s1, s2 = props
    f1, f2 = fold

    def prop(c):
        return int(s2[(int(s1[c >> 7]) << 7) | (c & 127)])

    def fcp(c):
        return c + int(f2[(int(f1[c >> 7]) << 7) | (c & 127)])

    def wordchar(c):
        return bool(prop(c) & (1 << 18))

    cps = [ord(ch) for ch in text]
    for s in range(len(cps)):
        if not (cjk or s == 0 or not wordchar(cps[s - 1])):
            continue
        node, j = root, s
        while j < len(cps):
            c = fcp(cps[j])
            lo, hi = int(fe[node]), int(fe[node + 1])
            nxt = -1
            while lo < hi:
                mid = (lo + hi) >> 1
                if int(ec[mid]) == c:
                    nxt = int(et[mid])
                    break
                if int(ec[mid]) < c:
                    lo = mid + 1
                else:
                    hi = mid
            if nxt < 0:
                break
            node = nxt
            j += 1
            if term[node] and (cjk or j >= len(cps) or not wordchar(cps[j])):
                return True
    return False


@pytest.mark.parametrize("lang", ["en", "da", "ja"])
def test_flattened_automaton_walk_equals_host_matcher(tmp_path, lang):
    write_lists(tmp_path)
    h = native.host()
    texts = corpus(400, seed=hash(lang) & 0xFFFF) + ["", "dummybadword", "日本語悪い", "ΣΑΣ."]
    cfg = parse_pipeline_config(cfg_yaml(tmp_path, lang))
    eng = Engine(cfg, backend="cpu", nthreads=2, badwords_dir=str(tmp_path))
    data, off = synth.pack(texts)
    res = eng.process(data, off)
    cpu_match = res.status == 1  # keep_fraction 0: filtered <=> matched
    fe, ec, et, term, roots, cjk = eng.badwords.flatten()
    s1, s2, _, _ = h.ucd_tables()
    f1, f2 = h.ucd_fold_tables()
    assert len(fe) == len(term) + 1 and fe[-1] == len(ec) == len(et)
    for i, t in enumerate(texts):
        got = kernel_walk(t, roots[lang], cjk[lang], (fe, ec, et, term), (s1, s2), (f1, f2))
        assert got == bool(cpu_match[i]), (i, t)
    assert cpu_match.sum() > 20 and (~cpu_match).sum() > 20


def test_fold_table_matches_icu_for_list_characters():
    h = native.host()
    f1, f2 = h.ucd_fold_tables()

    def fcp(c):
        return c + int(f2[(int(f1[c >> 7]) << 7) | (c & 127)])

    # simple default case folding (ICU u_foldCase, U_FOLD_CASE_DEFAULT)
    assert fcp(ord("A")) == ord("a") and fcp(ord("Σ")) == ord("σ") and fcp(ord("ς")) == ord("σ")
    assert fcp(0x212A) == ord("k") and fcp(0x1E9E) == ord("ß") and fcp(ord("ß")) == ord("ß")
    assert fcp(ord("İ")) == ord("İ")  # no simple fold (full fold is i + U+0307)
    assert fcp(0x10FFFF) == 0x10FFFF


@pytest.mark.gpu
@pytest.mark.parametrize("keep_fraction", [0.0, 0.4])
def test_device_badwords_equals_cpu(tmp_path, keep_fraction):
    from textblaster_amd.ops import hiprt

    assert hiprt.device_count() > 0
    write_lists(tmp_path)
    texts = corpus(3000, seed=3) + synth.make_corpus(500, 600, seed=4)
    meta = [(b'{"language":"%s"}' % random.Random(i).choice([b"en", b"da", b"ja", b"zz"])) if i % 4 else b""
            for i in range(len(texts))]
    data, off = synth.pack(texts)
    md = np.frombuffer(b"".join(meta), np.uint8).copy()
    mo = np.zeros(len(meta) + 1, np.int64)
    np.cumsum([len(m) for m in meta], out=mo[1:])
    mv = np.array([1 if m else 0 for m in meta], np.uint8)
    # With a C4 step in front, documents the device delegates to the CPU oracle draw their
    # keep-fraction numbers after the batch's other documents, so exact equality of the draws
    # is only expected without delegation (keep_fraction 0 makes the draws irrelevant).
    for with_c4 in ((False, True) if keep_fraction == 0.0 else (False,)):
        cfg = parse_pipeline_config(cfg_yaml(tmp_path, "en", keep_fraction, with_c4))
        kw = dict(keep_reasons=True, badwords_dir=str(tmp_path))
        a = Engine(cfg, backend="cuda", **kw).process(data, off, (md, mo, mv))
        b = Engine(cfg, backend="cpu", segmentation="icu", **kw).process(data, off, (md, mo, mv))
        np.testing.assert_array_equal(a.status, b.status)
        assert a.reasons == b.reasons
        assert rows_out(a) == rows_out(b)


def rows_out(res):
    """row -> (kept?, text, metadata); a batch result may hold several parts (delegated rows)."""
    out = {}
    for kind, parts in (("kept", res.kept), ("excluded", res.excluded)):
        for p in parts:
            for k, r in enumerate(p.rows):
                t = bytes(p.text_data[p.text_off[k]:p.text_off[k + 1]])
                m = bytes(p.meta_data[p.meta_off[k]:p.meta_off[k + 1]]) if p.meta_valid[k] else None
                out[int(r)] = (kind, t, m)
    return out
