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


# ---- in-pipeline matching (device pass + host draws), emulated on the CPU -------------------
def _bw_corpus(n, seed):
    """Synthetic web documents with list words sprinkled in (some on word boundaries, some
    inside words), plus per-document language metadata."""
    rng = random.Random(seed)
    texts = synth.make_corpus(n, 700, seed=seed)
    out = []
    for k, t in enumerate(texts):
        if k % 40 == 7:
            t = (t + "\n") * 12  # long documents: matches deep in later k_badwords_match segments
        r = rng.random()
        if r < 0.25:
            w = rng.choice(["dummybadword", "Exact Phrase", "GRIMT", "xdummybadwordx", "co-op"])
            cut = rng.randrange(len(t) + 1) if k % 40 != 7 else len(t) - rng.randrange(1, 40)
            t = t[:cut] + " " + w + " " + t[cut:]
        out.append(t)
    meta = [(b'{"language":"%s"}' % rng.choice([b"en", b"da", b"ja", b"zz"])) if i % 3 else b""
            for i in range(len(out))]
    return out, meta


def _pack_meta(meta):
    md = np.frombuffer(b"".join(meta), np.uint8).copy()
    mo = np.zeros(len(meta) + 1, np.int64)
    np.cumsum([len(m) for m in meta], out=mo[1:])
    mv = np.array([1 if m else 0 for m in meta], np.uint8)
    return md, mo, mv


BW_PIPE = """pipeline:
  - {type: GopherQualityFilter, min_doc_words: 20, max_doc_words: 100000, min_stop_words: 1}
%(pre)s  - {type: C4BadWordsFilter, keep_fraction: %(kf)s, fail_on_missing_language: false, default_language: en, seed: 11}
%(post)s  - {type: FineWebQualityFilter, line_punct_thr: 0.12, line_punct_exclude_zero: false, short_line_thr: 0.67, short_line_length: 30, char_duplicates_ratio: 0.01, new_line_ratio: 0.3}
%(tc)s"""
C4 = ("  - {type: C4QualityFilter, split_paragraph: true, remove_citations: true, filter_no_terminal_punct: false, "
      "min_num_sentences: 1, min_words_per_line: 1, max_word_length: 1000, filter_lorem_ipsum: true, "
      "filter_javascript: true, filter_curly_bracket: true, filter_policy: true}\n")
TC = "  - {type: TokenCounter, tokenizer_name: gpt2}\n"


CASES = [("pre", 0.4, True), ("pre", 0.0, False), ("post", 0.4, False), ("none", 1.0, True)]


@pytest.mark.parametrize("c4_where,kf,tc", CASES)
def test_emulated_inpipeline_badwords_equals_cpu(tmp_path, c4_where, kf, tc):
    """The GPU backend's flow (matches from the device pass, draws + decisions on the host, K16
    outputs with badwords-filtered documents moved to the excluded side) == the CPU oracle.
    A C4 rewrite after the step disables K16 (host assembly)."""
    _inpipeline_case(tmp_path, c4_where, kf, tc, "emulate")


@pytest.mark.gpu
@pytest.mark.parametrize("c4_where,kf,tc", CASES)
def test_device_inpipeline_badwords_equals_cpu(tmp_path, c4_where, kf, tc):
    """Same on the MI355X: k_badwords_match in the batch's pass sequence."""
    _inpipeline_case(tmp_path, c4_where, kf, tc, "cuda")


def _inpipeline_case(tmp_path, c4_where, kf, tc, backend):
    import os

    write_lists(tmp_path)
    texts, meta = _bw_corpus(1200, seed=21)
    data, off = synth.pack(texts)
    y = BW_PIPE % dict(pre=C4 if c4_where == "pre" else "", post=C4 if c4_where == "post" else "", kf=kf,
                       tc=TC if tc else "")
    cfg = parse_pipeline_config(y)
    tok_dir = os.path.join(os.path.dirname(__file__), "fixtures", "tokenizers")
    kw = dict(keep_reasons=True, badwords_dir=str(tmp_path), nthreads=4, tokenizer_dir=tok_dir)
    ea = Engine(cfg, backend=backend, **kw)
    a = ea.process(data, off, _pack_meta(meta))
    b = Engine(cfg, backend="cpu", segmentation="icu", **kw).process(data, off, _pack_meta(meta))
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    oa, ob = rows_out(a), rows_out(b)
    assert oa == ob
    bw_i = [i for i, s in enumerate(cfg.pipeline) if s.type == "C4BadWordsFilter"][0]
    n_bw = int(np.count_nonzero(b.fail_step == bw_i))
    assert n_bw > 20 if kf < 1.0 else n_bw == 0  # the step filtered documents (none at keep_fraction 1)
    if 0 < kf < 1 and c4_where != "post":
        # K16 stayed on: some kept-on-device documents were moved by the host's draws
        assert len(a.excluded) == 2


def test_emulated_badwords_pipelined_keeps_draw_order(tmp_path):
    """process_many over several batches draws the keep-fraction numbers in document order
    across batches, like the sequential CPU path."""
    write_lists(tmp_path)
    cfg = parse_pipeline_config(BW_PIPE % dict(pre="", post="", kf=0.5, tc=""))
    kw = dict(keep_reasons=True, badwords_dir=str(tmp_path), nthreads=4)
    batches = []
    for s in range(4):
        t, m = _bw_corpus(300, seed=40 + s)
        d, o = synth.pack(t)
        batches.append((d, o, _pack_meta(m)))
    a = [rows_out(r) for r in Engine(cfg, backend="emulate", **kw).process_many(batches)]
    eb = Engine(cfg, backend="cpu", segmentation="icu", **kw)
    b = [rows_out(eb.process(*x)) for x in batches]
    assert a == b


def test_meta_languages_and_gather_spans():
    h = native.host()
    meta = [b'{"language":"da","x":"1"}', b"", b'{"y":"z"}', b'{"language":"en"}', b"not json", b'{"language":"da"}']
    md, mo, mv = _pack_meta(meta)
    codes, names = h.meta_languages(md, mo, mv, 2)
    langs = [names[c] if c >= 0 else None for c in codes]
    assert langs == ["da", None, None, "en", None, "da"]
    t = np.frombuffer(b"aaabbcdddd", np.uint8).copy()
    o = np.array([0, 3, 5, 6, 10], np.int64)
    d, no = h.gather_spans(t, o, np.array([3, 1], np.int64), 2)
    assert bytes(d) == b"ddddbb" and list(no) == [0, 4, 6]
    with pytest.raises(ValueError):
        h.gather_spans(t, o, np.array([4], np.int64), 2)


@pytest.mark.parametrize("lang", ["en", "da", "ja"])
def test_hashed_table_walk_equals_host_matcher(tmp_path, lang):
    """bw_match_batch (the kernel's hashed-table walk, csrc/common/badwords.h) == the ICU
    oracle (BadWordsModule.matches) for every document, including dead/no-list skips."""
    write_lists(tmp_path)
    h = native.host()
    bw = h.BadWordsModule(str(tmp_path))
    for l in LISTS:
        bw.lookup(l)
    fe, ec, et, term, roots, cjk = bw.flatten()
    term = np.ascontiguousarray(term, dtype=np.uint8)
    tab = h.bw_build_table(fe, np.ascontiguousarray(ec).view(np.uint32), et, term)
    texts = corpus(1500, seed=hash(lang) & 0xFFF) + ["", "dummybadword", "日本語悪い", "ΣΑΣ."]
    data, off = synth.pack(texts)
    m = h.bw_match_batch(data, off, tab, root0=roots[lang], cjk0=int(cjk[lang]), nthreads=2)
    ref = np.array([bw.matches(lang, t) for t in texts])
    np.testing.assert_array_equal(m == 1, ref)
    dead = np.zeros(len(texts), np.uint8)
    dead[::5] = 2
    dead[1::5] = 3
    m2 = h.bw_match_batch(data, off, tab, root0=roots[lang], cjk0=int(cjk[lang]), dead=dead, dead_max=2)
    assert np.all(m2[::5] == -1) and np.array_equal(m2[1::5], m[1::5])
    roots_arr = np.full(len(texts), roots[lang], np.int32)
    roots_arr[::7] = -1
    m3 = h.bw_match_batch(data, off, tab, roots=roots_arr, cjk=np.full(len(texts), int(cjk[lang]), np.uint8))
    assert np.all(m3[::7] == -1)
