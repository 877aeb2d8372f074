"""Gopher repetition / quality filters and the text helpers they use (ports reference
gopher_rep.rs and gopher_quality.rs test modules)."""
import pytest

from textblaster_amd.data_model import TextDocument
from textblaster_amd.errors import DocumentFiltered
from textblaster_amd.pipeline.steps import GopherQualityFilter, GopherRepetitionFilter
from textblaster_amd.utils.text import find_all_duplicate, find_duplicates, find_top_duplicate, get_n_grams


def doc(content, id_="d"):
    return TextDocument(id=id_, source="test", content=content)


@pytest.fixture(params=["icu", "rules"])
def seg(request):
    return request.param


def reason_of(step, content):
    with pytest.raises(DocumentFiltered) as ei:
        step.process(doc(content))
    return ei.value.reason


# ---- helpers ----------------------------------------------------------------------------------

def test_get_n_grams():
    w = ["a", "b", "c", "d"]
    assert get_n_grams(w, 2) == ["a b", "b c", "c d"]
    assert get_n_grams(w, 1) == w
    assert get_n_grams(w, 4) == ["a b c d"]
    assert get_n_grams(w, 5) == []
    assert get_n_grams([], 2) == []
    assert get_n_grams(w, 0) == []


def test_find_duplicates():
    assert find_duplicates(["a", "b", "c"]) == (0, 0)
    assert find_duplicates(["a", "b", "a"]) == (1, 1)
    assert find_duplicates(["ab", "cd", "ab", "ef", "cd"]) == (2, 4)
    assert find_duplicates(["a", "a", "a"]) == (2, 2)
    assert find_duplicates([]) == (0, 0)


def test_find_top_duplicate():
    assert find_top_duplicate(["a", "a"]) == 2
    assert find_top_duplicate(["a", "a", "b", "b"]) == 2
    assert find_top_duplicate(["a b", "c d", "a b"]) == 6
    assert find_top_duplicate(["a", "b", "c"]) == 0
    assert find_top_duplicate(["aa", "aa", "b", "b"]) == 4
    assert find_top_duplicate(["a", "a", "a"]) == 3
    assert find_top_duplicate([]) == 0
    assert find_top_duplicate(["unique"]) == 0


def test_find_all_duplicate():
    assert find_all_duplicate(["a", "b", "c", "d", "e"], 2) == 0
    assert find_all_duplicate(["a", "b", "c", "d", "e"], 3) == 0
    assert find_all_duplicate(["a", "b", "c", "a", "b", "d"], 2) == 2
    assert find_all_duplicate(["a", "b", "a", "b", "a", "b"], 2) == 4
    assert find_all_duplicate(["a"] * 5, 2) == 4
    assert find_all_duplicate([], 2) == 0
    assert find_all_duplicate(["a", "b", "c", "d", "e"], 0) == 0
    assert find_all_duplicate(["a", "b", "c", "d", "e"], 6) == 0


# ---- repetition filter ------------------------------------------------------------------------

def rep(seg):
    return GopherRepetitionFilter(segmentation=seg)


def test_rep_permissive(seg):
    rep(seg).process(doc("This is a normal document.\nIt has multiple lines.\n\nAnd multiple paragraphs."))


def test_duplicate_paragraphs(seg):
    p1, p2 = "This is the first paragraph.", "This is the second paragraph."
    ok = f"{p1}\n\n{p2}\n\nAnother unique."
    f = rep(seg)
    f.dup_para_frac = 0.3
    f.process(doc(ok))
    assert "dup_para_frac (ratio 0.33, max 0.30)" in reason_of(f, f"{p1}\n\n{p2}\n\n{p1}")
    bad = f"{p1}\n\n{p1}\n\n{p1}"
    g = rep(seg)
    g.dup_para_char_frac = 2 * len(p1) / len(bad) - 0.01
    g.process(doc(ok))
    assert "dup_para_char_frac" in reason_of(g, bad)


def test_duplicate_lines(seg):
    l1, l2 = "This is line one.", "This is line two."
    ok = f"{l1}\n{l2}\nUnique line"
    f = rep(seg)
    f.dup_line_frac = 0.3
    f.process(doc(ok))
    assert "dup_line_frac (ratio 0.33, max 0.30)" in reason_of(f, f"{l1}\n{l2}\n{l1}")
    bad = f"{l1}\n{l1}\n{l1}"
    thr = 2 * len(l1) / len(bad) - 0.01
    g = rep(seg)
    g.dup_line_char_frac = thr
    g.process(doc(ok))
    r = reason_of(g, bad)
    assert r.startswith("dup_line_char_frac (ratio")
    assert f"max {thr:.2f}" in r


def test_top_n_grams(seg):
    f = rep(seg)
    f.top_n_grams = [(2, 0.3)]
    f.process(doc("a b c d e f a b g h i j"))
    assert "top_2_gram" in reason_of(f, "a b c a b d a b e a b")


def test_duplicate_n_grams(seg):
    f = rep(seg)
    f.dup_n_grams = [(2, 0.1)]
    assert "duplicated_2_n_grams" in reason_of(f, "a b c d e a b f g")
    f.process(doc("a b c d e f g h i"))


# ---- quality filter ---------------------------------------------------------------------------

def q(seg, **kw):
    f = GopherQualityFilter(segmentation=seg)
    for k, v in kw.items():
        setattr(f, k, v)
    return f


def test_quality_permissive(seg):
    q(seg).process(doc("This is a perfectly normal document with the and of words."))


def test_min_doc_words(seg):
    f = q(seg, min_doc_words=3)
    f.process(doc("Hello world test . !"))
    assert "gopher_short_doc (2 non-symbol words, required 3)" in reason_of(f, "Hello world . !")
    assert "gopher_short_doc (0 non-symbol words, required 3)" in reason_of(f, ". ! ?")


def test_max_doc_words(seg):
    f = q(seg, max_doc_words=3)
    f.process(doc("One two three ."))
    assert "gopher_long_doc (4 non-symbol words, max 3)" in reason_of(f, "One two three four .")


def test_avg_word_length(seg):
    f = q(seg, min_avg_word_length=3.0, max_avg_word_length=5.0)
    f.process(doc("cat words test ."))
    assert "gopher_below_avg_threshold (avg len 1.50, required 3.00)" in reason_of(f, "a it .")
    assert "gopher_above_avg_threshold (avg len 7.00, max 5.00)" in reason_of(f, "testing another .")
    assert ("gopher_below_avg_threshold (avg len 0.00, required 3.00 - 0 non-symbol words)"
            in reason_of(f, ". ! ."))


def test_symbol_word_ratio(seg):
    f = q(seg, max_symbol_word_ratio=0.1)
    f.process(doc("word1 word2 # word3 word4 word5 word6 word7 word8 word9 word10"))
    assert "gopher_too_many_hashes (ratio 0.25, max 0.10)" in reason_of(
        f, "word1 # word2 # word3 word4 word5 word6 word7 word8")
    f.process(doc(""))
    assert "gopher_too_many_hashes (ratio 1.00, max 0.10)" in reason_of(f, "#")
    f.process(doc("word1 word2 ... word3 word4 word5 word6 word7 word8 word9 word10"))
    assert "gopher_too_many_ellipsis_units (ratio 0.25, max 0.10)" in reason_of(
        f, "word1 ... word2 … word3 word4 word5 word6 word7 word8")


def test_bullet_lines(seg):
    f = q(seg, max_bullet_lines_ratio=0.5)
    f.process(doc("- item 1\n- item 2\nnormal line\nanother normal line"))
    assert "gopher_too_many_bullets (ratio 0.75, max 0.50)" in reason_of(f, "- item 1\n- item 2\n- item 3\nnormal line")
    f.process(doc(""))
    assert "gopher_too_many_bullets (ratio 1.00, max 0.50)" in reason_of(f, "- all bullets")


def test_ellipsis_lines(seg):
    f = q(seg, max_ellipsis_lines_ratio=0.5)
    f.process(doc("Line one...\nLine two…\nNormal line\nAnother normal"))
    assert "gopher_too_many_end_ellipsis_lines (ratio 0.75, max 0.50)" in reason_of(
        f, "Line one...\nLine two…\nLine three...\nNormal line")


def test_alpha_ratio(seg):
    f = q(seg, max_non_alpha_words_ratio=0.5)
    f.process(doc("word 123 word !!!"))
    exp = "gopher_below_alpha_threshold (alpha ratio {:.2f}, required min 0.50)"
    assert exp.format(1 / 3) in reason_of(f, "word 123 456 !!!")
    assert exp.format(0.0) in reason_of(f, "123 456 789 !!!")
    assert exp.format(0.0) in reason_of(f, "")


def test_stop_words(seg):
    f = q(seg, min_stop_words=2)
    f.process(doc("the quick brown fox and the lazy dog"))
    assert "gopher_too_few_stop_words (found 0, required 2)" in reason_of(f, "a quick brown fox is lazy")
    g = GopherQualityFilter(None, None, None, None, None, None, None, None, 1, ["custom", "words"], segmentation=seg)
    g.process(doc("this is a custom test with other words"))
    assert "gopher_too_few_stop_words (found 0, required 1)" in reason_of(g, "this is a regular sentence")
    h = q(seg, min_stop_words=0)
    h.process(doc("no stop words here"))
    h.min_stop_words = None
    h.process(doc("no stop words here"))


def _ref_top(words, n):
    if n == 0 or len(words) < n:
        return 0
    cnt = {}
    for i in range(len(words) - n + 1):
        g = " ".join(words[i:i + n])
        cnt[g] = cnt.get(g, 0) + 1
    m = max(cnt.values())
    return 0 if m <= 1 else max(len(g.encode()) * m for g, c in cnt.items() if c == m)


def _ref_all_dup(words, n):
    if n == 0 or len(words) < n:
        return 0
    seen, rep, i = set(), 0, 0
    while i + n <= len(words):
        g = "".join(words[i:i + n])
        if g in seen:
            rep += len(g.encode())
            i += n
        else:
            seen.add(g)
            i += 1
    return rep


def test_ngram_statistics_match_string_reference():
    """The host n-gram statistics (word hashes + exact verification, no n-gram strings) equal the
    string-building definitions, including concatenations that collide across word borders
    ("ab" + "c" == "a" + "bc") and multibyte words."""
    import random

    from textblaster_amd import native

    top = native.host().find_top_duplicate
    rng = random.Random(11)
    vocab = ["a", "b", "ab", "c", "bc", "abc", "the", "æble", "øl", "á", "中文", "x"]
    for _ in range(300):
        words = [rng.choice(vocab[:rng.randint(2, len(vocab))]) for _ in range(rng.randint(0, 60))]
        for n in range(1, 11):
            assert top(words, n) == _ref_top(words, n), (words, n)
            assert find_all_duplicate(words, n) == _ref_all_dup(words, n), (words, n)
