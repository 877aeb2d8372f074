"""FineWeb quality, language detection, token counter and text-utility behaviour (ports reference
fineweb_quality.rs, language_filter.rs, token_counter.rs and utils/text.rs test modules)."""
import os

import pytest

from textblaster_amd.config.pipeline import DEFAULT_STOP_CHARS
from textblaster_amd.data_model import TextDocument
from textblaster_amd.errors import DocumentFiltered, Unexpected
from textblaster_amd.pipeline.steps import FineWebQualityFilter, LanguageDetectionFilter, TokenCounter
from textblaster_amd.utils import text as tu

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "tokenizers")


def doc(content, id_="d"):
    return TextDocument(id=id_, source="test_source", content=content)


@pytest.fixture(params=["icu", "rules"])
def seg(request):
    return request.param


def fw(seg, **kw):
    f = FineWebQualityFilter(0.12, False, 0.67, 30, 0.95, 0.3, stop_chars=DEFAULT_STOP_CHARS, segmentation=seg)
    for k, v in kw.items():
        setattr(f, k, v)
    return f


def reason_of(step, content):
    with pytest.raises(DocumentFiltered) as ei:
        step.process(doc(content))
    return ei.value.reason


# ---- FineWeb ----------------------------------------------------------------------------------

@pytest.mark.parametrize("content", ["", "   \n\t   \n ", "\n\n\n"])
def test_fineweb_empty(seg, content):
    assert reason_of(fw(seg), content) == "empty"


def test_fineweb_line_punct(seg):
    c = "Line one\nLine two\nLine three\nLine four\nLine five\nLine six\nLine seven\nLine eight\nLine nine\nLine ten."
    assert reason_of(fw(seg), c).startswith("line_punct_ratio: 0.1000 < threshold 0.1200")
    fw(seg, short_line_thr=1.0).process(doc(
        "Line one is long enough and ends with a period.\nLine two is also long enough and ends with a question "
        "mark?\nLine three is also very long indeed and ends with an exclamation mark!"))
    fw(seg, line_punct_exclude_zero=True, short_line_thr=1.0).process(doc(
        "Looooooooong line one, no punctuation here\nLooooooooong line two, also no punctuation\n"
        "Looooooooong line three, definitely no punctuation"))
    assert reason_of(fw(seg), "Line one\nLine two\nLine three").startswith(
        "line_punct_ratio: 0.0000 < threshold 0.1200")


def test_fineweb_short_lines(seg):
    c = ("Short line.\nThis is another short one.\nWay too short.\nThis line is definitely longer than thirty "
         "characters to provide some balance.")
    assert reason_of(fw(seg), c).startswith("short_line_ratio: 0.7500 > threshold 0.6700")
    fw(seg).process(doc("This line is adequately long and should pass.\nSo is this one, it meets the criteria "
                        "perfectly.\nAnd another one just to be sure it's fine."))
    assert reason_of(fw(seg), "... --- !!!").startswith("short_line_ratio: 1.0000 > threshold 0.6700")


def test_fineweb_char_dup(seg):
    fw(seg, line_punct_thr=0.0, short_line_thr=1.0, new_line_ratio=1.0).process(
        doc("abcdefghijklmnopqrstuvwxyz.\n1234567890."))
    fw(seg, line_punct_thr=0.0, short_line_thr=1.0).process(doc("abcde fghij klmno pqrst uvwxyz."))
    f = fw(seg, line_punct_thr=0.0, short_line_thr=1.0, new_line_ratio=1.0, char_duplicates_ratio=0.66)
    assert reason_of(f, "Hello World\nHello World\nHello World").startswith("char_dup_ratio: 0.6667 > threshold 0.6600")


def test_fineweb_new_line_ratio(seg):
    f = fw(seg, line_punct_thr=0.0, short_line_thr=1.0)
    assert reason_of(f, "word.\nword.\nword.\nword.\nword.").startswith("list_ratio: 0.8000 > threshold 0.3000")
    fw(seg).process(doc("Many words on a single line with no newlines effectively. This should pass easily."))
    fw(seg).process(doc("Word one is long enough and ends with a period.\nWord two is also quite long and ends with a "
                        "period.\nWord three is suitably lengthy and ends with a period.\nWord four and five and six "
                        "are here and it ends with a period."))


def test_fineweb_passing(seg):
    fw(seg).process(doc(
        "This is a good line that ends with a period.\nAnother good line also ends with a question mark?\nShort "
        "lines are not too frequent here, which is great!\nCharacter duplication is hopefully not too high in this "
        "example text.\nAnd the ratio of newlines to words should be reasonable as well."))


# ---- language ---------------------------------------------------------------------------------

def test_language_allowed():
    out = LanguageDetectionFilter(0.8, ["eng"]).process(doc(
        "Sometimes, all you need to start the day right is a good coffee and someone greeting you smiling."))
    assert out.metadata["Detected language"] == "English"
    float(out.metadata["Detected language confidence"])


@pytest.mark.parametrize("content", ["Hej med dig. Dette er Dansk", "Jag talar lite svenska."])
def test_language_disallowed(content):
    r = reason_of(LanguageDetectionFilter(0.8, ["eng"]), content)
    assert 'Document is not any of the following languages: "eng"' in r


def test_language_low_confidence():
    f = LanguageDetectionFilter(0.99, ["eng"])
    with pytest.raises(DocumentFiltered) as ei:
        f.process(TextDocument(id="doc5", source="s", content="Text arrives out of thin air"))
    d = ei.value.document
    assert d.id == "doc5"
    assert d.metadata["Detected language"] == "English"
    assert "Language detection confidence is not satified" in ei.value.reason


# ---- token counter (stand-in tokenizer fixtures, see tools/make_test_tokenizers.py) -----------

@pytest.mark.parametrize("name,content,expected", [
    ("bert-base-uncased", "Hello, world! This is a test.", "11"),
    ("gpt2", "Hello, world! This is a test.", "9"),
    ("bert-base-uncased", "", "2"),
])
def test_token_counter(name, content, expected):
    tc = TokenCounter(name, tokenizer_dir=FIX)
    assert tc.process(doc(content)).metadata["token_count"] == expected


def test_token_counter_missing():
    with pytest.raises(Unexpected, match="Error in loading tokenizer"):
        TokenCounter("no-such-tokenizer-xyz", tokenizer_dir=FIX)


# ---- text utils -------------------------------------------------------------------------------

def test_split_sentences(seg):
    s = lambda t: tu.split_into_sentences(t, seg)  # noqa: E731
    assert s("") == [] and s("   ") == []
    assert s("Hello world.") == ["Hello world."]
    assert s("  Hello world.  ") == ["Hello world."]
    assert s("Dette er en sætning.") == ["Dette er en sætning."]
    assert s("SingleWord") == ["SingleWord"] and s("  SingleWord  ") == ["SingleWord"]
    exp = ["Første sætning.", "Anden sætning!", "Tredje sætning?"]
    assert s("Første sætning. Anden sætning! Tredje sætning?") == exp
    assert s("  Første sætning.   Anden sætning!  Tredje sætning?  ") == exp
    assert s(" Hello. How are you? Fine! ") == ["Hello.", "How are you?", "Fine!"]
    assert s("This is a sentence. This is another") == ["This is a sentence.", "This is another"]
    assert s("  This is a sentence.   This is another  ") == ["This is a sentence.", "This is another"]


def test_split_words(seg):
    w = lambda t: tu.split_into_words(t, seg)  # noqa: E731
    assert w("") == []
    assert w("hello") == ["hello"]
    assert w("hello world") == ["hello", "world"]
    assert w("hello, world!") == ["hello", "world"]
    assert w("first. second; third?") == ["first", "second", "third"]
    assert w("...leading") == ["leading"]
    assert w("trailing...") == ["trailing"]
    assert w("mid...dle") == ["mid", "dle"]
    assert w("hej med dig") == ["hej", "med", "dig"]
    assert w("en, to, tre!") == ["en", "to", "tre"]


def test_punctuation_set():
    for ch in ".,!?\"\u0000\u001f":
        assert ch in tu.PUNCTUATION
    for ch in "aA5":
        assert ch not in tu.PUNCTUATION


def test_danish_stop_words():
    assert tu.DANISH_STOP_WORDS
    assert "og" in tu.DANISH_STOP_WORDS and "er" in tu.DANISH_STOP_WORDS
    assert "hest" not in tu.DANISH_STOP_WORDS
