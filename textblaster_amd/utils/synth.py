"""Synthetic CommonCrawl-shaped documents (no network: the benchmark and tests generate data).

Documents are built from small per-language vocabularies and sentence templates with the
structural features the filters react to: lines and paragraphs, repeated lines/paragraphs and
n-grams, bullet and ellipsis lines, '#' tags, citations ``[1]``, curly brackets, "lorem ipsum",
"javascript", cookie/policy boilerplate, CRLF line ends, non-ASCII punctuation and emoji.
Length follows a log-normal distribution around ``mean_bytes`` (CommonCrawl-like heavy tail).
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np

VOCAB = {
    "eng": ("the of and to in is that for it with as was on be by this are from at or have an not "
            "they which you one were all we her she there would their will when who him been has more "
            "if no out do so can what up said about other into than its time only could new them man "
            "some these then two first may any like now my such make over our even most me state after "
            "also made many did must before back see through way where get much go well your know should "
            "down work year because come people just say each those take day good how long little use "
            "world government house city school water market report company system research data music "
            "history family children policy season energy health community business online service").split(),
    "dan": ("og i at det er en til på som de med han af for ikke der var mig sig men et har om vi min havde "
            "ham hun nu over da fra du ud sin dem os op man hans hvor eller hvad skal selv her alle vil "
            "blev kunne ind når være dog noget ville jo deres efter ned skulle denne end dette mit også "
            "under have dig anden hende mine alt meget sit sine vor mod disse hvis din nogle hos blive "
            "mange ad bliver hendes været thi jer sådan byen landet regeringen børn skole arbejde "
            "kommunen historie familie sundhed virksomhed forskning musik vand marked uge året").split(),
    "swe": ("och det att i en jag hon som han på den med var sig för så till är men ett om hade de av icke "
            "mig du henne då sin nu har inte hans honom skulle hennes där min man ej vid kunde något från "
            "ut när efter upp vi dem vara vad över än dig kan sina här ha mot alla under någon eller allt "
            "mycket sedan ju denna själv detta åt utan varit hur ingen mitt ni bli blev oss din dessa "
            "staden landet regeringen barn skolan arbete kommunen historia familj hälsa företag").split(),
    "nob": ("og i jeg det at en et den til er som på de med han av ikke der så var meg seg men ett har om "
            "vi min mitt ha hadde hun nå over da ved fra du ut sin dem oss opp man kan hans hvor eller "
            "hva skal selv sjøl her alle vil bli ble blitt kunne inn når være kom noen noe ville dere "
            "deres kun ja etter ned skulle denne for deg si sine sitt mot å meget hvorfor dette disse "
            "byen landet regjeringen barn skolen arbeid kommunen historie familie helse bedrift").split(),
    "nno": ("og i eg det at ein eit den til er som på dei med han av ikkje der så var meg seg men har om vi "
            "min mitt ha hadde ho no over da ved frå du ut sin dykk oss opp kan hans kvar eller kva skal "
            "sjølv her alle vil bli vart vore kunne inn når vere kom nokon noko ville dykkar berre ja "
            "etter ned skulle denne for deg si sine sitt mot å mykje kvifor dette desse korleis heime "
            "byen landet regjeringa born skulen arbeid kommunen historie familie helse bedrift").split(),
}

BOILER = ["We use cookies to improve your experience.", "Read our privacy policy and terms of use.",
          "Please enable javascript to view this page.", "Lorem ipsum dolor sit amet.",
          "function() { return 0; }"]


# ---- large-vocabulary (Zipf) lexicons -------------------------------------------------------
# Per language: the function words above at the head of a Zipf-Mandelbrot rank-frequency law
# (p(r) ~ 1 / (r + 2.7)^1.07, as measured on web text), followed by ~60,000 synthetic content
# words built from that language's syllable inventory (1-4 syllables: 3-14 letters, mean ~7), so
# word, n-gram and hash-table statistics resemble real text instead of a ~130-word vocabulary.
_SYLL = {
    "eng": (["b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "st", "tr",
             "pl", "ch", "sh", "th", "br", "cr", "gr", "fl", ""],
            ["a", "e", "i", "o", "u", "ea", "ou", "ai", "ee", "y"],
            ["", "", "n", "r", "s", "t", "nd", "st", "ck", "ng", "l", "m", "rt", "ss"]),
    "dan": (["b", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "sk", "sp", "st", "kr",
             "tr", "bl", "fl", "gr", "hv", ""],
            ["a", "e", "i", "o", "u", "y", "æ", "ø", "å", "ej", "ø"],
            ["", "", "n", "r", "s", "t", "d", "g", "k", "l", "nd", "st", "rt", "ns", "ld"]),
    "swe": (["b", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "sk", "sp", "st", "kr",
             "tr", "bl", "fr", "gr", "sj", ""],
            ["a", "e", "i", "o", "u", "y", "å", "ä", "ö", "ä"],
            ["", "", "n", "r", "s", "t", "d", "g", "k", "l", "nd", "st", "rt", "ng", "ck"]),
    "nob": (["b", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "sk", "sp", "st", "kr",
             "tr", "bl", "fl", "gr", "hv", ""],
            ["a", "e", "i", "o", "u", "y", "æ", "ø", "å", "ei", "ø"],
            ["", "", "n", "r", "s", "t", "d", "g", "k", "l", "nd", "st", "rt", "ns", "kk"]),
    "nno": (["b", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "sk", "sp", "st", "kj",
             "gj", "tr", "bl", "fl", "gr", "kv", ""],
            ["a", "e", "i", "o", "u", "y", "æ", "ø", "å", "ei", "au"],
            ["", "", "n", "r", "s", "t", "d", "g", "k", "l", "nd", "st", "rt", "ng", "kk"]),
}
ZIPF_TYPES = 60000
_LEX = {}


def lexicon(lang: str, n_types: int = ZIPF_TYPES):
    """(words, cumulative probabilities) of a language's Zipf lexicon (deterministic, cached)."""
    key = (lang, n_types)
    if key not in _LEX:
        rng = np.random.default_rng(90210 + sorted(_SYLL).index(lang))
        on, nu, co = _SYLL[lang]
        words = list(dict.fromkeys(VOCAB[lang]))
        seen = set(words)
        while len(words) < n_types:
            k = 1 + min(3, int(rng.poisson(1.1)))
            w = "".join(on[int(rng.integers(0, len(on)))] + nu[int(rng.integers(0, len(nu)))] + co[int(rng.integers(0, len(co)))]
                        for _ in range(k))
            if len(w) >= 2 and w not in seen:
                seen.add(w)
                words.append(w)
        r = np.arange(len(words), dtype=np.float64)
        p = 1.0 / np.power(r + 2.7, 1.07)
        _LEX[key] = (words, np.cumsum(p / p.sum()))
    return _LEX[key]


class _ZipfVocab:
    """Word sampler with the list interface make_doc uses (len / index), drawing by Zipf rank."""

    def __init__(self, lang: str):
        self.words, self.cdf = lexicon(lang)
        self._pending = None

    def draw(self, rng: np.random.Generator, k: int) -> List[str]:
        idx = np.searchsorted(self.cdf, rng.random(k), side="right")
        idx = np.minimum(idx, len(self.words) - 1)
        return [self.words[int(i)] for i in idx]


def _sentence(rng: np.random.Generator, vocab) -> str:
    n = int(rng.integers(4, 18))
    if isinstance(vocab, _ZipfVocab):
        words = vocab.draw(rng, n)
    else:
        words = [vocab[int(rng.integers(0, len(vocab)))] for _ in range(n)]
    words[0] = words[0].capitalize()
    r = rng.random()
    if r < 0.05:
        words.insert(int(rng.integers(1, n)), str(int(rng.integers(1, 2025))))
    elif r < 0.07:
        words.insert(int(rng.integers(1, n)), "#" + words[-1])
    end = rng.choice([".", ".", ".", ".", "!", "?", "...", "…", ":", ""], p=None)
    s = " ".join(words) + end
    if rng.random() < 0.03:
        s += f" [{int(rng.integers(1, 40))}]"
    if rng.random() < 0.01:
        s += " 😀"
    return s


def _pick(rng: np.random.Generator, vocab) -> str:
    if isinstance(vocab, _ZipfVocab):
        return vocab.draw(rng, 1)[0]
    return vocab[int(rng.integers(0, len(vocab)))]


def make_doc(rng: np.random.Generator, lang: str, target_bytes: int, vocab_kind: str = "small") -> str:
    vocab = VOCAB[lang] if vocab_kind == "small" else _ZipfVocab(lang)
    lines: List[str] = []
    size = 0
    prev_par: Optional[str] = None
    while size < target_bytes:
        r = rng.random()
        if r < 0.06 and lines:
            line = lines[int(rng.integers(0, len(lines)))]  # repeated line
        elif r < 0.10:
            line = "- " + _sentence(rng, vocab)
        elif r < 0.12:
            line = "• " + " ".join(_pick(rng, vocab) for _ in range(3))
        elif r < 0.13:
            line = BOILER[int(rng.integers(0, len(BOILER)))]
        elif r < 0.16:
            line = _pick(rng, vocab).capitalize()  # short heading
        else:
            line = " ".join(_sentence(rng, vocab) for _ in range(int(rng.integers(1, 5))))
        lines.append(line)
        size += len(line.encode()) + 1
        if rng.random() < 0.15:
            lines.append("")  # paragraph break
            if prev_par is not None and rng.random() < 0.1:
                lines.append(prev_par)
            prev_par = line
    sep = "\r\n" if rng.random() < 0.05 else "\n"
    text = sep.join(lines)
    if rng.random() < 0.1:
        text = "  " + text + "\n\n"
    return text


# Dictionary-segmented scripts (ICU word segmentation by dictionary: Han, Kana, Thai): snippets for
# the mixed-script corpus
CJK_SNIPPETS = ["日本語のテキストです。", "東京は日本の首都です", "中文分词测试", "北京欢迎你", "カタカナ",
                "ひらがなとカタカナ", "漢字", "人工知能"]
THAI_SNIPPETS = ["ภาษาไทย", "สวัสดีครับ", "ประเทศไทย"]


def make_cjk_doc(rng: np.random.Generator, target_bytes: int) -> str:
    """A document written in CJK (sentences of the snippets above), about ``target_bytes`` long."""
    lines, size = [], 0
    while size < target_bytes:
        line = "".join(CJK_SNIPPETS[int(rng.integers(0, len(CJK_SNIPPETS)))] for _ in range(int(rng.integers(2, 6))))
        lines.append(line)
        size += len(line.encode()) + 1
    return "\n".join(lines)


def make_corpus(n_docs: int, mean_bytes: int = 1024, seed: int = 0,
                langs=("eng", "dan", "swe", "nob", "nno"), lang_p=None, vocab: str = "small",
                mixed_script: bool = False) -> List[str]:
    """``vocab``: "small" (the ~130 function words per language, the original benchmark corpus)
    or "zipf" (60,000-type Zipf lexicons per language, see ``lexicon``). ``mixed_script``: 5 % of
    the documents get one CJK or Thai snippet inserted at a random word boundary and 1 % are
    written in CJK (the dictionary-segmented scripts a European-language crawl still contains)."""
    if vocab not in ("small", "zipf"):
        raise ValueError("vocab must be 'small' or 'zipf'")
    rng = np.random.default_rng(seed)
    sigma = 0.8
    mu = math.log(mean_bytes) - sigma * sigma / 2
    sizes = np.clip(rng.lognormal(mu, sigma, n_docs), 16, 64 * mean_bytes).astype(np.int64)
    langs = list(langs)
    choice = rng.choice(len(langs), size=n_docs, p=lang_p)
    docs = [make_doc(rng, langs[int(c)], int(s), vocab) for c, s in zip(choice, sizes)]
    if mixed_script:
        mrng = np.random.default_rng(seed + 4242)
        u = mrng.random(n_docs)
        for i in np.nonzero(u < 0.06)[0].tolist():
            if u[i] < 0.01:
                docs[i] = make_cjk_doc(mrng, int(sizes[i]))
                continue
            pool = THAI_SNIPPETS if mrng.random() < 0.3 else CJK_SNIPPETS
            snip = pool[int(mrng.integers(0, len(pool)))]
            t = docs[i]
            sp = [k for k in range(len(t)) if t[k] == " "]
            at = sp[int(mrng.integers(len(sp)))] + 1 if sp else 0
            docs[i] = t[:at] + snip + " " + t[at:]
    return docs


def long_tokens(rng: np.random.Generator) -> str:
    """A byte-level-BPE stress snippet: a long URL, a base64 blob, an indentation run or a dash rule
    (pre-tokens of 64+ bytes: long letter / digit / punctuation / whitespace runs)."""
    k = int(rng.integers(0, 5))
    if k == 0:
        path = "/".join("".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(rng.integers(8, 40))))
                        for _ in range(int(rng.integers(2, 6))))
        return f"https://www.{path[:30]}.example.com/{path}?id={int(rng.integers(1, 10**9))}&ref=" + \
            "".join(chr(97 + int(c)) for c in rng.integers(0, 26, 80))
    if k == 1:
        alpha = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/", np.uint8)
        return bytes(alpha[rng.integers(0, 64, int(rng.integers(100, 1200)))]).decode() + "=="
    if k == 2:
        return "\n" + " " * int(rng.integers(64, 400)) + "indented();"
    if k == 3:
        return "\n" + "-" * int(rng.integers(64, 300)) + "\n"
    return "".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(rng.integers(65, 600))))


def inject_long_tokens(texts: List[str], rate: float, seed: int = 0) -> List[str]:
    """A fraction ``rate`` of the documents gets a long_tokens() snippet at a random space."""
    rng = np.random.default_rng(8111 + seed)
    out = list(texts)
    for i in np.nonzero(rng.random(len(out)) < rate)[0].tolist():
        t = out[i]
        sp = [k for k in range(len(t)) if t[k] == " "]
        at = sp[int(rng.integers(len(sp)))] + 1 if sp else 0
        out[i] = t[:at] + long_tokens(rng) + " " + t[at:]
    return out


def inject_words(texts: List[str], list_path: str, rate: float, seed: int = 0) -> List[str]:
    """A fraction ``rate`` of the documents gets one entry of a word list (e.g. a C4 bad-words
    list) inserted after a random space, so a word-list filter has matches to act on."""
    with open(list_path, encoding="utf-8") as f:
        entries = [ln.strip() for ln in f if ln.strip()]
    rng = np.random.default_rng(7331 + seed)
    out = list(texts)
    for i in np.nonzero(rng.random(len(out)) < rate)[0].tolist():
        t = out[i]
        sp = [k for k in range(len(t)) if t[k] == " "]
        at = sp[int(rng.integers(len(sp)))] + 1 if sp else 0
        out[i] = t[:at] + entries[int(rng.integers(len(entries)))] + " " + t[at:]
    return out


def pack(texts: List[str]):
    """Pack strings into (uint8 data, int64 offsets) like an Arrow LargeUtf8 column."""
    enc = [t.encode("utf-8") for t in texts]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    data = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, dtype=np.uint8)
    return data, off
