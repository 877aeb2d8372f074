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


def _sentence(rng: np.random.Generator, vocab: List[str]) -> str:
    n = int(rng.integers(4, 18))
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


def make_doc(rng: np.random.Generator, lang: str, target_bytes: int) -> str:
    vocab = VOCAB[lang]
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
            line = "• " + " ".join(vocab[int(rng.integers(0, len(vocab)))] for _ in range(3))
        elif r < 0.13:
            line = BOILER[int(rng.integers(0, len(BOILER)))]
        elif r < 0.16:
            line = vocab[int(rng.integers(0, len(vocab)))].capitalize()  # short heading
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


def make_corpus(n_docs: int, mean_bytes: int = 1024, seed: int = 0,
                langs=("eng", "dan", "swe", "nob", "nno"), lang_p=None) -> List[str]:
    rng = np.random.default_rng(seed)
    sigma = 0.8
    mu = math.log(mean_bytes) - sigma * sigma / 2
    sizes = np.clip(rng.lognormal(mu, sigma, n_docs), 16, 64 * mean_bytes).astype(np.int64)
    langs = list(langs)
    choice = rng.choice(len(langs), size=n_docs, p=lang_p)
    return [make_doc(rng, langs[int(c)], int(s)) for c, s in zip(choice, sizes)]


def pack(texts: List[str]):
    """Pack strings into (uint8 data, int64 offsets) like an Arrow LargeUtf8 column."""
    enc = [t.encode("utf-8") for t in texts]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    data = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, dtype=np.uint8)
    return data, off
