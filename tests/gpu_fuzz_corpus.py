"""Seeded document generator for the large GPU-vs-ICU differential (test_gpu_differential.py):
slices of base documents from four pools — the small-vocabulary synthetic corpus, the Zipf
corpus, Unicode-heavy random text and the adversarial pool (UAX#29 fuzz characters, constructs
across chunk boundaries) — cut at random code points, spliced with CRLF / blank-line joins and
sprinkled with UAX#29 edge characters (combining marks, ZWJ / emoji sequences, regional
indicator runs, MidLetter / MidNum punctuation, NBSP and other spaces, Hebrew quotes,
Arabic-Indic digits). Cheap enough to build 200,000+ documents in a few seconds."""
import random

from adversarial import MOTIFS, adversarial_corpus
from test_uax29_fuzz import POOL

from textblaster_amd.utils import synth

EDGE_CHARS = ["́", "̈", "‍", "​", " ", " ", "　", "\U0001F1E9", "\U0001F1F0",
              "\U0001F44D\U0001F3FD", "\U0001F468‍\U0001F469", "א״ב", "١٢",
              "'", "’", ":", ".", ",", ";", "\r\n", "\r", "\n", "\n\n", "\t", "…", "...", "#",
              "[1]", "[2, 3]", "{", "}", "• ", "- ", "æøå", "İ", "Σ", "K"]

WORDS = ["the", "og", "och", "ikkje", "ikke", "privacy policy", "javascript", "lorem ipsum", "cookies",
         "don't", "U.S.A.", "3.14", "naïve", "Blåbærgrød", "Øresund", "straße", "ΣΑΣ", "İstanbul",
         "terms of use", "café", "co-operate", "e-mail", "1,000.5", "a.b.c"]


def _unicode_doc(rng: random.Random, n: int) -> str:
    out = []
    while sum(len(x) for x in out) < n:
        r = rng.random()
        if r < 0.45:
            out.append(rng.choice(WORDS))
            out.append(rng.choice([" ", " ", " ", ". ", ", ", "\n", "! ", "? "]))
        elif r < 0.75:
            out.append("".join(rng.choice(POOL) for _ in range(rng.randint(1, 6))))
        elif r < 0.9:
            out.append(rng.choice(EDGE_CHARS))
        else:
            out.append(rng.choice(MOTIFS))
    return "".join(out)


def base_pools(seed: int):
    rng = random.Random(seed)
    small = synth.make_corpus(3000, 1500, seed=seed)
    zipf = synth.make_corpus(2000, 1500, seed=seed + 1, vocab="zipf")
    uni = [_unicode_doc(rng, int(rng.lognormvariate(6.5, 0.8))) for _ in range(3000)]
    adv = adversarial_corpus(seed=seed + 2, n_pool=600)
    return [small, zipf, uni, adv]


def fuzz_docs(n: int, seed: int = 1234):
    pools = base_pools(seed)
    rng = random.Random(seed)
    weights = [0.35, 0.25, 0.25, 0.15]
    out = []
    for _ in range(n):
        pool = rng.choices(pools, weights)[0]
        d = rng.choice(pool)
        if d:
            ln = min(len(d), max(1, int(rng.lognormvariate(5.8, 1.0))))
            a = rng.randint(0, len(d) - ln)
            d = d[a:a + ln]
        r = rng.random()
        if r < 0.2:  # splice a second slice after a line / paragraph break
            e = rng.choice(rng.choice(pools))
            d = d + rng.choice(["\n", "\n\n", "\r\n", "\r\n\r\n", " ", ""]) + e[:rng.randint(0, 400)]
        if rng.random() < 0.3:  # a few edge characters at random code points
            for _ in range(rng.randint(1, 3)):
                k = rng.randint(0, len(d))
                d = d[:k] + rng.choice(EDGE_CHARS) + d[k:]
        if rng.random() < 0.05:  # repeated lines (Gopher / FineWeb duplicate statistics)
            line = d[:rng.randint(1, 80)]
            d = d + ("\n" + line) * rng.randint(2, 6)
        out.append(d)
    return out
