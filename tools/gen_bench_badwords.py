"""Synthetic bad-words list for benchmarks (no network: the LDNOOBW lists cannot be fetched).

400 pseudo-words from the English syllable inventory of utils/synth.py (seeded apart from the
Zipf lexicon, so they occur in benchmark text only where bench.py --badwords-rate injects them)
plus 40 two-word phrases: a trie with the fan-out of a real list, so the matching cost is
representative. Output: config/badwords/en (one entry per line)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from textblaster_amd.utils import synth  # noqa: E402


def words(n=400, seed=977):
    on, nu, co = synth._SYLL["eng"]
    rng = np.random.default_rng(seed)
    lex = set(synth.lexicon("eng")[0])
    out = []
    while len(out) < n:
        w = "".join(on[rng.integers(len(on))] + nu[rng.integers(len(nu))] + co[rng.integers(len(co))]
                    for _ in range(int(rng.integers(2, 4))))
        if 4 <= len(w) <= 14 and w not in lex and w not in out:
            out.append(w)
    return out


def main():
    w = words()
    rng = np.random.default_rng(5)
    phrases = [f"{w[int(rng.integers(len(w)))]} {w[int(rng.integers(len(w)))]}" for _ in range(40)]
    d = os.path.join(ROOT, "config", "badwords")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "en"), "w", encoding="utf-8") as f:
        f.write("\n".join(w + phrases) + "\n")


if __name__ == "__main__":
    main()
