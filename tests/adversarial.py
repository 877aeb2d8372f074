"""Adversarial documents for the device-vs-oracle differential tests: random strings from the
UAX#29 fuzz pool (tests/test_uax29_fuzz.py) at document scale, and constructs placed across
the 64-item chunk boundaries of the wave primitives (code point index and byte index 63/64,
127/128, 191/192, ...), where scans carry state between chunks."""
import random

from test_uax29_fuzz import POOL

MOTIFS = ["don't", "3.14", "U.S.A.", "a.b", "\r\n", "\n\n\n", "...", "…", "\U0001F1E9\U0001F1F0\U0001F1F8",
          "\U0001F468‍\U0001F469", "é", "#tag", "[12, 3]", "• bullet", "- dash", "א״ב", "Σ.",
          "word  word", " x", "1,000.5"]


def pool_docs(seed: int, n: int, max_len: int = 300):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(1, max_len)
        out.append("".join(rng.choice(POOL) for _ in range(k)))
    return out


def boundary_docs():
    out = []
    for motif in MOTIFS:
        for pad in (60, 61, 62, 63, 64, 65, 125, 126, 127, 128, 190, 191):
            # ASCII padding: code point index == byte index at the motif
            out.append("ab cd ef gh " * (pad // 12) + "x" * (pad % 12) + motif + " tail words here. End.")
            # 2-byte padding: the byte boundary falls elsewhere than the code point boundary
            out.append("æø " * (pad // 3) + motif + " more text follows. Done!")
    # repeated lines / n-grams whose repeats straddle chunks
    out.append(("the same line of words repeats here.\n" * 9) + "different ending")
    out.append(" ".join(["alpha beta gamma delta epsilon zeta"] * 30))
    out.append("ab c a bc ab c a bc " * 20)
    return out


def adversarial_corpus(seed: int = 3, n_pool: int = 400):
    return pool_docs(seed, n_pool) + boundary_docs()
