"""Text utilities with the reference semantics (reference src/utils/text.rs), backed by the C++
host runtime. ``backend`` selects the UAX#29 implementation: "icu" (ICU4C, the oracle) or
"rules" (this framework's rule engine, the same code the HIP kernels run)."""
from __future__ import annotations

from typing import List, Sequence, Tuple

from .. import native

# reference utils/text.rs:9-25 (kept for API parity; unused by the default pipeline)
DANISH_STOP_WORDS = (
    "ad af aldrig alle alt anden andet andre at bare begge blev blive bliver da de dem den denne der deres det "
    "dette dig din dine disse dit dog du efter ej eller en end ene eneste enhver er et far fem fik fire flere "
    "fleste for fordi forrige fra få får før god godt ham han hans har havde have hej helt hende hendes her hos "
    "hun hvad hvem hver hvilken hvis hvor hvordan hvorfor hvornår i ikke ind ingen intet ja jeg jer jeres jo kan "
    "kom komme kommer kun kunne lad lav lidt lige lille man mand mange med meget men mens mere mig min mine mit "
    "mod må ned nej ni nogen noget nogle nu ny nyt når nær næste næsten og også okay om op os otte over på se "
    "seks selv ser ses sig sige sin sine sit skal skulle som stor store syv så sådan tag tage thi ti til to tre "
    "ud under var ved vi vil ville vor vores være været"
).split()

_P_PUNCT = 1 << 11


def is_punctuation(ch: str) -> bool:
    """Membership in TextBlaster's PUNCTUATION set (reference utils/text.rs:28-57)."""
    return bool(native.host().props(ord(ch)) & _P_PUNCT)


class _PunctuationSet:
    def __contains__(self, ch) -> bool:
        return isinstance(ch, str) and len(ch) == 1 and is_punctuation(ch)


PUNCTUATION = _PunctuationSet()


def split_into_sentences(text: str, backend: str = "icu") -> List[str]:
    return native.host().split_into_sentences(text, backend)


def split_into_words(text: str, backend: str = "icu") -> List[str]:
    return native.host().split_into_words(text, backend)


def get_n_grams(words: Sequence[str], n: int) -> List[str]:
    if n == 0:
        return []
    return [" ".join(words[i:i + n]) for i in range(len(words) - n + 1)]


def find_duplicates(items: Sequence[str]) -> Tuple[int, int]:
    return tuple(native.host().find_duplicates(list(items)))


def find_top_duplicate(items: Sequence[str]) -> int:
    """reference text.rs:211-238 over arbitrary items: max(count) x len among the most frequent."""
    counts = {}
    for it in items:
        counts[it] = counts.get(it, 0) + 1
    if not counts:
        return 0
    mx = max(counts.values())
    if mx <= 1:
        return 0
    return max(len(k.encode()) * mx for k, v in counts.items() if v == mx)


def find_all_duplicate(words: Sequence[str], n: int) -> int:
    return native.host().find_all_duplicate(list(words), n)


def rust_lowercase(text: str) -> str:
    return native.host().rust_lowercase(text)
