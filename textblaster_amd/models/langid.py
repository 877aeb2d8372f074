"""Language identification model (stands in for lingua; reference language_filter.rs:35-93).

Architecture (csrc/common/langid.h): hashed character 1..4-grams of lowercased letter runs ->
per bucket an int16 row of fixed-point logit contributions to {English, Danish, Swedish,
Nynorsk, Bokmal} (P[65536, 8], 5 used, scale 1/1024) -> logits = sum of the document's rows /
#grams / 1024 + b -> softmax; the confidence is the top probability. The sums are exact integers,
so the device kernel (k_langid_features: one 16-byte gather per n-gram) and the CPU path agree
bit for bit. This is a fastText-style mean-of-embeddings model with its linear head folded into
the table ((mean E) W = mean (E W)); tools/train_langid.py trains the folded table directly.

Weights are produced offline by ``tools/train_langid.py`` from the text in
``models/data/langid_corpus`` and stored as a plain ``.npz`` (loaded with allow_pickle=False).
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import numpy as np

from .. import native

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DEFAULT_WEIGHTS = os.path.join(DATA_DIR, "langid_v2.npz")
LANGS = ("eng", "dan", "swe", "nno", "nob")
NAMES = ("English", "Danish", "Swedish", "Nynorsk", "Bokmal")


@dataclasses.dataclass
class LangidWeights:
    P: np.ndarray  # int16 [BUCKETS * ROW] fixed-point logit rows
    b: np.ndarray  # float32 [ROW]
    _native: Optional[object] = None

    def native(self):
        if self._native is None:
            self._native = native.host().LangidModel(self.P, self.b)
        return self._native

    def detect(self, text: str):
        """(language name or None, confidence) with the CPU arithmetic."""
        lang, conf = self.native().detect(text)
        return (NAMES[lang], conf) if lang >= 0 else (None, 0.0)


def load(path: str) -> LangidWeights:
    with np.load(path, allow_pickle=False) as z:
        if "P" not in z.files or "b" not in z.files:
            raise ValueError(f"language model {path} is not a hashed n-gram logit table (keys P, b)")
        P = np.ascontiguousarray(z["P"], dtype=np.int16).reshape(-1)
        b = np.ascontiguousarray(z["b"], dtype=np.float32).reshape(-1)
    h = native.host()
    if P.size != h.LID_BUCKETS * h.LID_ROW or b.size != h.LID_ROW:
        raise ValueError(f"language model {path} has the wrong shape")
    if np.any(P.reshape(-1, h.LID_ROW)[:, h.LID_LANGS:] != 0):
        raise ValueError(f"language model {path}: padding columns must be zero")
    return LangidWeights(P, b)


_default: Optional[LangidWeights] = None


def load_default() -> LangidWeights:
    global _default
    if _default is None:
        path = os.environ.get("TB_LANGID_MODEL", DEFAULT_WEIGHTS)
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"language-id weights not found at {path}; run `python tools/train_langid.py`")
        _default = load(path)
    return _default
