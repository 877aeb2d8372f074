"""Language identification model (stands in for lingua; reference language_filter.rs:35-93).

Architecture (fastText-style, survey H5): hashed character 1..3-grams of lowercased letter runs
-> mean of bf16 embedding rows E[65536, 32] (exact fixed-point sum) -> bf16 doc vector ->
logits = doc . W[32, 5(+pad 16)] + b -> softmax over {English, Danish, Swedish, Nynorsk, Bokmal}.
On the device the featurizer runs in the document kernel and the head is one
``v_mfma_f32_16x16x32_bf16`` per 16 documents; the CPU path uses the same arithmetic.

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
DEFAULT_WEIGHTS = os.path.join(DATA_DIR, "langid_v1.npz")
LANGS = ("eng", "dan", "swe", "nno", "nob")
NAMES = ("English", "Danish", "Swedish", "Nynorsk", "Bokmal")


@dataclasses.dataclass
class LangidWeights:
    emb: np.ndarray  # uint16 bf16 bits [BUCKETS * DIM]
    w: np.ndarray    # uint16 bf16 bits [DIM * PAD]
    b: np.ndarray    # float32 [PAD]
    _native: Optional[object] = None

    def native(self):
        if self._native is None:
            self._native = native.host().LangidModel(self.emb, self.w, self.b)
        return self._native

    def detect(self, text: str):
        """(language name or None, confidence) with the CPU arithmetic."""
        lang, conf = self.native().detect(text)
        return (NAMES[lang], conf) if lang >= 0 else (None, 0.0)


def load(path: str) -> LangidWeights:
    with np.load(path, allow_pickle=False) as z:
        emb = np.ascontiguousarray(z["emb"], dtype=np.uint16).reshape(-1)
        w = np.ascontiguousarray(z["w"], dtype=np.uint16).reshape(-1)
        b = np.ascontiguousarray(z["b"], dtype=np.float32).reshape(-1)
    h = native.host()
    if emb.size != h.LID_BUCKETS * h.LID_DIM or w.size != h.LID_DIM * h.LID_LANGS_PAD or b.size != h.LID_LANGS_PAD:
        raise ValueError(f"language model {path} has the wrong shape")
    # the device accumulates n-gram rows in int32 fixed point per lane (docproc.h
    # langid_features_bytes): |e| < 32 keeps every partial sum below 2^31
    emax = float(np.abs((emb.astype(np.uint32) << 16).view(np.float32)).max()) if emb.size else 0.0
    if not emax < 32.0:
        raise ValueError(f"language model {path}: embedding magnitude {emax} out of range (< 32)")
    return LangidWeights(emb, w, b)


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
