"""Language identification model (stands in for lingua; reference language_filter.rs:35-93).

Featurizer: hashed character 1..4-grams of lowercased letter runs (csrc/common/langid.h), 65536
buckets. Model (``langid_v3.npz``): fastText with a D = 32 document vector made of two 16-dim
  bags over one int8 embedding table (16 values per bucket, so a gather moves 16 bytes): the
  1- and 2-grams are summed into dims 0..15, the 3- and 4-grams into dims 16..31; a document's
  rows are summed exactly, the mean doc vector is quantised to
  integers |a| <= 255 with one exponent per document (block floating point: exact in bf16), and
  the 32 -> 5 linear head runs on the matrix cores as ``v_mfma_f32_16x16x32_bf16`` tiles of 16
  documents (k_langid_mfma) with integer bf16 weights. Every product and partial sum is an
  integer below 2^24, so the MFMA's fp32 output is exact and the CPU path computes the same
  records bit for bit. (Round 5's folded int16 logit table, "v2", lost its A/B to this model
  and was removed.)

Softmax over {English, Danish, Swedish, Nynorsk, Bokmal}; the confidence is the top probability.
Weights are produced offline by ``tools/train_langid.py`` from ``models/data/langid_corpus`` and
stored as plain ``.npz`` files (loaded with allow_pickle=False).
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import numpy as np

from .. import native

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DEFAULT_WEIGHTS = os.path.join(DATA_DIR, "langid_v3.npz")
LANGS = ("eng", "dan", "swe", "nno", "nob")
NAMES = ("English", "Danish", "Swedish", "Nynorsk", "Bokmal")
QMAX = 255  # |integer| of the v3 doc vectors and head weights: exact in bf16


@dataclasses.dataclass
class LangidWeights:
    b: np.ndarray                      # float32 [8] bias
    E: np.ndarray                      # int8 [BUCKETS * ROW_DIM] embedding rows (both bags)
    W: np.ndarray                      # int16 [DIM * LANGS] integer head, |W| <= 255
    w_scale: float                     # logit units per head unit
    _native: Optional[object] = None

    @property
    def version(self) -> int:
        return 3

    @property
    def description(self) -> str:
        return ("fastText int8 EmbeddingBag(65536 x 16) x 2 bags (1-2 / 3-4-grams) -> 32-dim doc vector -> "
                "bf16 MFMA head (v_mfma_f32_16x16x32_bf16)")

    @property
    def dtype(self) -> str:
        """Compute dtype of the model's math on the device (bench.py reports it)."""
        return "bf16"

    def native(self):
        if self._native is None:
            h = native.host()
            self._native = h.LangidModel(self.E, self.W, float(self.w_scale), self.b)
        return self._native

    def detect(self, text: str):
        """(language name or None, confidence) with the CPU arithmetic."""
        lang, conf = self.native().detect(text)
        return (NAMES[lang], conf) if lang >= 0 else (None, 0.0)

    def float_logits(self, text: str) -> Optional[np.ndarray]:
        """v3 logits of ``text`` by plain f64 inference (mean of the two bags, head, bias; no
        doc-vector quantisation): the reference the integer / MFMA path is checked against."""
        h = native.host()
        g, order = h.langid_buckets(text, True)
        if not g:
            return None
        rd = h.LID_ROW_DIM
        E = self.E.reshape(h.LID_BUCKETS, rd).astype(np.float64)
        g = np.asarray(g, dtype=np.int64)
        hi = np.asarray(order) >= 3
        v = np.concatenate([E[g[~hi]].sum(0), E[g[hi]].sum(0)]) / len(g)
        W = self.W.reshape(h.LID_DIM, h.LID_LANGS).astype(np.float64)
        return v @ W * self.w_scale + self.b[:h.LID_LANGS].astype(np.float64)

    def head_bf16_t(self) -> np.ndarray:
        """v3 head as the MFMA B operand: uint16 bf16 bits [16 columns][32 dims] (W transposed,
        languages zero-padded to 16 columns; the integers are exact in bf16)."""
        h = native.host()
        wt = np.zeros((16, h.LID_DIM), dtype=np.float32)
        wt[:len(LANGS), :] = self.W.reshape(h.LID_DIM, len(LANGS)).T
        return (wt.view(np.uint32) >> 16).astype(np.uint16)


def quantize_v3(E: np.ndarray, W: np.ndarray, b: np.ndarray) -> dict:
    """Float fastText weights (E [buckets, 16], shared by the two bags; W [32, langs]; b [langs])
    -> the v3 arrays: int8 E (per-tensor scale sE), integer W (|W| <= 255, scale sW),
    w_scale = sE * sW, b."""
    h = native.host()
    sE = float(np.abs(E).max()) / 127.0 or 1.0
    Eq = np.clip(np.rint(E / sE), -127, 127).astype(np.int8)
    sW = float(np.abs(W).max()) / QMAX or 1.0
    Wq = np.clip(np.rint(W / sW), -QMAX, QMAX).astype(np.int16)
    bb = np.zeros(h.LID_ROW, dtype=np.float32)
    bb[:len(b)] = b
    return {"E": Eq.reshape(-1), "W": Wq.reshape(-1), "w_scale": np.float64(sE * sW), "b": bb}


def load(path: str) -> LangidWeights:
    h = native.host()
    with np.load(path, allow_pickle=False) as z:
        files = set(z.files)
        if not {"E", "W", "w_scale", "b"} <= files:
            raise ValueError(f"language model {path} is not a fastText model (E, W, w_scale, b)")
        E = np.ascontiguousarray(z["E"], dtype=np.int8).reshape(-1)
        W = np.ascontiguousarray(z["W"], dtype=np.int16).reshape(-1)
        w_scale = float(np.asarray(z["w_scale"]).reshape(()))
        b = np.ascontiguousarray(z["b"], dtype=np.float32).reshape(-1)
    if E.size != h.LID_BUCKETS * h.LID_ROW_DIM or W.size != h.LID_DIM * h.LID_LANGS or b.size != h.LID_ROW:
        raise ValueError(f"language model {path} has the wrong shape")
    if np.any(np.abs(W.astype(np.int32)) > QMAX) or not w_scale > 0:
        raise ValueError(f"language model {path}: head out of range")
    return LangidWeights(b=b, E=E, W=W, w_scale=w_scale)


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
