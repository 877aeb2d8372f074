"""TokenCounter tokenizer (reference src/pipeline/token/token_counter.rs:8-43).

The reference calls ``Tokenizer::from_pretrained(name)`` (a Hugging Face Hub download). There is
no network here, so the name is resolved locally, in order:
  1. ``name`` is a path to a ``tokenizer.json`` file or to a directory containing one;
  2. ``<tokenizer_dir>/<name>/tokenizer.json`` (CLI ``--tokenizer-dir``, env ``TB_TOKENIZER_DIR``);
  3. the Hugging Face cache (``$HF_HOME`` / ``~/.cache/huggingface/hub/models--<name>/snapshots/*``).
Load failure raises ``Unexpected("Error in loading tokenizer")`` like the reference.

Counting = ``len(encode(text, add_special_tokens=True).tokens)``, batched through the Rust
tokenizers library's parallel ``encode_batch``.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional

from ..errors import Unexpected


def resolve_tokenizer_file(name: str, tokenizer_dir: Optional[str] = None) -> Optional[str]:
    cands = []
    if os.path.isfile(name):
        cands.append(name)
    if os.path.isdir(name):
        cands.append(os.path.join(name, "tokenizer.json"))
    for d in (tokenizer_dir, os.environ.get("TB_TOKENIZER_DIR")):
        if d:
            cands.append(os.path.join(d, name, "tokenizer.json"))
            cands.append(os.path.join(d, name.replace("/", "--"), "tokenizer.json"))
    hf = os.environ.get("HF_HOME", os.path.join(os.path.expanduser("~"), ".cache", "huggingface"))
    cands += sorted(glob.glob(os.path.join(hf, "hub", "models--" + name.replace("/", "--"), "snapshots", "*",
                                           "tokenizer.json")))
    for c in cands:
        if os.path.isfile(c):
            return c
    return None


class TokenCounterModel:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.path = path
        self.tok = Tokenizer.from_file(path)

    def count(self, texts: List[str]) -> List[int]:
        if not texts:
            return []
        encs = self.tok.encode_batch(texts, add_special_tokens=True)
        return [len(e.tokens) for e in encs]


def load_tokenizer(name: str, tokenizer_dir: Optional[str] = None) -> TokenCounterModel:
    path = resolve_tokenizer_file(name, tokenizer_dir)
    if path is None:
        raise Unexpected("Error in loading tokenizer")
    try:
        return TokenCounterModel(path)
    except Exception as e:  # noqa: BLE001 - any load failure maps to the reference's error
        raise Unexpected("Error in loading tokenizer") from e
