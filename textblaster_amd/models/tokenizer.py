"""TokenCounter tokenizer (reference src/pipeline/token/token_counter.rs:8-43).

The reference calls ``Tokenizer::from_pretrained(name)`` (a Hugging Face Hub download). There is
no network here, so the name is resolved locally, in order:
  1. ``name`` is a path to a ``tokenizer.json`` file or to a directory containing one;
  2. ``<tokenizer_dir>/<name>/tokenizer.json`` (CLI ``--tokenizer-dir``, env ``TB_TOKENIZER_DIR``);
  3. the Hugging Face cache (``$HF_HOME`` / ``~/.cache/huggingface/hub/models--<name>/snapshots/*``).
Load failure raises ``Unexpected("Error in loading tokenizer")`` like the reference.

Counting = ``len(encode(text, add_special_tokens=True).tokens)``, batched through the Rust
tokenizers library's parallel ``encode_batch``. GPT-2-style byte-level BPE tokenizers also get a
:class:`BpeSpec` (:meth:`TokenCounterModel.bpe_spec`): the merge table as an open-addressed hash
table plus the byte ids, which the device pipeline counts with (csrc/common/bpe.h, k_bpe_count)
and ``count_native`` runs on the host (same algorithm; documents it cannot count exactly are
counted by ``tokenizers``).
"""
from __future__ import annotations

import glob
import os
import dataclasses
import json
from typing import List, Optional

import numpy as np

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


def bytes_to_unicode() -> List[str]:
    """GPT-2's byte -> printable character map of the ByteLevel pre-tokenizer."""
    bs = list(range(33, 127)) + list(range(161, 173)) + list(range(174, 256))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    m = dict(zip(bs, cs))
    return [chr(m[b]) for b in range(256)]


MAX_ADDED = 8  # csrc/common/bpe.h kBpeMaxAdded


@dataclasses.dataclass
class BpeSpec:
    """Device tables of a byte-level BPE tokenizer (csrc/common/bpe.h DevBpe)."""
    byte_id: np.ndarray    # uint32 [256]
    keys: np.ndarray       # uint64 [mask + 1]
    vals: np.ndarray       # uint64 [mask + 1]
    mask: int
    added: np.ndarray      # uint8: added-token contents, concatenated
    added_off: List[int]   # [n_added + 1]
    post_add: int          # tokens the post-processor adds


def _post_add(pp) -> Optional[int]:
    """Special tokens the post-processor adds to a single sequence, None if not known."""
    if pp is None:
        return 0
    t = pp.get("type")
    if t == "ByteLevel":
        return 0
    if t in ("RobertaProcessing", "BertProcessing"):
        return 2
    if t == "TemplateProcessing":
        n = 0
        for piece in pp.get("single", []):
            if "SpecialToken" in piece:
                sp = pp.get("special_tokens", {}).get(piece["SpecialToken"]["id"])
                if sp is None:
                    return None
                n += len(sp.get("ids", []))
            elif "Sequence" not in piece:
                return None
        return n
    if t == "Sequence":
        tot = 0
        for q in pp.get("processors", []):
            k = _post_add(q)
            if k is None:
                return None
            tot += k
        return tot
    return None


def build_bpe_spec(tj: dict) -> Optional[BpeSpec]:
    """BpeSpec of a parsed tokenizer.json, or None when the tokenizer is not a byte-level BPE the
    device counter reproduces exactly (no normalizer, ByteLevel regex pre-tokenizer without prefix
    space, plain BPE merges, no truncation / padding, known post-processor)."""
    from .. import native

    m = tj.get("model") or {}
    if m.get("type") != "BPE" or m.get("dropout") not in (None, 0, 0.0) or m.get("continuing_subword_prefix") \
            or m.get("end_of_word_suffix") or m.get("ignore_merges"):
        return None
    if tj.get("normalizer") is not None or tj.get("truncation") is not None or tj.get("padding") is not None:
        return None
    pt = tj.get("pre_tokenizer")
    if pt is not None and pt.get("type") == "Sequence" and len(pt.get("pretokenizers", [])) == 1:
        pt = pt["pretokenizers"][0]
    if pt is None or pt.get("type") != "ByteLevel" or pt.get("add_prefix_space") or not pt.get("use_regex", True):
        return None
    post = _post_add(tj.get("post_processor"))
    if post is None:
        return None
    vocab = m.get("vocab") or {}
    b2u = bytes_to_unicode()
    if any(ch not in vocab for ch in b2u):
        return None
    byte_id = np.array([vocab[ch] for ch in b2u], dtype=np.uint32)
    a, b, rank, nid = [], [], [], []
    for i, mg in enumerate(m.get("merges") or []):
        if isinstance(mg, str):
            parts = mg.split(" ")
            if len(parts) != 2:
                return None
        else:
            parts = mg
        x, y = parts
        if x not in vocab or y not in vocab or (x + y) not in vocab:
            return None
        a.append(vocab[x])
        b.append(vocab[y])
        rank.append(i)
        nid.append(vocab[x + y])
    u32 = lambda v: np.array(v, dtype=np.uint32)  # noqa: E731
    keys, vals, mask = native.host().bpe_build_table(u32(a), u32(b), u32(rank), u32(nid))
    added = [t["content"].encode("utf-8") for t in tj.get("added_tokens") or [] if t.get("content")]
    if len(added) > MAX_ADDED:
        return None
    off = [0]
    for t in added:
        off.append(off[-1] + len(t))
    return BpeSpec(byte_id, keys, vals, int(mask), np.frombuffer(b"".join(added) or b"\0", dtype=np.uint8).copy(),
                   off if added else [], post)


class TokenCounterModel:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.path = path
        self.tok = Tokenizer.from_file(path)
        self._spec = False

    def count(self, texts: List[str]) -> List[int]:
        if not texts:
            return []
        encs = self.tok.encode_batch(texts, add_special_tokens=True)
        return [len(e.tokens) for e in encs]

    def bpe_spec(self) -> Optional[BpeSpec]:
        """Device/native tables when this is a byte-level BPE tokenizer (else None); built once."""
        if self._spec is False:
            with open(self.path, encoding="utf-8") as f:
                self._spec = build_bpe_spec(json.load(f))
        return self._spec

    def count_native(self, data: np.ndarray, off: np.ndarray, nthreads: int = 8) -> np.ndarray:
        """Token counts of packed UTF-8 documents with the native byte-level BPE counter (host
        emulation of k_bpe_count); documents it returns -2 for (added-token text, invalid UTF-8,
        pre-tokens over 64 bytes) are counted by ``tokenizers``. Needs :meth:`bpe_spec`."""
        from .. import native

        sp = self.bpe_spec()
        if sp is None:
            raise Unexpected("count_native needs a byte-level BPE tokenizer")
        out = native.host().bpe_count(np.ascontiguousarray(data, dtype=np.uint8), np.ascontiguousarray(off, np.int64),
                                      sp.byte_id, sp.keys, sp.vals, sp.mask, sp.added, sp.added_off, sp.post_add,
                                      nthreads).astype(np.int64)
        bad = np.nonzero(out < 0)[0]
        if len(bad):
            out[bad] = self.count([bytes(data[off[k]:off[k + 1]]).decode("utf-8", "replace") for k in bad.tolist()])
        return out


def train_synthetic_bpe(path: str, vocab_size: int = 50257, n_docs: int = 20000, seed: int = 1) -> str:
    """Train a GPT-2-format byte-level BPE tokenizer (ByteLevel pre-tokenizer and post-processor,
    ``<|endoftext|>`` special token, ``vocab_size`` entries) on the synthetic Zipf corpus and save
    it as ``path`` (kept if it already exists). There is no network for the real gpt2 files: this
    stands in for them with the same model type, pre-tokenizer and vocabulary size; the token
    counts differ from real GPT-2, the work per byte is of the same kind."""
    if os.path.isfile(path):
        return path
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors, trainers

    from ..utils import synth

    texts = synth.make_corpus(n_docs, 1024, seed=seed, vocab="zipf")
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.post_processor = processors.ByteLevel(trim_offsets=False)
    tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=["<|endoftext|>"], show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(texts, tr)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.{os.getpid()}.tmp"
    tok.save(tmp)
    os.replace(tmp, path)
    return path


def load_tokenizer(name: str, tokenizer_dir: Optional[str] = None) -> TokenCounterModel:
    path = resolve_tokenizer_file(name, tokenizer_dir)
    if path is None:
        raise Unexpected("Error in loading tokenizer")
    try:
        return TokenCounterModel(path)
    except Exception as e:  # noqa: BLE001 - any load failure maps to the reference's error
        raise Unexpected("Error in loading tokenizer") from e
