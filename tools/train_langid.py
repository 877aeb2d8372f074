"""Train the language-id weights (textblaster_amd/models/data/langid_v2.npz).

Model (csrc/common/langid.h): per hashed character 1..4-gram bucket an int16 row of fixed-point
logit contributions to the 5 languages (scale 1/1024) plus a bias; logits = mean of the
document's rows + b. Trained as a mean-mode EmbeddingBag(buckets, 5) + bias with softmax cross
entropy, then exported in fixed point (|P| < 32, clamped while training).

Training text: the hand-written sentences in models/data/langid_corpus/<lang>.txt (whole
sentences, runs of sentences and sentence fragments). Random word sequences from the
synthetic-corpus vocabularies (utils/synth.VOCAB) are off by default (--vocab-share 0), so the
benchmark corpus is not generated from the training text; the held-out evaluation
(tools/eval_langid.py, models/data/langid_eval) shares nothing with either. Features come from
the native featurizer (_tbhost.langid_buckets), so training and inference hash identically.
Label smoothing keeps the confidence of short texts moderate, like lingua's relative confidences.

    python tools/train_langid.py [--epochs 12] [--n 10000] [--out path]
"""
import argparse
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from textblaster_amd import native  # noqa: E402
from textblaster_amd.models.langid import DATA_DIR, LANGS  # noqa: E402
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--out", default=os.path.join(DATA_DIR, "langid_v2.npz"))
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
    table = torch.nn.EmbeddingBag(h.LID_BUCKETS, len(LANGS), mode="mean")
    torch.nn.init.zeros_(table.weight)
    bias = torch.nn.Parameter(torch.zeros(len(LANGS)))
    opt = torch.optim.Adam(list(table.parameters()) + [bias], lr=0.02)
    lossf = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    lim = 32767.0 / h.LID_SCALE
    bs = 256
    for ep in range(args.epochs):
        order = torch.randperm(len(feats))
        tot = 0.0
        for k in range(0, len(order), bs):
            idx = order[k:k + bs].tolist()
            flat = torch.from_numpy(np.concatenate([feats[i] for i in idx]))
            offs = torch.tensor([0] + list(np.cumsum([len(feats[i]) for i in idx])[:-1]))
            loss = lossf(table(flat, offs) + bias, labels[idx])
            opt.zero_grad()
            loss.backward()
            opt.step()
            with torch.no_grad():
                table.weight.clamp_(-lim, lim)
            tot += loss.item() * len(idx)
        print(f"epoch {ep} loss {tot / len(feats):.4f}", flush=True)
    P = np.zeros((h.LID_BUCKETS, h.LID_ROW), dtype=np.int16)
    P[:, :len(LANGS)] = np.clip(np.rint(table.weight.detach().numpy() * h.LID_SCALE), -32767, 32767).astype(np.int16)
    b = np.zeros(h.LID_ROW, dtype=np.float32)
    b[:len(LANGS)] = bias.detach().numpy()
    np.savez(args.out, P=P.reshape(-1), b=b)
    print("saved", args.out, os.path.getsize(args.out))


if __name__ == "__main__":
    main()
