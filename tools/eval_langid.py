"""Held-out evaluation of the language-id model (the LanguageDetectionFilter's detector).

The evaluation text (textblaster_amd/models/data/langid_eval/<lang>.txt) shares no sentence
with the training corpus (models/data/langid_corpus) and no vocabulary generator with the
synthetic benchmark corpus (utils/synth.VOCAB). The five files are parallel: the same 110
everyday statements written in each language, so only the language differs between classes.
A reliability table (accuracy per confidence bucket) shows how the confidence the filter gates
on (LanguageDetectionFilter min_confidence, 0.65 in the reference config) relates to accuracy.

Reported on two granularities: single sentences, and documents of 3 consecutive sentences
(the filter sees whole documents). Accuracy per language + confusion matrix (rows = truth).

    python tools/eval_langid.py [--model path.npz] [--out profiles/langid_eval.md]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from textblaster_amd.models.langid import DATA_DIR, LANGS, NAMES, load, load_default  # noqa: E402


def eval_sets():
    sets = {}
    for lang in LANGS:
        with open(os.path.join(DATA_DIR, "langid_eval", f"{lang}.txt"), encoding="utf-8") as f:
            sents = [s.strip() for s in f if s.strip()]
        docs = [" ".join(sents[i:i + 3]) for i in range(0, len(sents) - 2, 3)]
        sets[lang] = {"sentence": sents, "document": docs}
    return sets


def evaluate(model):
    res = {}
    for gran in ("sentence", "document"):
        conf = np.zeros((len(LANGS), len(LANGS) + 1), dtype=np.int64)  # last column: undetected
        for ti, lang in enumerate(LANGS):
            for text in eval_sets()[lang][gran]:
                name, _ = model.detect(text)
                pi = NAMES.index(name) if name in NAMES else len(LANGS)
                conf[ti, pi] += 1
        res[gran] = conf
    return res


BUCKETS = [0.0, 0.4, 0.5, 0.6, 0.65, 0.7, 0.8, 0.9, 1.0001]


def reliability(model, gran="sentence"):
    """[(lo, hi, n, correct)] over every held-out sample's (confidence, correct?)."""
    rows = [[lo, hi, 0, 0] for lo, hi in zip(BUCKETS[:-1], BUCKETS[1:])]
    for ti, lang in enumerate(LANGS):
        for text in eval_sets()[lang][gran]:
            name, conf = model.detect(text)
            ok = name == NAMES[ti]
            for r in rows:
                if r[0] <= conf < r[1]:
                    r[2] += 1
                    r[3] += int(ok)
                    break
    return rows


def report(res, rel=None) -> str:
    lines = ["# Language-id evaluation (held-out set)", "",
             "Model: `textblaster_amd/models/data/langid_v3.npz` (fastText int8 two-bag embedding + bf16 MFMA head),",
             "trained by `tools/train_langid.py` on `models/data/langid_corpus/` (~260-300 hand-written lines",
             "per language, ~20-25 KB each). Evaluation text: `textblaster_amd/models/data/langid_eval/`",
             "(110 parallel sentences per language, no overlap with the training corpus, not generated from",
             "the benchmark vocabulary). Lingua parity is unpinned (no lingua models offline).", ""]
    for gran, conf in res.items():
        acc = np.diag(conf[:, :len(LANGS)]) / conf.sum(1)
        lines.append(f"## {gran}s ({int(conf.sum())} samples)")
        lines.append("")
        lines.append("| truth \\ predicted | " + " | ".join(LANGS) + " | none | accuracy |")
        lines.append("|---|" + "---|" * (len(LANGS) + 2))
        for i, lang in enumerate(LANGS):
            lines.append(f"| {lang} | " + " | ".join(str(int(v)) for v in conf[i]) + f" | {100 * acc[i]:.1f}% |")
        tot = np.trace(conf[:, :len(LANGS)]) / conf.sum()
        lines.append("")
        lines.append(f"Overall accuracy: {100 * tot:.1f}%")
        lines.append("")
    for gran, rows in (rel or {}).items():
        lines.append(f"## reliability ({gran}s): accuracy per confidence bucket")
        lines.append("")
        lines.append("| confidence | samples | correct | accuracy |")
        lines.append("|---|---|---|---|")
        for lo, hi, n, c in rows:
            acc = f"{100 * c / n:.1f}%" if n else "-"
            lines.append(f"| [{lo:.2f}, {min(hi, 1.0):.2f}) | {n} | {c} | {acc} |")
        n_pass = sum(n for lo, _, n, _ in rows if lo >= 0.65)
        c_pass = sum(c for lo, _, _, c in rows if lo >= 0.65)
        n_all = sum(r[2] for r in rows)
        lines.append("")
        lines.append(f"At the reference gate (confidence >= 0.65): {n_pass}/{n_all} samples pass "
                     f"({100 * n_pass / max(n_all, 1):.1f}%), {100 * c_pass / max(n_pass, 1):.1f}% of them correctly labelled.")
        lines.append("")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    model = load(a.model) if a.model else load_default()
    text = report(evaluate(model), {g: reliability(model, g) for g in ("sentence", "document")})
    print(text)
    if a.out:
        with open(a.out, "w", encoding="utf-8") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
