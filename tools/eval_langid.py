"""Held-out evaluation of the language-id model (the LanguageDetectionFilter's detector).

The evaluation text (textblaster_amd/models/data/langid_eval/<lang>.txt) shares no sentence
with the training corpus (models/data/langid_corpus) and no vocabulary generator with the
synthetic benchmark corpus (utils/synth.VOCAB). The five files are parallel: the same 40
everyday statements written in each language, so only the language differs between classes.

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


def report(res) -> str:
    lines = ["# Language-id evaluation (held-out set)", "",
             "Model: `textblaster_amd/models/data/langid_v1.npz` (hashed char 1-3-gram bag, bf16 head).",
             "Evaluation text: `textblaster_amd/models/data/langid_eval/` (40 parallel sentences per language,",
             "no overlap with the training corpus, not generated from the benchmark vocabulary).", ""]
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
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    model = load(a.model) if a.model else load_default()
    text = report(evaluate(model))
    print(text)
    if a.out:
        with open(a.out, "w", encoding="utf-8") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
