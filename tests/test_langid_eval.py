"""Held-out accuracy of the bundled language-id model (tools/eval_langid.py; evaluation text
shares no sentence with the training corpus and is not generated from the benchmark
vocabulary). Lingua parity itself is unpinned (no lingua models offline): this pins the
detector's quality on real sentences of the five candidate languages."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from eval_langid import evaluate  # noqa: E402

from textblaster_amd.models.langid import LANGS, load_default  # noqa: E402


def test_heldout_accuracy():
    res = evaluate(load_default())
    sent, doc = res["sentence"], res["document"]
    acc_s = np.diag(sent[:, :len(LANGS)]) / sent.sum(1)
    acc_d = np.diag(doc[:, :len(LANGS)]) / doc.sum(1)
    assert sent.sum(1).min() >= 100  # >= 100 held-out sentences per language
    for i, lang in enumerate(LANGS):
        if lang in ("eng", "swe"):
            assert acc_s[i] >= 0.97 and acc_d[i] >= 0.97, (lang, acc_s[i], acc_d[i])
        elif lang == "dan":  # Danish / Bokmal share most trigrams on single sentences
            assert acc_s[i] >= 0.95 and acc_d[i] >= 0.97, (lang, acc_s[i], acc_d[i])
        else:  # Bokmal / Nynorsk: the close pair
            assert acc_s[i] >= 0.90 and acc_d[i] >= 0.97, (lang, acc_s[i], acc_d[i])
