"""Large GPU-vs-ICU differential (independent of the host emulation of the kernel source): 200,000
seeded documents from tests/gpu_fuzz_corpus.py — slices of the small-vocabulary and Zipf
synthetic corpora, Unicode-heavy random text (UAX#29 edge classes: combining marks, ZWJ / emoji
sequences, regional-indicator runs, MidLetter / MidNum punctuation, NBSP and other spaces,
Hebrew quotes, CR / CRLF) and the adversarial pool — through the device engine and through the
CPU engine with ICU4C segmentation (the oracle). Every document's status, first failing step,
reason string, output text and metadata must be identical. Needs an MI355X."""
import json
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gpu_fuzz_corpus import fuzz_docs  # noqa: E402

from textblaster_amd.utils import synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(REPO, "config", "bench_pipeline.yaml")
N = int(os.environ.get("TB_DIFF_N", "200000"))


def test_device_equals_icu_oracle_on_200k_fuzz_documents():
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine

    from test_emulated_device_path import outputs

    texts = fuzz_docs(N)
    data, off = synth.pack(texts)
    cfg = load_pipeline_config(CFG)
    a = Engine(cfg, backend="cuda", keep_reasons=True).process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", keep_reasons=True).process(data, off)
    bad = np.nonzero((a.status != b.status) | (a.fail_step != b.fail_step))[0]
    assert len(bad) == 0, [(int(k), texts[k][:80], int(a.fail_step[k]), int(b.fail_step[k])) for k in bad[:5]]
    assert a.reasons == b.reasons
    oa, ob = outputs(a), outputs(b)
    assert oa.keys() == ob.keys()
    diff = [k for k in oa if oa[k] != ob[k]]
    assert not diff, [(k, texts[k][:80], oa[k][2], ob[k][2]) for k in diff[:5]]
    # the corpus exercises every step: kept, excluded by several steps, CPU-routed documents
    assert len(set(int(x) for x in a.fail_step)) >= 4
    st = a.status
    assert (st == st.min()).sum() > 0 and (st == st.max()).sum() > 0
    meta = [m for _, _, m in oa.values() if m]
    assert any("Detected language confidence" in json.loads(m) for m in meta)
