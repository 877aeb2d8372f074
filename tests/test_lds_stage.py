"""LDS-resident short-document stage algorithm (csrc/common/lds_stage.h), run sequentially on the
host (emulate_stage_lds), against the generic algorithm (analyze_stage, emulate_stage) record
for record: the same allocation order as the device kernel, so the same documents overflow
their slice and take the retry path. Runs without a GPU."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from adversarial import adversarial_corpus  # noqa: E402
from test_emulated_device_path import EDGE  # noqa: E402

from textblaster_amd.config import load_pipeline_config
from textblaster_amd.pipeline.device import lds_buckets, lds_doc_slices, launch_order
from textblaster_amd.pipeline.plan import build_plan
from textblaster_amd.utils import synth


def _corpus():
    rng = np.random.default_rng(3)
    words = "the cat sat on the mat and the dog ran".split()
    rep = [" ".join(rng.choice(words[:int(rng.integers(2, 10))], size=int(rng.integers(20, 400)))) for _ in range(150)]
    danish = ["Jeg er ikke sikker på, at det er det rigtige. Det var også godt, når vi KAN være der.",
              "OG SÅ VAR DER IKKE MERE. Hun havde været der før, men ikke siden.",
              "Være eller ikke være, det er spørgsmålet. Også HER."]
    # segments longer than a 64-code-point chunk: long words, URLs, whitespace and punctuation
    # runs, word chars after long non-word runs (state carried across chunks)
    long_tokens = ["a" * 70 + " b", "x " + "y" * 130 + ".", "http://example.com/" + "q" * 150 + " end.",
                   " " * 150 + "word " + "\t" * 70 + "more", "." * 200 + "x", "-" * 90 + "ab" + "," * 70,
                   "\u0301" * 80 + "a", " " + "\u0301" * 70 + " x", "word" + "\u00e6" * 100 + " z",
                   ("ab" * 40 + " ") * 5, "1" * 100 + ".5 " + "2,000" * 30]
    return (synth.make_corpus(1200, 1100, seed=5) + EDGE + adversarial_corpus() + rep + danish * 3 + long_tokens
            + ["ab c a bc ab c a bc " * 20, "a b a b a b a b a b a b a b a b", "x y z\n\nx y z\nx y z",
               "abab ab ab abab " * 30, "aa aaa a aaaa aa a aaa " * 25])


@pytest.fixture(scope="module", params=["config/bench_pipeline.yaml", "config/pipeline_config.yaml"])
def setup(host, request):
    """The bench pipeline (English stop words) and the reference default pipeline (Danish stop
    words, some with non-ASCII letters)."""
    from textblaster_amd.models.langid import load_default

    cfg = load_pipeline_config(request.param)
    cfg.pipeline = [s for s in cfg.pipeline if s.type != "TokenCounter"]
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    texts = _corpus()
    data, off = synth.pack(texts)
    return steps, plan, load_default().native(), data, off


@pytest.mark.parametrize("per_byte,fixed", [(64, 4096), (10, 1024), (6, 512), (3, 256)])
def test_lds_records_equal_generic(host, setup, per_byte, fixed):
    steps, plan, lid, data, off = setup
    lens = np.diff(off)
    sl = np.where(lens <= 4096, np.minimum(per_byte * lens + fixed, 160 * 1024), 0).astype(np.uint32)
    retried_any = 0
    for idx in plan.stages:
        r0, f0 = host.emulate_stage(steps, idx, data, off, 8, lid, 10240)
        r1, f1, rt = host.emulate_stage_lds(steps, idx, data, off, sl, 8, lid)
        np.testing.assert_array_equal(r0, r1)
        np.testing.assert_array_equal(f0, f1)
        retried_any += int(rt.sum())
        if per_byte >= 64:
            assert rt.sum() == 0
    if per_byte <= 6:
        assert retried_any > 100  # the retry path is exercised


def test_lds_records_with_gate_skips(host, setup):
    steps, plan, lid, data, off = setup
    n = len(off) - 1
    dead = (np.arange(n) % 3 == 0).astype(np.uint8)
    sl = lds_doc_slices(np.diff(off), 4096, 10, 1024)
    for idx in plan.stages:
        r0, f0 = host.emulate_stage(steps, idx, data, off, 8, lid, 10240, dead)
        r1, f1, _ = host.emulate_stage_lds(steps, idx, data, off, sl, 8, lid, dead)
        np.testing.assert_array_equal(r0, r1)
        np.testing.assert_array_equal(f0, f1)


def test_bucket_planner_covers_positions_and_bounds_slices():
    rng = np.random.default_rng(1)
    lens = np.concatenate([rng.integers(0, 5000, 5000), [0, 1, 15, 16, 4096, 4097]]).astype(np.int64)
    perm = launch_order(lens)
    lp = lens[perm]
    n_long = int(np.count_nonzero(lens > 4096))
    b = lds_buckets(lp[n_long:], 10, 1024)
    assert b[0][0] == 0 and b[-1][1] == len(lp) - n_long
    for (p0, p1, sl), nxt in zip(b, b[1:] + [None]):
        assert p1 > p0 and sl % 256 == 0 and sl <= 159 * 1024
        assert sl >= 10 * int(lp[n_long + p0:n_long + p1].max()) + 1024  # the longest document fits
        if nxt is not None:
            assert nxt[0] == p1
    sl = lds_doc_slices(lens, 4096, 10, 1024)
    assert np.all((sl == 0) == (np.isin(np.arange(len(lens)), perm[:n_long])))
