"""Adversarial inputs on the CPU: the device algorithms' host emulation against the ICU oracle
on fuzz-pool documents and chunk-boundary cases, and forced hash collisions (keys cut to 2
bits inside canonicalize) leaving every record unchanged (equality is decided by byte /
id verification, never by a hash)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from adversarial import adversarial_corpus  # noqa: E402
from test_emulated_device_path import outputs  # noqa: E402

from textblaster_amd.config import load_pipeline_config  # noqa: E402
from textblaster_amd.pipeline.engine import Engine  # noqa: E402
from textblaster_amd.pipeline.plan import build_plan  # noqa: E402
from textblaster_amd.utils import synth  # noqa: E402


def test_emulated_path_equals_oracle_on_adversarial_corpus():
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    texts = adversarial_corpus()
    data, off = synth.pack(texts)
    a = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True).process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True).process(data, off)
    np.testing.assert_array_equal(a.status, b.status)
    np.testing.assert_array_equal(a.fail_step, b.fail_step)
    assert a.reasons == b.reasons
    oa, ob = outputs(a), outputs(b)
    diff = [k for k in oa if oa[k] != ob.get(k)]
    assert not diff, [texts[k] for k in diff[:3]]


def test_forced_hash_collisions_do_not_change_records(host):
    cfg = load_pipeline_config("config/pipeline_config.yaml")
    cfg.pipeline = [s for s in cfg.pipeline if s.type in ("GopherRepetitionFilter", "GopherQualityFilter",
                                                          "FineWebQualityFilter")]
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    texts = synth.make_corpus(400, 900, seed=5) + adversarial_corpus(7, 150)
    data, off = synth.pack(texts)
    for idx in plan.stages:
        ref, fl = host.emulate_stage(steps, idx, data, off, 4, None, 0, None, False)
        got, fl2 = host.emulate_stage(steps, idx, data, off, 4, None, 0, None, True)
        np.testing.assert_array_equal(fl, fl2)
        np.testing.assert_array_equal(ref, got)
