"""Host output formatting: the allocation-free Rust `{:.N}` / f64 Display formatters against
Python's correctly rounded formatting, and the direct-to-JSON metadata path of output assembly
against the map-based path (TB_META_FAST=0)."""
import os
import random
import struct

import numpy as np

from textblaster_amd.config import load_pipeline_config
from textblaster_amd.pipeline.engine import Engine
from textblaster_amd.utils import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fmt_fixed_matches_correct_rounding(host):
    rng = random.Random(5)
    vals = [0.0, -0.0, 0.125, 0.375, 2.675, 1.005, 0.5, 1.5, 2.5, 0.045, 0.00005, 123456.785, 1e13 + 0.5, 5e-324,
            0.30000000000000004, 99.995, -0.001, -2.5, 1e15, float("inf"), float("nan")]
    vals += [rng.random() * 10 ** rng.randint(-6, 12) for _ in range(20000)]
    vals += [k / 200.0 for k in range(2000)] + [k / 20000.0 for k in range(2000)]
    vals += [struct.unpack("<d", struct.pack("<Q", rng.getrandbits(62)))[0] for _ in range(2000)]
    for v in vals:
        for p in range(5):
            want = format(v, f".{p}f")
            if want in ("inf", "nan", "-inf"):
                continue
            assert host.fmt_fixed(v, p) == want, (v, p)


def test_fmt_f64_shortest_roundtrip(host):
    rng = random.Random(9)
    for _ in range(5000):
        v = rng.random() ** rng.randint(1, 40)
        s = host.fmt_f64(v)
        assert "e" not in s and float(s) == v


def _collect(eng, data, off, meta):
    res = eng.process(data, off, meta)
    out = []
    for part in res.kept + res.excluded:
        md, mo, mv = part.meta_data, part.meta_off, part.meta_valid
        for j, r in enumerate(part.rows):
            out.append((int(r), bytes(md[mo[j]:mo[j + 1]]) if mv[j] else None))
    return sorted(out)


def test_direct_json_metadata_equals_map_path(monkeypatch):
    cfg = load_pipeline_config(os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    eng = Engine(cfg, backend="cpu", segmentation="rules", nthreads=2)
    texts = synth.make_corpus(600, 600, seed=21)
    data, off = synth.pack(texts)
    monkeypatch.setenv("TB_META_FAST", "1")
    fast = _collect(eng, data, off, None)
    monkeypatch.setenv("TB_META_FAST", "0")
    slow = _collect(eng, data, off, None)
    assert fast == slow
    assert sum(1 for _, m in fast if m) > 500


def test_direct_json_metadata_with_input_metadata(monkeypatch):
    """Input metadata (the CLI path's common case): the direct path appends the steps' members to
    the input members; inputs holding a key a step writes, invalid JSON, empty objects, escapes and
    null rows must come out exactly as from the map-based path."""
    cfg = load_pipeline_config(os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    eng = Engine(cfg, backend="cpu", segmentation="rules", nthreads=2)
    texts = synth.make_corpus(600, 600, seed=22)
    data, off = synth.pack(texts)
    kinds = ['{"url":"https://example.com/%d"}', '{}', 'not json', '{"c4_filter_status":"x","a":"b"}',
             '{"Detected language":"xx"}', '{"k\\"q":"v\\\\n\\u00e6 \\u4e2d"}', '{"a":"1","b":"2","c":"3"}', None,
             # the canonical-text splice must fall back for every non-canonical form
             '{ "a": "1" }', '{"a":"1","a":"2"}', '{"a":1}', '{"a":"æ 中 ü","b":""}', '{"a":"x\ty"}', '{"a":"1",}',
             '{"":""}', '{"a":"1"}}', '{"a":"1","token_count":"3"}', "{" + ",".join(f'"k{j}":"v"' for j in range(17)) + "}",
             "{" + ",".join(f'"k{j}":"v"' for j in range(16)) + "}"]
    metas = [kinds[i % len(kinds)] for i in range(len(texts))]
    enc = [(m % i if "%d" in m else m).encode() if m is not None else b"" for i, m in enumerate(metas)]
    mo = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=mo[1:])
    md = np.frombuffer(b"".join(enc), dtype=np.uint8).copy()
    mv = np.array([m is not None for m in metas], dtype=np.uint8)
    monkeypatch.setenv("TB_META_FAST", "1")
    fast = _collect(eng, data, off, (md, mo, mv))
    monkeypatch.setenv("TB_META_FAST", "0")
    slow = _collect(eng, data, off, (md, mo, mv))
    assert fast == slow
    assert any(m and m.startswith(b'{"url"') for _, m in fast)


def test_native_pool_cpu_is_attributed_per_job(host):
    """The worker pool charges its jobs' CPU time to the submitting call site's tag (the e2e JSON's
    pool_cpu_seconds_by_job): output assembly shows up under "assemble"."""
    cfg = load_pipeline_config(os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    eng = Engine(cfg, backend="cpu", segmentation="rules", nthreads=2)
    texts = synth.make_corpus(400, 600, seed=23)
    data, off = synth.pack(texts)
    before = dict(host.pool_cpu_stats())
    eng.process(data, off)
    after = dict(host.pool_cpu_stats())
    assert after.get("assemble", 0.0) > before.get("assemble", 0.0)
    assert after.get("cpu_steps", 0.0) > before.get("cpu_steps", 0.0)
