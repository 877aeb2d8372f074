"""K16 (device resolve + output compaction, csrc/common/gate.h resolve_doc): the per-document
first failure, status and compacted kept / excluded texts computed from the device records must
equal the host resolver's — on the emulated device path here (same TB_HD function, same output
layout as k_resolve + k_compact), on the GPU in tests/test_gpu_e2e.py. Reference semantics:
executor.rs:32-46 (first failure wins) and producer_logic.rs:148-167 (kept / excluded routing)."""
import numpy as np
import pytest

from textblaster_amd import native
from textblaster_amd.config import load_pipeline_config
from textblaster_amd.pipeline import device as devmod
from textblaster_amd.pipeline.engine import Engine
from textblaster_amd.utils import metrics, synth

from test_emulated_device_path import EDGE, outputs


def _corpus(n=1200, seed=5):
    texts = synth.make_corpus(n, 900, seed=seed) + EDGE
    return synth.pack(texts)


def test_resolve_plan_built_for_device_only_pipelines():
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    eng = Engine(cfg, backend="emulate", nthreads=4)
    assert eng.device_runner.resolve_blob is not None
    assert len(eng.device_runner.resolve_blob) == native.host().SIZEOF_DEV_RESOLVE


def test_resolve_plan_refused_with_host_steps():
    # TokenCounter / C4BadWords run on the host: no device resolve, host assembly as before
    cfg = load_pipeline_config("tests/config/test_pipeline_config.yaml")
    eng = Engine(cfg, backend="emulate", nthreads=4)
    types = [s.type for s in cfg.pipeline]
    if "TokenCounter" in types or "C4BadWordsFilter" in types:
        assert eng.device_runner.resolve_blob is None


def test_device_resolve_outputs_equal_host_assembly(monkeypatch):
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    data, off = _corpus()
    before = metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get()
    a = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True).process(data, off)
    assert metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get() == before  # fast path taken
    monkeypatch.setenv("TB_TUNE", "device_resolve=0")
    b = Engine(cfg, backend="emulate", nthreads=4, keep_reasons=True).process(data, off)
    c = Engine(cfg, backend="cpu", segmentation="icu", nthreads=4, keep_reasons=True).process(data, off)
    for x in (b, c):
        np.testing.assert_array_equal(a.status, x.status)
        np.testing.assert_array_equal(a.fail_step, x.fail_step)
        assert a.reasons == x.reasons
        assert outputs(a) == outputs(x)
    # output parts are in document order, kept then excluded
    for p in a.kept + a.excluded:
        assert np.all(np.diff(p.rows) > 0)


def test_resolve_host_matches_decisions_per_document():
    """resolve_host over stage/C4 records == BatchState decisions (fail step, status, content)."""
    h = native.host()
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    eng = Engine(cfg, backend="emulate", nthreads=4)
    run = eng.device_runner
    data, off = _corpus(400, seed=9)
    res = run.run(data, off)
    r = res.resolved
    assert r is not None and r.err == 0
    n = len(off) - 1
    assert r.fail.shape == (n,) and r.status.shape == (n,)
    assert set(np.unique(r.status)).issubset({0, 1, 3})
    assert np.all((r.fail >= 0) == (r.status != 0))
    ((kr, ko, kt),), ((xr, xo, xt),) = r.parts()
    assert len(kr) == np.count_nonzero(r.status == 0) and len(xr) == np.count_nonzero(r.status == 1)
    assert ko[0] == 0 and ko[-1] == len(kt) and xo[0] == 0 and xo[-1] == len(xt)
    # a document filtered before the C4 step carries its input text
    c4 = [i for i, s in enumerate(cfg.pipeline) if s.type == "C4QualityFilter"][0]
    for k, d in enumerate(xr.tolist()):
        if r.fail[d] < c4:
            assert bytes(xt[xo[k]:xo[k + 1]]) == bytes(data[off[d]:off[d + 1]])
    del h


def test_resolve_disagreement_falls_back_to_host(monkeypatch):
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    data, off = _corpus(300, seed=3)
    eng = Engine(cfg, backend="emulate", nthreads=4)
    good = outputs(eng.process(data, off))
    orig = devmod.EmulatedRunner.run

    def corrupt(self, d, o, bw=None):
        res = orig(self, d, o, bw)
        res.resolved.status = res.resolved.status.copy()
        res.resolved.status[0] ^= 1  # flip one document's outcome
        return res

    monkeypatch.setattr(devmod.EmulatedRunner, "run", corrupt)
    before = metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get()
    bad = outputs(eng.process(data, off))
    assert metrics.DEVICE_RESOLVE_FALLBACK_TOTAL._value.get() == before + 1
    assert bad == good


@pytest.mark.parametrize("n", [0, 1, 5])
def test_resolve_tiny_batches(n):
    cfg = load_pipeline_config("config/bench_pipeline.yaml")
    texts = synth.make_corpus(n, 600, seed=1) if n else []
    data, off = synth.pack(texts)
    a = Engine(cfg, backend="emulate", nthreads=2).process(data, off)
    b = Engine(cfg, backend="cpu", segmentation="icu", nthreads=2).process(data, off)
    assert outputs(a) == outputs(b)


class _FakeDev:
    """Stand-in for a hiprt.DevArray (slicing + to_host) to exercise LazyVersions on the CPU."""

    def __init__(self, a):
        self.a = a
        self.fetches = 0

    def __getitem__(self, sl):
        return _FakeDev(self.a[sl])

    def to_host(self):
        self.fetches += 1
        return self.a.copy()


def test_lazy_versions_download_once_on_access():
    vb = _FakeDev(np.frombuffer(b"abcdefXXXX", np.uint8).copy())
    vo = _FakeDev(np.array([0, 2, 6], np.int64))
    lv = devmod.LazyVersions({1: (vb, vo)})
    assert list(lv) == [1] and len(lv) == 1
    assert vo.fetches == 0  # nothing downloaded yet
    d, o = lv[1]
    assert bytes(d) == b"abcdef" and o.tolist() == [0, 2, 6]
    assert vo.fetches == 1
    assert [k for k, _ in lv.items()] == [1] and vo.fetches == 1
