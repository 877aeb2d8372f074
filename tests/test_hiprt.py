"""Native HIP runtime layer (csrc/hip/runtime.hip via ops/hiprt.py): copies, fills, views,
pinned memory, events, the caching allocators and the strided scan kernel, against numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from textblaster_amd.ops import hiprt

    assert hiprt.device_count() > 0
    hiprt.set_device(0)
    return hiprt


def test_roundtrip_views_and_fill(rt):
    a = np.arange(1000, dtype=np.int64) * 7
    d = rt.to_device(a)
    assert np.array_equal(d.to_host(), a)
    assert np.array_equal(d[10:20].to_host(), a[10:20])
    assert np.array_equal(d.view(np.int32)[:4].to_host(), a.view(np.int32)[:4])
    z = rt.zeros(333, np.int16)
    assert not z.to_host().any()
    d[5:9].fill_(0)
    b = a.copy()
    b[5:9] = 0
    assert np.array_equal(d.to_host(), b)


def test_pinned_async_copies_and_events(rt):
    s = rt.Stream()
    n = 1 << 20
    src = rt.pinned(n, np.uint8)
    src[:] = np.random.default_rng(0).integers(0, 255, n, dtype=np.uint8)
    d = rt.empty(n, np.uint8)
    dst = rt.pinned(n, np.uint8)
    e0 = rt.Event(timing=True).record(s)
    d.copy_from_host(src, s)
    d.copy_to_host(dst, s)
    e1 = rt.Event(timing=True).record(s)
    e1.synchronize()
    assert e1.query()
    assert np.array_equal(src, dst)
    assert e0.elapsed_time(e1) >= 0.0


def test_scan_strided_matches_numpy(rt):
    rng = np.random.default_rng(1)
    for n in (1, 2, 63, 1024, 1025, 2047, 2048, 2049, 12295, 100_003, 600_001):
        src = rng.integers(0, 1000, 2 * n, dtype=np.int64)
        d = rt.to_device(src)
        out = rt.zeros(n, np.int64)
        rt.scan_strided_i64(d[1:], 2, n, out)
        assert np.array_equal(out.to_host(), np.cumsum(src[1::2])), n


def test_caching_allocator_reuses_blocks(rt):
    n = (37 << 20) + 12345               # an unusual size: its cached block is the only fit
    a = rt.empty(n, np.uint8)
    p = a.data_ptr()
    del a
    st0 = rt.cache_stats()
    assert st0["device_cached"] >= n
    b = rt.empty(n, np.uint8)
    assert b.data_ptr() == p            # the freed block came back from the cache
    assert rt.cache_stats()["device_in_use"] >= st0["device_in_use"] + n


def test_no_torch_in_device_path():
    """The single-GPU pipeline never imports PyTorch (start-up cost, profiles/r2_e2e)."""
    import subprocess
    import sys

    code = ("import sys, numpy as np\n"
            "from textblaster_amd.config import load_pipeline_config\n"
            "from textblaster_amd.pipeline.engine import Engine\n"
            "from textblaster_amd.utils import synth\n"
            "e = Engine(load_pipeline_config('config/bench_pipeline.yaml'), backend='cuda', device='cuda:0')\n"
            "d, o = synth.pack(synth.make_corpus(64, 512, seed=2))\n"
            "r = e.process(d, o)\n"
            "assert r.n_kept + r.n_excluded + len(r.error_rows) == 64\n"
            "print('torch' in sys.modules)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "False"
