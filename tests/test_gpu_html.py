"""K17 GPU HTML entity decoder (csrc/hip/html.hip) vs. the host C++ decoder (csrc/host/html.cpp),
which is the oracle of the reader's decode_html_entities step (reference parquet_reader.rs:177-179)."""
import numpy as np
import pytest

from textblaster_amd import native
from textblaster_amd.utils import synth

pytestmark = pytest.mark.gpu

PIECES = ["&amp;", "&lt;", "&gt;", "&quot;", "&nbsp;", "&AElig;", "&NotEqualTilde;", "&copy", "&#65;", "&#x41;",
          "&#X1F600;", "&#0;", "&#x110000;", "&#xD800;", "&#55296;", "&#;", "&#x;", "&;", "&", "&&amp;",
          "&amp", "&unknownentity;", "&#" + "0" * 70 + "65;", "&" + "a" * 45 + ";", "&ä;", "&#1114111;",
          "æøå", "plain ", "tekst ", "\n", "&eacute;", "&Eacute;", "&frac12;", "&#9;"]


def _corpus(rng, n):
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 120))
        out.append("".join(PIECES[int(j)] for j in rng.integers(0, len(PIECES), size=k)))
    out += ["", "&", "no entities at all " * 20, "x" * 63 + "&amp;", "x" * 64 + "&#" + "0" * 100 + "66;tail"]
    return out


def test_gpu_html_decode_matches_host():
    from textblaster_amd.ops import hiprt
    from textblaster_amd.ops.html import HtmlDecoder

    h = native.host()
    rng = np.random.default_rng(3)
    texts = _corpus(rng, 3000)
    data, off = synth.pack(texts)
    dec = HtmlDecoder("cuda:0")
    od, oo = dec.decode(hiprt.to_device(data), hiprt.to_device(off.astype(np.int64)))
    with hiprt.stream(dec.stream):
        od = od.to_host()
        oo = oo.to_host()
    for i, t in enumerate(texts):
        want = h.html_decode(t).encode("utf-8")
        got = bytes(od[oo[i]:oo[i + 1]])
        assert got == want, (i, t[:80], got[:80], want[:80])


def test_gpu_html_decode_host_arrays_like_batch_decoder():
    from textblaster_amd.ops.html import HtmlDecoder

    h = native.host()
    texts = ["a &amp; b", "plain", "&#x263A; &hearts;"]
    data, off = synth.pack(texts)
    want = h.html_decode_batch(np.ascontiguousarray(data), np.ascontiguousarray(off), 2)
    got = HtmlDecoder("cuda:0").decode_host(data, off)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    plain, poff = synth.pack(["no refs here", "none"])
    assert HtmlDecoder("cuda:0").decode_host(plain, poff) is None


def test_run_with_gpu_html_decode_equals_host_decode(tmp_path):
    """`run --html-decode gpu` writes the same Parquet outputs as the host decoder."""
    import os

    import pyarrow.parquet as pq

    from textblaster_amd.data_model import TextDocument
    from textblaster_amd.io.parquet import ParquetWriter
    from textblaster_amd.parallel.dist import DistContext
    from textblaster_amd.runner import RunConfig, run

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = os.path.join(repo, "config", "bench_pipeline.yaml")
    rng = np.random.default_rng(5)
    texts = [t + " " + s for t, s in zip(synth.make_corpus(800, 512, seed=4), _corpus(rng, 800))]
    inp = str(tmp_path / "in.parquet")
    w = ParquetWriter(inp)
    w.write_batch([TextDocument(f"h{i}", t, "html") for i, t in enumerate(texts)])
    w.close()
    tabs = {}
    for mode in ("cpu", "gpu"):
        o, e = str(tmp_path / f"{mode}.o.parquet"), str(tmp_path / f"{mode}.e.parquet")
        ctx = DistContext()
        ctx.device = "cuda:0"
        run(RunConfig(inp, o, e, cfg, backend="cuda", unit_rows=300, html_decode=mode), ctx)
        tabs[mode] = (pq.read_table(o), pq.read_table(e))
    for a, b in zip(tabs["cpu"], tabs["gpu"]):
        assert a.column("id").equals(b.column("id")) and a.column("text").equals(b.column("text"))
