"""Parquet text-column decoding on the device (csrc/hip/parquet.hip, ops/parquet_gpu.py) against
pyarrow's decoder of the same files: Snappy and stored chunks, data pages v1 and v2, PLAIN and
dictionary values (including the writer's dictionary -> PLAIN fallback), nulls, non-ASCII text,
long documents (Snappy copies beyond the 32 KB LDS history, multi-byte literal lengths) and
highly repetitive text (self-overlapping copies). The CPU part checks the page directory."""
import os
import random

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from textblaster_amd.io.parquet import string_column_buffers
from textblaster_amd.utils import synth


def _texts(seed: int, n: int):
    rng = random.Random(seed)
    base = synth.make_corpus(min(n, 400), 700, seed=seed)
    out = []
    for i in range(n):
        r = rng.random()
        if r < 0.05:
            out.append(None)
        elif r < 0.08:
            out.append("")
        elif r < 0.12:
            out.append("blåbærgrød ΣΑΣ 日本語 \U0001F44D " * rng.randint(1, 40))
        elif r < 0.14:
            out.append("a" * rng.randint(1, 5000))  # self-overlapping copies (offset 1)
        elif r < 0.16:
            # long document: copies reaching further back than the LDS history
            out.append(" ".join(rng.choice(base) for _ in range(rng.randint(60, 120))))
        else:
            out.append(rng.choice(base))
    return out


CASES = {
    "snappy_dict_v1": dict(compression="snappy", use_dictionary=True, data_page_version="1.0"),
    "snappy_plain_v1": dict(compression="snappy", use_dictionary=False, data_page_version="1.0"),
    "stored_plain_v1": dict(compression="none", use_dictionary=False, data_page_version="1.0"),
    "snappy_dict_v2": dict(compression="snappy", use_dictionary=True, data_page_version="2.0"),
    "snappy_plain_v2": dict(compression="snappy", use_dictionary=False, data_page_version="2.0"),
    "stored_dict_v2": dict(compression="none", use_dictionary=True, data_page_version="2.0"),
}


def _write(path, texts, opts, rg_rows=700):
    t = pa.table({"id": pa.array([str(i) for i in range(len(texts))]), "text": pa.array(texts, pa.string())})
    pq.write_table(t, path, row_group_size=rg_rows, **opts)


@pytest.mark.parametrize("case", sorted(CASES))
def test_page_directory_covers_every_row(tmp_path, case):
    from textblaster_amd import native
    from textblaster_amd.ops.parquet_gpu import page_table

    path = str(tmp_path / f"{case}.parquet")
    _write(path, _texts(3, 2000), CASES[case])
    pf = pq.ParquetFile(path)
    raw = np.fromfile(path, dtype=np.uint8)
    ci = [pf.schema.column(i).name for i in range(len(pf.schema))].index("text")
    for rg in range(pf.num_row_groups):
        cc = pf.metadata.row_group(rg).column(ci)
        start = min(cc.data_page_offset, cc.dictionary_page_offset or cc.data_page_offset) \
            if cc.has_dictionary_page else cc.data_page_offset
        chunk = raw[start:start + cc.total_compressed_size]
        pages = native.host().parquet_pages(chunk)
        assert pages[:, 1].max() + 0 <= len(chunk)
        codec = 1 if str(cc.compression).upper() == "SNAPPY" else 0
        t = page_table(chunk, codec, pf.schema.column(ci).max_definition_level,
                       pf.metadata.row_group(rg).num_rows)
        assert t is not None, case
        table, dict_page, data_idx, nbytes = t
        assert (dict_page >= 0) == bool(cc.has_dictionary_page)
        assert table["num_values"][data_idx].sum() == pf.metadata.row_group(rg).num_rows
        assert nbytes >= table["out_size"].sum()


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_gpu_text_column_equals_pyarrow(tmp_path, case):
    from textblaster_amd.ops import hiprt
    from textblaster_amd.ops.parquet_gpu import GpuTextColumn

    assert hiprt.device_count() > 0
    path = str(tmp_path / f"{case}.parquet")
    texts = _texts(11, 3000)
    _write(path, texts, CASES[case])
    dec = GpuTextColumn(path, "text", 0)
    assert dec.ok
    pf = pq.ParquetFile(path)
    for rg in range(pf.num_row_groups):
        got = dec.read(rg)
        assert got is not None, (case, rg, dec.stats)
        data, off, valid = got
        ref = pf.read_row_group(rg, columns=["text"]).column(0)
        rd, ro, rv = string_column_buffers(ref)
        np.testing.assert_array_equal(valid, rv if rv is not None else np.ones(len(ref), np.uint8))
        np.testing.assert_array_equal(off, ro)
        assert bytes(data) == bytes(rd)
    assert dec.stats["fallback"] == 0


@pytest.mark.gpu
def test_gpu_decode_run_equals_cpu_decode(tmp_path):
    """run(): the Parquet -> Parquet outputs are byte-identical with the text column decoded by
    pyarrow or on the device."""
    from textblaster_amd.runner import RunConfig, run

    path = str(tmp_path / "in.parquet")
    texts = [t if t is not None else "" for t in _texts(5, 4000)]
    _write(path, texts, dict(compression="snappy", use_dictionary=True), rg_rows=1500)
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config", "pipeline_config.yaml")
    outs = {}
    for mode in ("cpu", "gpu"):
        o, e = str(tmp_path / f"{mode}.o.parquet"), str(tmp_path / f"{mode}.e.parquet")
        tok = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "tokenizers")
        run(RunConfig(path, o, e, cfg, backend="cuda", unit_rows=1000, parquet_decode=mode, tokenizer_dir=tok))
        outs[mode] = (pq.read_table(o), pq.read_table(e))
    assert outs["cpu"][0].equals(outs["gpu"][0])
    assert outs["cpu"][1].equals(outs["gpu"][1])
