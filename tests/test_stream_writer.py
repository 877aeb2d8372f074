"""Parallel output path: units encoded to in-memory Parquet files on several threads and
appended in order by io.pqconcat.StreamConcat must read back exactly like one ParquetWriter
writing the same tables (reference parquet_writer.rs:69-164: one row group per batch)."""
import concurrent.futures as cf

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from textblaster_amd.io.parquet import OUTPUT_SCHEMA, ParquetWriter, encode_table
from textblaster_amd.io.pqconcat import StreamConcat


def _table(k, n):
    rng = np.random.default_rng(k)
    texts = ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(m))) + " ø&amp;" for m in rng.integers(0, 60, n)]
    return pa.Table.from_arrays([
        pa.array([f"id-{k}-{i}" for i in range(n)]), pa.array(["src"] * n), pa.array(texts),
        pa.array([i if i % 3 else None for i in range(n)], pa.int32()).cast(pa.date32()),
        pa.StructArray.from_arrays([pa.array([None] * n, pa.timestamp("us")), pa.array([None] * n, pa.timestamp("us"))],
                                   names=["start", "end"]),
        pa.array(['{"k":%d}' % i if i % 2 else None for i in range(n)])], schema=OUTPUT_SCHEMA)


def test_stream_concat_equals_single_writer(tmp_path):
    tables = [_table(k, n) for k, n in enumerate([5, 0, 17, 1, 300, 0, 42])]
    ref = tmp_path / "ref.parquet"
    w = ParquetWriter(str(ref))
    for t in tables:
        w.write_table(t)
    w.close()
    out = tmp_path / "out.parquet"
    sc = StreamConcat(str(out))
    with cf.ThreadPoolExecutor(4) as ex:
        for t, buf in zip(tables, ex.map(encode_table, tables)):
            if t.num_rows:
                sc.append(buf)
    assert sc.close()
    a, b = pq.read_table(ref), pq.read_table(out)
    assert a.schema == b.schema and a.equals(b)
    ma, mb = pq.ParquetFile(ref).metadata, pq.ParquetFile(out).metadata
    assert ma.num_row_groups == mb.num_row_groups == 5
    assert ma.num_rows == mb.num_rows
    # row groups are readable one by one at their shifted offsets
    pf = pq.ParquetFile(out)
    got = pa.concat_tables([pf.read_row_group(i) for i in range(pf.num_row_groups)])
    assert got.equals(a)


def test_stream_concat_empty(tmp_path):
    out = tmp_path / "e.parquet"
    sc = StreamConcat(str(out))
    assert not sc.close()
    ParquetWriter(str(out)).close()
    t = pq.read_table(out)
    assert t.num_rows == 0 and t.schema == OUTPUT_SCHEMA
