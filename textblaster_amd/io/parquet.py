"""Parquet input/output with the reference's schema and quirks (reference
src/pipeline/readers/parquet_reader.rs, src/pipeline/writers/parquet_writer.rs).

Input: required ``--text-column`` and ``--id-column`` (Utf8/LargeUtf8); optional ``source``
(fallback: the input path), ``added`` (Date32 interpreted as days-from-CE, or
Timestamp(us)), ``created`` (struct of two date/timestamp fields, both required),
``metadata`` (JSON object of strings; unparsable -> empty + warning). Text is HTML-entity
decoded. Rows with a null text or id are reported as errors and skipped.

Output columns (in order): ``id: Utf8 !null, source: Utf8 !null, text: Utf8 !null,
added: Date32 (days-from-CE, as the reference writes it), created: Struct{start, end:
Timestamp(us)}, metadata: Utf8 JSON (null when empty)``. Output and excluded files are always
created, even when empty.

The batched path never builds per-document Python objects: text/metadata columns go to the
engine as packed buffers, and id/source/added/created are carried as Arrow columns and taken
by row index for the outputs.
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import json
import logging
import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.parquet as pq

from .. import native
from ..data_model import TextDocument
from ..errors import ConfigError, IoError, ParquetError, Unexpected

log = logging.getLogger("textblaster_amd.io")

_EPOCH_CE_DAYS = _dt.date(1970, 1, 1).toordinal()  # days-from-CE of 1970-01-01 (719163)


@dataclasses.dataclass
class ParquetInputConfig:
    """reference config/parquet.rs:4-11"""

    path: str
    text_column: str = "text"
    id_column: str = "id"
    batch_size: Optional[int] = None


OUTPUT_SCHEMA = pa.schema([
    pa.field("id", pa.string(), nullable=False),
    pa.field("source", pa.string(), nullable=False),
    pa.field("text", pa.string(), nullable=False),
    pa.field("added", pa.date32(), nullable=True),
    pa.field("created", pa.struct([pa.field("start", pa.timestamp("us"), nullable=True),
                                   pa.field("end", pa.timestamp("us"), nullable=True)]), nullable=True),
    pa.field("metadata", pa.string(), nullable=True),
])


# ---------------------------------------------------------------------------------------------
# column helpers

def string_column_buffers(arr: pa.Array) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """(uint8 data, int64 offsets, uint8 validity or None) of a Utf8/LargeUtf8 array, zero-copy
    for the data buffer when possible."""
    if isinstance(arr, pa.ChunkedArray):
        arr = pa.concat_arrays(arr.chunks) if arr.num_chunks != 1 else arr.chunk(0)
    if pa.types.is_string(arr.type):
        off_t, width = np.int32, 4
    elif pa.types.is_large_string(arr.type):
        off_t, width = np.int64, 8
    else:
        raise Unexpected(f"expected a string column, got {arr.type}")
    n = len(arr)
    bufs = arr.buffers()
    offsets = np.frombuffer(bufs[1], dtype=off_t, count=n + 1 + arr.offset)[arr.offset:arr.offset + n + 1]
    offsets = offsets.astype(np.int64)
    start = int(offsets[0])
    data_buf = bufs[2]
    data = (np.frombuffer(data_buf, dtype=np.uint8) if data_buf is not None and data_buf.size
            else np.zeros(0, dtype=np.uint8))
    if start:
        offsets = offsets - start
    data = data[start:start + int(offsets[-1])]
    valid = None
    if arr.null_count:
        valid = np.asarray(arr.is_valid()).astype(np.uint8)
    return data, offsets, valid


def _date_days_from_ce(arr: pa.Array) -> pa.Array:
    """Date32/Timestamp column -> int32 'days from CE' as the reference reads it."""
    if pa.types.is_date32(arr.type):
        # Date32 values are taken as days-from-CE verbatim (reference parquet_reader.rs:49)
        return pc.cast(arr, pa.int32())
    if pa.types.is_timestamp(arr.type):
        days_epoch = pc.cast(pc.cast(arr, pa.timestamp("us")), pa.int64())
        vals = np.asarray(days_epoch.fill_null(0).to_numpy(zero_copy_only=False), dtype=np.int64)
        out = (np.floor_divide(vals, 86_400_000_000) + _EPOCH_CE_DAYS).astype(np.int32)
        return pa.array(out, type=pa.int32(), mask=np.asarray(arr.is_null()))
    return pa.nulls(len(arr), pa.int32())


def _timestamp_us(arr: pa.Array) -> pa.Array:
    if pa.types.is_timestamp(arr.type):
        return pc.cast(arr, pa.timestamp("us"))
    if pa.types.is_date32(arr.type):
        days = np.asarray(pc.cast(arr, pa.int32()).fill_null(0).to_numpy(zero_copy_only=False), dtype=np.int64)
        us = (days - _EPOCH_CE_DAYS) * 86_400_000_000
        return pa.array(us, type=pa.timestamp("us"), mask=np.asarray(arr.is_null()))
    return pa.nulls(len(arr), pa.timestamp("us"))


_RS_NAMES = {
    "int8": "Int8", "int16": "Int16", "int32": "Int32", "int64": "Int64", "uint8": "UInt8", "uint16": "UInt16",
    "uint32": "UInt32", "uint64": "UInt64", "float": "Float32", "double": "Float64", "halffloat": "Float16",
    "bool": "Boolean", "binary": "Binary", "large_binary": "LargeBinary", "null": "Null", "date32[day]": "Date32",
    "date64[ms]": "Date64", "string": "Utf8", "large_string": "LargeUtf8",
}


def arrow_rs_debug(t: pa.DataType) -> str:
    """Name of an Arrow type as arrow-rs's ``{:?}`` prints it (for the reference's messages)."""
    return _RS_NAMES.get(str(t), str(t))


@dataclasses.dataclass
class DocBatch:
    """One read batch in engine layout."""

    n: int
    text: Tuple[np.ndarray, np.ndarray]                 # packed UTF-8 (HTML-decoded)
    meta: Optional[Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]]
    ids: pa.Array
    source: pa.Array
    added: pa.Array          # int32 days-from-CE (nullable)
    created: pa.Array        # struct<start, end>
    error_rows: int = 0
    bytes_in: int = 0


class ParquetReader:
    """reference parquet_reader.rs:18-251"""

    def __init__(self, config: ParquetInputConfig, html_threads: int = 8, html_decoder=None):
        # like the reference, construction does not touch the file; errors surface on first use
        self.config = config
        self.html_threads = html_threads
        # optional device decoder (ops.html.HtmlDecoder, K17); default: the host C++ decoder
        self.html_decoder = html_decoder
        self._pf_obj = None

    @property
    def _pf(self) -> pq.ParquetFile:
        return self.open()._pf_obj

    def open(self) -> "ParquetReader":
        if self._pf_obj is not None:
            return self
        config = self.config
        try:
            pf = pq.ParquetFile(config.path)
        except FileNotFoundError as e:
            raise IoError(e) from e
        except (pa.ArrowInvalid, OSError) as e:
            raise ParquetError(e) from e
        schema = pf.schema_arrow
        names = schema.names
        for col in (config.text_column, config.id_column):
            if col not in names:
                raise ConfigError(f"Required column '{col}' not found in schema.")
        ttype = schema.field(config.text_column).type
        if not (pa.types.is_string(ttype) or pa.types.is_large_string(ttype)):
            raise ConfigError(f"Column '{config.text_column}' must be Utf8 or LargeUtf8, found: {arrow_rs_debug(ttype)}")
        self.has_source = "source" in names
        self.has_added = "added" in names
        self.has_created = "created" in names
        self.has_metadata = ("metadata" in names
                             and (pa.types.is_string(schema.field("metadata").type)
                                  or pa.types.is_large_string(schema.field("metadata").type)))
        self.columns = [config.text_column, config.id_column] + [
            c for c, ok in (("source", self.has_source), ("added", self.has_added), ("created", self.has_created),
                            ("metadata", self.has_metadata)) if ok and c not in (config.text_column, config.id_column)]
        self._pf_obj = pf
        return self

    @property
    def num_row_groups(self) -> int:
        return self._pf.num_row_groups

    def row_group_bytes(self) -> List[int]:
        md = self._pf.metadata
        return [md.row_group(i).total_byte_size for i in range(md.num_row_groups)]

    def row_group_rows(self) -> List[int]:
        md = self._pf.metadata
        return [md.row_group(i).num_rows for i in range(md.num_row_groups)]

    def read_row_group(self, rg: int, pf: Optional[pq.ParquetFile] = None, use_threads: bool = True) -> pa.Table:
        """The reader's columns of row group ``rg``."""
        pf = pf if pf is not None else self._pf
        return pf.read_row_group(rg, columns=self.columns, use_threads=use_threads)

    # -- batched engine path ------------------------------------------------------------------
    def iter_batches(self, batch_rows: int = 65536, row_groups: Optional[Sequence[int]] = None
                     ) -> Iterator[DocBatch]:
        it = self._pf.iter_batches(batch_size=batch_rows, row_groups=row_groups, columns=self.columns,
                                   use_threads=True)
        for rb in it:
            yield self._to_docbatch(rb)

    def _to_docbatch(self, rb: pa.RecordBatch) -> DocBatch:
        cfg = self.config
        text = rb.column(cfg.text_column)
        ids = rb.column(cfg.id_column)
        bad = None
        if text.null_count or ids.null_count:
            bad = np.asarray(pc.or_(text.is_null(), ids.is_null()))
            for r in np.nonzero(bad)[0][:5]:
                which = cfg.text_column if not text[int(r)].is_valid else cfg.id_column
                log.warning("Row %d has null %s column '%s'; skipping", r, "text" if which == cfg.text_column
                            else "id", which)
            keep = pa.array(~bad)
            rb = rb.filter(keep)
            text = rb.column(cfg.text_column)
            ids = rb.column(cfg.id_column)
        n = rb.num_rows
        data, off, _ = string_column_buffers(text)
        if self.html_decoder is not None:
            dec = self.html_decoder.decode_host(data, off)
        else:
            dec = native.host().html_decode_batch(np.ascontiguousarray(data), np.ascontiguousarray(off),
                                                  self.html_threads)
        if dec is not None:
            data, off = dec
        if not (pa.types.is_string(ids.type) or pa.types.is_large_string(ids.type)):
            ids = pc.cast(ids, pa.string())
        if self.has_source:
            src = rb.column("source")
            if not pa.types.is_string(src.type):
                src = pc.cast(src, pa.string())
            source = pc.fill_null(src, self.config.path)
        else:
            source = pa.array([self.config.path] * n, type=pa.string())
        added = _date_days_from_ce(rb.column("added")) if self.has_added else pa.nulls(n, pa.int32())
        created = self._created(rb, n)
        meta = None
        if self.has_metadata:
            md, mo, mv = string_column_buffers(rb.column("metadata"))
            meta = (np.ascontiguousarray(md), mo, mv)
        return DocBatch(n, (np.ascontiguousarray(data), off), meta, ids, source, added, created,
                        int(bad.sum()) if bad is not None else 0, int(off[-1]) if n else 0)

    def _created(self, rb: pa.RecordBatch, n: int) -> pa.Array:
        st = pa.struct([pa.field("start", pa.timestamp("us")), pa.field("end", pa.timestamp("us"))])
        if not self.has_created:
            return pa.StructArray.from_arrays([pa.nulls(n, pa.timestamp("us")), pa.nulls(n, pa.timestamp("us"))],
                                              fields=list(st))
        col = rb.column("created")
        if not pa.types.is_struct(col.type) or col.type.num_fields < 2:
            log.warning("'created' column is not a StructArray.")
            return pa.StructArray.from_arrays([pa.nulls(n, pa.timestamp("us")), pa.nulls(n, pa.timestamp("us"))],
                                              fields=list(st))
        a = _timestamp_us(col.field(0))
        b = _timestamp_us(col.field(1))
        both = pc.and_(a.is_valid(), b.is_valid())
        if col.null_count:
            both = pc.and_(both, col.is_valid())
        a = pc.if_else(both, a, pa.scalar(None, pa.timestamp("us")))
        b = pc.if_else(both, b, pa.scalar(None, pa.timestamp("us")))
        return pa.StructArray.from_arrays([a, b], fields=list(st))

    # -- per-document path (reference BaseReader::read_documents) ------------------------------
    def read_documents(self) -> Iterator[TextDocument]:
        """Yields TextDocument objects; rows with null text/id raise Unexpected when reached
        (iterate with ``iter_documents_results`` to get errors as values)."""
        for r in self.iter_documents_results():
            if isinstance(r, Exception):
                raise r
            yield r

    def iter_documents_results(self):
        cfg = self.config
        bs = cfg.batch_size or 1024
        h = native.host()
        for rb in self._pf.iter_batches(batch_size=bs, columns=self.columns):
            cols = {name: rb.column(name) for name in rb.schema.names}
            texts = cols[cfg.text_column].to_pylist()
            ids = cols[cfg.id_column].to_pylist()
            srcs = cols["source"].to_pylist() if self.has_source else None
            added = _date_days_from_ce(cols["added"]).to_pylist() if self.has_added else None
            created = self._created(rb, rb.num_rows).to_pylist()
            metas = cols["metadata"].to_pylist() if self.has_metadata else None
            for i in range(rb.num_rows):
                if texts[i] is None:
                    yield Unexpected(f"Row {i} has null text column '{cfg.text_column}'")
                    continue
                if ids[i] is None:
                    yield Unexpected(f"Row {i} has null id column '{cfg.id_column}'")
                    continue
                md = {}
                if metas is not None and metas[i] is not None:
                    parsed = h.parse_meta_json(metas[i])
                    if parsed is None:
                        log.warning("Failed to parse metadata JSON for id %s", ids[i])
                    else:
                        md = dict(parsed)
                a = added[i] if added is not None else None
                c = created[i]
                yield TextDocument(
                    id=str(ids[i]),
                    content=h.html_decode(texts[i]),
                    source=(srcs[i] if srcs is not None and srcs[i] is not None else cfg.path),
                    added=_dt.date.fromordinal(a) if a is not None and a > 0 else None,
                    created=(c["start"], c["end"]) if c and c["start"] is not None and c["end"] is not None else None,
                    metadata=md,
                )


class ParquetWriter:
    """reference parquet_writer.rs:49-164. Uncompressed by default (arrow-rs default
    WriterProperties); ``compression`` may be set (e.g. "snappy", "zstd")."""

    def __init__(self, path: str, compression: str = "none"):
        parent = os.path.dirname(os.path.abspath(path))
        try:
            os.makedirs(parent, exist_ok=True)
            self._w = pq.ParquetWriter(path, OUTPUT_SCHEMA, compression=compression)
        except OSError as e:
            raise IoError(e) from e
        self.path = path
        self.rows = 0

    def write_table(self, table: pa.Table) -> None:
        if table.num_rows:
            self._w.write_table(table)
            self.rows += table.num_rows

    def write_batch(self, documents: Sequence[TextDocument]) -> None:
        """Per-document API (reference BaseWriter::write_batch)."""
        if not documents:
            return
        h = native.host()
        ids, srcs, texts, added, cs, ce, metas = [], [], [], [], [], [], []
        for d in documents:
            ids.append(d.id)
            srcs.append(d.source)
            texts.append(d.content)
            added.append(d.added.toordinal() if d.added else None)
            if d.created:
                cs.append(d.created[0])
                ce.append(d.created[1])
            else:
                cs.append(None)
                ce.append(None)
            metas.append(h.serialize_meta_json(list(d.metadata.items())) if d.metadata else None)
        table = build_output_table(pa.array(ids, pa.string()), pa.array(srcs, pa.string()),
                                   pa.array(texts, pa.string()), pa.array(added, pa.int32()),
                                   pa.StructArray.from_arrays([pa.array(cs, pa.timestamp("us")),
                                                               pa.array(ce, pa.timestamp("us"))],
                                                              names=["start", "end"]),
                                   pa.array(metas, pa.string()))
        self.write_table(table)

    def close(self) -> None:
        if self._w is not None:
            self._w.close()
            self._w = None


def encode_table(table: pa.Table, compression: str = "none") -> pa.Buffer:
    """One table -> a complete Parquet file in memory, written exactly as ``ParquetWriter``
    would write it (same schema, properties and row groups). Encoders on several threads run
    concurrently (the encode releases the GIL); ``io.pqconcat.StreamConcat`` appends the
    results to one file without re-encoding."""
    sink = pa.BufferOutputStream()
    w = pq.ParquetWriter(sink, OUTPUT_SCHEMA, compression=compression)
    if table.num_rows:
        w.write_table(table)
    w.close()
    return sink.getvalue()


def build_output_table(ids, source, text, added_days_ce, created, metadata) -> pa.Table:
    added = pa.Array.from_buffers(pa.date32(), len(added_days_ce), added_days_ce.buffers(),
                                  offset=added_days_ce.offset)
    return pa.Table.from_arrays([ids, source, text, added, created, metadata], schema=OUTPUT_SCHEMA)


def packed_to_string_array(data: np.ndarray, off: np.ndarray, valid: Optional[np.ndarray] = None) -> pa.Array:
    """Engine output buffers -> Arrow string array (Utf8 when it fits int32 offsets)."""
    n = len(off) - 1
    mask_buf = None
    null_count = 0
    if valid is not None and len(valid) and not valid.all():
        mask_buf = pa.py_buffer(np.packbits(valid.astype(bool), bitorder="little"))
        null_count = int(n - valid.sum())
    data_buf = pa.py_buffer(np.ascontiguousarray(data))
    if off[-1] < 2**31 - 1:
        arr = pa.Array.from_buffers(pa.string(), n, [mask_buf, pa.py_buffer(off.astype(np.int32)), data_buf],
                                    null_count=null_count)
    else:
        arr = pa.Array.from_buffers(pa.large_string(), n, [mask_buf, pa.py_buffer(off), data_buf],
                                    null_count=null_count)
    return arr


def write_empty(path: str) -> None:
    ParquetWriter(path).close()
