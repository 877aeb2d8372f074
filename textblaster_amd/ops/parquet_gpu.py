"""Parquet text-column decoding on the GPU (csrc/hip/parquet.hip).

The reference reader decodes the ``text`` column on the CPU through the parquet crate
(reference src/data/readers/parquet_reader.rs:100-190); decompression and value decoding of that
column dominate the host side of a Parquet -> Parquet run (profiles/r3_e2e: ~1.5 CPU-µs per
document of reader threads). Here the host only parses page headers (csrc/host/parquet_pages.cpp)
and uploads the column chunk as stored; Snappy decompression, definition levels, PLAIN /
dictionary values and the packing into one UTF-8 buffer + int64 offsets run on the device.

Supported: flat BYTE_ARRAY columns (max repetition level 0, max definition level <= 1), SNAPPY or
UNCOMPRESSED chunks, data pages v1 (RLE definition levels) and v2, PLAIN / PLAIN_DICTIONARY /
RLE_DICTIONARY values. ``read`` returns None for anything else, and when the device reports
malformed input, so the caller decodes that row group with pyarrow.
"""
from __future__ import annotations

import os
import threading
from typing import Optional, Tuple

import numpy as np
import pyarrow.parquet as pq

from .. import native
from .kernels import _check

PQ_PAGE = np.dtype([("in_off", "<i8"), ("out_off", "<i8"), ("in_size", "<i4"), ("out_size", "<i4"),
                    ("raw", "<i4"), ("codec", "<i4"), ("kind", "<i4"), ("num_values", "<i4"),
                    ("encoding", "<i4"), ("def_len", "<i4"), ("rep_len", "<i4"), ("max_def", "<i4"),
                    ("row0", "<i8")])
_CODECS = {"SNAPPY": 1, "UNCOMPRESSED": 0}
_ENCODINGS = (0, 2, 8)  # PLAIN, PLAIN_DICTIONARY, RLE_DICTIONARY
_DICT_PAGE, _DATA_V1, _DATA_V2 = 2, 0, 3


def page_table(chunk: np.ndarray, codec: int, max_def: int, nrows: int):
    """Device page descriptors for one column chunk: (PQ_PAGE array, index of the dictionary page
    or -1, data page indices, page-buffer size), or None when the chunk uses something the device
    decoder does not handle."""
    pg = native.host().parquet_pages(chunk)
    out = []
    dict_page = -1
    data = []
    out_off = 0
    row = 0
    for r in pg:
        typ, data_off, comp, uncomp, nval, enc, def_enc, _nulls, def_len, rep_len, v2c = (int(v) for v in r)
        if typ not in (_DICT_PAGE, _DATA_V1, _DATA_V2):
            continue  # index pages carry no values
        if typ == _DICT_PAGE:
            if dict_page >= 0 or enc not in (0, 2):
                return None
            kind, raw, c = 0, 0, codec
        elif typ == _DATA_V1:
            if enc not in _ENCODINGS or (max_def > 0 and def_enc != 3):
                return None
            kind, raw, c = 1, 0, codec
        else:
            if enc not in _ENCODINGS or rep_len != 0 or (max_def == 0 and def_len != 0):
                return None
            kind, raw, c = 2, rep_len + def_len, (codec if v2c else 0)
            if raw > comp or raw > uncomp:
                return None
        if c == 0 and comp != uncomp:
            return None
        e = (data_off, out_off, comp, uncomp, raw, c, kind, nval, enc, def_len, rep_len, max_def,
             row if kind else 0)
        if kind == 0:
            dict_page = len(out)
        else:
            data.append(len(out))
            row += nval
        out.append(e)
        out_off += (uncomp + 7) & ~7
    if row != nrows or not data:
        return None
    if any(out[i][8] in (2, 8) for i in data) and dict_page < 0:
        return None
    return np.array(out, dtype=PQ_PAGE), dict_page, np.array(data, dtype=np.int32), out_off


def _wait(ev) -> None:
    """Waits for an event by polling with short sleeps: the reader threads must not spin a core
    each while the device decodes (hipEventSynchronize busy-waits on this runtime)."""
    import time

    while not ev.query():
        time.sleep(0.0002)


class _Ticker:
    """Accumulates (wall, thread CPU) seconds per stage into a shared dict."""

    def __init__(self, acc: dict, lock):
        import time

        self.time = time
        self.acc = acc
        self.lock = lock
        self.t = time.perf_counter()
        self.c = time.thread_time()

    def __call__(self, name: str) -> None:
        t, c = self.time.perf_counter(), self.time.thread_time()
        with self.lock:
            w, u = self.acc.get(name, (0.0, 0.0))
            self.acc[name] = (w + t - self.t, u + c - self.c)
        self.t, self.c = t, c


class GpuTextColumn:
    """Decodes one string column of a Parquet file, row group by row group, on a device. Safe to
    call from several reader threads (each decodes on its own stream)."""

    def __init__(self, path: str, column: str, device=0):
        from . import hiprt

        self.rt = hiprt
        self.device = hiprt.parse_device(device)
        self.lib = native.hip()
        if int(self.lib.tb_sizeof_pq_page()) != PQ_PAGE.itemsize:
            raise RuntimeError("libtbhip.so and ops/parquet_gpu.py disagree on the page descriptor")
        self.path = path
        try:
            self.pf = pq.ParquetFile(path)
        except Exception:  # the reader reports open errors with the reference's messages
            self.pf = None
        names = [self.pf.schema.column(i).name for i in range(len(self.pf.schema))] if self.pf is not None else []
        self.ci = names.index(column) if column in names else -1
        self.ok = self.ci >= 0
        if self.ok:
            sc = self.pf.schema.column(self.ci)
            self.max_def = int(sc.max_definition_level)
            self.ok = (sc.physical_type == "BYTE_ARRAY" and int(sc.max_repetition_level) == 0
                       and self.max_def <= 1 and sc.path.count(".") == 0)
        self.file_size = os.path.getsize(path) if self.ok else 0
        self._tls = threading.local()
        self.stats = {"row_groups": 0, "fallback": 0, "bytes_in": 0, "bytes_out": 0}
        # seconds (wall, thread CPU) per stage, summed over calls: file, table, launch, wait, gather
        self.timing = {}
        self._lock = threading.Lock()

    def _stream(self):
        s = getattr(self._tls, "stream", None)
        if s is None:
            self.rt.set_device(self.device)
            s = self._tls.stream = self.rt.Stream()
        return s

    def read(self, rg: int) -> Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
        """(data uint8, offsets int64 [rows + 1], valid uint8 [rows]) of row group ``rg``, or None
        (unsupported layout / malformed input: decode it on the host)."""
        if not self.ok:
            return None
        md = self.pf.metadata.row_group(rg)
        cc = md.column(self.ci)
        codec = _CODECS.get(str(cc.compression).upper())
        if codec is None:
            return self._fallback()
        start = cc.data_page_offset
        if cc.has_dictionary_page and cc.dictionary_page_offset is not None and cc.dictionary_page_offset > 0:
            start = min(start, cc.dictionary_page_offset)
        size = int(cc.total_compressed_size)
        if start < 0 or start + size > self.file_size:
            return self._fallback()
        rt = self.rt
        rt.set_device(self.device)
        tick = _Ticker(self.timing, self._lock)
        # the chunk goes from the file straight into page-locked memory (DMA'd to the device)
        chunk = rt.pinned(size, np.uint8)
        f = self._file()
        f.seek(start)
        if f.readinto(memoryview(chunk)) != size:
            return self._fallback()
        nrows = int(md.num_rows)
        tick("file")
        try:
            t = page_table(chunk, codec, self.max_def, nrows)
        except RuntimeError:
            t = None
        if t is None:
            return self._fallback()
        pages, dict_page, data_idx, buf_bytes = t
        tick("table")
        s = self._stream()
        lib = self.lib
        with rt.stream(s):
            d_chunk = rt.empty(max(size, 1), np.uint8)
            d_chunk.copy_from_host(chunk, s)
            d_pages = rt.empty(len(pages) * PQ_PAGE.itemsize, np.uint8)
            d_pages.copy_from_host(pages.view(np.uint8), s)
            d_data = rt.empty(len(data_idx), np.int32)
            d_data.copy_from_host(data_idx, s)
            pagebuf = rt.empty(max(buf_bytes, 8), np.uint8)
            err = rt.zeros(1, np.uint32, s)
            _check(lib.tb_pq_decompress(s.handle, d_chunk.data_ptr(), d_pages.data_ptr(), len(pages),
                                        pagebuf.data_ptr(), err.data_ptr()), "tb_pq_decompress")
            ndict = int(pages[dict_page]["num_values"]) if dict_page >= 0 else 0
            dict_off = rt.empty(max(ndict, 1), np.int64)
            dict_len = rt.empty(max(ndict, 1), np.int32)
            if dict_page >= 0:
                _check(lib.tb_pq_dict(s.handle, d_pages.data_ptr(), dict_page, pagebuf.data_ptr(), dict_off.data_ptr(),
                                      dict_len.data_ptr(), err.data_ptr()), "tb_pq_dict")
            src = rt.empty(max(nrows, 1), np.int64)
            lens = rt.empty(max(nrows, 1), np.int64)
            valid = rt.empty(max(nrows, 1), np.uint8)
            _check(lib.tb_pq_values(s.handle, d_pages.data_ptr(), d_data.data_ptr(), len(data_idx),
                                    pagebuf.data_ptr(), dict_off.data_ptr(), dict_len.data_ptr(), ndict,
                                    src.data_ptr(), lens.data_ptr(), valid.data_ptr(), nrows, err.data_ptr()),
                   "tb_pq_values")
            off = rt.zeros(nrows + 1, np.int64, s)
            rt.scan_strided_i64(lens, 1, nrows, off[1:], s)
            h_off = rt.pinned(nrows + 1, np.int64)
            h_valid = rt.pinned(max(nrows, 1), np.uint8)[:nrows]
            e = rt.pinned(1, np.uint32)
            off.copy_to_host(h_off, s)
            valid[:nrows].copy_to_host(h_valid, s)
            err.copy_to_host(e, s)
            tick("launch")
            _wait(s.record())
            tick("wait")
            if int(e[0]) != 0:
                return self._fallback()
            total = int(h_off[nrows])
            out = rt.empty(max(total, 1), np.uint8)
            _check(lib.tb_pq_gather(s.handle, pagebuf.data_ptr(), src.data_ptr(), off.data_ptr(), nrows,
                                    out.data_ptr()), "tb_pq_gather")
            # page-locked output: the engine uploads pinned batch inputs in place (zero copy)
            h_data = rt.pinned(max(total, 1), np.uint8)[:total]
            out[:total].copy_to_host(h_data, s)
            _wait(s.record())
            tick("gather")
        with self._lock:
            self.stats["row_groups"] += 1
            self.stats["bytes_in"] += size
            self.stats["bytes_out"] += total
        return h_data, h_off, h_valid

    def _file(self):  # noqa: E301
        f = getattr(self._tls, "file", None)
        if f is None:
            f = self._tls.file = open(self.path, "rb", buffering=0)
        return f

    def _fallback(self):
        with self._lock:
            self.stats["fallback"] += 1
        return None
