"""Parquet concatenation without decoding: column-chunk bytes are copied verbatim and only the
Thrift footer is rewritten (offsets shifted, row groups appended, row counts summed).

This replaces a decode + re-encode merge of the per-unit part files (the reference writes one
file from one producer, producer_logic.rs:109-196; here N ranks produce parts in parallel).
The merge is split so that every rank can copy its own parts into the final file at an
offset it gets from an all-gather of body sizes (AG1), and rank 0 only writes the footer:

    plan = part_layout(paths)                    # per rank: body bytes + shifted row groups
    sizes = all_gather(plan.body_bytes)          # AG1
    write_bodies(out_fd, plan, base_offset)      # every rank, pwrite/copy_file_range
    finish(out_path, [row groups of all ranks])  # rank 0: footer + magic

Only the Thrift compact protocol subset that Parquet's FileMetaData uses is implemented; it
is generic over field ids, so unknown fields survive the round trip untouched.
"""
from __future__ import annotations

import dataclasses
import os
import struct
from typing import List, Sequence, Tuple

MAGIC = b"PAR1"

# compact protocol type ids
T_STOP, T_TRUE, T_FALSE, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE, T_BINARY, T_LIST, T_SET, T_MAP, T_STRUCT = range(13)


class ThriftError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# compact protocol codec: a struct decodes to a list of [field_id, type, value]

class _Reader:
    __slots__ = ("b", "p")

    def __init__(self, b: bytes, p: int = 0):
        self.b = b
        self.p = p

    def byte(self) -> int:
        v = self.b[self.p]
        self.p += 1
        return v

    def varint(self) -> int:
        shift = v = 0
        while True:
            c = self.byte()
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7
            if shift > 70:
                raise ThriftError("varint too long")

    def zigzag(self) -> int:
        v = self.varint()
        return (v >> 1) ^ -(v & 1)

    def value(self, t: int):
        if t in (T_TRUE, T_FALSE):
            return t == T_TRUE
        if t == T_BYTE:
            return self.byte()
        if t in (T_I16, T_I32, T_I64):
            return self.zigzag()
        if t == T_DOUBLE:
            v = self.b[self.p:self.p + 8]
            self.p += 8
            return v
        if t == T_BINARY:
            n = self.varint()
            v = self.b[self.p:self.p + n]
            self.p += n
            return v
        if t in (T_LIST, T_SET):
            h = self.byte()
            n, et = h >> 4, h & 0x0F
            if n == 15:
                n = self.varint()
            if et in (T_TRUE, T_FALSE):
                return (et, [self.byte() == T_TRUE for _ in range(n)])
            return (et, [self.value(et) for _ in range(n)])
        if t == T_MAP:
            n = self.varint()
            if n == 0:
                return (0, 0, [])
            kv = self.byte()
            kt, vt = kv >> 4, kv & 0x0F
            return (kt, vt, [(self.value(kt), self.value(vt)) for _ in range(n)])
        if t == T_STRUCT:
            return self.struct()
        raise ThriftError(f"unknown compact type {t}")

    def struct(self) -> list:
        fields = []
        last = 0
        while True:
            h = self.byte()
            t = h & 0x0F
            if t == T_STOP:
                return fields
            d = h >> 4
            fid = last + d if d else self.zigzag()
            fields.append([fid, t, self.value(t)])
            last = fid


class _Writer:
    __slots__ = ("out",)

    def __init__(self):
        self.out = bytearray()

    def varint(self, v: int) -> None:
        while True:
            if v < 0x80:
                self.out.append(v)
                return
            self.out.append((v & 0x7F) | 0x80)
            v >>= 7

    def zigzag(self, v: int) -> None:
        self.varint((v << 1) ^ (v >> 63))

    def value(self, t: int, v) -> None:
        if t in (T_TRUE, T_FALSE):
            return
        if t == T_BYTE:
            self.out.append(v & 0xFF)
        elif t in (T_I16, T_I32, T_I64):
            self.zigzag(v)
        elif t == T_DOUBLE:
            self.out += v
        elif t == T_BINARY:
            self.varint(len(v))
            self.out += v
        elif t in (T_LIST, T_SET):
            et, items = v
            if len(items) < 15:
                self.out.append((len(items) << 4) | et)
            else:
                self.out.append(0xF0 | et)
                self.varint(len(items))
            if et in (T_TRUE, T_FALSE):
                self.out += bytes(T_TRUE if x else T_FALSE for x in items)
            else:
                for x in items:
                    self.value(et, x)
        elif t == T_MAP:
            kt, vt, items = v
            self.varint(len(items))
            if items:
                self.out.append((kt << 4) | vt)
                for k, x in items:
                    self.value(kt, k)
                    self.value(vt, x)
        elif t == T_STRUCT:
            self.struct(v)
        else:
            raise ThriftError(f"unknown compact type {t}")

    def struct(self, fields: list) -> None:
        last = 0
        for fid, t, v in fields:
            if t in (T_TRUE, T_FALSE):
                t = T_TRUE if v else T_FALSE
            d = fid - last
            if 0 < d <= 15:
                self.out.append((d << 4) | t)
            else:
                self.out.append(t)
                self.zigzag(fid)
            self.value(t, v)
            last = fid
        self.out.append(T_STOP)


def decode_struct(b: bytes) -> list:
    return _Reader(b).struct()


def encode_struct(fields: list) -> bytes:
    w = _Writer()
    w.struct(fields)
    return bytes(w.out)


def _get(fields: list, fid: int):
    for f in fields:
        if f[0] == fid:
            return f
    return None


# ---------------------------------------------------------------------------------------------
# FileMetaData surgery (parquet.thrift field ids)

FMD_SCHEMA, FMD_NUM_ROWS, FMD_ROW_GROUPS = 2, 3, 4
RG_COLUMNS, RG_FILE_OFFSET, RG_ORDINAL = 1, 5, 7
CC_FILE_OFFSET, CC_META, CC_OFFSET_INDEX, CC_COLUMN_INDEX = 2, 3, 4, 6
CMD_OFFSETS = (9, 10, 11, 14)   # data_page / index_page / dictionary_page / bloom_filter offsets


def read_footer(path: str) -> Tuple[int, int, list]:
    """(file size, body end = footer start, decoded FileMetaData)."""
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        head = f.read(4)
        f.seek(size - 8)
        tail = f.read(8)
        if head != MAGIC or tail[4:] != MAGIC:
            raise ThriftError(f"{path}: not a Parquet file (or an encrypted one)")
        flen = struct.unpack("<I", tail[:4])[0]
        start = size - 8 - flen
        f.seek(start)
        fmd = decode_struct(f.read(flen))
    return size, start, fmd


def parse_buffer(buf) -> Tuple[int, list]:
    """(body end = footer start, decoded FileMetaData) of a whole Parquet file held in memory."""
    mv = memoryview(buf)
    size = len(mv)
    if size < 12 or bytes(mv[:4]) != MAGIC or bytes(mv[size - 4:]) != MAGIC:
        raise ThriftError("buffer is not a Parquet file (or an encrypted one)")
    flen = struct.unpack("<I", bytes(mv[size - 8:size - 4]))[0]
    start = size - 8 - flen
    return start, decode_struct(bytes(mv[start:size - 8]))


def shift_row_group(rg: list, delta: int) -> None:
    """Adds ``delta`` to every absolute file offset of one RowGroup (in place)."""
    # 0 means "unset" for the deprecated file_offset fields, which then stay 0
    f = _get(rg, RG_FILE_OFFSET)
    if f is not None and f[2] > 0:
        f[2] += delta
    cols = _get(rg, RG_COLUMNS)
    for cc in (cols[2][1] if cols else []):
        for fid in (CC_FILE_OFFSET, CC_OFFSET_INDEX, CC_COLUMN_INDEX):
            g = _get(cc, fid)
            if g is not None and g[2] > 0:
                g[2] += delta
        if _get(cc, CC_OFFSET_INDEX) is not None:
            # page locations inside an offset index are absolute too; parts are written without
            # a page index (pyarrow's default), anything else is refused rather than corrupted
            raise ThriftError("part files with a page index cannot be concatenated")
        md = _get(cc, CC_META)
        if md is not None:
            for fid in CMD_OFFSETS:
                g = _get(md[2], fid)
                if g is not None:
                    g[2] += delta


@dataclasses.dataclass
class PartLayout:
    paths: List[str]
    bodies: List[Tuple[int, int]]        # (start, end) byte range of each part's body
    row_groups: List[list]               # decoded RowGroups, offsets relative to body start 0
    num_rows: int
    schema: bytes                        # encoded schema field (must match across parts)
    template: list                       # FileMetaData of the first part

    @property
    def body_bytes(self) -> int:
        return sum(e - s for s, e in self.bodies)


def part_layout(paths: Sequence[str]) -> PartLayout:
    bodies, rgs, rows, schema, template = [], [], 0, b"", []
    pos = 0
    for p in paths:
        _, end, fmd = read_footer(p)
        sch = encode_struct([_get(fmd, FMD_SCHEMA)])
        if not template:
            template, schema = fmd, sch
        elif sch != schema:
            raise ThriftError(f"{p}: schema differs from {paths[0]}")
        bodies.append((4, end))
        for rg in (_get(fmd, FMD_ROW_GROUPS) or [0, 0, (T_STRUCT, [])])[2][1]:
            shift_row_group(rg, pos - 4)     # relative to this layout's body start
            rgs.append(rg)
        pos += end - 4
        rows += (_get(fmd, FMD_NUM_ROWS) or [0, 0, 0])[2]
    return PartLayout(list(paths), bodies, rgs, rows, schema, template)


def write_bodies(fd: int, layout: PartLayout, base: int) -> None:
    """Copies every part body of ``layout`` into ``fd`` starting at absolute offset ``base``."""
    off = base
    for p, (s, e) in zip(layout.paths, layout.bodies):
        with open(p, "rb") as f:
            n = e - s
            done = 0
            while done < n:
                try:
                    k = os.copy_file_range(f.fileno(), fd, n - done, s + done, off + done)
                except (AttributeError, OSError):
                    f.seek(s + done)
                    chunk = f.read(min(n - done, 1 << 24))
                    k = os.pwrite(fd, chunk, off + done)
                if k <= 0:
                    raise OSError(f"short copy from {p}")
                done += k
        off += e - s


def footer_bytes(template: list, row_groups: List[list], num_rows: int) -> bytes:
    fmd = [list(f) for f in template]
    for f in fmd:
        if f[0] == FMD_NUM_ROWS:
            f[2] = num_rows
        elif f[0] == FMD_ROW_GROUPS:
            f[2] = (T_STRUCT, row_groups)
    if _get(fmd, FMD_ROW_GROUPS) is None:
        fmd.append([FMD_ROW_GROUPS, T_LIST, (T_STRUCT, row_groups)])
        fmd.sort(key=lambda f: f[0])
    for i, rg in enumerate(row_groups):
        o = _get(rg, RG_ORDINAL)
        if o is not None:
            o[2] = i
    return encode_struct(fmd)


def finish(fd: int, end_of_bodies: int, template: list, row_groups: List[list], num_rows: int) -> None:
    """Writes the leading magic, footer, footer length and trailing magic."""
    foot = footer_bytes(template, row_groups, num_rows)
    os.pwrite(fd, MAGIC, 0)
    os.pwrite(fd, foot + struct.pack("<I", len(foot)) + MAGIC, end_of_bodies)
    os.ftruncate(fd, end_of_bodies + len(foot) + 8)


def concat(paths: Sequence[str], out_path: str) -> int:
    """Single-process concatenation of ``paths`` into ``out_path``; returns the row count."""
    lay = part_layout(paths)
    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        write_bodies(fd, lay, 4)
        for rg in lay.row_groups:
            shift_row_group(rg, 4)
        finish(fd, 4 + lay.body_bytes, lay.template, lay.row_groups, lay.num_rows)
    finally:
        os.close(fd)
    return lay.num_rows


class StreamConcat:
    """Appends whole in-memory Parquet files (e.g. row groups encoded concurrently by several
    threads into ``pa.BufferOutputStream``s) to one output file in call order, without
    re-encoding: each body is written once at the running offset and its row groups are
    shifted there; ``close`` writes the merged footer. Returns False from ``close`` when nothing
    was appended (the caller writes an empty file with its schema)."""

    def __init__(self, path: str):
        self.path = path
        self.fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        self.pos = 4
        self.row_groups: List[list] = []
        self.num_rows = 0
        self.template: list = []
        self.schema = b""

    def append(self, buf) -> None:
        end, fmd = parse_buffer(buf)
        sch = encode_struct([_get(fmd, FMD_SCHEMA)])
        if not self.template:
            self.template, self.schema = fmd, sch
        elif sch != self.schema:
            raise ThriftError(f"{self.path}: appended file has a different schema")
        mv = memoryview(buf)[4:end]
        done = 0
        while done < len(mv):
            k = os.pwrite(self.fd, mv[done:], self.pos + done)
            if k <= 0:
                raise OSError(f"short write to {self.path}")
            done += k
        for rg in (_get(fmd, FMD_ROW_GROUPS) or [0, 0, (T_STRUCT, [])])[2][1]:
            shift_row_group(rg, self.pos - 4)
            self.row_groups.append(rg)
        self.pos += len(mv)
        self.num_rows += (_get(fmd, FMD_NUM_ROWS) or [0, 0, 0])[2]

    def close(self) -> bool:
        if self.fd < 0:
            return bool(self.template)
        try:
            if self.template:
                finish(self.fd, self.pos, self.template, self.row_groups, self.num_rows)
        finally:
            os.close(self.fd)
            self.fd = -1
        return bool(self.template)
