"""K17: HTML character-reference decoding of a packed text batch on the GPU (csrc/hip/html.hip).

The reference reader decodes every text cell with ``html_escape::decode_html_entities``
(reference src/data/readers/parquet_reader.rs:177-179). The host reader does the same with the
C++ decoder (csrc/host/html.cpp); this op is the device version of that decoder, bit-identical
to it (tests/test_gpu_html.py), for batches that are already packed as UTF-8 bytes + int64
offsets. Named references are found with one hashed probe (table built here). Two
launches, one wave per document: output sizes, then an on-device exclusive scan
of the sizes and the scatter of the decoded bytes.
"""
from __future__ import annotations

import threading
from typing import Tuple

import numpy as np

from .. import native
from .kernels import _check


def html_name_hash(name: bytes) -> int:
    """FNV-1a, the hash the device lookup uses (csrc/hip/html.hip name_hash)."""
    h = 2166136261
    for c in name:
        h = ((h ^ c) * 16777619) & 0xFFFFFFFF
    return h


def build_slots(names: bytes, noff) -> np.ndarray:
    """Open-addressing table (load factor <= 1/4, linear probing) of entity indices by name."""
    n = len(noff) - 1
    size = 1
    while size < 4 * n:
        size <<= 1
    slots = np.full(size, -1, dtype=np.int32)
    for e in range(n):
        k = html_name_hash(names[noff[e]:noff[e + 1]]) & (size - 1)
        while slots[k] >= 0:
            k = (k + 1) & (size - 1)
        slots[k] = e
    return slots


class HtmlDecoder:
    """Holds the entity table on one device; ``decode`` works on device arrays (ops/hiprt.py)."""

    def __init__(self, device="cuda:0"):
        from . import hiprt

        self.rt = hiprt
        self.device = hiprt.parse_device(device)
        self.lib = native.hip()
        hiprt.set_device(self.device)
        self.stream = hiprt.Stream()
        names, noff, vals, voff = native.host().html_entity_table()
        with hiprt.stream(self.stream):
            self.names = hiprt.to_device(np.frombuffer(names, dtype=np.uint8))
            self.name_off = hiprt.to_device(np.asarray(noff, dtype=np.int32))
            self.vals = hiprt.to_device(np.frombuffer(vals, dtype=np.uint8))
            self.val_off = hiprt.to_device(np.asarray(voff, dtype=np.int32))
            self.nent = len(noff) - 1
            slots = build_slots(names, noff)
            assert (slots < 0).any(), "the device probe loop needs an empty slot"
            self.slots = hiprt.to_device(slots)
        self.slot_mask = len(slots) - 1
        self._lock = threading.Lock()  # the reader pool calls decode_host from several threads

    def decode(self, data, off, host_off: np.ndarray = None):
        """data: uint8[N], off: int64[B+1] (device arrays) -> decoded (data', off') on the device,
        ordered on this decoder's stream. ``host_off``: the same offsets on the host, when the
        caller has them (skips the download for the bounds check)."""
        rt = self.rt
        if data.dtype != np.uint8 or off.dtype != np.int64:
            raise ValueError("html decode needs uint8 data and int64 offsets")
        ndocs = off.numel() - 1
        with rt.stream(self.stream):
            if ndocs <= 0:
                return data[:0], rt.zeros(off.numel(), np.int64)
            # the kernels trust the offsets: check the bounds and monotonicity before they index
            # device memory with them
            ho = host_off if host_off is not None else off.to_host()
            if len(ho) != ndocs + 1 or ho[0] < 0 or ho[-1] > data.numel() or bool((ho[1:] < ho[:-1]).any()):
                raise ValueError("html decode: offsets must be non-decreasing and within the data")
            lens = rt.empty(ndocs, np.int64)
            _check(self.lib.tb_html_sizes(self.stream.handle, data.data_ptr(), off.data_ptr(), ndocs,
                                          self.names.data_ptr(), self.name_off.data_ptr(), self.vals.data_ptr(),
                                          self.val_off.data_ptr(), self.nent, self.slots.data_ptr(), self.slot_mask,
                                          lens.data_ptr()), "tb_html_sizes")
            out_off = rt.zeros(ndocs + 1, np.int64)
            rt.scan_strided_i64(lens, 1, ndocs, out_off[1:])
            tot = np.zeros(1, np.int64)
            out_off[ndocs:].copy_to_host(tot, self.stream)
            self.stream.synchronize()
            total = int(tot[0])
            out = rt.empty(max(total, 1), np.uint8)
            _check(self.lib.tb_html_scatter(self.stream.handle, data.data_ptr(), off.data_ptr(), ndocs,
                                            self.names.data_ptr(), self.name_off.data_ptr(), self.vals.data_ptr(),
                                            self.val_off.data_ptr(), self.nent, self.slots.data_ptr(),
                                            self.slot_mask, out_off.data_ptr(), out.data_ptr()), "tb_html_scatter")
            return out[:total], out_off

    def decode_host(self, data: np.ndarray, off: np.ndarray):
        """Host arrays in, host arrays out (H2D, the two kernels, D2H); None when no document
        changes, like the host decoder's html_decode_batch."""
        rt = self.rt
        # look for '&' without a full-size boolean mask or copy (memchr in the host module)
        if data.size == 0 or not native.host().contains_byte(np.ascontiguousarray(data, dtype=np.uint8), ord("&")):
            return None
        o64 = np.ascontiguousarray(off, dtype=np.int64)
        with self._lock:
            rt.set_device(self.device)
            with rt.stream(self.stream):
                d = rt.to_device(np.ascontiguousarray(data, dtype=np.uint8))
                o = rt.to_device(o64)
                od, oo = self.decode(d, o, host_off=o64)
                return od.to_host(), oo.to_host()
