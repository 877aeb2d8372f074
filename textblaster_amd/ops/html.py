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
    """Holds the entity table on one device; ``decode`` works on device tensors."""

    def __init__(self, device="cuda:0"):
        import torch

        self.torch = torch
        self.device = torch.device(device)
        self.lib = native.hip()
        names, noff, vals, voff = native.host().html_entity_table()
        dev = self.device
        self.names = torch.from_numpy(np.frombuffer(names, dtype=np.uint8).copy()).to(dev)
        self.name_off = torch.tensor(noff, dtype=torch.int32, device=dev)
        self.vals = torch.from_numpy(np.frombuffer(vals, dtype=np.uint8).copy()).to(dev)
        self.val_off = torch.tensor(voff, dtype=torch.int32, device=dev)
        self.nent = len(noff) - 1
        slots = build_slots(names, noff)
        assert (slots < 0).any(), "the device probe loop needs an empty slot"
        self.slots = torch.from_numpy(slots).to(dev)
        self.slot_mask = len(slots) - 1
        self._lock = threading.Lock()  # the reader pool calls decode_host from several threads

    def _stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def decode(self, data, off) -> Tuple["torch.Tensor", "torch.Tensor"]:  # noqa: F821
        """data: uint8[N], off: int64[B+1] (CUDA tensors) -> decoded (data', off')."""
        torch = self.torch
        if data.dtype != torch.uint8 or off.dtype != torch.int64 or off.dim() != 1:
            raise ValueError("html decode needs uint8 data and int64 offsets")
        if data.device != self.device or off.device != self.device:
            raise ValueError("html decode inputs must live on " + str(self.device))
        ndocs = off.numel() - 1
        if ndocs <= 0:
            return data[:0], off.clone()
        # the kernels trust the offsets: check the bounds (and, cheaply on the device, monotonicity)
        # before they index device memory with them
        first, last = int(off[0].item()), int(off[-1].item())
        if first < 0 or last > data.numel() or bool((off[1:] < off[:-1]).any().item()):
            raise ValueError("html decode: offsets must be non-decreasing and within the data")
        data = data.contiguous()
        off = off.contiguous()
        lens = torch.empty(ndocs, dtype=torch.int64, device=self.device)
        _check(self.lib.tb_html_sizes(self._stream(), data.data_ptr(), off.data_ptr(), ndocs, self.names.data_ptr(),
                                      self.name_off.data_ptr(), self.vals.data_ptr(), self.val_off.data_ptr(),
                                      self.nent, self.slots.data_ptr(), self.slot_mask, lens.data_ptr()),
               "tb_html_sizes")
        out_off = torch.zeros(ndocs + 1, dtype=torch.int64, device=self.device)
        torch.cumsum(lens, 0, out=out_off[1:])
        total = int(out_off[-1].item())
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        _check(self.lib.tb_html_scatter(self._stream(), data.data_ptr(), off.data_ptr(), ndocs,
                                        self.names.data_ptr(), self.name_off.data_ptr(), self.vals.data_ptr(),
                                        self.val_off.data_ptr(), self.nent, self.slots.data_ptr(), self.slot_mask,
                                        out_off.data_ptr(), out.data_ptr()),
               "tb_html_scatter")
        return out[:total], out_off

    def decode_host(self, data: np.ndarray, off: np.ndarray):
        """Host arrays in, host arrays out (H2D, the two kernels, D2H); None when no document
        changes, like the host decoder's html_decode_batch."""
        torch = self.torch
        # look for '&' without a full-size boolean mask or copy (memchr in the host module)
        if data.size == 0 or not native.host().contains_byte(np.ascontiguousarray(data, dtype=np.uint8), ord("&")):
            return None
        with self._lock, torch.cuda.device(self.device):
            d = torch.from_numpy(np.ascontiguousarray(data)).to(self.device)
            o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(self.device)
            od, oo = self.decode(d, o)
            return od.cpu().numpy(), oo.cpu().numpy()
