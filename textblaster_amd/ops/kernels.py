"""ctypes bindings for libtbhip.so (csrc/hip/kernels.hip, html.hip, runtime.hip) and thin launch
helpers.

Device memory comes from the native runtime layer (ops/hiprt.py: caching HBM allocator,
``DevArray`` views); kernels are launched on the calling thread's current hiprt stream. Every
launch checks the returned hipError_t and raises — there is no silent fallback on a GPU box.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from ..errors import DeviceError

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_U32 = ctypes.c_uint32
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t

# Bumped with every change of an entry point's signature in the table below: a stale
# libtbhip.so with an older argument list would otherwise be called with the wrong arguments.
ABI_VERSION = 24

_SIGS = {
    "tb_stage_analyze": [_P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _U32, _P, _P, _P, _P, _P, _P, _U32, _P, _I32, _I32, _P,
                         _P, _P, _P, _P, _P],
    "tb_gr_split_wave": [_P, _P, _I32, _P, _I32, _I32, _I32, _P, _P, _U32, _P, _P, _P, _P, _P, _P, _U32, _I32, _P,
                         _I32],
    "tb_c4_pass_a": [_P, _P, _P, _P, _P, _I32, _P, _P, _P, _U32, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _I32, _P, _P,
                     _P, _P, _P],
    "tb_stage_analyze_blk": [_P, _P, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _U32, _P, _P, _P, _P, _P, _P,
                             _U32, _P, _P, _P, _I32, _U32, _I32, _P, _P, _I32, _P, _P, _P],
    "tb_sizeof_pre_doc": [],
    "tb_pre_decode": [_P, _P, _P, _P, _I32, _P, _P, _U32, _P, _P, _P, _P, _P],
    "tb_gr_dup_split": [_P, _P, _I32, _P, _I32, _I32, _I32, _P, _P, _U32, _P, _P, _P, _P, _P, _P, _U32, _P],
    "tb_sizeof_gr_export": [],
    "tb_c4_pass_a_blk": [_P, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _U32, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _P,
                         _P, _P, _P, _P],
    "tb_gate": [_P, _P, _P, _I32, _I32, _P, _P, _I32],
    "tb_sizeof_gate": [],
    "tb_resolve": [_P, _P, _P, _I32, _I32, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P],
    "tb_sizeof_resolve": [],
    "tb_block_threads": [],
    "tb_badwords_match": [_P, _P, _P, _I32, _P, _P, _I32, _I32, _P, _U32, _P, _U32, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                          _U32],
    "tb_langid_mfma": [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, ctypes.c_double, _P, _P, _I32, _P],
    "tb_langid_prepare": [_P, _P, _P],
    "tb_pre_wcanon": [_P, _P, _P, _P, _I32, _P, _P, _U32, _P, _U32, _P],
    "tb_langid_aux_bytes": [],
    "tb_c4_pass_b": [_P, _P, _P, _I32, _P, _P, _P, _P, _P],
    "tb_pow_table": [_P, _P, _U32],
    "tb_html_sizes": [_P, _P, _P, _I32, _P, _P, _P, _P, _I32, _P, _U32, _P],
    "tb_html_scatter": [_P, _P, _P, _I32, _P, _P, _P, _P, _I32, _P, _U32, _P, _P],
    "tb_bpe_count": [_P, _P, _P, _P, _P, _I32, _P],
    "tb_sizeof_bpe": [],
    "tb_abi_version": [],
    # native runtime layer (csrc/hip/runtime.hip)
    "tbrt_device_count": [_P], "tbrt_set_device": [_I32], "tbrt_get_device": [_P], "tbrt_device_sync": [],
    "tbrt_mem_info": [_P, _P], "tbrt_malloc": [_P, _SZ], "tbrt_free": [_P], "tbrt_host_alloc": [_P, _SZ],
    "tbrt_host_free": [_P], "tbrt_empty_cache": [], "tbrt_cache_stats": [_P], "tbrt_stream_create": [_P, _I32],
    "tbrt_stream_destroy": [_P], "tbrt_stream_sync": [_P], "tbrt_stream_priority_range": [_P, _P],
    "tbrt_event_create": [_P, _I32], "tbrt_event_destroy": [_P], "tbrt_event_record": [_P, _P],
    "tbrt_event_sync": [_P], "tbrt_event_query": [_P], "tbrt_event_elapsed": [_P, _P, _P],
    "tbrt_stream_wait_event": [_P, _P], "tbrt_memcpy_h2d": [_P, _P, _SZ, _P], "tbrt_memcpy_d2h": [_P, _P, _SZ, _P],
    "tbrt_memcpy_d2d": [_P, _P, _SZ, _P], "tbrt_memset": [_P, _I32, _SZ, _P],
    "tb_scan_strided_i64": [_P, _P, _I64, _I64, _P],
    "tb_phase_slots": [],
    "tb_stage_waves": [],
    "tb_sizeof_plan": [],
    "tb_sizeof_stage": [],
    "tb_sizeof_c4": [],
}


def _dict_ptrs(dict_in):
    """(moff, bits, words) device arrays of docproc.h DictIn as three pointers (0 for None)."""
    if dict_in is None:
        return 0, 0, 0
    return tuple(_ptr(a) for a in dict_in)


# docproc.h PreDoc (checked against tb_sizeof_pre_doc)
PRE_DOC = np.dtype([("off", "<u8"), ("prop", "<u8"), ("wbm", "<u8"), ("nl_pos", "<u8"), ("nl_len", "<u8"),
                    ("n", "<u4"), ("C", "<u4"), ("dict", "<u4"), ("NL", "<u4"), ("tcs", "<u4"), ("tce", "<u4"),
                    ("nl_a", "<u4"), ("nl_e", "<u4"), ("wtmp", "<u8"), ("wcs", "<u8"), ("wce", "<u8"),
                    ("wbs", "<u8"), ("wbe", "<u8"), ("wal", "<u8"), ("W", "<u4"), ("pad", "<u4"),
                    ("wh", "<u8"), ("wtab", "<u8"), ("wk", "<u8"), ("wpb", "<u8"), ("wcsum", "<u8"),
                    ("wslot", "<u8"), ("wid", "<u8"), ("wl", "<u8"), ("wready", "<u4"), ("pad2", "<u4")])
PRE_WCHUNK = 2048  # kernels.hip kPreWChunk
PRE_TILE = 16384  # kernels.hip kPreTile


class DevBpe(ctypes.Structure):
    """csrc/common/bpe.h DevBpe (checked against tb_sizeof_bpe)."""
    _fields_ = [("byte_id", _P), ("keys", _P), ("vals", _P), ("cls1", _P), ("cls2", _P), ("added", _P),
                ("mask", _U32), ("n_added", _I32), ("added_off", _I32 * 9), ("post_add", _I32)]


class BpeTables:
    """A byte-level BPE tokenizer's tables in HBM (models/tokenizer.py BpeSpec) and the kernel's
    parameter block pointing at them."""

    def __init__(self, spec, cls_tables):
        from . import hiprt

        self.arrays = [hiprt.to_device(a) for a in (spec.byte_id, spec.keys, spec.vals, cls_tables[0], cls_tables[1],
                                                    spec.added)]
        if len(spec.added_off) > 9:
            raise DeviceError("bpe: too many added tokens")
        st = DevBpe()
        st.byte_id, st.keys, st.vals, st.cls1, st.cls2, st.added = [a.data_ptr() for a in self.arrays]
        st.mask = spec.mask
        st.n_added = max(len(spec.added_off) - 1, 0)
        for i, v in enumerate(spec.added_off):
            st.added_off[i] = v
        st.post_add = spec.post_add
        self.struct = st


def declare(lib: ctypes.CDLL) -> None:
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_size_t if name.startswith("tb_sizeof") else ctypes.c_int


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise DeviceError(f"{what} failed with hipError_t {rc}")


class Kernels:
    """Launch helpers bound to one device (holds the Unicode tables in HBM)."""

    def __init__(self, device: int):
        from .. import native
        from . import hiprt

        self.device = device
        self.lib = native.hip()
        h = native.host()
        if self.lib.tb_abi_version() != ABI_VERSION:
            raise DeviceError(f"libtbhip.so ABI {self.lib.tb_abi_version()} != {ABI_VERSION}; rebuild")
        if (self.lib.tb_sizeof_plan() != h.SIZEOF_DEV_PLAN or self.lib.tb_sizeof_stage() != h.SIZEOF_DEV_STAGE
                or self.lib.tb_sizeof_gate() != h.SIZEOF_DEV_GATE
                or self.lib.tb_sizeof_resolve() != h.SIZEOF_DEV_RESOLVE):
            raise DeviceError("libtbhip.so and _tbhost disagree on the device plan layout; rebuild")
        self.sizeof_gr_export = int(self.lib.tb_sizeof_gr_export())
        if int(self.lib.tb_sizeof_pre_doc()) != PRE_DOC.itemsize:
            raise DeviceError("libtbhip.so and ops/kernels.py disagree on PreDoc; rebuild")
        s1, s2, l1, l2 = h.ucd_tables()
        self.tabs = [hiprt.to_device(a) for a in (s1, s2, l1, l2)]
        self._pw = None
        self._pw_n = 0

    @staticmethod
    def stream() -> int:
        from . import hiprt

        return hiprt.current_stream().handle

    def pow_table(self, n: int):
        if n > self._pw_n:
            from . import hiprt

            cap = max(n, 1 << 16)
            cap = 1 << (cap - 1).bit_length()
            # B^0..B^cap followed by B^-0..B^-cap (k_pow_table)
            self._pw = hiprt.empty(2 * cap + 2, np.int64)
            _check(self.lib.tb_pow_table(self.stream(), self._pw.data_ptr(), cap), "tb_pow_table")
            # other slots' streams read the table right away with no event ordering them after
            # the kernel that fills it: growth is rare (documents over ~2 MB), so wait for it here
            hiprt.current_stream().synchronize()
            self._pw_n = cap
        return self._pw, self._pw_n

    def stage_analyze(self, plan, stage, bytes_, off, perm, ndocs, scratch, scratch_off, pw, pw_n, rec, flags,
                      lds_bytes=0, prof=None, waves=0, nblocks=0, dead=None, line_stats=None, gr_export=None,
                      dict_in=None):
        """k_stage_analyze_wave; ``dict_in`` = (moff, bits, words) device arrays or None each
        (docproc.h DictIn: the word sources of dictionary-script documents); ``line_stats`` (uint32, >= 4 * (total bytes / 8 + 16 ndocs) + 16): the
        C4 line export (docproc.h StageOut::line_stats), document d at 4 * (off[d] / 8 + 16 d).
        ``gr_export`` (zeroed, >= nblocks descriptors): split mode, every launched document exports
        its word arrays and gr_split_wave finishes its n-gram orders."""
        t = self.tabs
        if gr_export is not None and gr_export.nbytes < max(nblocks, 0) * self.sizeof_gr_export:
            raise DeviceError("stage_analyze: export buffer too small")
        rc = self.lib.tb_stage_analyze(
            self.stream(), plan.data_ptr(), stage.data_ptr(), bytes_.data_ptr(), off.data_ptr(), _ptr(perm), ndocs,
            scratch.data_ptr(), scratch_off.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(), t[1].data_ptr(),
            t[2].data_ptr(), t[3].data_ptr(), rec.data_ptr(), flags.data_ptr(), lds_bytes, _ptr(prof), waves, nblocks,
            _ptr(dead), _ptr(line_stats), _ptr(gr_export), *_dict_ptrs(dict_in))
        _check(rc, "tb_stage_analyze")

    def gr_export_wave_bytes(self, n_docs: int) -> int:
        """Bytes of a zeroed wave export buffer: n_docs descriptors, then k_gr_ngrams' list of the
        documents its LDS arrays cannot hold (NgRest: 16-byte header + a u32 per document)."""
        return n_docs * self.sizeof_gr_export + 16 + 4 * n_docs

    def gr_split_wave(self, stage, gr_step, perm, n_docs, n_tasks, ndocs, gr_export, pw, pw_n, rec, flags, lds_bytes,
                      block=True, prof=None, n_big=0):
        """The n-gram orders of the wave documents stage_analyze exported (n_tasks = the
        GopherRepetition step's duplicated + top orders): launch positions [0, n_big) one wave per
        (document, order) (k_gr_split_wave), the rest with ``block`` one workgroup per document
        (k_gr_ngrams); without ``block`` k_gr_split_wave for all."""
        if not 0 <= n_big <= n_docs:
            raise DeviceError("gr_split_wave: n_big out of range")
        if gr_export.nbytes < self.gr_export_wave_bytes(n_docs) or perm.numel() < n_docs:
            raise DeviceError("gr_split_wave: operand shapes")
        t = self.tabs
        rc = self.lib.tb_gr_split_wave(self.stream(), stage.data_ptr(), gr_step, perm.data_ptr(), n_docs, n_tasks,
                                       ndocs, gr_export.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(),
                                       t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), rec.data_ptr(),
                                       flags.data_ptr(), lds_bytes, 1 if block else 0, _ptr(prof), int(n_big))
        _check(rc, "tb_gr_split_wave")

    def stage_analyze_blk(self, plan, stage, bytes_, off, perm_long, nlong, ndocs, scratch, scratch_off, pw, pw_n,
                          rec, flags, lds_bytes=0, prof=None, dead=None, gr_export=None, n_split=0, split_bytes=0,
                          threads=512, line_stats=None, pre=None, n_pre=0, dict_in=None):
        """k_stage_analyze_blk; ``gr_export`` (zeroed, >= n_split descriptors): the first n_split
        launch positions longer than ``split_bytes`` export their word arrays (split mode)."""
        t = self.tabs
        if gr_export is not None and gr_export.nbytes < n_split * self.sizeof_gr_export:
            raise DeviceError("stage_analyze_blk: export buffer too small")
        if not 0 <= n_split <= nlong:
            raise DeviceError("stage_analyze_blk: n_split out of range")
        rc = self.lib.tb_stage_analyze_blk(
            self.stream(), plan.data_ptr(), stage.data_ptr(), bytes_.data_ptr(), off.data_ptr(), perm_long.data_ptr(),
            nlong, ndocs, scratch.data_ptr(), scratch_off.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(),
            t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), rec.data_ptr(), flags.data_ptr(), lds_bytes, _ptr(prof),
            _ptr(dead), _ptr(gr_export), n_split if gr_export is not None else 0, split_bytes, int(threads),
            _ptr(line_stats), _ptr(pre), int(n_pre) if pre is not None else 0, *_dict_ptrs(dict_in))
        _check(rc, "tb_stage_analyze_blk")

    def pre_decode(self, bytes_, off, perm_pre, npre, dead, pre, tiles_max, cnt):
        """k_pre_count / k_pre_decode / k_pre_wb: code points and word-break marks of
        the first ``npre`` long documents over many workgroups; ``pre``: PRE_DOC descriptors
        (device), ``cnt``: int64 [npre * tiles_max]."""
        if perm_pre.numel() < npre or cnt.numel() < npre * tiles_max or pre.nbytes < npre * PRE_DOC.itemsize:
            raise DeviceError("pre_decode: operand shapes")
        t = self.tabs
        rc = self.lib.tb_pre_decode(self.stream(), bytes_.data_ptr(), off.data_ptr(), perm_pre.data_ptr(), npre,
                                    _ptr(dead), pre.data_ptr(), int(tiles_max), cnt.data_ptr(), t[0].data_ptr(),
                                    t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr())
        _check(rc, "tb_pre_decode")

    def pre_wcanon(self, bytes_, off, perm_pre, npre, dead, pre, chunks_max, pw, pw_n, flags):
        """k_pre_wcanon / k_pre_wsum: GopherRepetition's word hashes, canonical word ids
        and concatenation-hash arrays of the ``npre`` pre-pass documents over many workgroups (after
        pre_decode; ``chunks_max`` >= ceil(max words / PRE_WCHUNK))."""
        if perm_pre.numel() < npre or pre.nbytes < npre * PRE_DOC.itemsize or chunks_max <= 0:
            raise DeviceError("pre_wcanon: operand shapes")
        rc = self.lib.tb_pre_wcanon(self.stream(), bytes_.data_ptr(), off.data_ptr(), perm_pre.data_ptr(), npre,
                                    _ptr(dead), pre.data_ptr(), int(chunks_max), pw.data_ptr(), pw_n,
                                    flags.data_ptr())
        _check(rc, "tb_pre_wcanon")

    def gr_dup_split(self, stage, gr_step, perm, n_split, n_tasks, ndocs, gr_export, pw, pw_n, rec, flags, lds_bytes,
                     cursor):
        """k_gr_dup_split: persistent workgroups take (split document, task) pairs from an atomic
        cursor (``cursor``: a uint32 device word of this launch, reset by the call; keep it alive
        until the kernel completes); n_tasks = the GopherRepetition step's duplicated + top n-gram
        orders + duplicated lines + paragraphs."""
        if gr_export.nbytes < n_split * self.sizeof_gr_export or perm.numel() < n_split or cursor.nbytes < 4:
            raise DeviceError("gr_dup_split: operand shapes")
        t = self.tabs
        rc = self.lib.tb_gr_dup_split(self.stream(), stage.data_ptr(), gr_step, perm.data_ptr(), n_split, n_tasks, ndocs,
                                      gr_export.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(), t[1].data_ptr(),
                                      t[2].data_ptr(), t[3].data_ptr(), rec.data_ptr(), flags.data_ptr(), lds_bytes,
                                      cursor.data_ptr())
        _check(rc, "tb_gr_dup_split")

    def c4_pass_a_blk(self, c4, bytes_, off, perm_long, nlong, ndocs, scratch, scratch_off, pw, pw_n, rec, src, flags,
                      lds_bytes=0, prof=None, dead=None, line_stats=None, c4_words=None, dict_lines=None):
        t = self.tabs
        dl = dict_lines or (None, None)
        rc = self.lib.tb_c4_pass_a_blk(
            self.stream(), c4.data_ptr(), bytes_.data_ptr(), off.data_ptr(), perm_long.data_ptr(), nlong, ndocs,
            scratch.data_ptr(), scratch_off.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(), t[1].data_ptr(),
            t[2].data_ptr(), t[3].data_ptr(), rec.data_ptr(), src.data_ptr(), flags.data_ptr(), lds_bytes, _ptr(prof),
            _ptr(dead), _ptr(line_stats), _ptr(c4_words), _ptr(dl[0]), _ptr(dl[1]))
        _check(rc, "tb_c4_pass_a_blk")

    def badwords_match(self, bytes_, off, ndocs, table, fold, matched, root=None, cjk=None, root0=-1, cjk0=0,
                       dead=None, dead_max=0, seg_bytes=2048, seg_doc=None, seg_idx=None):
        """k_badwords_match over documents [0, ndocs) of (bytes_, off): ``table`` is the hashed trie
        table (uint32 [4 * slots], csrc/common/badwords.h); per document root/cjk arrays, or one
        root0/cjk0 for all; documents with 0 < dead <= dead_max are skipped (matched -1). The first
        launch covers the first ``seg_bytes`` of every document; ``seg_doc`` / ``seg_idx`` (int32,
        the documents' further segments) add a second launch over those segments."""
        t = self.tabs
        f1, f2 = fold
        slots = table.numel() // 4
        if slots < 1 or slots & (slots - 1) or matched.numel() < ndocs or off.numel() < ndocs + 1:
            raise DeviceError("badwords_match: operand shapes")
        for a in (root, cjk, dead):
            if a is not None and a.numel() < ndocs:
                raise DeviceError("badwords_match: per-document array shorter than the batch")
        if (seg_doc is None) != (seg_idx is None) or (seg_doc is not None and seg_doc.numel() != seg_idx.numel()):
            raise DeviceError("badwords_match: segment lists")
        for sd, si in ((None, None), (seg_doc, seg_idx)):
            nitems = ndocs if sd is None else sd.numel()
            if sd is not None and nitems == 0:
                continue
            rc = self.lib.tb_badwords_match(
                self.stream(), bytes_.data_ptr(), off.data_ptr(), nitems, _ptr(root), _ptr(cjk), int(root0), int(cjk0),
                _ptr(dead), int(dead_max), table.data_ptr(), slots - 1, t[0].data_ptr(), t[1].data_ptr(),
                t[2].data_ptr(), t[3].data_ptr(), f1.data_ptr(), f2.data_ptr(), matched.data_ptr(), _ptr(sd), _ptr(si),
                int(seg_bytes))
            _check(rc, "tb_badwords_match")

    def langid_prepare(self, E):
        """The pair table of k_langid_mfma (orders 1 + 2 of every position over a 32-letter alphabet,
        + a zero row) built on the device from the embedding table ``E`` (E + 128, uint8); once per
        model. Returns the device buffer to pass as ``aux``."""
        from .. import native
        from . import hiprt

        h = native.host()
        if E.numel() != h.LID_BUCKETS * h.LID_ROW_DIM:
            raise DeviceError("langid_prepare: operand shapes")
        aux = hiprt.empty(int(self.lib.tb_langid_aux_bytes()), np.uint8)
        _check(self.lib.tb_langid_prepare(self.stream(), E.data_ptr(), aux.data_ptr()), "tb_langid_prepare")
        hiprt.current_stream().synchronize()
        return aux

    def langid_mfma(self, bytes_, off, perm, ndocs, E, aux, WT, w_scale, bias, rec, width, prof=None):
        """k_langid_mfma (v3 model): fastText int8 embedding bag + bf16 MFMA head, 16 documents per
        tile; the language record of every document into ``rec`` (document d at rec[d * width]).
        ``E``: the embedding table as E + 128, uint8 [buckets * 16], ``aux``: its pair table
        (langid_prepare), ``WT``: bf16 bits [16 * 32] (head transposed), ``bias``: float32 [8]
        (csrc/common/langid.h)."""
        from .. import native

        h = native.host()
        t = self.tabs
        if (E.numel() != h.LID_BUCKETS * h.LID_ROW_DIM or WT.numel() != 16 * h.LID_DIM or bias.numel() != h.LID_ROW
                or width < 2 or rec.numel() < ndocs * width or not w_scale > 0
                or aux.numel() != int(self.lib.tb_langid_aux_bytes())):
            raise DeviceError("langid_mfma: operand shapes")
        rc = self.lib.tb_langid_mfma(
            self.stream(), bytes_.data_ptr(), off.data_ptr(), _ptr(perm), ndocs, t[0].data_ptr(), t[1].data_ptr(),
            t[2].data_ptr(), t[3].data_ptr(), E.data_ptr(), aux.data_ptr(), WT.data_ptr(), float(w_scale),
            bias.data_ptr(), rec.data_ptr(), width, _ptr(prof))
        _check(rc, "tb_langid_mfma")

    def c4_pass_a(self, c4, bytes_, off, perm, ndocs, scratch, scratch_off, pw, pw_n, rec, src, flags, lds_bytes=0,
                  prof=None, nblocks=0, dead=None, line_stats=None, c4_words=None, dict_lines=None):
        """k_c4_pass_a; ``line_stats``: the line export of a stage over the same content version
        (trimmed spans, word counts and longest words of the Rust lines: documents without a
        citation skip decode, lines and words when split_paragraph is set). ``c4_words`` (uint32
        per document, preset to 0xFFFFFFFF): the rewrite's word count on the export path.
        ``dict_lines`` = (offsets int64, data uint32): host ICU line statistics of dictionary-script
        documents (docproc.h DictLines)."""
        t = self.tabs
        dl = dict_lines or (None, None)
        rc = self.lib.tb_c4_pass_a(
            self.stream(), c4.data_ptr(), bytes_.data_ptr(), off.data_ptr(), _ptr(perm), ndocs, scratch.data_ptr(),
            scratch_off.data_ptr(), pw.data_ptr(), pw_n, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
            t[3].data_ptr(), rec.data_ptr(), src.data_ptr(), flags.data_ptr(), lds_bytes, _ptr(prof), nblocks,
            _ptr(dead), _ptr(line_stats), _ptr(c4_words), _ptr(dl[0]), _ptr(dl[1]))
        _check(rc, "tb_c4_pass_a")

    def c4_pass_b(self, bytes_, off, ndocs, scratch, scratch_off, src, new_off, out):
        rc = self.lib.tb_c4_pass_b(self.stream(), bytes_.data_ptr(), off.data_ptr(), ndocs, scratch.data_ptr(),
                                   scratch_off.data_ptr(), src.data_ptr(), new_off.data_ptr(), out.data_ptr())
        _check(rc, "tb_c4_pass_b")

    def gate(self, gate, recs, ndocs, flags, dead, code, max_slot, need):
        """k_gate: mark documents that a step of the finished pass filtered (dead[doc] = code).
        ``need``: int64 fields per document the gate's steps read from each record buffer (the
        kernel trusts the blob's prefix/width, so the buffers are checked here)."""
        if not 0 < code <= 255:
            raise DeviceError("gate code out of range")
        if max_slot >= len(recs) or len(recs) > 8 or dead.numel() < ndocs or flags.numel() < ndocs:
            raise DeviceError("gate: operand shapes")
        if any(r.numel() < need * ndocs for r in recs):
            raise DeviceError("gate: a record buffer is smaller than the gate's steps read")
        arr = (ctypes.c_void_p * 8)(*([r.data_ptr() for r in recs] + [None] * (8 - len(recs))))
        rc = self.lib.tb_gate(self.stream(), gate.data_ptr(), ctypes.cast(arr, ctypes.c_void_p), len(recs), ndocs,
                              flags.data_ptr(), dead.data_ptr(), code)
        _check(rc, "tb_gate")

    def bpe_tables(self, spec) -> BpeTables:
        from .. import native

        if self.lib.tb_sizeof_bpe() != ctypes.sizeof(DevBpe):
            raise DeviceError("libtbhip.so DevBpe layout differs from the binding; rebuild")
        return BpeTables(spec, native.host().bpe_classes())

    def bpe_count(self, tabs: BpeTables, text, off, n_dev, n_max: int, counts):
        """k_bpe_count: token counts of documents k < min(n_dev[0], n_max) (csrc/hip/bpe.hip);
        ``n_dev``: optional one-element int64 device array (the kept count of K16)."""
        if off.numel() < n_max + 1 or counts.numel() < n_max or off.dtype != np.int64 or counts.dtype != np.int32:
            raise DeviceError("bpe_count: operand shapes")
        rc = self.lib.tb_bpe_count(self.stream(), ctypes.byref(tabs.struct), text.data_ptr(), off.data_ptr(),
                                   _ptr(n_dev), n_max, counts.data_ptr())
        _check(rc, "tb_bpe_count")

    def resolve(self, rp, recs, ndocs, flags, versions, fail, status, fver, lanes, sc, out, out_off, rows, err):
        """K16: k_resolve + four scans + k_compact (see tb_resolve). ``recs``: record buffers by
        slot; ``versions``: [(bytes, offsets)] by content version; the rest are outputs/scratch."""
        if len(recs) > 8 or not 1 <= len(versions) <= 8:
            raise DeviceError("resolve: too many record buffers or versions")
        if (flags.numel() < ndocs or fail.numel() < ndocs or status.numel() < ndocs or fver.numel() < ndocs
                or lanes.numel() < 4 * ndocs or sc.numel() < 4 * ndocs or out_off.numel() < ndocs + 1
                or rows.numel() < ndocs or err.numel() < 1 or any(vo.numel() != ndocs + 1 for _, vo in versions)):
            raise DeviceError("resolve: operand shapes")
        ra = (ctypes.c_void_p * 8)(*([r.data_ptr() for r in recs] + [None] * (8 - len(recs))))
        vb = (ctypes.c_void_p * 8)(*([b.data_ptr() for b, _ in versions] + [None] * (8 - len(versions))))
        vo = (ctypes.c_void_p * 8)(*([o.data_ptr() for _, o in versions] + [None] * (8 - len(versions))))
        rc = self.lib.tb_resolve(self.stream(), rp.data_ptr(), ctypes.cast(ra, ctypes.c_void_p), len(recs), ndocs,
                                 flags.data_ptr(), ctypes.cast(vb, ctypes.c_void_p), ctypes.cast(vo, ctypes.c_void_p),
                                 len(versions), fail.data_ptr(), status.data_ptr(), fver.data_ptr(), lanes.data_ptr(),
                                 sc.data_ptr(), out.data_ptr(), out.numel(), out_off.data_ptr(), rows.data_ptr(),
                                 err.data_ptr())
        _check(rc, "tb_resolve")
