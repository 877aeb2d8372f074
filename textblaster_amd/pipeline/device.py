"""Device (MI355X) execution of the record-producing and content-rewriting steps for one batch.

Per batch: the packed UTF-8 text (uint8 bytes + int64 offsets, the Arrow LargeUtf8 layout) is
staged into HBM once; every device stage then reads it in place. C4 passes produce the next
content version directly in HBM (sizes -> device scan -> scatter), so later stages never go
back to the host. Records, per-document flags and the final content version are copied back
once at the end of the batch.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import native
from ..errors import DeviceError
from ..ops.kernels import PRE_DOC, PRE_TILE, PRE_WCHUNK
from ..utils import metrics, tracing
from .plan import ExecPlan
from . import tuning
from .tuning import DeviceTuning

SCRATCH_ALIGN = 256


@dataclasses.dataclass
class DeviceResult:
    stage_recs: List[np.ndarray]            # per stage: int64 [width_total * ndocs]
    c4_recs: Dict[int, np.ndarray]          # step index -> int64 [7 * ndocs]
    versions: Dict[int, Tuple[np.ndarray, np.ndarray]]  # v >= 1 -> (bytes, offsets)
    flags: np.ndarray                       # uint32 [ndocs]; nonzero -> recompute on the CPU path
    timings: Dict[str, float]
    # Step gating (csrc/common/gate.h): dead[doc] = k > 0 -> passes >= k skipped the document
    # (a step of pass k-1 or earlier filtered it on the device); pass_of_step: step -> pass index
    dead: Optional[np.ndarray] = None
    pass_of_step: Optional[Dict[int, int]] = None
    # K16 (device resolve + compaction, csrc/common/gate.h resolve_doc): per document the first
    # failing step and status, and the final contents of kept then excluded documents compacted
    # into one buffer. None when the pipeline has host steps (TB_DEVICE_RESOLVE=0: off).
    resolved: Optional["Resolved"] = None
    # C4BadWords steps matched on the device (k_badwords_match over the content version the step
    # reads): step -> int8 [ndocs] (-1 skipped / no list, 0 no match, 1 match)
    bw_matched: Optional[Dict[int, np.ndarray]] = None


@dataclasses.dataclass
class BwInput:
    """Per batch and C4BadWords step: the hashed trie table of every loaded list (``gen`` names
    it, so the device copy is uploaded once) and per document the root of its language's trie —
    one ``root0`` / ``cjk0`` for all documents, or per-document ``roots`` / ``cjk`` arrays."""
    gen: int
    table: np.ndarray                 # uint32 [4 * slots] (csrc/common/badwords.h)
    roots: Optional[np.ndarray] = None  # int32 [ndocs], -1: no list
    cjk: Optional[np.ndarray] = None    # uint8 [ndocs]
    root0: int = -1
    cjk0: int = 0


@dataclasses.dataclass
class Resolved:
    fail: np.ndarray        # int32 [ndocs]: first failing step, -1 kept, 1<<30 delegated
    status: np.ndarray      # uint8 [ndocs]: 0 kept, 1 filtered, 3 delegated (CPU path)
    out: np.ndarray         # uint8: kept texts, then excluded texts
    out_off: np.ndarray     # int64 [ndocs + 1]: start of output k (first nk + nx + 1 valid)
    rows: np.ndarray        # int32 [ndocs]: document of output k
    err: int = 0            # nonzero: the compaction ran out of room (never with the C4 bound)
    ver: Optional[np.ndarray] = None  # uint8 [ndocs]: content version each document's output came from
    # trailing TokenCounter steps counted on the device (k_bpe_count): step -> int32 count of kept
    # output k (k < number kept; -2: count it on the host)
    tokens: Optional[Dict[int, np.ndarray]] = None

    # kept outputs a host step filtered afterwards (C4BadWords keep-fraction draws): bool over
    # the device's kept outputs; they move to the excluded side (Engine._device_resolve_agrees)
    moved: Optional[np.ndarray] = None

    def counts(self):
        return int(np.count_nonzero(self.status == 0)), int(np.count_nonzero(self.status == 1))

    def n_kept_final(self) -> int:
        nk, _ = self.counts()
        return nk - (int(np.count_nonzero(self.moved)) if self.moved is not None else 0)

    def kept_tokens(self, step: int) -> Optional[np.ndarray]:
        """k_bpe_count results of the final kept outputs (moved ones dropped)."""
        dev = (self.tokens or {}).get(step)
        if dev is None:
            return None
        nk, _ = self.counts()
        dev = dev[:nk]
        return dev[~self.moved] if self.moved is not None else dev

    def parts(self, nthreads: int = 8):
        """([(kept rows, offsets, text)], [(excluded ...), ...]): views of the compacted buffer; with
        ``moved``, the kept side is gathered without them and they form a second excluded part."""
        nk, nx = self.counts()
        o = self.out_off
        kb, tot = int(o[nk]), int(o[nk + nx])
        kept = (self.rows[:nk].astype(np.int64), o[:nk + 1], self.out[:kb])
        excl = (self.rows[nk:nk + nx].astype(np.int64), o[nk:nk + nx + 1] - kb, self.out[kb:tot])
        if self.moved is None or not self.moved.any():
            return [kept], [excl]
        h = native.host()
        ko = np.ascontiguousarray(o[:nk + 1])
        stay = np.nonzero(~self.moved)[0].astype(np.int64)
        gone = np.nonzero(self.moved)[0].astype(np.int64)
        kd, ko2 = h.gather_spans(self.out, ko, stay, nthreads)
        md, mo2 = h.gather_spans(self.out, ko, gone, nthreads)
        return [(kept[0][stay], ko2, kd)], [excl, (kept[0][gone], mo2, md)]


class LazyVersions(dict):
    """Content versions >= 1 left in HBM (K16 mode: the outputs come compacted from the device, so
    the host needs the versions only when it falls back to host assembly). Indexing or iterating
    items downloads them once."""

    def __init__(self, dev):
        super().__init__()
        self._dev = dict(dev)

    def _fetch(self):
        for v, (vb, vo) in sorted(self._dev.items()):
            ho = vo.to_host()
            dict.__setitem__(self, v, (vb[: int(ho[-1])].to_host() if int(ho[-1]) else np.zeros(0, np.uint8), ho))
        self._dev = {}

    def __getitem__(self, v):
        if self._dev:
            self._fetch()
        return dict.__getitem__(self, v)

    def items(self):
        if self._dev:
            self._fetch()
        return dict.items(self)

    def keys(self):
        return set(self._dev) | set(dict.keys(self))

    def __iter__(self):
        return iter(sorted(self.keys()))

    def __len__(self):
        return len(self.keys())


def trailing_token_counters(plan: ExecPlan) -> List[int]:
    """TokenCounter steps after the last filtering step (the reference's default config ends with
    one): they never filter, and they count the kept documents' final contents."""
    out = []
    for sp in reversed(plan.steps):
        if sp.type != "TokenCounter":
            break
        out.append(sp.index)
    return out[::-1]


def dict_marks_wanted(plan: ExecPlan, steps_native, tune: Optional[DeviceTuning] = None) -> bool:
    """Does a stage over the original text segment words (GopherQuality / GopherRepetition /
    FineWeb)? Then the host computes ICU word marks for the dictionary-script documents of every
    batch (text.h dict_word_marks) and they stay on the device (TB_TUNE dict_marks=0: CPU path)."""
    if not (tune or tuning.from_env()).dict_marks:
        return False
    kinds = ("GopherQualityFilter", "GopherRepetitionFilter", "FineWebQualityFilter")
    return any(plan.stage_version[s] == 0 and any(plan.steps[i].type in kinds for i in idx)
               for s, idx in enumerate(plan.stages))


def resolve_entries(plan: ExecPlan, stage_layout):
    """K16 plan: (entries, c4_versions) over every pipeline step in order — entries are (step,
    record slot, prefix) with slots = [stage 0 .. stage S-1, C4 step 0 ..] — or None when a step
    runs on the host (a TokenCounter in front of a filter, a C4 rewrite after C4BadWords).
    C4BadWords steps are skipped (see below). Trailing TokenCounter
    steps never filter, so K16 resolves the steps before them; the counts are added afterwards
    (k_bpe_count on the kept outputs, or the host tokenizer)."""
    entries, vers = [], []
    ns = len(plan.stages)
    trailing = set(trailing_token_counters(plan))
    # C4BadWords decides with keep-fraction draws on the host (document order): K16 resolves the
    # device steps as if it passed every document, and the host moves the documents it filters
    # afterwards; exact only while no content rewrite follows it (then their outputs are the
    # contents the step saw)
    bw = [sp.index for sp in plan.steps if sp.type == "C4BadWordsFilter"]
    if bw and any(sp.type == "C4QualityFilter" and sp.index > bw[0] for sp in plan.steps):
        return None
    for sp in plan.steps:
        if sp.index in trailing or sp.type == "C4BadWordsFilter":
            continue
        if sp.stage >= 0:
            pos = plan.stages[sp.stage].index(sp.index)
            _, _, prefix = stage_layout[sp.stage][1][pos]
            entries.append((sp.index, sp.stage, prefix))
            vers.append(-1)
        elif sp.c4_pass >= 0:
            entries.append((sp.index, ns + plan.c4_steps.index(sp.index), 0))
            vers.append(sp.version_out)
        else:
            return None
    if ns + len(plan.c4_steps) > 8 or plan.n_versions > native.host().MAX_VERSIONS or not entries:
        return None
    return entries, vers


def build_resolve(plan: ExecPlan, stage_layout, steps_native) -> Optional[bytes]:
    r = resolve_entries(plan, stage_layout)
    if r is None:
        return None
    try:
        return native.host().build_resolve(steps_native, r[0], r[1])
    except ValueError:  # a step without a device decision (e.g. > 16 n-gram orders)
        return None


def launch_order(lens: np.ndarray) -> np.ndarray:
    """Longest-first launch permutation (coarse 16-byte buckets: a stable radix sort on 16-bit
    keys instead of a comparison sort of int64 lengths)."""
    keys = (65535 - np.minimum(lens >> 4, 65535)).astype(np.uint16)
    return np.argsort(keys, kind="stable").astype(np.int32)


def lds_doc_slices(lens: np.ndarray, long_doc_bytes: int, per_byte: float, fixed: int, ratio: float = 1.25):
    """Per document the LDS slice k_stage_lds runs it with (0: a long-document workgroup runs it),
    exactly as DeviceRunner launches the buckets (used by the host emulation)."""
    perm = launch_order(lens)
    n_long = int(np.count_nonzero(lens > long_doc_bytes)) if long_doc_bytes > 0 else 0
    out = np.zeros(len(lens), dtype=np.uint32)
    lp = lens[perm]
    for p0, p1, sl in lds_buckets(lp[n_long:], per_byte, fixed, ratio):
        out[perm[n_long + p0:n_long + p1]] = sl
    return out


class _Slot:
    """Per in-flight batch resources: pinned input staging buffer and device scratch arena.
    Two slots alternate, so batch k+1 can be staged and launched while batch k's results are
    still being resolved on the host."""

    def __init__(self):
        self.pinned = None
        self.scratch = None
        self.scratch_c4 = None
        self.h2d_done = None  # event: the pinned staging buffer may be rewritten after it
        # per-slot streams (compute, language-id bag, long-document kernels, C4 wave / long, and
        # the copies): a batch's kernels only order against the batch that used the slot before
        # it, so batch k+1 starts while batch k's tail (long documents, C4, FineWeb, D2H) runs.
        # With the default layout these alias two streams per slot (see DeviceRunner).
        self.main = self.s_lid = self.s_blk = self.s_c4 = self.s_c4blk = None
        self.s_h2d = self.s_d2h = None


class PendingBatch:
    """A submitted batch: kernels and D2H copies are queued on the stream; ``wait()`` blocks on
    the completion event and returns host views of the results."""

    def __init__(self, runner, ndocs, event, stage_recs, c4_recs, versions, flags, t_submit, keep, dead=None,
                 resolved=None, bw=None):
        self.runner = runner
        self.ndocs = ndocs
        self.event = event
        self._stage_recs = stage_recs
        self._c4_recs = c4_recs
        self._versions = versions
        self._flags = flags
        self._dead = dead
        self._t_submit = t_submit
        self._keep = keep  # device tensors that must stay alive until the event completes
        self._resolved = resolved
        self._bw = bw or {}

    def wait(self) -> DeviceResult:
        import time

        t0 = time.perf_counter()
        with tracing.trace_range("tb.gpu_wait"):
            self.event.synchronize()
        t1 = time.perf_counter()
        stage_recs = list(self._stage_recs)
        c4_recs = dict(self._c4_recs)
        if isinstance(self._versions, LazyVersions):
            host_versions = self._versions
        else:
            host_versions = {}
            for ver, (vb, vo) in self._versions.items():
                host_versions[ver] = (vb[: int(vo[-1])], vo)
        fl = self._flags.view(np.uint32)
        dead = self._dead
        if self.runner.phase_prof:
            self.runner.collect_phase_prof(self._keep)
        kt = {}
        for item in self._keep or ():
            if isinstance(item, tuple) and len(item) == 3 and item[0] == "ktime":
                e0, e1 = item[2]
                # (a timing event may sit behind the batch's completion event on a side stream)
                e1.synchronize()
                kt[item[1]] = kt.get(item[1], 0.0) + e0.elapsed_time(e1) / 1000.0
        for name, sec in kt.items():
            metrics.GPU_KERNEL_SECONDS.labels(name).observe(sec)
        self._keep = None
        timings = dict(self._t_submit)
        timings["gpu_wait"] = t1 - t0
        res = None
        if self._resolved is not None:
            fail, st, out, out_off, rows, err, ver = self._resolved[:7]
            tokens = {si: t for si, t in self._resolved[7:]} or None
            res = Resolved(fail, st, out, out_off, rows, int(err[0]), ver, tokens)
        bwm = {i: m[:self.ndocs] for i, m in self._bw.items()} or None
        return DeviceResult(stage_recs, c4_recs, host_versions, fl, timings, dead, self.runner.pass_of_step, res, bwm)


KIND_LANGID = 4  # DevStep kind of LanguageDetectionFilter in a stage layout (csrc/common/devplan.h)
KIND_GOPHER_REP = 2
KIND_GOPHER_QUALITY = 1
KIND_FINEWEB = 3


def line_stats_stages(plan: ExecPlan, stage_layout, tune: Optional[DeviceTuning] = None) -> Dict[int, int]:
    """C4 line export (docproc.h export_line_stats): per content version read by a C4 pass, the
    first stage of that version that segments words and Rust lines (GopherQuality / FineWeb);
    it exports every line's trimmed span, word count and longest word, and the C4 pass reads them
    instead of decoding and segmenting the text again. TB_TUNE c4_line_stats=0 turns it off."""
    out: Dict[int, int] = {}
    if not (tune or tuning.from_env()).c4_line_stats:
        return out
    c4_versions = {plan.steps[i].version_in for i in plan.c4_steps}
    for si, sv in enumerate(plan.stage_version):
        kinds = {kind for kind, _, _ in stage_layout[si][1]}
        if sv in c4_versions and sv not in out and kinds & {KIND_GOPHER_QUALITY, KIND_FINEWEB}:
            out[sv] = si
    return out


def plan_passes(plan: ExecPlan, stage_layout, steps_native, gating: bool, lid_gate: bool = True):
    """Device passes in execution order (stages and C4 rewrites, by content version), the pass of
    every device step, and per pass (except the last) the gate blob over the steps it produced
    records for.

    With gating, a stage that holds the language-id step next to other steps is preceded by a
    ("lid", s) pass: the language-id kernel runs first, its gate marks the documents
    the language filter drops, and the stage kernels skip them (the reference never runs the
    later filters on those documents: executor.rs:30-57). TB_LID_GATE=0 keeps one pass."""
    h = native.host()
    passes = []
    for ver in range(plan.n_versions):
        for s, sv in enumerate(plan.stage_version):
            if sv != ver:
                continue
            kinds = [k for k, _, _ in stage_layout[s][1]]
            if gating and lid_gate and KIND_LANGID in kinds and len(kinds) > 1:
                passes.append(("lid", s))
            passes.append(("stage", s))
        passes += [("c4", i) for i in plan.c4_steps if plan.steps[i].version_in == ver]
    pass_of_step: Dict[int, int] = {}
    gates: Dict[int, bytes] = {}
    for p, (kind, x) in enumerate(passes):
        if kind in ("stage", "lid"):
            sel = [(j, prefix, width) for j, (k, width, prefix) in zip(plan.stages[x], stage_layout[x][1])
                   if (kind == "lid") == (k == KIND_LANGID) or (kind == "stage" and ("lid", x) not in passes)]
            entries = [(j, 0, prefix) for j, prefix, _ in sel]
            need = max(prefix + width for _, prefix, width in sel)
        else:
            entries = [(x, 0, 0)]
            need = 7  # C4 record width
        for j, _, _ in entries:
            pass_of_step[j] = p
        if gating and p + 1 < len(passes) and p + 1 <= 255:
            # need: int64 record fields per document the gate reads (checked at launch)
            gates[p] = (h.build_gate(steps_native, entries), need)
    return passes, pass_of_step, gates


BW_SEG_BYTES = 2048  # start positions per k_badwords_match wave


def bw_segments(lens: np.ndarray, growth: int, seg: int):
    """(doc, segment) lists of k_badwords_match's second launch: segments 1.. of every document
    whose length bound (input length + the content growth its C4 rewrites allow) exceeds one
    segment, so long documents are spread over waves instead of one wave walking them whole."""
    bound = lens.astype(np.int64) + int(growth)
    extra = np.maximum((bound + seg - 1) // seg - 1, 0)
    idx = np.nonzero(extra)[0]
    if not len(idx):
        z = np.zeros(0, dtype=np.int32)
        return z, z
    cnt = extra[idx]
    seg_doc = np.repeat(idx, cnt).astype(np.int32)
    starts = np.cumsum(cnt) - cnt
    seg_idx = (np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(starts, cnt) + 1).astype(np.int32)
    return seg_doc, seg_idx


def bw_dead_max(plan: ExecPlan, passes, pass_of_step: Dict[int, int]) -> Dict[int, int]:
    """Per C4BadWords step q: the device passes [0, q) hold only steps before it, so a document a
    gate marked dead <= q never reached the step (dead = k: the gate of pass k-1 filtered it);
    documents dead after a later pass did reach it and still need their match."""
    out = {}
    for sp in plan.steps:
        if sp.type != "C4BadWordsFilter":
            continue
        later = [p for j, p in pass_of_step.items() if j > sp.index]
        out[sp.index] = min(later) if later else len(passes)
    return out


class DeviceRunner:
    N_SLOTS = 2

    def __init__(self, steps_native, plan: ExecPlan, device, langid=None, max_batch_bytes: int = 384 << 20,
                 token_counters=None, slots: Optional[int] = None, host_threads: int = 8,
                 tune: Optional[DeviceTuning] = None):
        from ..ops import hiprt

        # operating points (pipeline/tuning.py: defaults with their A/B evidence, TB_TUNE overrides)
        self.tune = tu = (tune or tuning.from_env()).replace(slots=slots or None)
        self.rt = hiprt
        hiprt.set_blocking_events(tu.event_blocking)
        self.host_threads = max(1, int(host_threads))
        # dictionary-script documents: word marks from the host's ICU segmentation (stage kernels
        # of the original text) instead of the CPU path for the whole document
        self.dict_marks = dict_marks_wanted(plan, steps_native, tu)
        with tracing.trace_range("tb.init.hip_context"):
            self.device = hiprt.parse_device(device)
            if self.device >= hiprt.device_count():
                raise DeviceError(f"no HIP device {self.device}")
            hiprt.set_device(self.device)
        self.plan = plan
        self.steps = steps_native
        h = native.host()
        # Streams. The box exposes GPU_MAX_HW_QUEUES=4 hardware queues per process. The default
        # layout ("6") has exactly four streams that carry kernels — per slot one compute stream
        # (wave kernels, C4, language-id head, gates) and one side stream (long-document
        # workgroup kernels first, then the language-id bag; high priority so the long-document
        # tail is dispatched early) — plus one upload and one download stream shared by the
        # slots, which carry only DMA copies. Measured on the 1-GPU bench (profiles/r2_streams/):
        # 6 -> 44.5 ms/step, 13 (5 per slot + copies, the round-1 layout) -> 45-47.5,
        # 4 (copies folded into the slot streams) -> 50, 5 (one shared copy stream) -> 55: an
        # upload must never queue behind a download. The other layouts lost their A/Bs and were
        # removed; TB_TUNE streams=serial puts everything on one stream (exclusive kernel timings).
        blk_prio = tu.blk_priority
        self.stream_layout = tu.streams
        # Batches in flight on the device. Each slot holds its own scratch arena (<= 176 B per text
        # byte, x1.25 headroom): three slots keep the GPU fed (interleaved A/B, 20-step headline
        # bench: 35.3 vs 38.6 ms/step, profiles/r2_slots/ab.txt) and fit 288 GB of HBM with
        # 384 MB device batches; a smaller device gets two. `slots` (run --slots) or TB_TUNE
        # slots=N overrides.
        if tu.slots:
            self.N_SLOTS = max(1, int(tu.slots))
        else:
            try:
                _, total = hiprt.mem_info()
            except Exception:  # noqa: BLE001 - no info: the conservative choice
                total = 0
            per_slot = int(1.25 * 176 * max_batch_bytes) + (2 << 30)  # arena + staged/output buffers
            self.N_SLOTS = 3 if total >= 3 * per_slot + (8 << 30) else 2
        self.slots = [_Slot() for _ in range(self.N_SLOTS)]
        if self.stream_layout == "serial":
            one = hiprt.Stream()
            for sl in self.slots:
                sl.main = sl.s_lid = sl.s_blk = sl.s_c4 = sl.s_c4blk = sl.s_h2d = sl.s_d2h = one
        else:
            h2d, d2h = hiprt.Stream(), hiprt.Stream()
            for sl in self.slots:
                sl.main = sl.s_c4 = hiprt.Stream()
                sl.s_blk = sl.s_lid = sl.s_c4blk = hiprt.Stream(priority=blk_prio)
                sl.s_h2d, sl.s_d2h = h2d, d2h
        init = self.slots[0].main
        with hiprt.stream(init):
            from ..ops.kernels import Kernels

            with tracing.trace_range("tb.init.kernels"):
                self.k = Kernels(self.device)
            plan_b, stage_bs = h.build_device_plan(steps_native, plan.stages)
            self.plan_t = self._to_dev(plan_b)
            self.stage_ts = [self._to_dev(b) for b in stage_bs]
            self.stage_layout = [h.stage_layout(b) for b in stage_bs]
            self.c4_ts = {i: self._to_dev(h.build_c4(steps_native[i])) for i in plan.c4_steps}
            self.has_lid = any(steps_native[i].kind == h.StepKind.LanguageDetection
                               for st in plan.stages for i in st)
            self.lid_b = self.lid_E = self.lid_WT = None
            self.lid_w_scale = 0.0
            if self.has_lid:
                if langid is None:
                    raise DeviceError("LanguageDetectionFilter needs a language-id model")
                self.lid_b = hiprt.to_device(np.ascontiguousarray(langid.b, dtype=np.float32))
                # int8 embedding rows, biased to E + 128 as bytes for the kernel's SWAR sums
                # (2 MB, L2-resident), + the bf16 MFMA head operand
                self.lid_E = hiprt.to_device((langid.E.astype(np.int16) + 128).astype(np.uint8))
                self.lid_aux = self.k.langid_prepare(self.lid_E)  # 1-/2-gram pair table
                self.lid_WT = hiprt.to_device(np.ascontiguousarray(langid.head_bf16_t()).reshape(-1))
                self.lid_w_scale = float(langid.w_scale)
            self.c4_growth = int(h.C4_MAX_GROWTH)
            # gate=0 disables step gating (every pass runs over every document)
            self.gating = tu.gate
            self.passes, self.pass_of_step, gates = plan_passes(
                plan, self.stage_layout, steps_native, self.gating, tu.lid_gate and self.has_lid)
            self.gate_ts = {p: self._to_dev(b) for p, (b, _) in gates.items()}
            self.bw_dead_max = bw_dead_max(plan, self.passes, self.pass_of_step)
            self.gate_need = {p: need for p, (_, need) in gates.items()}
            # K16: device resolve + output compaction when every step runs on the device
            self.resolve_t = None
            if tu.device_resolve:
                blob = build_resolve(plan, self.stage_layout, steps_native)
                if blob is not None:
                    self.resolve_t = self._to_dev(blob)
                    # int64 fields per document read from each record buffer (launch-time check)
                    self.resolve_need = [w for w, _ in self.stage_layout] + [7] * len(plan.c4_steps)
            # trailing TokenCounter steps with a byte-level BPE tokenizer: counted on the device
            # after K16 (token_counters: [(step, BpeSpec)]; device_tokens=0 leaves them to the host)
            self.bpe = []
            if self.resolve_t is not None and tu.device_tokens:
                self.bpe = [(i, self.k.bpe_tables(sp)) for i, sp in (token_counters or [])]
            # B^k for the hashes, shared read-only by both slots: allocated once (longer spans
            # fall back to powmod61 in the kernels)
            with tracing.trace_range("tb.init.pow_table"):
                self.k.pow_table(1 << 22)
            init.synchronize()  # uploads and the table are complete before any slot stream reads them
        # LDS arena per document (one wave per workgroup): the stage kernel is built for W
        # waves/SIMD (tb_stage_waves) = 4 W waves/CU, so 160 KB / 4 W each costs no occupancy
        self.stage_waves = int(self.k.lib.tb_stage_waves())
        self.lds_bytes = tu.lds_bytes or (163840 // (4 * self.stage_waves)) & ~255
        self.lds_bytes_c4 = tu.lds_bytes_c4
        # documents longer than this run one workgroup (4 waves) each instead of one wave
        self.long_doc_bytes = tu.long_doc_bytes
        # three long-document workgroups per CU (with the register budget of k_stage_analyze_blk,
        # csrc/hip/kernels.hip TB_BLK_WPE)
        self.lds_bytes_blk = tu.lds_bytes_blk
        self.block_threads = int(self.k.lib.tb_block_threads())  # threads of the long-document workgroups
        # LDS slice of the split-order workgroups (k_gr_dup_split)
        self.lds_bytes_dup = tu.lds_bytes_dup or self.lds_bytes_blk
        # SURVEY 5.7 split: documents longer than this finish their duplicated n-gram orders in one
        # workgroup per order (k_gr_dup_split) instead of one after another in their stage
        # workgroup; 0 disables. Never below the long-document threshold (wave documents cannot
        # export: their arrays may live in LDS).
        self.split_doc_bytes = tu.split_doc_bytes
        if self.split_doc_bytes > 0:
            self.split_doc_bytes = max(self.split_doc_bytes, self.long_doc_bytes)
        # documents of at least this size get their code points and word-break marks
        # from the multi-workgroup pre-pass (k_pre_*) before their stage workgroup runs; 0
        # disables. Never below 64 KiB (smaller documents use the packed code point layout).
        self.pre_doc_bytes = tu.pre_doc_bytes
        # pre_wcanon=0: the pre-pass documents' word hashing and canonicalisation stay in their
        # stage workgroup (gopher_rep_record) instead of k_pre_wcanon's many workgroups
        self.pre_wcanon = tu.pre_wcanon
        if self.pre_doc_bytes > 0:
            self.pre_doc_bytes = max(self.pre_doc_bytes, 65536, self.long_doc_bytes)
        # per stage: (position of its GopherRepetition step, number of split tasks = its duplicated
        # + top n-gram orders + duplicated lines + duplicated paragraphs)
        self.gr_split = {}
        for si, idx in enumerate(plan.stages):
            grs = [k for k, (kind, _, _) in enumerate(self.stage_layout[si][1]) if kind == KIND_GOPHER_REP]
            if len(grs) == 1:
                st = steps_native[idx[grs[0]]]
                if st.n_dup + st.n_top > 0:
                    self.gr_split[si] = (grs[0], st.n_dup + st.n_top + 2)
        self.line_stats_stage = line_stats_stages(plan, self.stage_layout, tu)
        # scratch bytes per text byte (one pass, split documents): devplan.h; scratch_rate=a:b
        # overrides for A/B runs (larger only: smaller slices send documents to the CPU path)
        self.scratch_rates = (max(int(h.SCRATCH_PER_BYTE), tu.scratch_rate[0]),
                              max(int(h.SCRATCH_PER_BYTE_SPLIT), tu.scratch_rate[1]))
        # wave documents finish their n-gram orders in one wave per (document, order)
        # (k_gr_split_wave) or, below ngram_big_bytes, one workgroup per document (k_gr_ngrams:
        # 256 words, ~5.5 bytes per word on natural text; a document with more words runs the
        # generic code in that workgroup)
        self.lds_bytes_split = tu.lds_bytes_split
        self.ngram_block = tu.ngram_block
        self.ngram_big_bytes = tu.ngram_big_bytes
        # pinned inputs DMA'd in place (no host staging copy); zero_copy=0 forces the copy
        self.zero_copy = tu.zero_copy
        # phase_prof=1: per-document phase cycle counters (s_memtime stamps) for profiling
        self.phase_prof = tu.phase_prof
        self.phase_totals: Dict[str, np.ndarray] = {}
        self.phase_docs: Dict[str, int] = {}
        self.copy_threads = tu.copy_threads
        self._next_slot = 0
        self._bw_table = None  # (gen, device copy) of the hashed bad-words trie table
        self._bw_fold = None

    def bind_thread(self) -> None:
        """Make this runner's GPU the current device of the calling thread (HIP's current device
        is per thread; helper threads that launch work for this runner call this first)."""
        self.rt.set_device(self.device)

    def synchronize(self) -> None:
        """Wait for all queued device work (error recovery drains the queues before it frees)."""
        self.rt.synchronize()

    def _bw_tables(self, bw: BwInput):
        """Device copies of the case-fold tables and of the batch's trie table (uploaded once per
        table generation, on the calling stream before any kernel that reads them)."""
        rt = self.rt
        if self._bw_fold is None:
            f1, f2 = native.host().ucd_fold_tables()
            self._bw_fold = (rt.to_device(f1), rt.to_device(f2))
        if self._bw_table is None or self._bw_table[0] != bw.gen:
            self._bw_table = (bw.gen, rt.to_device(np.ascontiguousarray(bw.table, dtype=np.uint32)))
        return self._bw_table[1], self._bw_fold

    def _to_dev(self, b: bytes):
        return self.rt.to_device(np.frombuffer(bytes(b), dtype=np.uint8))

    def _stage_inputs(self, slot: _Slot, arrays, keep=None):
        """One H2D transfer for the per-batch inputs: arrays are packed at 256-byte aligned
        offsets into the slot's pinned buffer, copied with one DMA, and returned as typed views
        of the device buffer. An input that already lives in page-locked memory (hiprt.pinned,
        e.g. a reader that decodes into pinned batch buffers) is not copied on the host at all: its
        own DMA reads it in place (it is appended to ``keep`` so it outlives the copy)."""
        rt = self.rt
        offs, total = [], 0
        direct = [bool(self.zero_copy and a.nbytes >= (1 << 20) and a.flags.c_contiguous and rt.is_pinned(a))
                  for a in arrays]
        for a in arrays:
            offs.append(total)
            total += (a.nbytes + SCRATCH_ALIGN - 1) // SCRATCH_ALIGN * SCRATCH_ALIGN
        total = max(total, SCRATCH_ALIGN)
        packed = max([o + (a.nbytes + SCRATCH_ALIGN - 1) // SCRATCH_ALIGN * SCRATCH_ALIGN
                      for a, o, d in zip(arrays, offs, direct) if not d] + [SCRATCH_ALIGN])
        if slot.h2d_done is not None:
            slot.h2d_done.synchronize()  # the previous DMA out of this buffer has finished
        if slot.pinned is None or slot.pinned.nbytes < packed:
            slot.pinned = None
            slot.pinned = rt.pinned(int(packed * 1.25))
        hv = slot.pinned
        h = native.host()
        for a, o, d in zip(arrays, offs, direct):
            if a.nbytes and not d:
                h.parallel_copy(hv, o, np.ascontiguousarray(a).view(np.uint8).reshape(-1), self.copy_threads)
        # H2D on the upload stream: batch k+1's upload overlaps batch k's kernels
        dev = rt.empty(total, np.uint8)
        if any(direct):
            # the packed (small) arrays and each pinned input as separate DMAs
            o0 = 0
            for a, o, d in zip(arrays, offs, direct):
                if d:
                    if o > o0:
                        dev[o0:o].copy_from_host(hv[o0:o], slot.s_h2d)
                    dev[o:o + a.nbytes].copy_from_host(a.view(np.uint8).reshape(-1), slot.s_h2d)
                    if keep is not None:
                        keep.append(a)
                    o0 = o + (a.nbytes + SCRATCH_ALIGN - 1) // SCRATCH_ALIGN * SCRATCH_ALIGN
            if packed > o0:
                dev[o0:packed].copy_from_host(hv[o0:packed], slot.s_h2d)
        else:
            dev.copy_from_host(hv[:total], slot.s_h2d)
        ev = slot.s_h2d.record()
        slot.h2d_done = ev
        metrics.H2D_BYTES_TOTAL.inc(total)
        rt.current_stream().wait_event(ev)
        out = []
        for a, o in zip(arrays, offs):
            out.append(dev[o:o + a.nbytes].view(a.dtype) if a.nbytes else dev[o:o].view(a.dtype))
        return out, dev

    def _pre_decode(self, vb, vo, d_perm, long_lens: np.ndarray, dead, keep, flags=None, with_words=False):
        """SURVEY 5.7 pre-pass for the longest documents (launch positions [0, n_pre), sorted by
        length): device arrays for their code points and word-break marks, filled by k_pre_* on
        the current stream. Returns (PreDoc descriptors as a uint8 device array, n_pre)."""
        if self.pre_doc_bytes <= 0 or not len(long_lens):
            return None, 0
        big = np.nonzero(long_lens >= self.pre_doc_bytes)[0]
        if not len(big):
            return None, 0
        n_pre = int(big[-1]) + 1
        lens = long_lens[:n_pre].astype(np.int64)
        if bool((lens < self.pre_doc_bytes).any()) or n_pre > 65535:
            return None, 0  # the launch order is not the length order: no prefix to hand over
        al = lambda v: (v + 255) & ~255  # noqa: E731
        sz_off, sz_prop = al(4 * (lens + 1)), al(2 * (lens + 1))
        sz_wbm = al(4 * 2 * ((lens + 1 + 63) // 64))
        sz_nl = al(4 * (lens // 2 + 2))  # runs of '\n': at most one per two bytes
        sz_wt = al(4 * 8 * ((lens + 63) // 64 + 1))  # per 64-code-point chunk: 3 + 3 + 1 + 1 words
        sz_w = al(4 * (lens + 1))  # word arrays (words <= code points)
        sz_wa = al(lens + 1)
        per = sz_off + sz_prop + sz_wbm + 2 * sz_nl + sz_wt + 4 * sz_w + sz_wa
        # GopherRepetition's word arrays (k_pre_wcanon): wh / wk / wpb (8 B), wslot / wid / wl (4 B)
        # per word, the 1.5 W + 2-slot table, 4 sums per 2048-word chunk
        wcanon = bool(self.gr_split) and with_words
        if wcanon:
            sz_w8 = al(8 * (lens + 2))
            sz_tab = al(8 * (lens + lens // 2 + 3))
            sz_cs = al(8 * 4 * ((lens + PRE_WCHUNK - 1) // PRE_WCHUNK + 1))
            per = per + 3 * sz_w8 + 3 * al(4 * (lens + 2)) + sz_tab + sz_cs
        base = np.zeros(n_pre + 1, np.int64)
        np.cumsum(per, out=base[1:])
        rt = self.rt
        buf = rt.empty(int(base[-1]), np.uint8)
        p0 = buf.data_ptr()
        h = np.zeros(n_pre, dtype=PRE_DOC)
        h["off"] = p0 + base[:-1]
        h["prop"] = p0 + base[:-1] + sz_off
        h["wbm"] = p0 + base[:-1] + sz_off + sz_prop
        h["nl_pos"] = p0 + base[:-1] + sz_off + sz_prop + sz_wbm
        h["nl_len"] = p0 + base[:-1] + sz_off + sz_prop + sz_wbm + sz_nl
        o = p0 + base[:-1] + sz_off + sz_prop + sz_wbm + 2 * sz_nl
        h["wtmp"] = o
        h["wcs"] = o + sz_wt
        h["wce"] = o + sz_wt + sz_w
        h["wbs"] = o + sz_wt + 2 * sz_w
        h["wbe"] = o + sz_wt + 3 * sz_w
        h["wal"] = o + sz_wt + 4 * sz_w
        if wcanon:
            q = o + sz_wt + 4 * sz_w + sz_wa
            sz_w4 = al(4 * (lens + 2))
            for name in ("wh", "wk", "wpb"):
                h[name] = q
                q = q + sz_w8
            for name in ("wslot", "wid", "wl"):
                h[name] = q
                q = q + sz_w4
            h["wtab"] = q
            h["wcsum"] = q + sz_tab
        h["n"] = lens
        h["tcs"] = 0xFFFFFFFF
        d_pre = rt.empty(n_pre * PRE_DOC.itemsize, np.uint8)
        hp = h.view(np.uint8)
        d_pre.copy_from_host(hp, rt.current_stream())
        tiles_max = int((int(lens.max()) + PRE_TILE - 1) // PRE_TILE)
        cnt = rt.empty(n_pre * tiles_max, np.int64)
        self.k.pre_decode(vb, vo, d_perm[:n_pre], n_pre, dead, d_pre, tiles_max, cnt)
        if wcanon:
            pw, pw_n = self.k.pow_table(int(lens.max()) + 16)
            chunks_max = int((int(lens.max()) + 1 + PRE_WCHUNK - 1) // PRE_WCHUNK)
            self.k.pre_wcanon(vb, vo, d_perm[:n_pre], n_pre, dead, d_pre, chunks_max, pw, pw_n, flags)
        keep += [buf, d_pre, cnt, hp]
        return d_pre, n_pre

    def _langid(self, vb, vo, d_perm, ndocs, scratch, d_soff, rec, width, flags, prof):
        """Language-id records of a content version: k_langid_mfma (embedding bag + bf16 MFMA
        head, one 16-document tile per workgroup; no scratch)."""
        self.k.langid_mfma(vb, vo, d_perm, ndocs, self.lid_E, self.lid_aux, self.lid_WT, self.lid_w_scale,
                           self.lid_b, rec, width, prof)

    def _scratch_for(self, slot: _Slot, nbytes: int, which: str = "stage"):
        attr = "scratch" if which == "stage" else "scratch_c4"
        cur = getattr(slot, attr)
        if cur is None or cur.numel() < nbytes:
            # the old arena stays alive in the keep list of the batch that last used it
            setattr(slot, attr, None)
            cur = self.rt.empty(int(nbytes * 1.25) + (1 << 20), np.uint8)
            setattr(slot, attr, cur)
        return cur

    def _record(self, stream):
        return stream.record()

    def _ktimed(self, keep, name: str):
        """Context manager: HIP events around the launches inside it on the current stream; the
        elapsed time lands in tb_gpu_kernel_seconds{kernel=name} when the batch is collected."""
        import contextlib

        rt = self.rt

        @contextlib.contextmanager
        def cm():
            st = rt.current_stream()
            e0 = rt.Event(timing=True).record(st)
            yield
            e1 = rt.Event(timing=True).record(st)
            keep.append(("ktime", name, (e0, e1)))

        return cm()

    def _prof_buf(self, ndocs, keep, name):
        if not self.phase_prof:
            return None
        t = self.rt.zeros(ndocs * 32, np.int64)
        keep.append(("prof", name, t))
        return t

    def collect_phase_prof(self, keep) -> None:
        for item in keep:
            if isinstance(item, tuple) and len(item) == 3 and item[0] == "prof":
                _, name, t = item
                a = t.to_host().reshape(-1, 32).sum(0)
                self.phase_totals[name] = self.phase_totals.get(name, 0) + a
                self.phase_docs[name] = self.phase_docs.get(name, 0) + t.numel() // 32

    def phase_report(self) -> str:
        names = {0: "start", 1: "decode", 2: "dict", 3: "prefix_hash", 4: "words", 5: "lines", 6: "gopher_quality",
                 7: "gr_lines_paras", 8: "gr_word_hash", 9: "gr_top_ngrams", 10: "gr_dup_ngrams", 11: "fineweb",
                 12: "langid", 13: "gr_dup_walk", 14: "gr_dup_canon", 15: "gr_top_canon", 16: "c4_lorem", 17: "c4_decode", 18: "c4_lines", 19: "c4_cite", 20: "c4_words",
                 21: "c4_codes", 22: "c4_join", 23: "c4_sentences",
                 24: "gr_nl_runs", 25: "gr_line_dup", 26: "gr_word_hash8", 27: "gr_word_canon", 28: "gq_words",
                 29: "gq_bytes", 30: "rust_lines"}
        lines = []
        for k, tot in self.phase_totals.items():
            nd = max(1, self.phase_docs[k])
            allc = float(np.sum(tot))
            lines.append(f"{k}: {allc / nd:,.0f} cycles/doc (wave lifetime, summed phases)")
            for i in np.nonzero(tot)[0]:
                lines.append(f"   {names.get(int(i), i):>16}: {tot[i] / nd:>12,.0f}  ({100 * tot[i] / allc:5.1f}%)")
        return "\n".join(lines)

    def submit(self, data: np.ndarray, off: np.ndarray, bw: Optional[Dict[int, BwInput]] = None) -> PendingBatch:
        """Stage inputs, enqueue every device stage and the D2H copies; returns immediately.
        ``bw``: inputs of the pipeline's C4BadWords steps (Engine._bw_inputs)."""
        import time

        t0 = time.perf_counter()
        slot = self.slots[self._next_slot]
        self._next_slot = (self._next_slot + 1) % self.N_SLOTS
        with self.rt.stream(slot.main):
            return self._submit_on(slot, data, off, t0, bw or {})

    def _submit_on(self, slot: "_Slot", data: np.ndarray, off: np.ndarray, t0: float,
                   bw: Dict[int, BwInput]) -> PendingBatch:
        import time

        rt = self.rt
        h = native.host()
        ndocs = len(off) - 1
        lens = np.diff(off)
        perm = launch_order(lens)
        lens_perm = lens[perm]
        # scratch slice per document (devplan.h scratch_bytes_for_dev): the split rate for the
        # documents whose n-gram orders run in split tasks (k_gr_dup_split over the workgroup
        # documents past split_doc_bytes, k_gr_split_wave over wave documents past ngram_big_bytes)
        r_one, r_split = self.scratch_rates
        rate = np.full(ndocs, r_one, dtype=np.int64)
        if self.gr_split:
            is_long = lens > self.long_doc_bytes if self.long_doc_bytes > 0 else np.zeros(ndocs, bool)
            split = np.zeros(ndocs, bool)
            if self.split_doc_bytes > 0:
                split |= is_long & (lens > self.split_doc_bytes)
            split |= ~is_long & (lens > self.ngram_big_bytes)
            rate[split] = r_split
        per_doc = 4096 + rate * (lens + 64)
        per_doc = (per_doc + SCRATCH_ALIGN - 1) // SCRATCH_ALIGN * SCRATCH_ALIGN
        # slices in dispatch (perm) order: scratch_off[k] is the slice of the k-th launched
        # document, so the waves resident at one time share one contiguous window of the arena
        # (TLB and cache locality) instead of slices scattered over ~50 GB
        scratch_off = np.zeros(ndocs + 1, dtype=np.int64)
        np.cumsum(per_doc[perm], out=scratch_off[1:])
        maxlen = int(lens.max()) if ndocs else 0
        n_long = int(np.count_nonzero(lens > self.long_doc_bytes)) if self.long_doc_bytes > 0 else 0
        # perm is longest first: [0, n_long) workgroup docs, then the wave docs
        direct_keep: List = []
        # per-document bad-words roots / CJK flags and the long documents' segment lists travel in
        # the same upload
        bw_arrays = [((i, "root" if a.dtype == np.int32 else "cjk"), a) for i in sorted(bw)
                     for a in (bw[i].roots, bw[i].cjk) if a is not None]
        for _, a in bw_arrays:
            if len(a) != ndocs:
                raise DeviceError("badwords: per-document inputs do not match the batch")
        for v in sorted({self.plan.steps[i].version_in for i in bw}):
            sd, si = bw_segments(lens, self.c4_growth * v, BW_SEG_BYTES)
            if len(sd):
                bw_arrays += [((v, "seg_doc"), sd), ((v, "seg_idx"), si)]
        dict_arrays = []
        dict_c4_keys = []  # C4 steps with host line statistics (their two arrays follow the marks)
        if self.dict_marks and ndocs:
            with tracing.trace_range("tb.dict_marks"):
                moff, mbits = h.dict_word_marks(data, off, self.host_threads)
            if len(mbits):
                dict_arrays = [moff, mbits]
                metrics.DICT_MARKED_DOCS_TOTAL.inc(int(np.count_nonzero(moff >= 0)))
                # C4 steps on the original text: the per-line ICU word statistics of the marked
                # documents that may hold a citation (their C4 pass segments processed lines)
                for i in self.plan.c4_steps:
                    if self.plan.steps[i].version_in == 0:
                        lo, ld = h.dict_c4_lines(data, off, moff, bool(self.steps[i].remove_citations),
                                                 self.host_threads)
                        if len(ld):
                            dict_c4_keys.append(i)
                            dict_arrays += [lo, ld]
        with tracing.trace_range("tb.stage_h2d"):
            staged_views, staged = self._stage_inputs(
                slot, [data if len(data) else np.zeros(1, np.uint8), off, perm, scratch_off]
                + [np.ascontiguousarray(a) for _, a in bw_arrays] + dict_arrays, direct_keep)
        d_bytes, d_off, d_perm, d_soff = staged_views[:4]
        bw_dev = {key: d for (key, _), d in zip(bw_arrays, staged_views[4:4 + len(bw_arrays)])}
        # per content version: the word sources of its dictionary-script documents (DictIn)
        nd_arr = len(dict_arrays)
        dv = staged_views[len(staged_views) - nd_arr:] if nd_arr else []
        dict_in = {0: (dv[0], dv[1], None)} if nd_arr else {}
        dict_lines = {i: (dv[2 + 2 * k], dv[3 + 2 * k]) for k, i in enumerate(dict_c4_keys)}
        scratch = self._scratch_for(slot, int(scratch_off[-1]))
        # grows (new tensor, on this slot's stream) only for documents over 2 MB; the batch keeps a
        # reference to the table it used, so the other slot's kernels never see it freed
        pw, pw_n = self.k.pow_table(2 * maxlen + 64)
        flags = rt.zeros(ndocs, np.int32)
        dead = rt.zeros(ndocs, np.uint8) if self.gate_ts else None
        pass_idx = 0
        t1 = time.perf_counter()
        versions = {0: (d_bytes, d_off, len(data))}
        stage_recs_d: List = [None] * len(self.plan.stages)
        c4_recs_d = {}
        keep = [staged, scratch, pw] + direct_keep
        # Independent work runs concurrently on side streams (events order the dependencies):
        #   language-id bag (s_lid) | long-doc workgroup kernels (s_blk) | wave kernels (main)
        #   | C4 pass A/B of the same content version (s_c4, own scratch arena)
        # Block and wave kernels touch disjoint documents, so they share the stage arena.
        main = rt.current_stream()
        ready = {0: self._record(main)}
        tails = []
        c4_scratch = None
        pre_v0 = None  # (descriptors, n_pre) of the version-0 pre-pass
        for ver in range(self.plan.n_versions):
            vb, vo, vlen = versions[ver]
            main.wait_event(ready[ver])
            # uint32 [4 * (bytes / 8 + 16 * documents) + 16]: document d's region at
            # 4 * (off[d] / 8 + 16 d) (docproc.h line_stats_base)
            lstats = None
            if ver in self.line_stats_stage:
                lstats = rt.empty(4 * (vlen // 8 + 16 * ndocs) + 16, np.uint32)
                keep.append(lstats)
            for s, sv in enumerate(self.plan.stage_version):
                if sv != ver:
                    continue
                width_total, layout = self.stage_layout[s]
                rec = rt.zeros(width_total * ndocs, np.int64)
                lid_at = [(width, prefix) for kind, width, prefix in layout if kind == KIND_LANGID]
                ev_pre = self._record(main)  # rec zeroed
                keep.append(ev_pre)
                ev_lid = ev_blk = None
                prof = self._prof_buf(ndocs, keep, f"stage{s}")
                lid_pass = ("lid", s) in self.passes
                if lid_pass:
                    # language-id pass first (records + gate on the side stream); the stage kernels
                    # below skip the documents it filters
                    slot.s_lid.wait_event(ev_pre)
                    with rt.stream(slot.s_lid):
                        with self._ktimed(keep, "langid"):
                            for width, prefix in lid_at:
                                self._langid(vb, vo, d_perm, ndocs, scratch, d_soff, rec[prefix * ndocs:], width,
                                             flags, self._prof_buf(ndocs, keep, f"langid{s}"))
                        if pass_idx in self.gate_ts:
                            self.k.gate(self.gate_ts[pass_idx], [rec], ndocs, flags, dead, pass_idx + 1, 0,
                                        self.gate_need[pass_idx])
                        ev_pre = self._record(slot.s_lid)
                        keep.append(ev_pre)
                    main.wait_event(ev_pre)
                    pass_idx += 1
                skip = dead if pass_idx > 0 else None
                ls_out = lstats if self.line_stats_stage.get(ver) == s else None
                # long documents first: with the 4-stream layout the workgroup kernels and the
                # language-id bag share the side stream, and the long-document tail must start early
                if n_long:
                    slot.s_blk.wait_event(ev_pre)
                    n_split, gx = 0, None
                    if s in self.gr_split and self.split_doc_bytes > 0:
                        # launch positions [0, n_split) hold every document over the split size
                        huge = np.nonzero(lens[perm[:n_long]] > self.split_doc_bytes)[0]
                        if len(huge):
                            n_split = int(huge[-1]) + 1
                            # zeroed on the stream of the kernels that write and read it
                            gx = rt.zeros(n_split * self.k.sizeof_gr_export, np.uint8, slot.s_blk)
                            keep.append(gx)
                    # the split export slots are indexed by launch position
                    esz = self.k.sizeof_gr_export
                    with rt.stream(slot.s_blk), self._ktimed(keep, f"stage{s}_blk"):
                        # (the original text only: the host knows no lengths of rewritten versions); once
                        # per batch: every stage reading version 0 reuses it (read-only, same stream)
                        if ver == 0 and pre_v0 is None:
                            pre_v0 = self._pre_decode(vb, vo, d_perm, lens[perm[:n_long]], skip, keep, flags,
                                                      self.pre_wcanon)
                        pre, n_pre = pre_v0 if ver == 0 else (None, 0)
                        # launch positions [0, n_pre): the pre-pass kernel instantiation, the rest the common one
                        bt = self.block_threads
                        segs = ((0, n_pre, bt, True), (n_pre, n_long, bt, False))
                        for a0, a1, thr, with_pre in segs:
                            if a1 <= a0:
                                continue
                            ns = max(0, min(n_split, a1) - a0)
                            self.k.stage_analyze_blk(self.plan_t, self.stage_ts[s], vb, vo, d_perm[a0:a1], a1 - a0,
                                                     ndocs, scratch, d_soff[a0:], pw, pw_n, rec, flags,
                                                     self.lds_bytes_blk, prof, skip,
                                                     gx[a0 * esz:] if (gx is not None and ns) else None, ns,
                                                     self.split_doc_bytes, thr, ls_out,
                                                     pre if with_pre else None, a1 - a0 if with_pre else 0,
                                                     dict_in.get(ver))
                        if n_split:
                            gr_pos, n_tasks = self.gr_split[s]
                            cur = rt.empty(1, np.uint32)
                            keep.append(cur)
                            self.k.gr_dup_split(self.stage_ts[s], gr_pos, d_perm[:n_split], n_split, n_tasks, ndocs,
                                                gx, pw, pw_n, rec, flags, self.lds_bytes_dup, cur)
                        ev_blk = self._record(slot.s_blk)
                        keep.append(ev_blk)
                if lid_at and not lid_pass:
                    # language ID next to the stage kernels: it writes only its own record columns
                    slot.s_lid.wait_event(ev_pre)
                    with rt.stream(slot.s_lid), self._ktimed(keep, "langid"):
                        for width, prefix in lid_at:
                            self._langid(vb, vo, d_perm, ndocs, scratch, d_soff, rec[prefix * ndocs:], width,
                                         flags, self._prof_buf(ndocs, keep, f"langid{s}"))
                        ev_lid = self._record(slot.s_lid)
                        keep.append(ev_lid)
                if n_long < ndocs:
                    nw = ndocs - n_long
                    gxw = None
                    if s in self.gr_split:
                        # split mode: the wave documents' n-gram orders run one wave per (document,
                        # order) after the stage kernel (k_gr_split_wave)
                        gxw = rt.zeros(self.k.gr_export_wave_bytes(nw), np.uint8)
                        keep.append(gxw)
                    with self._ktimed(keep, f"stage{s}"):
                        self.k.stage_analyze(self.plan_t, self.stage_ts[s], vb, vo, d_perm[n_long:], ndocs,
                                             scratch, d_soff[n_long:], pw, pw_n, rec, flags,
                                             self.lds_bytes, prof, self.stage_waves, nw, skip, ls_out, gxw,
                                             dict_in.get(ver))
                        if gxw is not None:
                            gr_pos, n_tasks = self.gr_split[s]
                            # wave documents longer than ngram_big_bytes (a prefix: perm is longest
                            # first) take one wave per order, the rest one workgroup each
                            n_big = int(np.count_nonzero(lens_perm[n_long:] > self.ngram_big_bytes))
                            self.k.gr_split_wave(self.stage_ts[s], gr_pos, d_perm[n_long:], nw, n_tasks - 2, ndocs,
                                                 gxw, pw, pw_n, rec, flags, self.lds_bytes_split, self.ngram_block,
                                                 self._prof_buf(ndocs, keep, f"ngram{s}"), n_big)
                if ev_lid is not None:
                    main.wait_event(ev_lid)
                if ev_blk is not None:
                    main.wait_event(ev_blk)
                if pass_idx in self.gate_ts:
                    self.k.gate(self.gate_ts[pass_idx], [rec], ndocs, flags, dead, pass_idx + 1, 0,
                                        self.gate_need[pass_idx])
                pass_idx += 1
                stage_recs_d[s] = rec
            c4_here = [i for i in self.plan.c4_steps if self.plan.steps[i].version_in == ver]
            for i in c4_here:
                # The C4 pass reuses the stage arena: it starts after every stage kernel of its
                # content version (it waits for the gate on the compute stream), and the stages of
                # the next version start after its pass B (ready event).
                c4_scratch = scratch
                rec = rt.zeros(7 * ndocs, np.int64)
                src = rt.zeros(2 * ndocs, np.int64)
                new_off = rt.zeros(ndocs + 1, np.int64)
                # the rewrite's word count per document (kNoWords unless C4 pass A's export path
                # set it): the word source of the next version's dictionary-script documents
                c4w = None
                if self.dict_marks and ver in dict_in:
                    c4w = rt.empty(ndocs, np.uint32).fill_(0xFF)
                    keep.append(c4w)
                    dict_in[ver + 1] = (None, None, c4w)
                cap = vlen + self.c4_growth * ndocs + 16  # device rewrites never grow more (kC4MaxGrowth)
                out = rt.empty(cap, np.uint8)
                ev_main = self._record(main)
                slot.s_c4.wait_event(ev_main)
                slot.s_c4.wait_event(ready[ver])
                keep.append(ev_main)
                skip = dead if pass_idx > 0 else None
                prof = self._prof_buf(ndocs, keep, f"c4_step{i}")
                ev_c4blk = None
                if n_long:
                    # long documents (workgroup kernel) next to the wave kernel: disjoint docs
                    ev_c4 = self._record(slot.s_c4)
                    slot.s_c4blk.wait_event(ev_c4)
                    keep.append(ev_c4)
                    with rt.stream(slot.s_c4blk):
                        self.k.c4_pass_a_blk(self.c4_ts[i], vb, vo, d_perm[:n_long], n_long, ndocs, c4_scratch,
                                             d_soff, pw, pw_n, rec, src, flags, self.lds_bytes_blk, prof, skip,
                                             lstats, c4w, dict_lines.get(i))
                        ev_c4blk = self._record(slot.s_c4blk)
                        keep.append(ev_c4blk)
                with rt.stream(slot.s_c4), self._ktimed(keep, f"c4_step{i}"):
                    if n_long < ndocs:
                        self.k.c4_pass_a(self.c4_ts[i], vb, vo, d_perm[n_long:], ndocs, c4_scratch, d_soff[n_long:], pw,
                                         pw_n, rec, src, flags, self.lds_bytes_c4, prof, ndocs - n_long, skip,
                                         lstats, c4w, dict_lines.get(i))
                    if ev_c4blk is not None:
                        slot.s_c4.wait_event(ev_c4blk)
                    rt.scan_strided_i64(src[1:], 2, ndocs, new_off[1:])
                    self.k.c4_pass_b(vb, vo, ndocs, c4_scratch, d_soff, src, new_off, out)
                    if pass_idx in self.gate_ts:
                        self.k.gate(self.gate_ts[pass_idx], [rec], ndocs, flags, dead, pass_idx + 1, 0,
                                        self.gate_need[pass_idx])
                    ev = self._record(slot.s_c4)
                pass_idx += 1
                versions[ver + 1] = (out, new_off, cap)
                ready[ver + 1] = ev
                tails.append(ev)
                c4_recs_d[i] = rec
                keep.append(src)
        for ev in tails:
            main.wait_event(ev)
        bw_d = {}
        for i in sorted(bw):
            # C4BadWords: match every document that reached the step on the content version it
            # reads; the keep-fraction draws and the decision stay on the host (document order)
            x = bw[i]
            sp = self.plan.steps[i]
            vb, vo, _ = versions[sp.version_in]
            table, fold = self._bw_tables(x)
            m = rt.empty(max(ndocs, 1), np.int8)
            v = sp.version_in
            with self._ktimed(keep, "badwords"):
                self.k.badwords_match(vb, vo, ndocs, table, fold, m, bw_dev.get((i, "root")), bw_dev.get((i, "cjk")),
                                      x.root0, x.cjk0, dead, self.bw_dead_max[i], BW_SEG_BYTES,
                                      bw_dev.get((v, "seg_doc")), bw_dev.get((v, "seg_idx")))
            keep += [table, m]
            bw_d[i] = m
        res_d = None
        if self.resolve_t is not None:
            # K16 on the compute stream after every pass: first failure, status, and the final
            # contents of kept / excluded documents compacted into one buffer (the host then only
            # formats metadata). Output bound: a C4 rewrite grows a document by <= C4_MAX_GROWTH.
            recs = [r for r in stage_recs_d] + [c4_recs_d[i] for i in self.plan.c4_steps]
            vlist = [(versions[v][0], versions[v][1]) for v in range(self.plan.n_versions)]
            cap = len(data) + self.c4_growth * (self.plan.n_versions - 1) * ndocs + 16
            r_fail = rt.empty(ndocs, np.int32)
            r_status = rt.empty(ndocs, np.uint8)
            r_ver = rt.empty(ndocs, np.uint8)
            r_lanes = rt.empty(4 * ndocs, np.int64)
            r_sc = rt.empty(4 * ndocs, np.int64)
            r_out = rt.empty(max(cap, 1), np.uint8)
            r_off = rt.zeros(ndocs + 1, np.int64)
            r_rows = rt.empty(ndocs, np.int32)
            r_err = rt.zeros(1, np.int32)
            if any(r.numel() < need * ndocs for r, need in zip(recs, self.resolve_need)):
                raise DeviceError("resolve: a record buffer is smaller than the resolve plan reads")
            with self._ktimed(keep, "resolve"):
                self.k.resolve(self.resolve_t, recs, ndocs, flags.view(np.uint32), vlist, r_fail, r_status, r_ver,
                               r_lanes, r_sc, r_out, r_off, r_rows, r_err)
            keep += [r_fail, r_status, r_ver, r_lanes, r_sc, r_out, r_off, r_rows, r_err]
            res_d = (r_fail, r_status, r_out, r_off, r_rows, r_err, r_ver)
            for si, tabs in self.bpe:
                # the kept outputs are r_out[r_off[k]:r_off[k + 1]], k < the kept count (the last
                # entry of the kept-count scan, read by the kernel)
                r_tok = rt.empty(ndocs, np.int32)
                with self._ktimed(keep, "bpe_count"):
                    self.k.bpe_count(tabs, r_out, r_off, r_sc[3 * ndocs - 1:3 * ndocs], ndocs, r_tok)
                keep.append(r_tok)
                res_d = res_d + ((si, r_tok),)
        # D2H into pinned host buffers on the download stream (the slot's compute stream in the
        # 4-stream layout: it is last in line there anyway), then one completion event
        done = self._record(main)
        d2h_s = slot.s_d2h
        if d2h_s is not main:
            d2h_s.wait_event(done)

        def d2h(t):
            ht = rt.pinned(t.numel(), t.dtype)
            t.copy_to_host(ht, d2h_s)
            return ht

        h_stage = [d2h(r) if r is not None else None for r in stage_recs_d]
        h_c4 = {i: d2h(r) for i, r in c4_recs_d.items()}
        h_versions = {}
        h_res = None
        if res_d is not None:
            h_res = tuple(d2h(t) for t in res_d[:7]) + tuple((si, d2h(t)) for si, t in res_d[7:])
        if h_res is not None:
            # K16: the compacted outputs replace the versions on the host path; they stay in HBM
            # (downloaded only if the host has to assemble this batch itself)
            h_versions = LazyVersions({v: versions[v][:2] for v in range(1, self.plan.n_versions)})
        else:
            for ver in range(1, self.plan.n_versions):
                vb, vo, _ = versions[ver]
                h_versions[ver] = (d2h(vb), d2h(vo))
        h_flags = d2h(flags)
        h_dead = d2h(dead) if dead is not None else None
        h_bw = {i: d2h(m) for i, m in bw_d.items()}
        ev = self._record(d2h_s)
        keep += [stage_recs_d, c4_recs_d, versions, flags, dead, ready, tails, done]
        t2 = time.perf_counter()
        return PendingBatch(self, ndocs, ev, h_stage, h_c4, h_versions, h_flags,
                            {"stage_h2d": t1 - t0, "launch": t2 - t1}, keep, h_dead, h_res, h_bw)

    def run(self, data: np.ndarray, off: np.ndarray, bw: Optional[Dict[int, BwInput]] = None) -> DeviceResult:
        return self.submit(data, off, bw).wait()


class EmulatedRunner:
    """Host emulation of :class:`DeviceRunner` (same records, versions and flags, computed by the
    C++ port of the device algorithms). Drives the exact resolve path of the GPU backend on a
    machine without a GPU (``Engine(backend="emulate")``): used by CPU tests and for profiling
    the host side of the device pipeline."""

    def __init__(self, steps_native, plan: ExecPlan, langid=None, nthreads: int = 8, gating: Optional[bool] = None,
                 gate_corrupt: int = 0, token_counters=None, tune: Optional[DeviceTuning] = None):
        h = native.host()
        self.steps = steps_native
        self.plan = plan
        self.nthreads = nthreads
        self.lid = langid.native() if langid is not None else None
        _, stage_bs = h.build_device_plan(steps_native, plan.stages)
        self.stage_layout = [h.stage_layout(b) for b in stage_bs]
        tu = tune or tuning.from_env()
        if gating is None:
            gating = tu.gate
        self.passes, self.pass_of_step, self.gates = plan_passes(
            plan, self.stage_layout, steps_native, gating, tu.lid_gate)
        self.bw_dead_max = bw_dead_max(plan, self.passes, self.pass_of_step)
        self.line_stats_stage = line_stats_stages(plan, self.stage_layout, tu)
        # test hook: additionally mark every k-th document dead after the first pass (a wrong
        # device gate), to exercise the resolver's recovery path
        self.gate_corrupt = gate_corrupt
        self.resolve_blob = None
        if tu.device_resolve:
            self.resolve_blob = build_resolve(plan, self.stage_layout, steps_native)
        self.bpe = []
        if self.resolve_blob is not None and tu.device_tokens:
            self.bpe = list(token_counters or [])
        self.dict_marks = dict_marks_wanted(plan, steps_native, tu)

    def run(self, data: np.ndarray, off: np.ndarray, bw: Optional[Dict[int, BwInput]] = None) -> DeviceResult:
        import time

        h = native.host()
        t0 = time.perf_counter()
        ndocs = len(off) - 1
        flags = np.zeros(ndocs, dtype=np.uint32)
        versions = {0: (data, off)}
        stage_recs: List[Optional[np.ndarray]] = [None] * len(self.plan.stages)
        c4_recs = {}
        dead = np.zeros(ndocs, dtype=np.uint8) if self.gates else None
        lid_rec = {}
        lstats = {}  # content version -> the C4 line export buffer (as on the device)
        # content version -> the word sources of its dictionary-script documents (DeviceRunner)
        dict_in = {}
        if self.dict_marks and ndocs:
            moff, mbits = h.dict_word_marks(data, off, self.nthreads)
            if len(mbits):
                dict_in[0] = dict(dict_moff=moff, dict_bits=mbits)
        dict_lines = {}
        if 0 in dict_in:
            for i in self.plan.c4_steps:
                if self.plan.steps[i].version_in == 0:
                    lo, ld = h.dict_c4_lines(data, off, dict_in[0]["dict_moff"], bool(self.steps[i].remove_citations),
                                             self.nthreads)
                    if len(ld):
                        dict_lines[i] = dict(dict_loff=lo, dict_ldata=ld)
        for p, (kind, x) in enumerate(self.passes):
            skip = dead if p > 0 else None
            if kind == "lid":
                # the whole stage once (the language-id columns are what this pass produces; the
                # other columns are recomputed below for the documents the gate leaves alive)
                vd, vo = versions[self.plan.stage_version[x]]
                rec, fl = h.emulate_stage(self.steps, self.plan.stages[x], vd, vo, self.nthreads, self.lid, 0, skip)
                lid_rec[x] = rec
                # the language-id kernels flag nothing: their records are exact for every script, so
                # a document this gate filters never goes to the CPU path (dictionary scripts are
                # flagged by the segmentation passes of the documents that reach them)
                fl = np.zeros(ndocs, dtype=np.uint32)
            elif kind == "stage":
                sv = self.plan.stage_version[x]
                vd, vo = versions[sv]
                ls = None
                if self.line_stats_stage.get(sv) == x:
                    ls = lstats[sv] = np.empty(h.line_stats_words(vo), dtype=np.uint32)
                rec, fl = h.emulate_stage(self.steps, self.plan.stages[x], vd, vo, self.nthreads, self.lid, 0, skip,
                                          line_stats=ls, **dict_in.get(sv, {}))
                if x in lid_rec:
                    for k, width, prefix in self.stage_layout[x][1]:
                        if k == KIND_LANGID:
                            rec[prefix * ndocs:(prefix + width) * ndocs] = lid_rec[x][prefix * ndocs:(prefix + width) * ndocs]
                stage_recs[x] = rec
            else:
                vin = self.plan.steps[x].version_in
                vd, vo = versions[vin]
                c4w = None
                if vin in dict_in:
                    c4w = np.full(ndocs, 0xFFFFFFFF, dtype=np.uint32)
                    dict_in[self.plan.steps[x].version_out] = dict(dict_words=c4w)
                rec, nd, no, fl = h.emulate_c4(self.steps[x], vd, vo, self.nthreads, 0, skip,
                                               line_stats=lstats.get(vin), c4_words=c4w, **dict_lines.get(x, {}))
                c4_recs[x] = rec
                versions[self.plan.steps[x].version_out] = (nd, no)
            flags |= fl
            if p in self.gates:
                h.gate_host(self.gates[p][0], [rec], ndocs, flags, dead, p + 1)
                if p == 0 and self.gate_corrupt > 0:
                    extra = np.arange(0, ndocs, self.gate_corrupt)
                    dead[extra[dead[extra] == 0]] = 1
        host_versions = {v: versions[v] for v in range(1, self.plan.n_versions)}
        bwm = {}
        for i, x in sorted((bw or {}).items()):
            # k_badwords_match's walk (csrc/common/badwords.h bw_match_doc), same skip rule
            vd, vo = versions[self.plan.steps[i].version_in]
            bwm[i] = h.bw_match_batch(vd, vo, np.ascontiguousarray(x.table, dtype=np.uint32), x.roots, x.cjk, x.root0,
                                      x.cjk0, dead, self.bw_dead_max[i], self.nthreads)
        resolved = None
        if self.resolve_blob is not None:
            recs = list(stage_recs) + [c4_recs[i] for i in self.plan.c4_steps]
            vl = [versions[v] for v in range(self.plan.n_versions)]
            fail, st, out, out_off, rows = h.resolve_host(self.resolve_blob, recs, ndocs, flags,
                                                          [np.ascontiguousarray(d) for d, _ in vl],
                                                          [np.ascontiguousarray(o) for _, o in vl])
            resolved = Resolved(fail, st, out, out_off, rows)
            if self.bpe:
                # k_bpe_count's algorithm (csrc/common/bpe.h) over the kept outputs
                nk = int(np.count_nonzero(st == 0))
                ko = np.ascontiguousarray(out_off[:nk + 1])
                resolved.tokens = {
                    si: h.bpe_count(out, ko, sp.byte_id, sp.keys, sp.vals, sp.mask, sp.added, sp.added_off,
                                    sp.post_add, self.nthreads) for si, sp in self.bpe}
        return DeviceResult(stage_recs, c4_recs, host_versions, flags, {"emulate": time.perf_counter() - t0}, dead,
                            self.pass_of_step, resolved, bwm or None)
