"""Batched pipeline engine: the in-process replacement of the reference's producer/worker loop
(reference worker_logic.rs:140-193 + producer_logic.rs:109-196).

One ``Engine`` holds a validated pipeline, its device plan and models. ``process()`` takes one
batch of documents (packed UTF-8 + optional metadata JSON column) and returns kept / excluded
outputs with the same per-document semantics as the reference executor: steps in YAML order,
the first filtering step wins, metadata of every executed step is kept, C4 rewrites content.

Backends:
  * ``cuda``: record/rewrite steps on the MI355X (HIP kernels), decisions + output assembly in
    the C++ host runtime; documents flagged by the device (dictionary scripts, hash collisions,
    scratch overflow) are recomputed on the CPU path with the ICU oracle.
  * ``emulate``: the ``cuda`` resolve path with device records computed by the host port of
    the kernels (no GPU needed; tests and profiling).
  * ``cpu``: the C++ CPU path (multithreaded); segmentation by our UAX#29 rules ("rules") or by
    ICU4C ("icu", the oracle).
"""
from __future__ import annotations

import collections
import dataclasses
import os
import time
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .. import native
from ..config.pipeline import PipelineConfig
from ..errors import ConfigError, DeviceError, Unexpected
from ..utils import tracing
from .plan import ExecPlan, build_plan
from . import tuning
from .tuning import DeviceTuning

# per-document device flag bits (csrc/common/docproc.h DocFlag)
DOC_NEEDS_CPU = 1
DOC_OVERFLOW = 2


@dataclasses.dataclass
class OutputPart:
    rows: np.ndarray          # int64 row indices into the input batch
    text_data: np.ndarray     # uint8
    text_off: np.ndarray      # int64 [len(rows)+1]
    meta_data: np.ndarray     # uint8
    meta_off: np.ndarray      # int64
    meta_valid: np.ndarray    # uint8 (0 -> null metadata)


@dataclasses.dataclass
class BatchResult:
    n_docs: int
    kept: List[OutputPart]
    excluded: List[OutputPart]
    error_rows: np.ndarray
    fail_step: np.ndarray      # int32 per doc (-1 kept), CPU-delegated docs included
    status: np.ndarray         # uint8 per doc: 0 kept, 1 filtered, 2 error
    reasons: Dict[int, str]    # filled only when requested
    timings: Dict[str, float]
    n_delegated: int = 0
    # process_many: the CPU-path recomputation of the delegated documents, still running on the
    # engine's delegation thread ((future, rows)); merged before the result is handed out
    deferred: Optional[Tuple] = None

    @property
    def n_kept(self) -> int:
        return int(sum(len(p.rows) for p in self.kept))

    @property
    def n_excluded(self) -> int:
        return int(sum(len(p.rows) for p in self.excluded))


def _gate_mismatch(n: int, p: int) -> None:
    import logging

    from ..utils import metrics

    logging.getLogger("textblaster_amd.engine").warning(
        "device gate skipped %d document(s) in pass %d that the resolver finds alive; recomputing them on the CPU path",
        n, p)
    metrics.GATE_MISMATCH_DOCS_TOTAL.inc(n)


def default_threads() -> int:
    # a rank pinned to its CPU set (parallel/placement.py) sizes its pool from the set's thread
    # budget (readers and writers take their share of the same CPUs)
    from ..parallel import placement

    cpus = placement.bound_cpus()
    if cpus is not None and not os.environ.get("TB_THREADS"):
        return placement.thread_budget(len(cpus)).pool
    # the GPU boxes expose every CPU of the host through the affinity mask but give one GPU a
    # share of them (OMP_NUM_THREADS); honour explicit limits first
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    for var in ("TB_THREADS", "OMP_NUM_THREADS"):
        env = os.environ.get(var)
        if env and env.isdigit() and int(env) > 0:
            # torch.distributed.run exports OMP_NUM_THREADS=1 to every rank when it was unset;
            # that is its default for math libraries, not a CPU budget for our host runtime
            if var == "OMP_NUM_THREADS" and int(env) == 1 and local_world > 1:
                continue
            return int(env)
    try:
        ncpu = max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    return max(1, min(32, ncpu // max(1, local_world))) if local_world > 1 else ncpu


class Engine:
    def __init__(self, cfg: PipelineConfig, backend: str = "auto", device: Optional[str] = None,
                 nthreads: Optional[int] = None, segmentation: str = "rules", langid=None,
                 tokenizer_dir: Optional[str] = None, badwords_dir: Optional[str] = None,
                 keep_reasons: bool = False, tokenizer_file: Optional[str] = None,
                 fault_inject: Optional[str] = None, tokenizers=None, badwords=None,
                 max_batch_bytes: Optional[int] = None, slots: Optional[int] = None,
                 tune: Optional[DeviceTuning] = None):
        self.cfg = cfg
        self._cpu_engine = None
        self._n_submitted = 0
        self._fault = _parse_fault(fault_inject or os.environ.get("TB_FAULT_INJECT", ""))
        import threading

        self._submit_lock = threading.RLock()
        # CPU-path work of delegated documents (process_many): one thread, so it overlaps the next
        # batches' resolve / assembly on the consumer thread (the native pools do the heavy part)
        self._deleg_pool = None
        self._async_delegation = False
        # device operating points (pipeline/tuning.py; TB_TUNE, run --batch-bytes / --slots)
        self.tune = (tune or tuning.from_env()).replace(batch_bytes=max_batch_bytes or None, slots=slots or None)
        # process_many on the GPU backend submits from a helper thread (prefetch_thread=0: off)
        self.prefetch_threads = self.tune.prefetch_thread
        # text bytes per device batch (scratch 80-176 B per text byte per in-flight slot: 384 MB of
        # text -> at most ~85 GB of HBM per slot, three slots in flight on a 288 GB MI355X)
        self.max_batch_bytes = int(self.tune.batch_bytes)
        self.h = native.host()
        self.plan: ExecPlan = build_plan(cfg)
        self.steps = [self.h.make_step(s.native_dict()) for s in cfg.pipeline]
        self.nthreads = nthreads or default_threads()
        self.segmentation = segmentation
        self.keep_reasons = keep_reasons
        if backend == "auto":
            backend = "cuda" if _cuda_available() else "cpu"
        self.backend = backend
        types = [s.type for s in cfg.pipeline]
        self.langid = None
        if "LanguageDetectionFilter" in types:
            from ..models.langid import load_default

            with tracing.trace_range("tb.init.langid"):
                self.langid = langid or load_default()
        self.lid_native = self.langid.native() if self.langid is not None else None
        self.tokenizers: Dict[int, object] = dict(tokenizers or {})
        for i, s in enumerate(cfg.pipeline):
            if s.type == "TokenCounter" and i not in self.tokenizers:
                from ..models.tokenizer import load_tokenizer

                self.tokenizers[i] = load_tokenizer(tokenizer_file or s.params.tokenizer_name, tokenizer_dir)
        self.badwords = badwords
        if "C4BadWordsFilter" in types and self.badwords is None:
            bw_dirs = [s.params.cache_base_path for s in cfg.pipeline
                       if s.type == "C4BadWordsFilter" and s.params.cache_base_path]
            d = badwords_dir or (bw_dirs[0] if bw_dirs else os.path.join("data", "c4_badwords"))
            with tracing.trace_range("tb.init.badwords"):
                self.badwords = self.h.BadWordsModule(d)
        # C4BadWords steps: on the GPU backends the matching runs in the batch's device pass
        # sequence (k_badwords_match); languages and keep-fraction draws stay on the host. The lock
        # serialises the word-list loading of the submitter and consumer threads.
        self._bw_steps = [i for i, s in enumerate(cfg.pipeline) if s.type == "C4BadWordsFilter"]
        self._bw_lock = threading.Lock()
        self._bw_nolist = set()
        self.device_runner = None
        # trailing TokenCounter steps (after every filter) whose tokenizer is a byte-level BPE are
        # counted by the device path on the kept outputs (k_bpe_count); the others on the host
        from .device import trailing_token_counters

        self._trailing_tc = set(trailing_token_counters(self.plan))
        token_counters = []
        if backend in ("cuda", "emulate"):
            for i in sorted(self._trailing_tc):
                spec_fn = getattr(self.tokenizers.get(i), "bpe_spec", None)
                spec = spec_fn() if spec_fn is not None else None
                if spec is not None:
                    token_counters.append((i, spec))
        if backend == "emulate":
            from .device import EmulatedRunner

            self.device_runner = EmulatedRunner(self.steps, self.plan, self.langid, self.nthreads,
                                                token_counters=token_counters, tune=self.tune)
        if backend == "cuda":
            for st in self.steps:
                ok, why = self.h.device_supported(st)
                if not ok:
                    raise ConfigError(f"step {st.name} cannot run on the device: {why}")
            from .device import DeviceRunner

            with tracing.trace_range("tb.init.device_runner"):
                self.device_runner = DeviceRunner(self.steps, self.plan, device or "cuda", self.langid,
                                                  max_batch_bytes=self.max_batch_bytes, token_counters=token_counters,
                                                  host_threads=self.nthreads, tune=self.tune)

    # ------------------------------------------------------------------------------------------
    def process(self, data: np.ndarray, off: np.ndarray, meta: Optional[Tuple] = None,
                row_base: int = 0) -> BatchResult:
        """Run the pipeline over one batch. ``meta`` = (data uint8, off int64, valid uint8) or None."""
        return self._merge_deferred(self.finish(self.submit(data, off, meta, row_base)))

    def process_many(self, batches: Iterable, on_error: str = "raise") -> Iterator[BatchResult]:
        """Pipelined processing of an iterable of ``(data, off, meta)`` batches: batch k+1 is
        staged and its kernels queued on the GPU before batch k is resolved and assembled on the
        host, so device work and host work overlap. Results are yielded in input order.

        ``on_error="recover"``: a batch whose device work fails (HIP error, out of memory, an
        injected fault) is re-run split in two halves, and if that fails too, on the CPU oracle
        path; the failure is logged and counted, the run continues."""
        # Device batches are bounded in bytes (the per-document scratch arena is <= 176x the text):
        # a large input batch runs as several sub-batches whose results are merged back.
        groups: Dict[int, List] = {}
        sizes: Dict[int, int] = {}

        def expand():
            for g, item in enumerate(batches):
                subs = self._split_by_bytes(item)
                sizes[g] = len(subs)
                groups[g] = []
                for base, sub in subs:
                    yield g, base, sub

        def submit_item(g, base, item):
            try:
                return (g, base, item, self.submit(item[0], item[1], item[2] if len(item) > 2 else None))
            except Exception as e:  # noqa: BLE001 - handled per on_error
                return (g, base, item, e)

        self._async_delegation = self.backend in ("cuda", "emulate")
        try:
            if self.prefetch_threads and self.backend in ("cuda", "emulate"):
                yield from self._deferred_in_order(self._process_threaded(expand(), submit_item, on_error, groups,
                                                                          sizes))
                return
            yield from self._deferred_in_order(self._process_serial(expand(), submit_item, on_error, groups, sizes))
        finally:
            self._async_delegation = False

    def _process_serial(self, items, submit_item, on_error, groups, sizes):
        pending = None
        for g, base, item in items:
            cur = submit_item(g, base, item)
            if pending is not None:
                out = self._collect_group(pending, on_error, groups, sizes)
                if out is not None:
                    yield out
            pending = cur
        if pending is not None:
            out = self._collect_group(pending, on_error, groups, sizes)
            if out is not None:
                yield out

    # results whose delegated documents are still on the CPU path, at most this many held back
    DEFERRED_DEPTH = 3

    def _deferred_in_order(self, results) -> Iterator[BatchResult]:
        """Yields results in order once their delegated (CPU-path) documents are merged in; the
        CPU work of batch k runs while batches k+1.. are resolved and assembled."""
        held: collections.deque = collections.deque()
        try:
            for r in results:
                held.append(r)
                while held and (held[0].deferred is None or held[0].deferred[0].done()
                                or len(held) > self.DEFERRED_DEPTH):
                    yield self._merge_deferred(held.popleft())
            while held:
                yield self._merge_deferred(held.popleft())
        finally:
            for r in held:  # an early exit: the CPU jobs finish before their inputs go away
                if r.deferred is not None:
                    r.deferred[0].result()

    @staticmethod
    def _merge_deferred(result: BatchResult) -> BatchResult:
        if result.deferred is None:
            return result
        fut, delegated = result.deferred
        result.deferred = None
        t0 = time.perf_counter()
        sub2 = fut.result()
        result.kept += sub2.kept
        result.excluded += sub2.excluded
        result.error_rows = np.concatenate([result.error_rows, sub2.error_rows])
        result.fail_step[delegated] = sub2.fail_step
        result.status[delegated] = sub2.status
        result.reasons.update(sub2.reasons)
        result.n_delegated = len(delegated)
        result.timings["delegated_wait"] = time.perf_counter() - t0
        return result

    def _process_threaded(self, items, submit_item, on_error, groups, sizes):
        """process_many with a submitter thread: input staging (pinned copy + H2D) and kernel
        launches of the next batches run on their own thread while this thread resolves and
        assembles the current one, so the host critical path is max(staging, resolve+assemble)
        instead of their sum.

        In flight: up to N_SLOTS - 1 submitted batches wait in the hand-off queue, plus the one the
        submitter holds (blocked on put) and the one being collected, so N_SLOTS + 1 batches may be
        outstanding while only N_SLOTS device slots exist. Reusing a slot is still safe: its pinned
        staging buffer is rewritten only after the previous upload's h2d_done event, and its scratch
        arena is written only by kernels ordered on the slot's stream behind the previous batch's
        kernels. Batches dropped by an early exit are synchronised before their buffers go back to
        the caching allocator (which does not track streams)."""
        import queue
        import threading

        # submitted batches waiting for the consumer: one fewer than the device's batch slots
        depth = max(1, getattr(self.device_runner, "N_SLOTS", 2) - 1)
        q: "queue.Queue" = queue.Queue(maxsize=depth)
        stop = threading.Event()
        _END = object()

        def producer():
            try:
                tracing.name_os_thread("tb-submit")
                bind = getattr(self.device_runner, "bind_thread", None)
                if bind is not None:
                    bind()
                for g, base, item in items:
                    if stop.is_set():
                        break
                    q.put(submit_item(g, base, item))
            except BaseException as e:  # noqa: BLE001 - re-raised on the consumer thread
                q.put(("__error__", e))
            finally:
                q.put(_END)

        th = threading.Thread(target=producer, name="tb-submit", daemon=True)
        th.start()
        try:
            while True:
                x = q.get()
                if x is _END:
                    break
                if x[0] == "__error__":
                    raise x[1]
                out = self._collect_group(x, on_error, groups, sizes)
                if out is not None:
                    yield out
        finally:
            stop.set()
            drained = []
            while th.is_alive():
                try:
                    drained.append(q.get(timeout=0.05))
                except queue.Empty:
                    pass
            th.join()
            while True:
                try:
                    drained.append(q.get_nowait())
                except queue.Empty:
                    break
            if any(x is not _END for x in drained):
                # submitted but never collected: their kernels and copies may still be running on
                # buffers the caching allocator would hand out again once these objects die
                sync = getattr(self.device_runner, "synchronize", None)
                if sync is not None:
                    sync()

    # HBM scratch of the generic document kernels per device batch: at most 176 B per text byte
    # (80 for documents without the n-gram split) plus a fixed ~15 KB per document
    # (csrc/common/devplan.h scratch_bytes_for_dev); batches of many short documents are also cut
    # at that scratch budget (a 384 MB batch of 200-byte documents would need ~80 GB otherwise)
    SCRATCH_PER_BYTE = 176
    SCRATCH_PER_DOC = 176 * 64 + 4096

    def host_buffer(self, nbytes: int) -> np.ndarray:
        """A uint8 host buffer for batch text: page-locked (hiprt.pinned) on the GPU backend, so a
        producer that decodes into it lets the batch upload DMA straight from it (DeviceRunner
        skips the staging copy); plain memory otherwise."""
        if self.backend == "cuda":
            from ..ops import hiprt

            return hiprt.pinned(max(int(nbytes), 1))[: int(nbytes)]
        return np.empty(int(nbytes), dtype=np.uint8)

    def _split_by_bytes(self, item):
        data, off = item[0], item[1]
        meta = item[2] if len(item) > 2 else None
        n = len(off) - 1
        if self.backend == "cpu" or n <= 1:
            return [(0, item)]
        nbytes = int(off[-1]) - int(off[0])
        budget = self.SCRATCH_PER_BYTE * self.max_batch_bytes
        if nbytes <= self.max_batch_bytes and self.SCRATCH_PER_BYTE * nbytes + self.SCRATCH_PER_DOC * n <= budget:
            return [(0, item)]
        # cumulative scratch need of documents [0, k): 176 B x bytes + the per-document constant
        need = self.SCRATCH_PER_BYTE * (off - off[0]) + self.SCRATCH_PER_DOC * np.arange(n + 1, dtype=np.int64)
        out, a = [], 0
        while a < n:
            # largest b with off[b] - off[a] <= byte budget and scratch(a, b) <= scratch budget
            b1 = int(np.searchsorted(off, off[a] + self.max_batch_bytes, side="right")) - 1
            b2 = int(np.searchsorted(need, need[a] + budget, side="right")) - 1
            b = min(n, max(min(b1, b2), a + 1))
            out.append((a, _slice_batch(data, off, meta, a, b)))
            a = b
        return out

    def _collect_group(self, pending, on_error, groups, sizes):
        g, base, item, sub = pending
        res = self._finish_or_recover((item, sub), on_error)
        groups[g].append((base, res))
        if len(groups[g]) < sizes[g]:
            return None
        parts = groups.pop(g)
        if len(parts) == 1:
            return parts[0][1]
        return _concat_results([self._merge_deferred(r) for _, r in parts], [b for b, _ in parts])

    def _finish_or_recover(self, pending, on_error: str) -> BatchResult:
        item, sub = pending
        if not isinstance(sub, Exception):
            try:
                return self.finish(sub)
            except Exception as e:  # noqa: BLE001
                sub = e
        if on_error != "recover":
            raise sub
        return self.recover(item[0], item[1], item[2] if len(item) > 2 else None, sub)

    def recover(self, data, off, meta, err: BaseException) -> BatchResult:
        """Re-run a failed batch: halves on the same backend, then the CPU oracle path."""
        import logging

        from ..utils import metrics

        log = logging.getLogger("textblaster_amd.engine")
        n = len(off) - 1
        log.warning("batch of %d docs failed on %s (%s: %s); recovering", n, self.backend, type(err).__name__, err)
        drain = getattr(self.device_runner, "synchronize", None)
        if drain is not None:
            try:  # work queued by the failed submission finishes before its buffers are reused
                drain()
            except Exception:  # noqa: BLE001 - a sticky device error surfaces again on the retry
                pass
        metrics.BATCH_FAILURES_TOTAL.labels(type(err).__name__).inc()
        if self.backend != "cpu" and n > 1 and not _is_sticky(err):
            try:
                h = n // 2
                parts = [self.process(*_slice_batch(data, off, meta, 0, h)),
                         self.process(*_slice_batch(data, off, meta, h, n))]
                return _concat_results(parts, [0, h])
            except Exception as e2:  # noqa: BLE001
                log.warning("split retry failed too (%s: %s); using the CPU path", type(e2).__name__, e2)
        metrics.CPU_FALLBACK_DOCS_TOTAL.inc(n)
        return self._cpu_fallback().process(data, off, meta)

    def _cpu_fallback(self) -> "Engine":
        if self._cpu_engine is None:
            self._cpu_engine = Engine(self.cfg, backend="cpu", nthreads=self.nthreads, segmentation="icu",
                                      langid=self.langid, keep_reasons=self.keep_reasons,
                                      tokenizers=self.tokenizers, badwords=self.badwords)
        return self._cpu_engine

    def submit(self, data: np.ndarray, off: np.ndarray, meta: Optional[Tuple] = None, row_base: int = 0):
        with self._submit_lock, tracing.trace_range("tb.submit"):  # submitter thread and recovery may both submit
            ts = time.perf_counter()
            sub = self._submit(data, off, meta, row_base)
            sub.submit_s = time.perf_counter() - ts
            return sub

    def _submit(self, data: np.ndarray, off: np.ndarray, meta: Optional[Tuple] = None, row_base: int = 0):
        t0 = time.perf_counter()
        self._n_submitted += 1
        if self._fault is not None and not self._fault.get("fired") and self._n_submitted == self._fault["batch"]:
            self._fault["fired"] = True
            if self._fault["kind"] == "oom":
                raise MemoryError("injected device out-of-memory (TB_FAULT_INJECT)")
            raise DeviceError("injected kernel fault (TB_FAULT_INJECT)")
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        dev = None
        if self.backend in ("cuda", "emulate"):
            bw = self._bw_inputs(len(off) - 1, meta) if self._bw_steps else None
            submit = getattr(self.device_runner, "submit", None)
            dev = submit(data, off, bw) if submit is not None else self.device_runner.run(data, off, bw)
        return _Submitted(data, off, meta, row_base, dev, t0)

    def _bw_inputs(self, ndocs: int, meta) -> Dict[int, object]:
        """Per C4BadWords step: the hashed trie table and each document's list root (language =
        input metadata "language", else the step's default_language; reference
        c4_filters.rs:464-468). Lists load here, once per language."""
        from .device import BwInput

        codes, names = None, []
        if meta is not None and meta[0] is not None:
            md, mo, mv = meta
            codes, names = self.h.meta_languages(np.ascontiguousarray(md, dtype=np.uint8),
                                                 np.ascontiguousarray(mo, dtype=np.int64),
                                                 None if mv is None else np.ascontiguousarray(mv, dtype=np.uint8),
                                                 self.nthreads)
            if not (codes >= 0).any():
                codes = None
        out = {}
        with self._bw_lock:
            for i in self._bw_steps:
                langs = list(names) + [self.cfg.pipeline[i].params.default_language]
                fe, ec, et, term, roots, cjk, gen, table = self._badwords_automaton(set(langs))
                rl = np.array([roots.get(l, -1) for l in langs], dtype=np.int32)
                cl = np.array([1 if cjk.get(l, False) else 0 for l in langs], dtype=np.uint8)
                if codes is None:
                    out[i] = BwInput(gen, table, root0=int(rl[-1]), cjk0=int(cl[-1]))
                else:
                    ix = np.where(codes >= 0, codes, len(names))
                    out[i] = BwInput(gen, table, roots=rl[ix], cjk=cl[ix])
        return out

    def finish(self, sub: "_Submitted") -> BatchResult:
        with tracing.trace_range("tb.finish"):
            return self._finish(sub)

    def _finish(self, sub: "_Submitted") -> BatchResult:
        data, off, meta, row_base, t0 = sub.data, sub.off, sub.meta, sub.row_base, sub.t0
        ndocs = len(off) - 1
        md, mo, mv = meta if meta is not None else (None, None, None)
        tf = time.perf_counter()
        bs = self.h.BatchState(data, off, md, mo, mv, self.nthreads)
        timings: Dict[str, float] = {"batch_state": time.perf_counter() - tf}
        delegated = np.zeros(0, dtype=np.int64)
        resolved = None
        if sub.dev is not None:
            tw = time.perf_counter()
            res = sub.dev.wait() if hasattr(sub.dev, "wait") else sub.dev
            timings.update(res.timings)
            t1 = time.perf_counter()
            timings["wait_total"] = t1 - tw
            delegated = np.nonzero(res.flags)[0].astype(np.int64)
            if len(delegated):
                bs.delegate(delegated)
            resolved = getattr(res, "resolved", None)
            vid = {0: 0}
            if resolved is not None:
                # versions are registered (index v) only if the host assembles this batch
                vid.update({v: v for v in res.versions})
            else:
                for v in sorted(res.versions):
                    vd, vo = res.versions[v]
                    vid[v] = bs.add_version(np.ascontiguousarray(vd), np.ascontiguousarray(vo))
            dead = getattr(res, "dead", None)
            gate_checked = set()
            agreed = False
            for sp in self.plan.steps:
                st = self.steps[sp.index]
                p = res.pass_of_step.get(sp.index, 0) if dead is not None else 0
                if p > 0 and p not in gate_checked:
                    # documents the device skipped in this pass must already be filtered here;
                    # any that are still alive (a gate disagreement) go to the CPU path
                    gate_checked.add(p)
                    bad = np.nonzero((dead != 0) & (dead <= p) & (bs.fail_step() < 0))[0].astype(np.int64)
                    if len(bad):
                        _gate_mismatch(len(bad), p)
                        bs.delegate(bad)
                        delegated = np.union1d(delegated, bad).astype(np.int64)
                if sp.stage >= 0:
                    width_total, layout = self.device_runner.stage_layout[sp.stage]
                    pos = self.plan.stages[sp.stage].index(sp.index)
                    _, width, prefix = layout[pos]
                    rec = res.stage_recs[sp.stage][prefix * ndocs:(prefix + width) * ndocs]
                    bs.apply_records(st, sp.index, np.ascontiguousarray(rec), -1)
                elif sp.c4_pass >= 0:
                    bs.apply_records(st, sp.index, res.c4_recs[sp.index], vid[sp.version_out])
                else:
                    matched = (res.bw_matched or {}).get(sp.index) if sp.type == "C4BadWordsFilter" else None
                    if matched is not None and dead is not None:
                        # the device matched only documents no pass before the step filtered
                        q = self.device_runner.bw_dead_max[sp.index]
                        bad = np.nonzero((dead != 0) & (dead <= q) & (bs.fail_step() < 0))[0].astype(np.int64)
                        if len(bad):
                            _gate_mismatch(len(bad), q)
                            bs.delegate(bad)
                            delegated = np.union1d(delegated, bad).astype(np.int64)
                    if resolved is not None and sp.index in self._trailing_tc and not agreed:
                        # every filter's records are applied: the device's kept outputs must be the
                        # host's alive documents before the counter reads them
                        agreed = True
                        if not self._device_resolve_agrees(bs, resolved):
                            resolved = None
                            self._register_versions(bs, res)
                    self._host_step(bs, sp.index, ndocs, resolved, matched)
            if resolved is not None and not agreed and not self._device_resolve_agrees(bs, resolved):
                resolved = None
                self._register_versions(bs, res)
            timings["resolve"] = time.perf_counter() - t1
        else:
            t1 = time.perf_counter()
            self._run_cpu_steps(bs, 0, len(self.steps), ndocs, self.segmentation)
            timings["cpu_pipeline"] = time.perf_counter() - t1
        t2 = time.perf_counter()
        with tracing.trace_range("tb.assemble"):
            result = self._collect(bs, ndocs, timings, resolved)
        if len(delegated):
            if self._async_delegation:
                # recomputed on the delegation thread while the next batches are resolved; rows
                # are shifted by row_base below, so the merge happens after that shift too
                import concurrent.futures as cf

                if self._deleg_pool is None:
                    # two batches' CPU work side by side (each also spreads over the native pool)
                    self._deleg_pool = cf.ThreadPoolExecutor(max_workers=2, thread_name_prefix="tb-delegate",
                                                             initializer=tracing.name_os_thread,
                                                             initargs=("tb-delegate",))
                rb = row_base
                presets = self._lid_presets(res, ndocs, delegated) if sub.dev is not None else None

                def job(rows=delegated, presets=presets):
                    r2 = self._process_delegated(data, off, meta, rows, presets)
                    if rb:
                        for p in r2.kept + r2.excluded:
                            p.rows = p.rows + rb
                    return r2

                result.deferred = (self._deleg_pool.submit(job), delegated)
                result.n_delegated = len(delegated)
            else:
                sub2 = self._process_delegated(data, off, meta, delegated,
                                               self._lid_presets(res, ndocs, delegated) if sub.dev is not None else None)
                result.kept += sub2.kept
                result.excluded += sub2.excluded
                result.error_rows = np.concatenate([result.error_rows, sub2.error_rows])
                result.fail_step[delegated] = sub2.fail_step
                result.status[delegated] = sub2.status
                result.reasons.update(sub2.reasons)
                result.n_delegated = len(delegated)
        timings["assemble"] = time.perf_counter() - t2
        timings["finish"] = time.perf_counter() - tf
        timings["submit"] = sub.submit_s
        timings["total"] = time.perf_counter() - t0
        if row_base:
            for p in result.kept + result.excluded:
                p.rows = p.rows + row_base
        return result

    @staticmethod
    def _register_versions(bs, res) -> None:
        """Content versions >= 1 into the batch state (host assembly after a K16 disagreement)."""
        for v in sorted(res.versions):
            vd, vo = res.versions[v]
            if bs.add_version(np.ascontiguousarray(vd), np.ascontiguousarray(vo)) != v:
                raise Unexpected("content version registration order")

    def _run_cpu_steps(self, bs, begin: int, end: int, ndocs: int, seg: str) -> None:
        a = begin
        for i in range(begin, end):
            if self.cfg.pipeline[i].type == "TokenCounter":
                if i > a:
                    bs.run_cpu(self.steps, a, i, seg, self.lid_native, self.badwords)
                self._host_step(bs, i, ndocs)
                a = i + 1
        if end > a:
            bs.run_cpu(self.steps, a, end, seg, self.lid_native, self.badwords)

    def _host_step(self, bs, i: int, ndocs: int, resolved=None, matched=None) -> None:
        st = self.steps[i]
        t = self.cfg.pipeline[i].type
        if t == "TokenCounter":
            alive = bs.alive_indices()
            rec = np.full(ndocs, -1, dtype=np.int64)
            if len(alive) and resolved is not None and resolved.n_kept_final() == len(alive):
                # K16 agreed: final kept output k is alive[k]; its count came from k_bpe_count (or
                # -2: added-token text / a pre-token over 64 bytes -> the tokenizer, like
                # unsupported tokenizers)
                dev = resolved.kept_tokens(i)
                cnt = dev.astype(np.int64) if dev is not None else np.full(len(alive), -2, np.int64)
                bad = np.nonzero(cnt < 0)[0]
                from ..utils import metrics

                metrics.BPE_HOST_DOCS_TOTAL.inc(len(bad))
                metrics.BPE_DEVICE_DOCS_TOTAL.inc(len(cnt) - len(bad))
                if len(bad):
                    o = resolved.out_off
                    ko = np.nonzero(~resolved.moved)[0] if resolved.moved is not None else np.arange(len(alive))
                    cnt[bad] = self.tokenizers[i].count(
                        [bytes(resolved.out[o[k]:o[k + 1]]).decode("utf-8", "replace") for k in ko[bad].tolist()])
                rec[alive] = cnt
            elif len(alive):
                texts = bs.contents(alive)
                rec[alive] = self.tokenizers[i].count(texts)
            bs.apply_records(st, i, rec, -1)
        elif t == "C4BadWordsFilter":
            with self._bw_lock:
                if matched is not None:
                    bs.apply_badwords_device(st, i, self.badwords, np.ascontiguousarray(matched, dtype=np.int8))
                else:
                    bs.apply_badwords(st, i, self.badwords)
        else:
            raise Unexpected(f"{t} is not a host step")

    def _badwords_automaton(self, needed) -> Tuple:
        """Flattened tries of every loaded bad-words list and their hashed transition table
        (rebuilt when a batch needs a language whose list was loaded since). A list that cannot
        be loaded gets no root: the host step raises the same error the CPU path does."""
        a = getattr(self, "_bw_flat", None)
        if a is None or any(l not in a[4] and l not in self._bw_nolist for l in needed):
            for l in needed:
                try:
                    if not self.badwords.lookup(l)[1]:
                        self._bw_nolist.add(l)
                except RuntimeError:
                    self._bw_nolist.add(l)
            fe, ec, et, term, roots, cjk = self.badwords.flatten()
            term = np.ascontiguousarray(term, dtype=np.uint8)
            table = self.h.bw_build_table(fe, np.ascontiguousarray(ec).view(np.uint32), et, term)
            self._bw_gen = getattr(self, "_bw_gen", 0) + 1
            a = self._bw_flat = (fe, ec, et, term, roots, cjk, self._bw_gen, table)
        return a

    def _lid_presets(self, res, ndocs: int, rows: np.ndarray):
        """Device records of the language-ID steps for documents ``rows``: the record needs no
        segmentation and is exact for every script, so the CPU path of delegated documents
        applies it instead of recomputing it.

        Only steps whose stage reads the input text (content version 0) qualify: after a
        C4QualityFilter the device's rewritten text of a delegated document is not the text the
        CPU path rewrites (k_c4_pass_a stops at a dictionary script and leaves the version
        empty). A row is eligible only if no scratch overflow was flagged for it and no device
        gate skipped it in or before the language-ID pass. Returns ``(presets, eligible)``:
        ``presets[step]`` is the flat record array over ``rows`` and ``eligible`` a bool mask
        over ``rows`` (ineligible rows recompute every step on the CPU path)."""
        out = {}
        eligible = np.ones(len(rows), dtype=bool)
        if res is None or not len(rows):
            return out, eligible
        flags = getattr(res, "flags", None)
        if flags is not None:
            eligible &= (np.asarray(flags)[rows] & DOC_OVERFLOW) == 0
        dead = getattr(res, "dead", None)
        for sp in self.plan.steps:
            if sp.stage < 0 or self.cfg.pipeline[sp.index].type != "LanguageDetectionFilter":
                continue
            if self.plan.stage_version[sp.stage] != 0:
                continue
            _, layout = self.device_runner.stage_layout[sp.stage]
            pos = self.plan.stages[sp.stage].index(sp.index)
            _, width, prefix = layout[pos]
            rec = np.asarray(res.stage_recs[sp.stage][prefix * ndocs:(prefix + width) * ndocs])
            out[sp.index] = np.ascontiguousarray(rec.reshape(ndocs, width)[rows]).reshape(-1)
            if dead is not None:
                p = res.pass_of_step.get(sp.index, 0)
                d = np.asarray(dead)[rows]
                eligible &= ~((d != 0) & (d <= p))
        return out, eligible

    def _process_delegated(self, data, off, meta, rows: np.ndarray, presets=None) -> BatchResult:
        """CPU path of delegated documents ``rows``; ``presets`` = ``_lid_presets`` output.
        Rows whose device language-ID record is not usable run every step on the CPU."""
        if presets is None or not presets[0]:
            return self._process_subset_cpu(data, off, meta, rows)
        recs, eligible = presets
        if eligible.all():
            return self._process_subset_cpu(data, off, meta, rows, recs)
        parts = []
        ok = np.nonzero(eligible)[0]
        bad = np.nonzero(~eligible)[0]
        if len(ok):
            sub_recs = {}
            for i, rec in recs.items():
                w = len(rec) // len(rows)
                sub_recs[i] = np.ascontiguousarray(rec.reshape(len(rows), w)[ok]).reshape(-1)
            parts.append((ok, self._process_subset_cpu(data, off, meta, rows[ok], sub_recs)))
        parts.append((bad, self._process_subset_cpu(data, off, meta, rows[bad])))
        fail = np.zeros(len(rows), dtype=parts[0][1].fail_step.dtype)
        status = np.zeros(len(rows), dtype=parts[0][1].status.dtype)
        out = BatchResult(len(rows), [], [], np.zeros(0, dtype=np.int64), fail, status, {}, {})
        errs = []
        for pos, r in parts:
            out.kept += r.kept
            out.excluded += r.excluded
            errs.append(r.error_rows)
            fail[pos] = r.fail_step
            status[pos] = r.status
            out.reasons.update(r.reasons)
        out.error_rows = np.concatenate(errs)
        return out

    def _process_subset_cpu(self, data, off, meta, rows: np.ndarray, presets=None) -> BatchResult:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        # (native gathers: one memcpy per document, no Python loop over the rows)
        sub_data, sub_off = self.h.gather_spans(np.ascontiguousarray(data, dtype=np.uint8),
                                                np.ascontiguousarray(off, dtype=np.int64), rows, self.nthreads)
        sub_data = np.asarray(sub_data)[:int(sub_off[-1])]
        sub_meta = None
        if meta is not None and meta[0] is not None:
            md, mo, mv = meta
            smd, smo = self.h.gather_spans(np.ascontiguousarray(md, dtype=np.uint8),
                                           np.ascontiguousarray(mo, dtype=np.int64), rows, self.nthreads)
            smd = np.asarray(smd)[:int(smo[-1])]
            smv = mv[rows] if mv is not None else None
            sub_meta = (np.ascontiguousarray(smd, dtype=np.uint8), smo, smv)
        md2, mo2, mv2 = sub_meta if sub_meta else (None, None, None)
        bs = self.h.BatchState(np.ascontiguousarray(sub_data, dtype=np.uint8), sub_off, md2, mo2, mv2, self.nthreads)
        a = 0
        for i in sorted(presets or {}):
            # a device-exact record (language ID): applied, the steps before it run on the CPU
            if i > a:
                self._run_cpu_steps(bs, a, i, len(rows), "icu")
            bs.apply_records(self.steps[i], i, presets[i], -1)
            a = i + 1
        self._run_cpu_steps(bs, a, len(self.steps), len(rows), "icu")
        res = self._collect(bs, len(rows), {})
        for p in res.kept + res.excluded:
            p.rows = rows[p.rows]
        res.error_rows = rows[res.error_rows]
        res.reasons = {int(rows[k]): v for k, v in res.reasons.items()}
        return res

    def _device_resolve_agrees(self, bs, resolved) -> bool:
        """The host re-derived every decision from the device records (apply_records); the
        device-compacted outputs are used only when both agree on every document's first failing
        step and status, and the compaction did not run out of room. Otherwise the batch is
        assembled on the host (counted in tb_device_resolve_fallback_total).

        The one allowed difference: a C4BadWords step (resolved on the device as passing every
        document) filtered a document the device kept or filtered at a later step; its output is
        the same text (no rewrite follows the step, resolve_entries), so kept ones move to the
        excluded side (``resolved.moved``) and the others keep their place."""
        hf, hs = bs.fail_step(), bs.status()
        ok = resolved.err == 0
        if ok:
            diff = np.nonzero((hf != resolved.fail) | (hs != resolved.status))[0]
            if len(diff):
                df, ds = resolved.fail[diff], resolved.status[diff]
                ok = bool(len(self._bw_steps)) and bool(np.all(
                    np.isin(hf[diff], self._bw_steps) & (hs[diff] == 1) & (ds <= 1) & ((df < 0) | (df > hf[diff]))))
                if ok:
                    nk, _ = resolved.counts()
                    moved_docs = diff[ds == 0]
                    resolved.moved = np.isin(resolved.rows[:nk], moved_docs) if len(moved_docs) else None
        if ok and resolved.ver is not None:
            # the content version the device compacted each output from must be the host's too
            out = resolved.status <= 1
            ok = bool(np.array_equal(resolved.ver[out].astype(np.int32), bs.cur_version()[out]))
        if not ok:
            import logging

            from ..utils import metrics

            resolved.moved = None
            logging.getLogger("textblaster_amd.engine").warning(
                "device resolve disagrees with the host decisions (or overflowed); assembling this batch on the host")
            metrics.DEVICE_RESOLVE_FALLBACK_TOTAL.inc()
        return ok

    def _collect(self, bs, ndocs: int, timings, resolved=None) -> BatchResult:
        status = bs.status()
        fail = bs.fail_step()
        kept_rows = np.nonzero(status == 0)[0].astype(np.int64)
        excl_rows = np.nonzero(status == 1)[0].astype(np.int64)
        err_rows = np.nonzero(status == 2)[0].astype(np.int64)
        if resolved is not None:
            # K16: texts were compacted on the device (kept, then excluded, document order — the
            # rows above; documents a host step filtered afterwards in a second excluded part);
            # only the metadata columns are built here
            sides = []
            for side in resolved.parts(self.nthreads):
                out = []
                for rows, off, text in side:
                    _, _, md, mo, mv = bs.assemble(rows, False)
                    out.append(OutputPart(rows, text, off, md, mo, mv))
                sides.append(out)
            kept_parts, excl_parts = sides
        else:
            kept_parts, excl_parts = [], []
            for rows, dst in ((kept_rows, kept_parts), (excl_rows, excl_parts)):
                td, to, md, mo, mv = bs.assemble(rows)
                dst.append(OutputPart(rows, td, to, md, mo, mv))
        reasons = {}
        if self.keep_reasons and len(excl_rows):
            reasons = dict(zip(excl_rows.tolist(), bs.reasons(excl_rows)))
        return BatchResult(ndocs, kept_parts, excl_parts, err_rows, fail, status, reasons, timings)

    def step_names(self) -> List[str]:
        return [s.type for s in self.cfg.pipeline]


def _parse_fault(spec: str):
    """``kind@batch`` (kind: kernel | oom, batch: 1-based submit counter), e.g. ``kernel@3``."""
    if not spec:
        return None
    kind, _, at = spec.partition("@")
    if kind not in ("kernel", "oom") or not at.isdigit():
        raise ConfigError(f"bad fault injection spec {spec!r} (expected kernel@N or oom@N)")
    return {"kind": kind, "batch": int(at), "fired": False}


def _is_sticky(err: BaseException) -> bool:
    """A GPU memory access fault poisons the HIP context; retrying on the device is pointless."""
    msg = str(err).lower()
    return "illegal" in msg or "memory access fault" in msg or "hiperrorlaunchfailure" in msg


def _slice_batch(data, off, meta, a: int, b: int):
    o = off[a:b + 1]
    d = data[o[0]:o[-1]]
    o = o - o[0]
    m = None
    if meta is not None and meta[0] is not None:
        md, mo, mv = meta
        mo2 = mo[a:b + 1]
        m = (md[mo2[0]:mo2[-1]], mo2 - mo2[0], mv[a:b] if mv is not None else None)
    return np.ascontiguousarray(d), np.ascontiguousarray(o), m


def _concat_results(parts: List[BatchResult], bases: List[int]) -> BatchResult:
    kept, excluded, errs, reasons = [], [], [], {}
    for r, base in zip(parts, bases):
        for p in r.kept:
            p.rows = p.rows + base
            kept.append(p)
        for p in r.excluded:
            p.rows = p.rows + base
            excluded.append(p)
        errs.append(r.error_rows + base)
        reasons.update({k + base: v for k, v in r.reasons.items()})
    timings: Dict[str, float] = {}
    for r in parts:
        for k, v in r.timings.items():
            timings[k] = timings.get(k, 0.0) + v
    return BatchResult(sum(r.n_docs for r in parts), kept, excluded, np.concatenate(errs),
                       np.concatenate([r.fail_step for r in parts]), np.concatenate([r.status for r in parts]),
                       reasons, timings, sum(r.n_delegated for r in parts))


@dataclasses.dataclass
class _Submitted:
    data: np.ndarray
    off: np.ndarray
    meta: Optional[Tuple]
    row_base: int
    dev: object          # PendingBatch / DeviceResult / None (cpu)
    t0: float
    submit_s: float = 0.0


def _cuda_available() -> bool:
    """A HIP device is visible (asked through the native runtime layer, no PyTorch import)."""
    try:
        from ..ops import hiprt

        return hiprt.device_count() > 0
    except Exception:
        return False
