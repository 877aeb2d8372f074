"""End-to-end Parquet -> pipeline -> Parquet run: the in-process replacement of the reference's
producer + worker pair (reference producer_logic.rs:23-230, worker_logic.rs:136-283,
bin/producer.rs, bin/worker.rs).

Work decomposition
  The input is cut into *units*: row-group slices of at most ``unit_rows`` rows. Units are the
  output and checkpoint granularity; the units of one row group form a *group*, the scheduling
  granularity (a row group is decoded once, by one rank). Ranks pull groups from a shared atomic
  cursor (``DistContext.claim``: ``store.add`` on the process group's store), the
  competing-consumer equivalent of the reference's work queue (worker_logic.rs:241-283,
  utils/common.rs:91-94 ``basic_qos``): a rank whose documents cost more per byte (very long
  documents run at a fraction of the short-document rate on the GPU) or whose GPU is busier
  takes fewer groups, so the ranks finish together. ``run --schedule static`` restores contiguous
  ranges balanced by bytes (``parallel.dist.shard_ranges``). Documents never cross GPUs.

Per rank, four stages overlap (bounded queues, the heavy native calls release the GIL):
  reader thread   Parquet decode + HTML-entity decode + packing    (unit k+2)
  GPU stream      H2D, HIP kernels, D2H (Engine.process_many)      (unit k+1)
  main thread     resolve + output assembly                        (unit k)
  writer thread   Arrow assembly + Parquet encode                  (unit k-1)

Outputs
  * single rank, no checkpointing: rows stream straight into ``output_file`` / ``excluded_file``;
  * otherwise every unit writes ``<work_dir>/parts/u<unit>.{kept,excluded}.parquet`` and appends a
    line to ``<work_dir>/manifest.rank<r>.jsonl`` once both files are closed. ``resume=True``
    skips units already in a manifest. At the end the parts are concatenated in unit order
    (row order = input order) into the two final files *without re-encoding*: rank r copies the
    parts of a contiguous unit range (whoever processed them) at an offset from an all-gather
    of sizes (AG1), rank 0 writes the rewritten footers (io/pqconcat.py); the work dir is
    removed unless ``keep_parts``.
  Counters (docs, kept, excluded, errors, per-step filtered) are all-reduced while the job
  runs by a heartbeat thread (parallel/heartbeat.py; it also turns a dead peer into a
  non-zero exit) and once more over RCCL at the end (AR1); rank 0 serves the global view on
  the metrics endpoint.
"""
from __future__ import annotations

import collections
import dataclasses
import hashlib
import json
import logging
import os
import queue
import resource
import shutil
import threading
import time
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from .config.pipeline import PipelineConfig, load_pipeline_config
from .errors import PipelineError, Unexpected
from .io.parquet import (DocBatch, ParquetInputConfig, ParquetReader, ParquetWriter, build_output_table,
                         encode_table, packed_to_string_array)
from .parallel.dist import DistContext, shard_ranges
from .parallel.heartbeat import Heartbeat
from .utils import metrics, tracing

log = logging.getLogger("textblaster_amd.runner")


@dataclasses.dataclass
class RunConfig:
    input_file: str
    output_file: str = "output_processed.parquet"
    excluded_file: str = "excluded.parquet"
    pipeline_config: str = "config/pipeline_config.yaml"
    text_column: str = "text"
    id_column: str = "id"
    backend: str = "auto"              # auto | cuda | cpu
    segmentation: str = "icu"          # CPU backend segmentation: icu (oracle) | rules
    unit_rows: int = 65536
    threads: Optional[int] = None
    work_dir: Optional[str] = None     # checkpoint dir (default: <output_file>.work when needed)
    resume: bool = False
    checkpoint: bool = False           # force the part-file path on a single rank
    keep_parts: bool = False
    compression: str = "none"
    tokenizer_dir: Optional[str] = None
    badwords_dir: Optional[str] = None
    html_decode: str = "cpu"           # input HTML entity decoding: cpu (C++ host) | gpu (K17 kernels)
    metrics_port: Optional[int] = None
    progress_interval: float = 1.0
    tokenizer_file: Optional[str] = None
    # row groups decoded / units encoded concurrently; None: the rank's thread budget when it is pinned to a CPU set (parallel/placement.py), else 8 / 4
    read_threads: Optional[int] = None
    write_threads: Optional[int] = None
    claim_ahead: Optional[int] = None    # groups a rank may hold ahead of its main loop (default readers + 3)
    batch_bytes: Optional[int] = None    # device batch bytes (default 384 MB; TB_TUNE batch_bytes)
    slots: Optional[int] = None          # device batches in flight (default: auto, 3 when HBM allows; TB_TUNE slots)
    fault_inject: Optional[str] = None   # debug: "kernel@N" / "oom@N" (N = 1-based batch), "rank@N[:R]",
                                         # "slow@SECONDS[:R]" (rank R sleeps after every unit)
    schedule: str = "dynamic"            # dynamic (shared cursor) | static (byte-balanced ranges)


@dataclasses.dataclass
class RunStats:
    docs: int = 0
    kept: int = 0
    excluded: int = 0
    errors: int = 0
    bytes_in: int = 0
    seconds: float = 0.0
    units: int = 0
    units_skipped: int = 0
    delegated: int = 0
    step_filtered: List[int] = dataclasses.field(default_factory=list)
    phase_seconds: Dict[str, float] = dataclasses.field(default_factory=dict)  # rank 0's own view
    rank_units: List[int] = dataclasses.field(default_factory=list)  # units processed per rank
    rank_busy: List[float] = dataclasses.field(default_factory=list)  # main-loop seconds per rank
    # per rank: [CPUs, pool threads, reader threads, writer threads, first CPU, last CPU] (CPUs 0:
    # not pinned, first / last -1)
    rank_cpus: List[List[int]] = dataclasses.field(default_factory=list)

    @property
    def docs_per_sec(self) -> float:
        return self.docs / self.seconds if self.seconds > 0 else 0.0

    def vector(self, nsteps: int) -> np.ndarray:
        sf = list(self.step_filtered) + [0] * (nsteps - len(self.step_filtered))
        return np.asarray([self.docs, self.kept, self.excluded, self.errors, self.bytes_in, self.delegated] + sf,
                          dtype=np.int64)

    @classmethod
    def from_vector(cls, v: np.ndarray, seconds: float, units: int, skipped: int) -> "RunStats":
        v = [int(x) for x in v]
        return cls(v[0], v[1], v[2], v[3], v[4], seconds, units, skipped, v[5], v[6:])


# ---------------------------------------------------------------------------------------------
# units

@dataclasses.dataclass(frozen=True)
class Unit:
    index: int
    row_group: int
    start: int
    stop: int
    est_bytes: float


def plan_units(reader: ParquetReader, unit_rows: int) -> List[Unit]:
    units = []
    for rg, (n, b) in enumerate(zip(reader.row_group_rows(), reader.row_group_bytes())):
        for s in range(0, n, unit_rows):
            e = min(n, s + unit_rows)
            units.append(Unit(len(units), rg, s, e, b * (e - s) / max(n, 1)))
    return units


def _fingerprint(path: str, unit_rows: int, pipeline_path: str) -> str:
    st = os.stat(path)
    h = hashlib.sha256()
    h.update(f"{os.path.abspath(path)}|{st.st_size}|{int(st.st_mtime)}|{unit_rows}".encode())
    with open(pipeline_path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


class _UnitReader:
    """Reads units in order, caching the last decoded row group (consecutive units usually share
    it)."""

    def __init__(self, reader: ParquetReader, own_file: bool = False):
        self.reader = reader
        self._rg = -1
        self._tbl = None
        self.seconds = 0.0
        self.cpu = 0.0  # CPU seconds of the threads that read through this object
        self.lock = threading.Lock()
        # worker threads open their own ParquetFile (a reader object is not shared across threads)
        self._pf = pq.ParquetFile(reader.config.path, memory_map=True) if own_file else None
        # several reader threads decode row groups side by side: Arrow's own column threads on
        # top of that only add contention (measured slower)
        self._use_threads = not own_file

    def read(self, u: Unit) -> DocBatch:
        t0, c0 = time.perf_counter(), time.thread_time()
        try:
            with tracing.trace_range("tb.read"):
                return self._read(u)
        finally:
            self.seconds += time.perf_counter() - t0
            self.cpu += time.thread_time() - c0

    def _read(self, u: Unit) -> DocBatch:
        if u.row_group != self._rg:
            pf = self._pf if self._pf is not None else self.reader._pf
            with tracing.trace_range("tb.read_row_group"):
                self._tbl = self.reader.read_row_group(u.row_group, pf, self._use_threads)
            self._rg = u.row_group
        t = self._tbl.slice(u.start, u.stop - u.start).combine_chunks()
        batches = t.to_batches()
        rb = batches[0] if batches else pa.RecordBatch.from_pylist([], schema=t.schema)
        with tracing.trace_range("tb.to_docbatch"):
            return self.reader._to_docbatch(rb)


# ---------------------------------------------------------------------------------------------
# output assembly

def part_table(batch: DocBatch, part) -> pa.Table:
    rows = pa.array(part.rows, type=pa.int64())
    text = packed_to_string_array(part.text_data, part.text_off)
    meta = packed_to_string_array(part.meta_data, part.meta_off, part.meta_valid)
    return build_output_table(batch.ids.take(rows).cast(pa.string()), batch.source.take(rows),
                              text, batch.added.take(rows), batch.created.take(rows), meta)


class _Sink:
    """Receives every unit's two encoded Parquet files (kept, excluded) in unit order."""

    def commit(self, unit: Unit, kept: Tuple[pa.Buffer, int], excluded: Tuple[pa.Buffer, int], counts: Dict) -> None:
        raise NotImplementedError

    def close(self) -> None:
        pass


class _DirectSink(_Sink):
    """Single rank without checkpoints: row groups are appended straight to the two outputs."""

    def __init__(self, rc: RunConfig):
        from .io.pqconcat import StreamConcat

        self.rc = rc
        self.outs = []
        for path in (rc.output_file, rc.excluded_file):
            parent = os.path.dirname(os.path.abspath(path))
            os.makedirs(parent, exist_ok=True)
            self.outs.append(StreamConcat(path))

    def commit(self, unit, kept, excluded, counts):
        for out, (buf, rows) in zip(self.outs, (kept, excluded)):
            if rows:
                out.append(buf)

    def close(self):
        for out in self.outs:
            if not out.close():        # nothing appended: a valid empty file with the schema
                ParquetWriter(out.path, self.rc.compression).close()


class _PartSink(_Sink):
    def __init__(self, rc: RunConfig, work_dir: str, rank: int):
        self.rc = rc
        self.parts = os.path.join(work_dir, "parts")
        os.makedirs(self.parts, exist_ok=True)
        self.manifest = open(os.path.join(work_dir, f"manifest.rank{rank}.jsonl"), "a", encoding="utf-8")

    def commit(self, unit, kept, excluded, counts):
        for kind, (buf, _) in (("kept", kept), ("excluded", excluded)):
            final = os.path.join(self.parts, f"u{unit.index:07d}.{kind}.parquet")
            tmp = final + ".tmp"
            with open(tmp, "wb") as f:
                f.write(memoryview(buf))
            os.replace(tmp, final)
        self.manifest.write(json.dumps(dict(unit=unit.index, **counts)) + "\n")
        self.manifest.flush()
        os.fsync(self.manifest.fileno())

    def close(self):
        self.manifest.close()


def read_manifests(work_dir: str) -> Dict[int, Dict]:
    done = {}
    if not os.path.isdir(work_dir):
        return done
    for name in sorted(os.listdir(work_dir)):
        if name.startswith("manifest.rank") and name.endswith(".jsonl"):
            with open(os.path.join(work_dir, name), encoding="utf-8") as f:
                for line in f:
                    line = line.strip()
                    if not line:
                        continue
                    try:
                        rec = json.loads(line)
                    except json.JSONDecodeError:
                        continue  # a torn last line from a crash: the unit is redone
                    done[int(rec["unit"])] = rec
    return done


def merge_parts(work_dir: str, my_units: List[int], rc: RunConfig, ctx: Optional[DistContext] = None) -> None:
    """Concatenates the part files into the two final files without re-encoding them
    (io/pqconcat.py). Every rank copies the parts of its own (contiguous) unit range at an
    offset from an all-gather of body sizes (AG1); rank 0 then writes the footers. Row order
    is unit order = input order."""
    from .io import pqconcat

    ctx = ctx or DistContext()
    rank, world = ctx.rank, ctx.world_size
    parts = os.path.join(work_dir, "parts")
    outs = (("kept", rc.output_file), ("excluded", rc.excluded_file))
    lays = []
    for kind, _ in outs:
        paths = [os.path.join(parts, f"u{u:07d}.{kind}.parquet") for u in my_units]
        for p in paths:
            if not os.path.exists(p):
                raise Unexpected(f"missing part file {p}; rerun with --resume")
        lays.append(pqconcat.part_layout(paths))
    sizes = ctx.all_gather_counts([lay.body_bytes for lay in lays])          # AG1: [world, 2]
    if rank == 0:
        for _, path in outs:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            os.close(os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644))
    ctx.barrier()
    for k, ((kind, path), lay) in enumerate(zip(outs, lays)):
        base = 4 + int(sizes[:rank, k].sum())
        fd = os.open(path, os.O_WRONLY)
        try:
            pqconcat.write_bodies(fd, lay, base)
        finally:
            os.close(fd)
        for rg in lay.row_groups:
            pqconcat.shift_row_group(rg, base)
        rec = [[1, pqconcat.T_LIST, (pqconcat.T_STRUCT, lay.row_groups)],
               [2, pqconcat.T_I64, lay.num_rows],
               [3, pqconcat.T_BINARY, pqconcat.encode_struct(lay.template) if lay.template else b""]]
        with open(os.path.join(work_dir, f"footer.{kind}.rank{rank}.bin"), "wb") as f:
            f.write(pqconcat.encode_struct(rec))
    ctx.barrier()
    if rank == 0:
        for k, (kind, path) in enumerate(outs):
            rgs, rows, template, schema = [], 0, None, None
            for r in range(world):
                with open(os.path.join(work_dir, f"footer.{kind}.rank{r}.bin"), "rb") as f:
                    rec = pqconcat.decode_struct(f.read())
                fields = {fid: v for fid, _, v in rec}
                rgs += fields[1][1]
                rows += fields[2]
                if fields[3]:
                    t = pqconcat.decode_struct(fields[3])
                    sch = pqconcat.encode_struct([x for x in t if x[0] == pqconcat.FMD_SCHEMA])
                    if template is None:
                        template, schema = t, sch
                    elif sch != schema:
                        raise Unexpected(f"rank {r} wrote {kind} parts with a different schema")
            fd = os.open(path, os.O_WRONLY)
            try:
                if template is None:       # no unit anywhere: a valid empty file
                    os.close(fd)
                    fd = -1
                    ParquetWriter(path, rc.compression).close()
                else:
                    pqconcat.finish(fd, 4 + int(sizes[:, k].sum()), template, rgs, rows)
            finally:
                if fd >= 0:
                    os.close(fd)
    ctx.barrier()


# ---------------------------------------------------------------------------------------------

class _Prefetcher:
    """Drives ``gen`` on its own thread, keeping up to ``depth`` items ready. Started before the
    engine is built, so Parquet decoding overlaps HIP context creation and kernel loading
    instead of following them. ``close`` stops the thread (also when nothing was consumed)."""

    def __init__(self, gen: Iterator, depth: int):
        self.q: queue.Queue = queue.Queue(maxsize=max(1, depth))
        self.err: List[BaseException] = []
        self.stop = threading.Event()
        self._end = object()
        self._gen = gen
        self.t = threading.Thread(target=lambda: (tracing.name_os_thread("tb-prefetch"), self._work()),
                                  name="tb-prefetch", daemon=True)
        self.t.start()

    def _put(self, item) -> bool:
        while not self.stop.is_set():
            try:
                self.q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _work(self):
        try:
            for item in self._gen:
                if not self._put(item):
                    break
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            self.err.append(e)
        finally:
            self._put(self._end)
            close = getattr(self._gen, "close", None)
            if close is not None and self.stop.is_set():
                close()

    def __iter__(self):
        while True:
            item = self.q.get()
            if item is self._end:
                break
            yield item
        if self.err:
            raise self.err[0]

    def close(self):
        self.stop.set()
        self.t.join(timeout=60)


def unit_groups(units: List[Unit]) -> List[List[Unit]]:
    """Consecutive units of one row group (the scheduling granularity)."""
    groups: List[List[Unit]] = []
    for u in units:
        if groups and groups[-1][0].row_group == u.row_group:
            groups[-1].append(u)
        else:
            groups.append([u])
    return groups


class _ClaimGate:
    """Bounds the groups a rank holds (claimed, not yet handed to the engine) to ``ahead``: the
    reader thread takes a token before each claim, the main loop returns it when it passes a
    group's last unit to the engine (whose own in-flight depth is a few batches).
    Without it the reader's prefetch would claim groups a busy rank cannot start for a while
    (the reference's ``basic_qos(prefetch_count)``, utils/common.rs:91-94)."""

    def __init__(self, ahead: int):
        self.ahead = max(1, ahead)
        self.sem = threading.Semaphore(self.ahead)
        self.last: set = set()
        self.closed = False

    def done(self, unit_index: int) -> None:
        if unit_index in self.last:
            self.last.discard(unit_index)
            self.sem.release()


def _claimed(ctx: DistContext, key: str, groups: List[List[Unit]], claimed: List[int],
             gate: _ClaimGate) -> Iterator[List[Unit]]:
    """The groups this rank takes from the shared cursor ``key``, one claim each, lazily: a claim
    is made only when the rank holds fewer than ``gate``'s bound of unprocessed groups."""
    while True:
        while not gate.sem.acquire(timeout=0.1):
            if gate.closed:
                return
        i = ctx.claim(key, 1)
        if i >= len(groups):
            return
        claimed.append(i)
        gate.last.add(groups[i][-1].index)
        yield groups[i]


def _read_units(reader: ParquetReader, groups, nthreads: int, timer: _UnitReader, window: Optional[int] = None):
    """Yields (unit, DocBatch) of the row-group ``groups`` (an iterable, consumed lazily) in
    order. Row groups are decoded by up to ``nthreads`` worker threads at once (Parquet
    decompression + HTML-entity decoding dominate the input side); each row group is read once
    and sliced into its units.

    At most ``window`` groups (default ``nthreads + 1``) are taken from ``groups`` and not yet
    yielded. ``groups`` may block on a claim gate whose tokens come back only after yielded
    groups reach the main loop; so the next group is taken only after the previous one was
    yielded, and a gate bound of ``window`` or more can never starve the reader."""
    import concurrent.futures as cf

    def load(group: List[Unit]):
        r = _UnitReader(reader, own_file=nthreads > 1)
        out = [(u, r.read(u)) for u in group]
        with timer.lock:
            timer.seconds += r.seconds
            timer.cpu += r.cpu
        return out

    if nthreads <= 1:
        for g in groups:
            yield from load(g)
        return
    window = max(1, min(nthreads + 1, window or nthreads + 1))
    with cf.ThreadPoolExecutor(max_workers=nthreads, thread_name_prefix="tb-reader",
                               initializer=tracing.name_os_thread, initargs=("tb-reader",)) as ex:
        pending: collections.deque = collections.deque()
        it = iter(groups)
        exhausted = False
        while True:
            while not exhausted and len(pending) < window:
                g = next(it, None)
                if g is None:
                    exhausted = True
                    break
                pending.append(ex.submit(load, g))
            if not pending:
                return
            yield from pending.popleft().result()


class _Writer:
    """Output side of the run. A pool of encoder threads turns each unit's kept / excluded rows
    into two in-memory Parquet files concurrently (Arrow assembly and Parquet encoding release
    the GIL); one committer thread hands them to the sink in unit order (appending row groups
    to the final files, or writing checkpoint parts). ``submit`` blocks when ``depth`` units
    are pending. reference parquet_writer.rs:69-164 writes one row group per batch on the
    producer thread."""

    def __init__(self, sink: _Sink, compression: str = "none", threads: int = 4, depth: Optional[int] = None):
        import concurrent.futures as cf

        self.sink = sink
        self.compression = compression
        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, threads), thread_name_prefix="tb-encode",
                                          initializer=tracing.name_os_thread, initargs=("tb-encode",))
        self.q: queue.Queue = queue.Queue(maxsize=depth or max(1, threads) + 2)
        self.err: List[BaseException] = []
        self.seconds = 0.0
        self.cpu_encode = 0.0  # CPU seconds of the encoder threads / the committer thread
        self.cpu_write = 0.0
        self._lock = threading.Lock()
        self.t = threading.Thread(target=lambda: (tracing.name_os_thread("tb-writer"), self._run()), name="tb-writer",
                                  daemon=True)
        self.t.start()

    def _encode(self, job):
        t0, c0 = time.perf_counter(), time.thread_time()
        batch, res, unit, counts = job
        with tracing.trace_range("tb.part_table"):
            kept, exc = self._tables(batch, res)
        with tracing.trace_range("tb.encode"):
            out = (unit, (encode_table(kept, self.compression), kept.num_rows),
                   (encode_table(exc, self.compression), exc.num_rows), counts)
        with self._lock:
            self.seconds += time.perf_counter() - t0
            self.cpu_encode += time.thread_time() - c0
        return out

    def _run(self):
        while True:
            fut = self.q.get()
            if fut is None:
                return
            try:
                unit, kept, exc, counts = fut.result()
                if self.err:
                    continue
                t0, c0 = time.perf_counter(), time.thread_time()
                with tracing.trace_range("tb.write"):
                    self.sink.commit(unit, kept, exc, counts)
                with self._lock:
                    self.seconds += time.perf_counter() - t0
                    self.cpu_write += time.thread_time() - c0
            except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
                self.err.append(e)

    @staticmethod
    def _tables(batch, res):
        kept = part_table(batch, res.kept[0]) if len(res.kept) == 1 else pa.concat_tables(
            [part_table(batch, p) for p in res.kept])
        exc = part_table(batch, res.excluded[0]) if len(res.excluded) == 1 else pa.concat_tables(
            [part_table(batch, p) for p in res.excluded])
        if len(res.kept) > 1:
            kept = _sort_by_row(kept, np.concatenate([p.rows for p in res.kept]))
        if len(res.excluded) > 1:
            exc = _sort_by_row(exc, np.concatenate([p.rows for p in res.excluded]))
        return kept, exc

    def submit(self, job):
        if self.err:
            raise self.err[0]
        self.q.put(self.pool.submit(self._encode, job))

    def close(self):
        self.q.put(None)
        self.t.join()
        self.pool.shutdown(wait=True)
        if not self.err:
            self.sink.close()
        else:
            try:
                self.sink.close()
            except BaseException:  # noqa: BLE001 - the first error wins
                pass
        if self.err:
            raise self.err[0]


def _sort_by_row(tbl: pa.Table, rows: np.ndarray) -> pa.Table:
    order = np.argsort(rows, kind="stable")
    return tbl.take(pa.array(order))


def resolve_threads(rc: RunConfig):
    """(pool, readers, writers) of this rank: explicit settings first (RunConfig / the CLI, and
    TB_THREADS for the pool), then the thread budget of the CPU set
    the rank is pinned to (placement.thread_budget: all three within its CPUs), else the
    one-rank defaults (pool = the process's CPU share, 8 readers, 4 writers)."""
    from .parallel import placement
    from .pipeline.engine import default_threads

    cpus = placement.bound_cpus()
    bud = placement.thread_budget(len(cpus)) if cpus is not None else None

    def pick(v, env, dflt):
        if v is not None:
            return int(v)
        e = os.environ.get(env) if env else None
        if e and e.isdigit() and int(e) > 0:
            return int(e)
        return dflt

    pool = pick(rc.threads, "TB_THREADS", bud.pool if bud else default_threads())
    read = pick(rc.read_threads, None, bud.read if bud else 8)
    write = pick(rc.write_threads, None, bud.write if bud else 4)
    return pool, read, write


def run(rc: RunConfig, ctx: Optional[DistContext] = None, cfg: Optional[PipelineConfig] = None,
        engine=None) -> RunStats:
    """Process ``rc.input_file`` end to end; returns the global (all-rank) statistics."""
    from .parallel import placement
    from .pipeline.engine import Engine

    ctx = ctx or DistContext()
    n_pool, n_read, n_write = resolve_threads(rc)
    rc = dataclasses.replace(rc, threads=n_pool, read_threads=n_read, write_threads=n_write)
    rank, world = ctx.rank, ctx.world_size
    cfg = cfg or load_pipeline_config(rc.pipeline_config)
    nsteps = len(cfg.pipeline)
    t_start = time.perf_counter()
    ru_start = resource.getrusage(resource.RUSAGE_SELF)
    rank_fault = _parse_rank_fault(rc.fault_inject, world)
    slow = _parse_slow(rc.fault_inject, world)
    html_dec = None
    if rc.html_decode == "gpu":
        dev = ctx.device if ctx.device is not None else ("cuda" if rc.backend == "cuda" else None)
        if dev is None:
            raise PipelineError("--html-decode gpu needs a GPU rank")
        from .ops.html import HtmlDecoder

        html_dec = HtmlDecoder(dev)
    elif rc.html_decode != "cpu":
        raise PipelineError(f"unknown html decode backend {rc.html_decode!r} (cpu | gpu)")
    reader = ParquetReader(ParquetInputConfig(rc.input_file, rc.text_column, rc.id_column), html_decoder=html_dec)
    units = plan_units(reader, rc.unit_rows)
    use_parts = world > 1 or rc.checkpoint or rc.resume
    work_dir = rc.work_dir or (rc.output_file + ".work")
    done: Dict[int, Dict] = {}
    if use_parts:
        if rank == 0:
            os.makedirs(work_dir, exist_ok=True)
            fp = _fingerprint(rc.input_file, rc.unit_rows, rc.pipeline_config) if os.path.exists(
                rc.pipeline_config) else None
            plan_path = os.path.join(work_dir, "plan.json")
            if rc.resume and os.path.exists(plan_path):
                with open(plan_path, encoding="utf-8") as f:
                    old = json.load(f)
                if old.get("fingerprint") != fp or old.get("n_units") != len(units):
                    raise Unexpected(f"--resume: {work_dir} was written for a different input/config "
                                     f"(fingerprint {old.get('fingerprint')} != {fp}); remove it to start over")
            elif not rc.resume:
                for name in os.listdir(work_dir):
                    if name.startswith("manifest.rank"):
                        os.remove(os.path.join(work_dir, name))
                shutil.rmtree(os.path.join(work_dir, "parts"), ignore_errors=True)
            with open(plan_path, "w", encoding="utf-8") as f:
                json.dump({"fingerprint": fp, "n_units": len(units), "unit_rows": rc.unit_rows,
                           "input": os.path.abspath(rc.input_file)}, f)
        ctx.barrier()
        if rc.resume:
            done = read_manifests(work_dir)
    if rc.schedule not in ("dynamic", "static"):
        raise PipelineError(f"unknown schedule {rc.schedule!r} (dynamic | static)")
    # merge ranges: contiguous by unit index, balanced by bytes (whoever processed the units)
    shard = shard_ranges([u.est_bytes for u in units], world)[rank]
    mine = [units[i] for i in shard]
    claimed: List[int] = []
    # groups a rank may hold ahead of its main loop: enough for the decode threads and the
    # engine's batches in flight
    ahead = rc.claim_ahead or 0
    gate = _ClaimGate(ahead if ahead > 0 else rc.read_threads + 3)
    if rc.schedule == "static":
        groups_it = unit_groups([u for u in mine if u.index not in done])
        accounted = mine          # this rank reports the resumed units of its own range
    else:
        # every rank builds the same group list (same manifests), then pulls from one cursor. With
        # too few row groups to spread (< 4 per rank) every unit is its own claim: ranks then may
        # decode the same row group, but all of them get work
        todo_all = [u for u in units if u.index not in done]
        groups_all = unit_groups(todo_all)
        if world > 1 and len(groups_all) < 4 * world:
            groups_all = [[u] for u in todo_all]
        groups_it = _claimed(ctx, ctx.next_key("units"), groups_all, claimed, gate)
        accounted = units if rank == 0 else []
    local = RunStats(step_filtered=[0] * nsteps)
    for u in accounted:
        if u.index in done:
            rec = done[u.index]
            local.docs += rec["docs"]
            local.kept += rec["kept"]
            local.excluded += rec["excluded"]
            local.errors += rec["errors"]
            for i, c in enumerate(rec.get("step_filtered", [])):
                local.step_filtered[i] += c
            local.units_skipped += 1
    metrics.RANK.set(rank)
    metrics.WORLD_SIZE.set(world)
    if rank == 0 and rc.metrics_port is not None:
        metrics.setup_prometheus_metrics(rc.metrics_port)
    # input decoding starts now and overlaps the engine (HIP context, kernels, model) set-up
    ureader = _UnitReader(reader)
    source = _Prefetcher(_read_units(reader, groups_it, rc.read_threads, ureader, window=gate.ahead),
                         depth=rc.read_threads + 2)
    try:
        if engine is None:
            backend = rc.backend
            device = ctx.device if backend in ("cuda", "auto") else None
            with tracing.trace_range("tb.engine_init"):
                engine = Engine(cfg, backend=backend, device=device, nthreads=rc.threads,
                                max_batch_bytes=rc.batch_bytes, slots=rc.slots,
                                segmentation=rc.segmentation, tokenizer_dir=rc.tokenizer_dir,
                                badwords_dir=rc.badwords_dir, tokenizer_file=rc.tokenizer_file,
                                fault_inject=None if (rank_fault is not None or slow is not None) else rc.fault_inject)
    except BaseException:
        source.close()
        raise
    log.info("rank %d/%d: schedule=%s, %d units already done, backend=%s, CPUs %s, threads: pool %d, "
             "readers %d, writers %d", rank, world, rc.schedule, local.units_skipped, engine.backend,
             os.environ.get("TB_CPU_SET", "(not pinned)"), engine.nthreads, rc.read_threads, rc.write_threads)

    hb = Heartbeat(ctx, len(local.vector(nsteps)), interval=rc.progress_interval,
                   on_global=_publish_global if rank == 0 else None)
    hb.update(local.vector(nsteps))
    sink = _PartSink(rc, work_dir, rank) if use_parts else _DirectSink(rc)
    writer = _Writer(sink, rc.compression, rc.write_threads)
    last_report = time.perf_counter()
    last_docs = local.docs
    inflight: collections.deque = collections.deque()

    def feed():
        for unit, batch in source:
            inflight.append((unit, batch))
            gate.done(unit.index)  # handed to the engine (its own in-flight depth is bounded)
            yield batch.text[0], batch.text[1], batch.meta

    t_loop = time.perf_counter()
    setup_s = t_loop - t_start
    try:
        t_prev = time.perf_counter()
        for res in engine.process_many(feed(), on_error="recover"):
            unit, batch = inflight.popleft()
            now = time.perf_counter()
            dt, t_prev = now - t_prev, now
            fs = res.fail_step
            step_counts = np.bincount(fs[(res.status == 1) & (fs >= 0)], minlength=nsteps)[:nsteps] \
                if len(fs) else np.zeros(nsteps, dtype=np.int64)
            counts = dict(docs=batch.n + batch.error_rows, kept=res.n_kept, excluded=res.n_excluded,
                          errors=int(len(res.error_rows)) + batch.error_rows,
                          step_filtered=[int(x) for x in step_counts])
            with tracing.trace_range("tb.writer_submit"):
                writer.submit((batch, res, unit, counts))
            local.docs += counts["docs"]
            local.kept += counts["kept"]
            local.excluded += counts["excluded"]
            local.errors += counts["errors"]
            local.bytes_in += batch.bytes_in
            local.delegated += res.n_delegated
            for i, c in enumerate(step_counts):
                local.step_filtered[i] += int(c)
            local.units += 1
            _update_metrics(cfg, res, batch, counts, step_counts, dt)
            hb.update(local.vector(nsteps))
            hb.check()
            if slow is not None and slow[1] == rank:
                time.sleep(slow[0])
            if rank_fault is not None and rank_fault[1] == rank and local.units == rank_fault[0]:
                log.error("rank %d: injected rank failure after %d unit(s) (--fault-inject rank@...)", rank,
                          local.units)
                logging.shutdown()
                os._exit(17)
            now = time.perf_counter()
            if now - last_report >= rc.progress_interval:
                speed = (local.docs - last_docs) / (now - last_report)
                log.info("Processed: %d, Filtered: %d, Errored: %d | Speed: %.2f docs/sec", local.kept,
                         local.excluded, local.errors, speed)
                last_report, last_docs = now, local.docs
    finally:
        gate.closed = True
        source.close()
        writer.close()
    busy = time.perf_counter() - t_loop  # this rank's own work (hb.finish waits for the others)
    hb.finish(local.vector(nsteps))
    phase = {"setup": setup_s, "read": ureader.seconds, "write": writer.seconds,
             "main_loop": time.perf_counter() - t_loop,
             # CPU seconds by thread group: Parquet decode (reader threads; their HTML decoding runs
             # on the native pool, counted under "other"), output encode, part commits; other = the
             # process total minus those (main loop, engine threads, native pools)
             "cpu_read": ureader.cpu, "cpu_encode": writer.cpu_encode, "cpu_write": writer.cpu_write}
    ru_end = resource.getrusage(resource.RUSAGE_SELF)
    phase["cpu_total"] = (ru_end.ru_utime - ru_start.ru_utime) + (ru_end.ru_stime - ru_start.ru_stime)
    phase["cpu_other"] = phase["cpu_total"] - phase["cpu_read"] - phase["cpu_encode"] - phase["cpu_write"]
    log.info("rank %d phases: %s", rank, {k: round(v, 3) for k, v in phase.items()})
    elapsed = time.perf_counter() - t_start
    total_vec = ctx.all_reduce_sum(local.vector(nsteps))
    elapsed_max = ctx.all_reduce_max(elapsed)
    units_done = int(ctx.all_reduce_sum([local.units])[0])
    skipped = int(ctx.all_reduce_sum([local.units_skipped])[0])
    stats = RunStats.from_vector(total_vec, elapsed_max, units_done, skipped)
    stats.phase_seconds = phase
    per_rank = ctx.all_gather_counts([local.units, int(round(busy * 1e6))])
    stats.rank_units = [int(x) for x in per_rank[:, 0]]
    stats.rank_busy = [float(x) / 1e6 for x in per_rank[:, 1]]
    cpus = placement.bound_cpus()
    cpu_row = [len(cpus) if cpus else 0, engine.nthreads, rc.read_threads, rc.write_threads,
               min(cpus) if cpus else -1, max(cpus) if cpus else -1]
    stats.rank_cpus = [[int(v) for v in row] for row in ctx.all_gather_counts(cpu_row)]
    if use_parts:
        ctx.barrier()
        t_merge = time.perf_counter()
        merge_parts(work_dir, [u.index for u in mine], rc, ctx)
        phase["merge"] = time.perf_counter() - t_merge
        if rank == 0 and not rc.keep_parts:
            shutil.rmtree(work_dir, ignore_errors=True)
        ctx.barrier()
    stats.seconds = ctx.all_reduce_max(time.perf_counter() - t_start)
    tracing.dump_timeline(f".rank{rank}" if world > 1 else "")
    if rank == 0:
        metrics.set_global_counts(stats.docs, stats.kept, stats.excluded, stats.errors)
    return stats


def _publish_global(v: np.ndarray) -> None:
    metrics.set_global_counts(int(v[0]), int(v[1]), int(v[2]), int(v[3]))


def _parse_slow(spec: Optional[str], world: int) -> Optional[Tuple[float, int]]:
    """``slow@SECONDS[:R]``: rank R (default: the last rank) sleeps SECONDS after every unit
    (debug: a straggler, for the scheduling tests)."""
    if not spec or not spec.startswith("slow@"):
        return None
    sec, _, r = spec[5:].partition(":")
    try:
        return float(sec), int(r) if r else world - 1
    except ValueError:
        raise PipelineError(f"bad fault injection spec {spec!r} (expected slow@SECONDS or slow@SECONDS:R)") from None


def _parse_rank_fault(spec: Optional[str], world: int) -> Optional[Tuple[int, int]]:
    """``rank@N[:R]``: rank R (default: the last rank) dies after its N-th unit (debug)."""
    if not spec or not spec.startswith("rank@"):
        return None
    at, _, r = spec[5:].partition(":")
    if not at.isdigit() or (r and not r.isdigit()):
        raise PipelineError(f"bad fault injection spec {spec!r} (expected rank@N or rank@N:R)")
    return int(at), int(r) if r else world - 1


def _update_metrics(cfg, res, batch, counts, step_counts, dt) -> None:
    metrics.TASKS_PROCESSED_TOTAL.inc(counts["kept"])
    metrics.TASKS_FILTERED_TOTAL.inc(counts["excluded"])
    metrics.TASKS_FAILED_TOTAL.inc(counts["errors"])
    metrics.RESULTS_RECEIVED_TOTAL.inc(counts["docs"])
    metrics.RESULTS_SUCCESS_TOTAL.inc(counts["kept"])
    metrics.RESULTS_FILTERED_TOTAL.inc(counts["excluded"])
    metrics.RESULTS_ERROR_TOTAL.inc(counts["errors"])
    metrics.TASK_PROCESSING_DURATION_SECONDS.observe(dt)
    metrics.BYTES_PROCESSED_TOTAL.inc(batch.bytes_in)
    metrics.DELEGATED_DOCS_TOTAL.inc(res.n_delegated)
    if dt > 0:
        metrics.DOCS_PER_SECOND.set(counts["docs"] / dt)
    for phase, sec in res.timings.items():
        metrics.GPU_PHASE_SECONDS.labels(phase).observe(sec)
    for i, c in enumerate(step_counts):
        if c:
            metrics.STEP_FILTERED_TOTAL.labels(str(i), cfg.pipeline[i].type).inc(int(c))
