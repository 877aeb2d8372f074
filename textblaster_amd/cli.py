"""Command line (reference src/bin/producer.rs, src/bin/worker.rs, config/producer.rs,
config/worker.rs).

    python -m textblaster_amd run       -i in.parquet [-o out.parquet] [-e excluded.parquet] [-c cfg.yaml] ...
    python -m textblaster_amd producer  (same as run: the reference's producer flags + the pipeline config)
    python -m textblaster_amd worker    --validate-config [-c cfg.yaml]
    python -m textblaster_amd worker    [-c cfg.yaml] < tasks.jsonl > outcomes.jsonl
    python -m textblaster_amd validate-config cfg.yaml

There is no RabbitMQ: ``run``/``producer`` execute the whole pipeline in-process on the local
GPUs (``--gpus N`` starts one process per GPU through torch.distributed.run; under torchrun the
ranks are read from the environment). The reference's queue flags (``-a/--amqp-addr``,
``-q/--task-queue``, ``-r/--results-queue``, ``--prefetch-count``) are accepted with the same
defaults and ignored. ``worker`` without ``--validate-config`` reads task JSON lines (the
reference's message format) from stdin and writes outcome JSON lines to stdout.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from typing import List, Optional

DEFAULT_AMQP = "amqp://guest:guest@localhost:5672/%2f"
DEFAULT_CONFIG = "config/pipeline_config.yaml"


class _JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        return json.dumps({
            "timestamp": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created))
            + f".{int(record.msecs * 1000):06d}Z",
            "level": record.levelname,
            "fields": {"message": record.getMessage()},
            "target": record.name,
        })


class DailyFileHandler(logging.Handler):
    """JSON log lines into ``<dir>/<name>.log.<YYYY-MM-DD>`` (local date), switching files when
    the date changes — the file layout of the reference's tracing_appender::rolling::daily
    (bin/producer.rs:57-83)."""

    def __init__(self, log_dir: str, name: str, today=None):
        super().__init__()
        import datetime

        self.dir, self.name = log_dir, name
        self._today = today or (lambda: datetime.date.today().isoformat())
        self._date = None
        self._fh = None

    def path_for(self, date: str) -> str:
        return os.path.join(self.dir, f"{self.name}.log.{date}")

    def emit(self, record: logging.LogRecord) -> None:
        try:
            d = self._today()
            if d != self._date or self._fh is None:
                if self._fh is not None:
                    self._fh.close()
                self._fh = open(self.path_for(d), "a", encoding="utf-8")
                self._date = d
            self._fh.write(self.format(record) + "\n")
            self._fh.flush()
        except Exception:  # noqa: BLE001 - logging must never raise
            self.handleError(record)

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None
        super().close()


def setup_logging(log_dir: Optional[str], name: str, console_level: str = "WARNING") -> None:
    """Console at WARNING, JSON lines at INFO (or $TB_LOG) into daily files
    ``<log_dir>/<name>.log.<YYYY-MM-DD>`` (reference: tracing console=warn, daily rolling JSON
    file ./log/<name>.log)."""
    root = logging.getLogger()
    root.handlers.clear()
    level = (os.environ.get("TB_LOG") or os.environ.get("RUST_LOG") or "INFO").upper()
    root.setLevel(level if level in ("DEBUG", "INFO", "WARNING", "WARN", "ERROR", "CRITICAL") else "INFO")
    con = logging.StreamHandler(sys.stderr)
    con.setLevel(console_level)
    con.setFormatter(logging.Formatter("%(levelname)s %(name)s: %(message)s"))
    root.addHandler(con)
    if log_dir:
        try:
            os.makedirs(log_dir, exist_ok=True)
            fh = DailyFileHandler(log_dir, name)
            fh.setFormatter(_JsonFormatter())
            root.addHandler(fh)
        except OSError as e:
            logging.getLogger("textblaster_amd").warning("cannot open log file in %s: %s", log_dir, e)


def _queue_flags(p: argparse.ArgumentParser) -> None:
    g = p.add_argument_group("reference queue flags (accepted, unused: no RabbitMQ in this engine)")
    g.add_argument("-a", "--amqp-addr", default=DEFAULT_AMQP)
    g.add_argument("-q", "--task-queue", default="task_queue")
    g.add_argument("-r", "--results-queue", default="results_queue")
    g.add_argument("--prefetch-count", type=int, default=10)


def _u16(s: str) -> int:
    v = int(s)
    if not 0 <= v <= 65535:
        raise argparse.ArgumentTypeError(f"{v} is not in 0..=65535")
    return v


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="textblaster_amd", description="MI355X text-quality filtering engine")
    sub = ap.add_subparsers(dest="command")

    for name in ("run", "producer"):
        p = sub.add_parser(name, help="filter a Parquet file end to end")
        p.add_argument("-i", "--input-file", required=True, help="Path to the input Parquet file")
        p.add_argument("--text-column", default="text", help="Text column name in the Parquet file")
        p.add_argument("--id-column", default="id", help="ID column name in the Parquet file")
        p.add_argument("-o", "--output-file", default="output_processed.parquet")
        p.add_argument("-e", "--excluded-file", default="excluded.parquet")
        p.add_argument("--metrics-port", type=_u16, default=None)
        p.add_argument("-c", "--pipeline-config", default=DEFAULT_CONFIG)
        _queue_flags(p)
        p.add_argument("--gpus", "--devices", dest="gpus", type=int, default=None,
                       help="number of local GPUs (one process each); default: all visible GPUs")
        p.add_argument("--backend", default="auto", choices=["auto", "cuda", "cpu"])
        p.add_argument("--cpu", dest="backend", action="store_const", const="cpu",
                       help="run the CPU oracle path (same as --backend cpu)")
        p.add_argument("--segmentation", default="icu", choices=["icu", "rules"],
                       help="UAX#29 implementation of the CPU backend")
        p.add_argument("--unit-rows", type=int, default=65536, help="rows per processing/checkpoint unit")
        p.add_argument("--threads", type=int, default=None,
                       help="native pool threads per rank (default: the rank's CPU budget)")
        p.add_argument("--read-threads", type=int, default=None,
                       help="Parquet reader threads per rank (default 8, or the rank's CPU budget share)")
        p.add_argument("--write-threads", type=int, default=None,
                       help="output encoder threads per rank (default 4, or the rank's CPU budget share)")
        p.add_argument("--batch-bytes", type=int, default=None,
                       help="text bytes per device batch (default 384 MiB: scratch is 80-176 B per byte)")
        p.add_argument("--slots", type=int, default=None,
                       help="device batches in flight per GPU (default: 3 when HBM allows)")
        p.add_argument("--claim-ahead", type=int, default=None,
                       help="row groups a rank may claim ahead of its main loop (reference prefetch_count "
                            "semantics; default readers + 3)")
        p.add_argument("--schedule", choices=("dynamic", "static"), default="dynamic",
                       help="row groups across ranks: a shared claim cursor (dynamic) or byte-balanced "
                            "contiguous ranges (static)")
        p.add_argument("--resume", action="store_true", help="skip units recorded in the work dir manifest")
        p.add_argument("--checkpoint", action="store_true", help="write per-unit parts + manifest (resumable)")
        p.add_argument("--work-dir", default=None, help="checkpoint dir (default <output-file>.work)")
        p.add_argument("--keep-parts", action="store_true")
        p.add_argument("--compression", default="none", help="Parquet codec (none, snappy, zstd, ...)")
        p.add_argument("--tokenizer-dir", default=None, help="local dir holding <name>/tokenizer.json")
        p.add_argument("--tokenizer-file", default=None, help="tokenizer.json used by every TokenCounter step")
        p.add_argument("--langid-model", default=None, help="language-id weights (.npz); default: bundled model")
        p.add_argument("--fault-inject", default=None, help="debug: kernel@N or oom@N (fail the N-th batch once), rank@N[:R] (rank R dies after N units), "
                            "slow@SECONDS[:R] (rank R sleeps after every unit)")
        p.add_argument("--badwords-dir", default=None, help="dir holding the C4 bad-words lists (<lang> files)")
        p.add_argument("--html-decode", choices=("cpu", "gpu"), default="cpu",
                       help="decode HTML entities of the input text on the host (default) or the GPU")
        p.add_argument("--log-dir", default="./log")

    w = sub.add_parser("worker", help="validate a config, or process task JSON lines from stdin")
    _queue_flags(w)
    w.add_argument("-c", "--pipeline-config", default=DEFAULT_CONFIG)
    w.add_argument("--metrics-port", type=_u16, default=None)
    w.add_argument("--validate-config", action="store_true", help="Validate the pipeline configuration and exit")
    w.add_argument("--segmentation", default="icu", choices=["icu", "rules"])
    w.add_argument("--tokenizer-dir", default=None)
    w.add_argument("--log-dir", default="./log")

    v = sub.add_parser("validate-config", help="validate a pipeline configuration file")
    v.add_argument("path", nargs="?", default=DEFAULT_CONFIG)
    return ap


def validate_config_cmd(path: str) -> int:
    from .config.pipeline import load_pipeline_config
    from .errors import PipelineError

    try:
        load_pipeline_config(path)
    except PipelineError as e:
        print(f"Configuration '{path}' is invalid: {e}", file=sys.stderr)
        return 1
    print(f"Configuration '{path}' is valid.")
    return 0


def _visible_gpus() -> int:
    from .parallel.launch import visible_gpu_count

    return visible_gpu_count()


def _relaunch_distributed(n: int, argv: List[str]) -> int:
    """Start ``n`` ranks via torch.distributed.run as a child process (never exec)."""
    from .parallel.launch import spawn_ranks

    return spawn_ranks(n, ["-m", "textblaster_amd"] + argv)


def run_cmd(args, argv: List[str]) -> int:
    from .errors import PipelineError
    from .parallel import dist
    from .parallel.heartbeat import RankFailure
    from .runner import RunConfig, run

    under_launcher = "WORLD_SIZE" in os.environ
    if args.backend == "cpu":
        ngpu = args.gpus or 0       # CPU ranks (gloo) when --gpus is given with --cpu
    else:
        ngpu = args.gpus if args.gpus is not None else _visible_gpus()
    if not under_launcher and ngpu > 1:
        from .parallel.launch import strip_flag

        shared = os.environ.get("TB_SHARED_GPU", "") not in ("", "0")  # all ranks on GPU 0 (dist.py)
        if args.backend != "cpu" and args.gpus is not None and _visible_gpus() < ngpu and not shared:
            print(f"Error: --gpus {ngpu} requested but only {_visible_gpus()} GPU(s) are visible", file=sys.stderr)
            return 2
        # strip --gpus so the children do not relaunch
        return _relaunch_distributed(ngpu, strip_flag(strip_flag(argv, "--gpus"), "--devices"))

    backend = args.backend
    if backend == "auto":
        backend = "cuda" if ngpu >= 1 else "cpu"
    ctx = dist.init_from_env(backend="nccl" if backend == "cuda" else "gloo")
    rank = ctx.rank
    setup_logging(args.log_dir, "producer" if ctx.world_size == 1 else f"producer.rank{rank}")
    log = logging.getLogger("textblaster_amd")
    if args.amqp_addr != DEFAULT_AMQP:
        log.warning("--amqp-addr is ignored: documents are processed in-process (no RabbitMQ)")
    log.info("Producer started.")
    log.info("Input file: %s", args.input_file)
    log.info("Output File: %s", args.output_file)
    if args.langid_model:
        os.environ["TB_LANGID_MODEL"] = args.langid_model
    rc = RunConfig(
        input_file=args.input_file, output_file=args.output_file, excluded_file=args.excluded_file,
        pipeline_config=args.pipeline_config, text_column=args.text_column, id_column=args.id_column,
        backend=backend, segmentation=args.segmentation, unit_rows=args.unit_rows, threads=args.threads,
        work_dir=args.work_dir, resume=args.resume, checkpoint=args.checkpoint, keep_parts=args.keep_parts,
        compression=args.compression, tokenizer_dir=args.tokenizer_dir, badwords_dir=args.badwords_dir,
        html_decode=args.html_decode, metrics_port=args.metrics_port, tokenizer_file=args.tokenizer_file,
        fault_inject=args.fault_inject, read_threads=args.read_threads, write_threads=args.write_threads,
        batch_bytes=args.batch_bytes, slots=args.slots, claim_ahead=args.claim_ahead, schedule=args.schedule)
    try:
        stats = run(rc, ctx)
    except RankFailure as e:
        # a peer is gone: collective teardown could block on it, so leave right away
        log.error("Run failed: %s", e)
        print(f"Error: {e}", file=sys.stderr, flush=True)
        logging.shutdown()
        os._exit(3)
    except PipelineError as e:
        log.error("Run failed: %s", e)
        print(f"Error: {e}", file=sys.stderr)
        ctx.destroy()
        return 1
    if rank == 0:
        from .config.pipeline import load_pipeline_config

        names = [s.type for s in load_pipeline_config(args.pipeline_config).pipeline]
        lines = [
            "--------------------",
            "Processing Summary:",
            f"  Documents Read: {stats.docs}",
            f"    - Kept (output): {stats.kept}",
            f"    - Filtered (excluded): {stats.excluded}",
            f"    - Errors: {stats.errors}",
        ]
        for i, n in enumerate(names):
            if i < len(stats.step_filtered):
                lines.append(f"      filtered by step {i} {n}: {stats.step_filtered[i]}")
        lines += [
            f"  Ranks: {ctx.world_size} ({backend}), units: {stats.units} (+{stats.units_skipped} resumed)",
            f"  Units per rank: {stats.rank_units} | busy seconds per rank: "
            f"{[round(b, 3) for b in stats.rank_busy]}",
            "  CPU sets per rank: " + "; ".join(
                f"r{r}: " + (f"cpus {c[4]}-{c[5]} ({c[0]})" if c[0] else "not pinned")
                + f", pool {c[1]}, readers {c[2]}, writers {c[3]}" for r, c in enumerate(stats.rank_cpus)),
            f"  Time: {stats.seconds:.2f} s | Speed: {stats.docs_per_sec:.2f} docs/sec",
            f"  Output File: {args.output_file}",
            f"  Excluded File: {args.excluded_file}",
            "--------------------",
        ]
        for ln in lines:
            log.info(ln)
            print(ln)
    ctx.destroy()
    return 0


def worker_cmd(args) -> int:
    if args.validate_config:
        return validate_config_cmd(args.pipeline_config)
    setup_logging(args.log_dir, "worker")
    from .config.pipeline import load_pipeline_config
    from .data_model import outcome_to_json
    from .errors import PipelineError
    from .pipeline.executor import PipelineExecutor, build_pipeline_from_config, execute_processing_pipeline
    from .utils import metrics

    log = logging.getLogger("textblaster_amd.worker")
    try:
        cfg = load_pipeline_config(args.pipeline_config)
        ex = PipelineExecutor(build_pipeline_from_config(cfg, args.tokenizer_dir, args.segmentation))
    except PipelineError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    metrics.setup_prometheus_metrics(args.metrics_port)
    log.info("Worker starting (stdin -> stdout).")
    out = sys.stdout.buffer
    for line in sys.stdin.buffer:
        line = line.strip()
        if not line:
            continue
        outcome = execute_processing_pipeline(line, ex)
        if outcome is not None:
            out.write(outcome_to_json(outcome) + b"\n")
    out.flush()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0].startswith("-") and argv[0] not in ("-h", "--help"):
        argv = ["run"] + argv  # bare producer-style flags
    ap = build_parser()
    args = ap.parse_args(argv)
    if args.command in ("run", "producer"):
        return run_cmd(args, argv)
    if args.command == "worker":
        return worker_cmd(args)
    if args.command == "validate-config":
        return validate_config_cmd(args.path)
    ap.print_help()
    return 2
