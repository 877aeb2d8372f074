"""Message-level producer API (reference src/producer_logic.rs:21-230), kept for users who drive
the pipeline per document (e.g. their own queue between processes) instead of with ``run``.

* :func:`publish_tasks` reads the Parquet input in 1024-row batches and hands one task message
  (the reference's ``TextDocument`` JSON) per document to ``publish``; read errors are counted
  and skipped, like the producer does.
* :func:`aggregate_results_from_stream` consumes ``ProcessingOutcome`` values until
  ``published_count`` arrived (or the stream ends), writing ``Success`` documents to the output
  file and ``Filtered`` documents to the excluded file in batches of 500; ``Error`` outcomes are
  counted and dropped. Both files are always created. Returns
  ``(outcomes_received, success, filtered)``.

``run`` (runner.py) is the high-throughput path; these functions exist for API parity.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import time
from typing import Callable, Iterable, Optional, Tuple

from .data_model import Error, Filtered, ProcessingOutcome, Success, TextDocument
from .errors import PipelineError
from .io.parquet import ParquetInputConfig, ParquetReader, ParquetWriter
from .utils import metrics

log = logging.getLogger("textblaster_amd.producer")

PARQUET_WRITE_BATCH_SIZE = 500  # reference producer_logic.rs:21
PARQUET_READ_BATCH_SIZE = 1024  # reference producer_logic.rs:37


@dataclasses.dataclass
class ProducerArgs:
    """reference config/producer.rs:5-47 (queue fields are accepted for compatibility)."""

    input_file: str
    text_column: str = "text"
    id_column: Optional[str] = "id"
    amqp_addr: str = "amqp://guest:guest@localhost:5672/%2f"
    task_queue: str = "task_queue"
    results_queue: str = "results_queue"
    prefetch_count: int = 10
    output_file: str = "output_processed.parquet"
    excluded_file: str = "excluded.parquet"
    metrics_port: Optional[int] = None


def publish_tasks(args: ProducerArgs, publish: Callable[[bytes], None]) -> int:
    """Publishes every readable document as task JSON; returns the number published."""
    reader = ParquetReader(ParquetInputConfig(args.input_file, args.text_column, args.id_column or "id",
                                              PARQUET_READ_BATCH_SIZE))
    published = 0
    read_errors = 0
    t0 = time.perf_counter()
    for item in reader.iter_documents_results():
        if isinstance(item, Exception):
            log.warning("Failed to read document: %s", item)
            read_errors += 1
            metrics.TASK_PUBLISH_ERRORS_TOTAL.inc()
            continue
        t = time.perf_counter()
        publish(item.to_json())
        metrics.TASK_PUBLISHING_DURATION_SECONDS.observe(time.perf_counter() - t)
        metrics.TASKS_PUBLISHED_TOTAL.inc()
        metrics.ACTIVE_TASKS_IN_FLIGHT.inc()
        published += 1
    log.info("Finished publishing %d tasks in %.2fs. Read/Serialization Errors: %d", published,
             time.perf_counter() - t0, read_errors)
    return published


def aggregate_results_from_stream(args: ProducerArgs, stream: Iterable[ProcessingOutcome],
                                  published_count: int) -> Tuple[int, int, int]:
    for path in (args.output_file, args.excluded_file):
        parent = os.path.dirname(os.path.abspath(path))
        os.makedirs(parent, exist_ok=True)
    out = ParquetWriter(args.output_file)
    exc = ParquetWriter(args.excluded_file)
    results, excluded = [], []
    received = success = filtered = 0
    it = iter(stream)
    try:
        while received < published_count:
            try:
                outcome = next(it)
            except StopIteration:
                log.warning("Outcome stream closed before all outcomes received.")
                break
            received += 1
            metrics.RESULTS_RECEIVED_TOTAL.inc()
            metrics.ACTIVE_TASKS_IN_FLIGHT.dec()
            if isinstance(outcome, Success):
                success += 1
                metrics.RESULTS_SUCCESS_TOTAL.inc()
                results.append(outcome.document)
                if len(results) >= PARQUET_WRITE_BATCH_SIZE:
                    out.write_batch(results)
                    results.clear()
            elif isinstance(outcome, Filtered):
                filtered += 1
                metrics.RESULTS_FILTERED_TOTAL.inc()
                excluded.append(outcome.document)
                if len(excluded) >= PARQUET_WRITE_BATCH_SIZE:
                    exc.write_batch(excluded)
                    excluded.clear()
            elif isinstance(outcome, Error):
                metrics.RESULTS_ERROR_TOTAL.inc()
        if results:
            out.write_batch(results)
        if excluded:
            exc.write_batch(excluded)
    finally:
        out.close()
        exc.close()
    log.info("Finished consuming (Received %d/%d).", received, published_count)
    return received, success, filtered


def run_in_process(args: ProducerArgs, executor) -> Tuple[int, int, int]:
    """publish -> execute_processing_pipeline -> aggregate, all in this process, per document:
    the reference's message flow without a broker (tests, small jobs)."""
    from .pipeline.executor import execute_processing_pipeline

    tasks = []
    n = publish_tasks(args, tasks.append)
    outcomes = (o for o in (execute_processing_pipeline(t, executor) for t in tasks) if o is not None)
    return aggregate_results_from_stream(args, outcomes, n)
