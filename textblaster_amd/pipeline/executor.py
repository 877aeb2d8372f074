"""Per-document executor (reference src/executor.rs) and worker-side outcome mapping
(reference src/worker_logic.rs:36-193).

``PipelineExecutor.run_single`` runs the steps in order and stops at the first error, wrapping
it as ``StepError(step_name, source)``. ``execute_processing_pipeline`` maps a serialized task
to a ``ProcessingOutcome``: ``Success``, ``Filtered`` (a ``DocumentFiltered`` directly inside the
``StepError``), or ``None`` for every other failure, updating the worker metrics like the
reference does. The batched engine (engine.py) implements the same semantics for throughput.
"""
from __future__ import annotations

import asyncio
import logging
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Iterable, List, Optional, Sequence, Union

from ..config.pipeline import PipelineConfig
from ..data_model import Filtered, ProcessingOutcome, Success, TextDocument
from ..errors import DocumentFiltered, PipelineError, SerializationError, StepError, Unexpected
from ..utils import metrics
from .steps import ProcessingStep, step_from_config

log = logging.getLogger("textblaster_amd.executor")


class PipelineExecutor:
    def __init__(self, steps: Sequence[ProcessingStep]):
        if not steps:
            log.warning("Pipeline created with no steps.")
        self.steps: List[ProcessingStep] = list(steps)

    def run_single(self, document: TextDocument) -> TextDocument:
        doc = document
        for step in self.steps:
            log.debug("Running step: %s", step.name())
            try:
                doc = step.process(doc)
            except PipelineError as e:
                raise StepError(step.name(), e) from e
            except Exception as e:  # noqa: BLE001 - a step bug is an unexpected pipeline error
                raise StepError(step.name(), Unexpected(str(e))) from e
        return doc

    async def run_single_async(self, document: TextDocument) -> TextDocument:
        doc = document
        for step in self.steps:
            try:
                doc = await step.process_async(doc)
            except PipelineError as e:
                raise StepError(step.name(), e) from e
        return doc

    def run_batch_parallel(self, documents: Iterable[TextDocument], max_workers: Optional[int] = None
                           ) -> List[Union[TextDocument, PipelineError]]:
        """Runs documents concurrently; returns results in input order (the reference returns
        completion order from FuturesUnordered, so callers must not rely on order there)."""
        docs = list(documents)

        def one(d):
            try:
                return self.run_single(d)
            except PipelineError as e:
                return e

        with ThreadPoolExecutor(max_workers=max_workers) as ex:
            return list(ex.map(one, docs))

    async def run_batch_parallel_async(self, documents: Iterable[TextDocument]
                                       ) -> List[Union[TextDocument, PipelineError]]:
        async def one(d):
            try:
                return await self.run_single_async(d)
            except PipelineError as e:
                return e

        return list(await asyncio.gather(*(one(d) for d in documents)))


def build_pipeline_from_config(config: PipelineConfig, tokenizer_dir: Optional[str] = None,
                               segmentation: str = "icu") -> List[ProcessingStep]:
    """reference worker_logic.rs:39-134 (a TokenCounter that cannot load raises, the
    reference panics)."""
    steps = []
    for i, sc in enumerate(config.pipeline):
        log.debug("Adding step %d: %s", i, sc.type)
        steps.append(step_from_config(sc, tokenizer_dir, segmentation))
    if not steps:
        log.warning("Warning: Building an empty pipeline from configuration!")
    else:
        log.info("Pipeline built successfully with %d steps.", len(steps))
    return steps


def execute_processing_pipeline(data: bytes, executor: PipelineExecutor) -> Optional[ProcessingOutcome]:
    """JSON task bytes -> outcome (reference worker_logic.rs:140-193)."""
    metrics.ACTIVE_PROCESSING_TASKS.inc()
    t0 = time.perf_counter()
    try:
        try:
            doc = TextDocument.from_json(data)
        except SerializationError as e:
            log.error("Failed to deserialize task message: %s", e)
            metrics.TASK_DESERIALIZATION_ERRORS_TOTAL.inc()
            return None
        try:
            processed = executor.run_single(doc)
            metrics.TASKS_PROCESSED_TOTAL.inc()
            return Success(processed)
        except StepError as e:
            if isinstance(e.source, DocumentFiltered):
                metrics.TASKS_FILTERED_TOTAL.inc()
                return Filtered(e.source.document, e.source.reason)
            log.error("Pipeline step %s failed: %s", e.step_name, e.source)
            metrics.TASKS_FAILED_TOTAL.inc()
            return None
        except PipelineError as e:
            log.error("Unexpected pipeline error: %s", e)
            metrics.TASKS_FAILED_TOTAL.inc()
            return None
    finally:
        metrics.TASK_PROCESSING_DURATION_SECONDS.observe(time.perf_counter() - t0)
        metrics.ACTIVE_PROCESSING_TASKS.dec()
