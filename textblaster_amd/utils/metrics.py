"""Prometheus metrics (reference src/utils/prometheus_metrics.rs:16-201).

The reference's producer/worker metric names are kept (with the double-counting and
never-incremented bugs fixed: every counter is incremented exactly once per event), plus
device-side metrics. ``setup_prometheus_metrics(port)`` serves ``GET /metrics`` on
``0.0.0.0:<port>`` from a background thread; in a multi-GPU run rank 0 serves the
all-reduced global view (``set_global_counts``).
"""
from __future__ import annotations

import logging
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest, start_http_server

REGISTRY = CollectorRegistry(auto_describe=True)
log = logging.getLogger("textblaster_amd.metrics")

# ---- producer (reference :16-86) ----
TASKS_PUBLISHED_TOTAL = Counter("producer_tasks_published_total", "Total number of tasks published.",
                                registry=REGISTRY)
TASK_PUBLISH_ERRORS_TOTAL = Counter("producer_task_publish_errors_total",
                                    "Total number of errors during task publishing (serialization, read errors).",
                                    registry=REGISTRY)
RESULTS_RECEIVED_TOTAL = Counter("producer_results_received_total", "Total number of results/outcomes received.",
                                 registry=REGISTRY)
RESULTS_SUCCESS_TOTAL = Counter("producer_results_success_total", "Total number of successful results.",
                                registry=REGISTRY)
RESULTS_FILTERED_TOTAL = Counter("producer_results_filtered_total", "Total number of filtered results.",
                                 registry=REGISTRY)
RESULTS_ERROR_TOTAL = Counter("producer_results_error_total", "Total number of error results.", registry=REGISTRY)
RESULT_DESERIALIZATION_ERRORS_TOTAL = Counter("producer_result_deserialization_errors_total",
                                              "Total number of errors deserializing results.", registry=REGISTRY)
ACTIVE_TASKS_IN_FLIGHT = Gauge("producer_active_tasks_in_flight",
                               "Number of tasks published but not yet resolved.", registry=REGISTRY)
TASK_PUBLISHING_DURATION_SECONDS = Histogram("producer_task_publishing_duration_seconds",
                                             "Histogram of batch staging latencies.", registry=REGISTRY)

# ---- worker (reference :89-143) ----
TASKS_PROCESSED_TOTAL = Counter("worker_tasks_processed_total", "Total number of tasks processed by the worker.",
                                registry=REGISTRY)
TASKS_FILTERED_TOTAL = Counter("worker_tasks_filtered_total", "Total number of tasks filtered by the pipeline.",
                               registry=REGISTRY)
TASKS_FAILED_TOTAL = Counter("worker_tasks_failed_total", "Total number of tasks that resulted in a pipeline error.",
                             registry=REGISTRY)
TASK_DESERIALIZATION_ERRORS_TOTAL = Counter("worker_task_deserialization_errors_total",
                                            "Total number of errors deserializing incoming task messages.",
                                            registry=REGISTRY)
OUTCOME_PUBLISH_ERRORS_TOTAL = Counter("worker_outcome_publish_errors_total",
                                       "Total number of errors publishing outcome messages.", registry=REGISTRY)
TASK_PROCESSING_DURATION_SECONDS = Histogram("worker_task_processing_duration_seconds",
                                             "Histogram of task (per-document API) or batch processing durations.",
                                             registry=REGISTRY)
ACTIVE_PROCESSING_TASKS = Gauge("worker_active_processing_tasks", "Number of tasks currently being processed.",
                                registry=REGISTRY)

# ---- new: engine / device ----
STEP_FILTERED_TOTAL = Counter("tb_step_filtered_total", "Documents filtered, by pipeline step.",
                              ["step_index", "step"], registry=REGISTRY)
DOCS_PER_SECOND = Gauge("tb_docs_per_second", "Throughput of the last batch (documents/second).",
                        registry=REGISTRY)
BYTES_PROCESSED_TOTAL = Counter("tb_bytes_processed_total", "Input text bytes processed.", registry=REGISTRY)
H2D_BYTES_TOTAL = Counter("tb_h2d_bytes_total", "Bytes staged host-to-device.", registry=REGISTRY)
GPU_PHASE_SECONDS = Histogram("tb_gpu_phase_seconds", "Per-batch time by phase.", ["phase"], registry=REGISTRY)
GPU_KERNEL_SECONDS = Histogram("tb_gpu_kernel_seconds", "Per-batch device time of each kernel group (HIP events).",
                               ["kernel"], registry=REGISTRY,
                               buckets=(0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, float("inf")))
DELEGATED_DOCS_TOTAL = Counter("tb_cpu_delegated_docs_total",
                               "Documents recomputed on the CPU oracle path (dictionary scripts, collisions).",
                               registry=REGISTRY)
DICT_MARKED_DOCS_TOTAL = Counter("tb_dict_marked_docs_total",
                                 "Dictionary-script documents kept on the device with host ICU word marks.",
                                 registry=REGISTRY)
BATCH_FAILURES_TOTAL = Counter("tb_batch_failures_total", "Batches whose device work failed (then recovered).",
                               ["error"], registry=REGISTRY)
CPU_FALLBACK_DOCS_TOTAL = Counter("tb_cpu_fallback_docs_total",
                                  "Documents re-run on the CPU oracle path after a device failure.", registry=REGISTRY)
GATE_MISMATCH_DOCS_TOTAL = Counter("tb_gate_mismatch_docs_total",
                                   "Documents a device step gate skipped that the host resolver found alive "
                                   "(recomputed on the CPU path; expected 0).", registry=REGISTRY)
DEVICE_RESOLVE_FALLBACK_TOTAL = Counter("tb_device_resolve_fallback_total",
                                        "Batches whose device resolve/compaction (K16) disagreed with the host "
                                        "decisions and were assembled on the host (expected 0).", registry=REGISTRY)
BPE_HOST_DOCS_TOTAL = Counter("tb_bpe_host_docs_total",
                              "Kept documents whose TokenCounter count the device handed to the host tokenizer "
                              "(added-token text or a pre-token over 64 bytes).", registry=REGISTRY)
BPE_DEVICE_DOCS_TOTAL = Counter("tb_bpe_device_docs_total",
                                "Kept documents whose TokenCounter count came from k_bpe_count.", registry=REGISTRY)
RANK = Gauge("tb_rank", "Data-parallel rank of this process.", registry=REGISTRY)
WORLD_SIZE = Gauge("tb_world_size", "Number of data-parallel ranks.", registry=REGISTRY)
GLOBAL_DOCS = Gauge("tb_global_docs_total", "All-reduced document counters (rank 0).", ["kind"],
                    registry=REGISTRY)

_server_started: Optional[int] = None


def setup_prometheus_metrics(port: Optional[int]) -> None:
    """Serve /metrics on 0.0.0.0:port (no-op when port is None)."""
    global _server_started
    if port is None:
        log.info("Metrics endpoint disabled (no --metrics-port).")
        return
    if _server_started == port:
        return
    start_http_server(port, addr="0.0.0.0", registry=REGISTRY)
    _server_started = port
    log.info("Prometheus metrics endpoint listening on 0.0.0.0:%d/metrics", port)


def render() -> bytes:
    return generate_latest(REGISTRY)


def set_global_counts(docs: int, kept: int, excluded: int, errors: int) -> None:
    GLOBAL_DOCS.labels("docs").set(docs)
    GLOBAL_DOCS.labels("kept").set(kept)
    GLOBAL_DOCS.labels("excluded").set(excluded)
    GLOBAL_DOCS.labels("errors").set(errors)
