"""Live global counters (AR1 while the job runs) and rank-failure detection.

The reference's Prometheus endpoints are per process (utils/prometheus_metrics.rs:172-196)
and a dead worker is only noticed through broker redelivery (worker_logic.rs:273-278). Here
ranks own different numbers of units, so a per-batch collective on the main thread would
mismatch between ranks. Instead every rank runs a small thread that all-reduces
``[done, cumulative counters...]`` every ``interval`` seconds over a side ``gloo`` group (host
counters, so they stay on the host: no device round trip, no contention with RCCL work on the
GPU). All ranks iterate in lockstep and stop on the iteration where every rank reports done.
Rank 0 publishes each reduced vector (``on_global``), so its ``/metrics`` shows the job-wide
view while the job runs.

A collective that fails or times out (a dead or hung peer) marks the beat as failed; the main
thread checks ``failed`` after every batch and aborts the rank with :class:`RankFailure`
(non-zero exit, restartable with ``--resume`` from the manifest). The end-of-run RCCL
collectives have their own timeout (``TB_COLLECTIVE_TIMEOUT``, ``dist.init_from_env``).
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
from typing import Callable, Optional

import numpy as np

from ..errors import PipelineError

log = logging.getLogger("textblaster_amd.heartbeat")


class RankFailure(PipelineError):
    pass


class Heartbeat:
    def __init__(self, ctx, width: int, interval: float = 1.0,
                 on_global: Optional[Callable[[np.ndarray], None]] = None,
                 timeout_s: Optional[float] = None):
        self.ctx = ctx
        self.width = width
        self.interval = interval
        self.on_global = on_global
        self._vec = np.zeros(width, dtype=np.int64)
        self._lock = threading.Lock()
        self._done = threading.Event()
        self.failed: Optional[str] = None
        self.rounds = 0
        self.last_global = np.zeros(width, dtype=np.int64)
        self._group = None
        self._thread: Optional[threading.Thread] = None
        if ctx.initialized and ctx.world_size > 1:
            import torch.distributed as td

            t = float(timeout_s or os.environ.get("TB_HEARTBEAT_TIMEOUT", "120"))
            # every rank creates the side group at the same point of run()
            self._group = td.new_group(backend="gloo", timeout=datetime.timedelta(seconds=t))
            self._thread = threading.Thread(target=self._run, name="tb-heartbeat", daemon=True)
            self._thread.start()

    def update(self, vec) -> None:
        with self._lock:
            self._vec = np.asarray(vec, dtype=np.int64).copy()

    def check(self) -> None:
        if self.failed:
            raise RankFailure(f"rank {self.ctx.rank}: a peer rank failed ({self.failed}); "
                              f"rerun with --resume to continue from the manifest")

    def _run(self) -> None:
        import torch
        import torch.distributed as td

        try:
            while True:
                done = self._done.wait(self.interval)
                with self._lock:
                    v = np.concatenate([[1 if done else 0], self._vec]).astype(np.int64)
                t = torch.from_numpy(v)
                td.all_reduce(t, op=td.ReduceOp.SUM, group=self._group)
                g = t.numpy()
                self.rounds += 1
                self.last_global = g[1:].copy()
                if self.on_global is not None:
                    self.on_global(self.last_global)
                if int(g[0]) == self.ctx.world_size:
                    return
        except Exception as e:  # noqa: BLE001 - reported to the main thread
            self.failed = f"{type(e).__name__}: {e}"
            log.error("rank %d: heartbeat collective failed: %s", self.ctx.rank, self.failed)

    def finish(self, vec=None) -> np.ndarray:
        """Final counters in, wait until every rank is done; returns the last global vector."""
        if vec is not None:
            self.update(vec)
        self._done.set()
        if self._thread is not None:
            self._thread.join()
            if self._group is not None and not self.failed:
                import torch.distributed as td

                td.destroy_process_group(self._group)
                self._group = None
        else:
            self.last_global = self._vec.copy()
            if self.on_global is not None:
                self.on_global(self.last_global)
        self.check()
        return self.last_global
