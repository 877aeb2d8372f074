"""Data parallelism over the GPUs of one node: one process per GPU, torch.distributed with the
``nccl`` backend (= RCCL over xGMI on ROCm), ``gloo`` for CPU-only runs and tests.

The reference scales with competing consumers on a RabbitMQ queue (utils/common.rs,
worker_logic.rs:241-283). Here document data never crosses GPUs: each rank owns a
deterministic, contiguous shard of the input row groups (balanced by byte size) and the only
collectives are tiny counter vectors:

  AR1  all_reduce(SUM) of per-step/per-reason document counters (int64, < 1 KB)
  AG1  all_gather of per-rank kept/excluded counts (part-file bookkeeping for the merge)
  BAR  barrier before the final merge

These are latency-bound (tens of µs over xGMI), so one collective per batch is plenty.
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional, Sequence

import numpy as np


@dataclasses.dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: Optional[str] = None

    @property
    def initialized(self) -> bool:
        return self.backend is not None

    def _torch(self):
        import torch
        import torch.distributed as td

        return torch, td

    def _tensor(self, arr: np.ndarray):
        torch, _ = self._torch()
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if self.backend == "nccl":
            t = t.to(self.device)
        return t

    def barrier(self) -> None:
        if self.initialized:
            _, td = self._torch()
            if self.backend == "nccl":
                td.barrier(device_ids=[self.local_rank])
            else:
                td.barrier()

    def all_reduce_sum(self, arr) -> np.ndarray:
        a = np.asarray(arr, dtype=np.int64)
        if not self.initialized:
            return a.copy()
        _, td = self._torch()
        t = self._tensor(a)
        td.all_reduce(t, op=td.ReduceOp.SUM)
        return t.cpu().numpy()

    def all_reduce_sum_async(self, arr) -> "PendingReduce":
        """Non-blocking all_reduce(SUM) of a small int64 vector (AR1); ``.wait()`` returns it."""
        a = np.asarray(arr, dtype=np.int64)
        if not self.initialized:
            return PendingReduce(None, a.copy())
        _, td = self._torch()
        t = self._tensor(a)
        return PendingReduce(td.all_reduce(t, op=td.ReduceOp.SUM, async_op=True), t)

    def all_reduce_max(self, x: float) -> float:
        if not self.initialized:
            return float(x)
        _, td = self._torch()
        t = self._tensor(np.asarray([x], dtype=np.float64))
        td.all_reduce(t, op=td.ReduceOp.MAX)
        return float(t.cpu().numpy()[0])

    def all_gather_counts(self, arr) -> np.ndarray:
        a = np.asarray(arr, dtype=np.int64).reshape(-1)
        if not self.initialized:
            return a.reshape(1, -1)
        torch, td = self._torch()
        t = self._tensor(a)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        td.all_gather(out, t)
        return np.stack([o.cpu().numpy() for o in out])

    def destroy(self) -> None:
        if self.initialized:
            _, td = self._torch()
            td.destroy_process_group()
            self.backend = None


class PendingReduce:
    def __init__(self, work, tensor):
        self.work = work
        self.tensor = tensor

    def wait(self) -> np.ndarray:
        if self.work is not None:
            self.work.wait()
            self.work = None
            self.tensor = self.tensor.cpu().numpy()
        return self.tensor


def init_from_env(backend: str = "nccl") -> DistContext:
    """Initialise from torchrun's env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ctx = DistContext(rank, world, local)
    if backend == "nccl":
        import torch

        torch.cuda.set_device(local)
        ctx.device = f"cuda:{local}"
    if world > 1:
        import torch.distributed as td

        import datetime

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a dead or hung peer turns into an error after this long instead of a silent hang
        kwargs = {"timeout": datetime.timedelta(seconds=float(os.environ.get("TB_COLLECTIVE_TIMEOUT", "600")))}
        if backend == "nccl":
            import torch

            kwargs["device_id"] = torch.device(f"cuda:{local}")
        td.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
        ctx.backend = backend
    return ctx


def shard_ranges(sizes: Sequence[int], world: int) -> List[range]:
    """Contiguous shards of items (row groups) balanced by total size (prefix-sum split)."""
    sizes = np.asarray(sizes, dtype=np.float64)
    n = len(sizes)
    if n == 0:
        return [range(0, 0) for _ in range(world)]
    csum = np.concatenate([[0.0], np.cumsum(sizes)])
    total = csum[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(csum, target, side="left"))
        k = max(bounds[-1], min(n, k))
        bounds.append(k)
    bounds.append(n)
    return [range(bounds[r], bounds[r + 1]) for r in range(world)]
