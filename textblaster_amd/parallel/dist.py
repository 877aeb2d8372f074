"""Data parallelism over the GPUs of one node: one process per GPU, torch.distributed with the
``nccl`` backend (= RCCL over xGMI on ROCm), ``gloo`` for CPU-only runs and tests.

The reference scales with competing consumers on a RabbitMQ queue (utils/common.rs,
worker_logic.rs:241-283). Here document data never crosses GPUs: ranks pull row groups from a
shared atomic cursor (``DistContext.claim``, the process group's store), so a rank that is slower
(longer documents, a busier GPU) simply takes fewer, and the only collectives are tiny counter
vectors:

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
        """Non-blocking all_reduce(SUM) of a small int64 vector (AR1); ``.wait()`` returns it.

        With RCCL the vector goes up and comes back through pinned host memory on a dedicated
        torch stream (non-blocking copies): nothing touches the null stream, so the reduction
        never waits for (or holds up) the document kernels of the native runtime's streams."""
        a = np.asarray(arr, dtype=np.int64)
        if not self.initialized:
            return PendingReduce(None, a.copy())
        torch, td = self._torch()
        if self.backend != "nccl":
            t = self._tensor(a)
            return PendingReduce(td.all_reduce(t, op=td.ReduceOp.SUM, async_op=True), t)
        if getattr(self, "_ar_stream", None) is None:
            self._ar_stream = torch.cuda.Stream(device=self.device, priority=-1)
        host = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
        with torch.cuda.stream(self._ar_stream):
            t = host.to(self.device, non_blocking=True)
            work = td.all_reduce(t, op=td.ReduceOp.SUM, async_op=True)
        return PendingReduce(work, t, host, self._ar_stream)

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

    def claim(self, key: str, n: int = 1) -> int:
        """Atomically takes ``n`` items of the shared counter ``key``; returns the index of the first
        one (every rank sees each index exactly once). Over a process group this is the group's
        key-value store (``store.add``: the rendezvous TCPStore under torchrun); without one a
        process-local counter. The competing-consumer equivalent of the reference's work queue
        (utils/common.rs:91-94 basic_qos, worker_logic.rs:241-283)."""
        n = int(n)
        if not self.initialized:
            cnt = self.__dict__.setdefault("_claims", {})
            first = cnt.get(key, 0)
            cnt[key] = first + n
            return first
        _, td = self._torch()
        store = td.distributed_c10d._get_default_store()
        return int(store.add(key, n)) - n

    def next_key(self, prefix: str) -> str:
        """A key unique to this call site's n-th use (all ranks make the same sequence of calls)."""
        seq = self.__dict__.get("_key_seq", 0)
        self.__dict__["_key_seq"] = seq + 1
        return f"tb/{prefix}/{seq}"

    def destroy(self) -> None:
        if self.initialized:
            _, td = self._torch()
            td.destroy_process_group()
            self.backend = None


class PendingReduce:
    def done(self) -> bool:
        """True once wait() would not block."""
        return self.work is None or self.work.is_completed()

    def __init__(self, work, tensor, host=None, stream=None):
        self.work = work
        self.tensor = tensor
        self.host = host
        self.stream = stream

    def wait(self) -> np.ndarray:
        if self.work is not None:
            if self.stream is not None:
                import torch

                with torch.cuda.stream(self.stream):
                    self.work.wait()  # orders the stream after the collective
                    self.host.copy_(self.tensor, non_blocking=True)
                self.stream.synchronize()
                self.tensor = self.host.numpy()
            else:
                self.work.wait()
                self.tensor = self.tensor.cpu().numpy()
            self.work = None
        return self.tensor


def _hip_initialised() -> bool:
    """Has this process already loaded (and so initialised) the native HIP runtime layer?"""
    import sys

    from .. import native

    return getattr(native, "_hip", None) is not None or "torch" in sys.modules and _torch_hip_initialised()


def _torch_hip_initialised() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001
        return False


def init_from_env(backend: str = "nccl", force_pg: Optional[bool] = None) -> DistContext:
    """Initialise from torchrun's env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT).

    A process group exists when WORLD_SIZE > 1, or at world size 1 when ``force_pg`` (default:
    env ``TB_FORCE_PG=1``) asks for one: then the per-step AR1 / AG1 / BAR collectives of the
    multi-GPU path run (and are timed) on a single GPU too, over a one-rank RCCL communicator
    (an in-process HashStore, no rendezvous). Without a group nothing imports torch: a one-GPU
    run only needs the native HIP runtime."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)) or world)
    # this rank's CPUs (its GPU's NUMA node, shared evenly with the node's other ranks), before
    # any HIP call: the runtime's threads, the native pools and the pinned buffers follow it
    from . import placement

    placement.bind_rank(local, local_world)
    if force_pg is None:
        force_pg = os.environ.get("TB_FORCE_PG", "") not in ("", "0")
    ctx = DistContext(rank, world, local)
    # TB_SHARED_GPU=1: every rank runs its engine on GPU 0 (functional multi-rank runs of the
    # device path on a one-GPU box); the group then uses gloo, since RCCL needs one GPU per rank.
    # TB_DIST_BACKEND overrides the process-group backend either way.
    shared = os.environ.get("TB_SHARED_GPU", "") not in ("", "0")
    pg_backend = os.environ.get("TB_DIST_BACKEND") or ("gloo" if shared else backend)
    if pg_backend not in ("nccl", "gloo"):
        raise ValueError(f"TB_DIST_BACKEND must be nccl or gloo, not {pg_backend!r}")
    if shared and pg_backend == "nccl" and world > 1:
        # RCCL needs one GPU per rank: with every rank on GPU 0 the communicator cannot form
        raise ValueError("TB_SHARED_GPU=1 puts every rank on GPU 0; use TB_DIST_BACKEND=gloo (the default "
                         "with TB_SHARED_GPU), an RCCL group needs one GPU per rank")
    if backend == "nccl":
        ctx.device = f"cuda:{0 if shared else local}"
    if world > 1 or force_pg:
        import datetime

        import torch
        import torch.distributed as td

        if pg_backend == "nccl":
            # RCCL and torch add their own streams next to the engine's eight; with the box's
            # default of 4 hardware queues per process they land behind document kernels on a
            # shared queue (measured: a one-rank group with no collective at all took the
            # 1-GPU bench from 35.6 to 47.9 ms/step; 8 queues: 37.0). The setting only takes
            # effect before the first HIP call of a process, so the launchers put it into the
            # environment of the processes they start (parallel/launch.py rank_env); here it
            # is applied only while this process has not touched HIP yet.
            if not _hip_initialised():
                q = pg_hw_queues()
                if q:
                    os.environ["GPU_MAX_HW_QUEUES"] = q
            # the collective streams at high priority: a counter reduction is never queued
            # behind a batch's kernels
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
            torch.cuda.set_device(local)
        # a dead or hung peer turns into an error after this long instead of a silent hang
        kwargs = {"timeout": datetime.timedelta(seconds=float(os.environ.get("TB_COLLECTIVE_TIMEOUT", "600")))}
        if pg_backend == "nccl":
            kwargs["device_id"] = torch.device(f"cuda:{local}")
        if world == 1:
            kwargs["store"] = td.HashStore()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        td.init_process_group(backend=pg_backend, rank=rank, world_size=world, **kwargs)
        ctx.backend = pg_backend
    return ctx


def pg_hw_queues() -> Optional[str]:
    """Hardware queues a process with an RCCL group should start with: TB_PG_HW_QUEUES if set
    ("0": keep the inherited value), else an operator's GPU_MAX_HW_QUEUES, else 8."""
    q = os.environ.get("TB_PG_HW_QUEUES")
    if q is not None:
        return None if q in ("", "0") else q
    return os.environ.get("GPU_MAX_HW_QUEUES") or "8"


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
