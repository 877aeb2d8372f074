"""Process-per-GPU launching without touching HIP in the launcher.

``bench.py --gpus N`` and ``run --gpus N`` start ``torch.distributed.run`` as a *child*
process (never exec: exec from a process that has initialised the GPU takes the machine
down on this pool), so the launcher must decide N before any HIP call. GPUs are counted from
the visibility env vars or the KFD topology in sysfs; ``torch.cuda.device_count()`` is the last
resort (it does not initialise the runtime on this image).
"""
from __future__ import annotations

import glob
import os
import socket
import subprocess
import sys
from typing import List, Optional

_VIS_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _kfd_gpu_nodes() -> Optional[int]:
    nodes = glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")
    if not nodes:
        return None
    n = 0
    for p in nodes:
        try:
            with open(p, encoding="ascii", errors="replace") as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count":
                        n += int(v) > 0
                        break
        except OSError:
            continue
    return n


def visible_gpu_count() -> int:
    """Number of GPUs this process may use, determined without initialising HIP."""
    total = _kfd_gpu_nodes()
    if total is None:
        try:
            import torch

            total = int(torch.cuda.device_count())
        except Exception:  # noqa: BLE001
            total = 0
    for var in _VIS_VARS:
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() not in ("", "-1")]
            total = min(total, len(ids)) if total else len(ids)
    return total


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def strip_flag(argv: List[str], flag: str) -> List[str]:
    """argv without ``flag VALUE`` / ``flag=VALUE`` (so children do not relaunch)."""
    out: List[str] = []
    skip = False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == flag:
            skip = True
            continue
        if a.startswith(flag + "="):
            continue
        out.append(a)
    return out


def spawn_ranks(n: int, target: List[str], port: Optional[int] = None) -> int:
    """Run ``target`` (``[script.py, args...]`` or ``["-m", module, args...]``) on ``n`` local
    ranks under torch.distributed.run as a child process; returns its exit code."""
    port = port or int(os.environ.get("TB_MASTER_PORT", "0")) or free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}"] + list(target)
    return subprocess.call(cmd, env=rank_env(os.environ))


def rank_env(base) -> dict:
    """Environment of the rank processes: set here, in the launcher, because the hardware-queue
    count is read once, at a process's first HIP call (a rank may touch HIP before it builds its
    process group)."""
    from .dist import pg_hw_queues

    env = dict(base)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = "127.0.0.1"
    env.setdefault("OMP_NUM_THREADS", "1")
    q = pg_hw_queues()
    if q:
        env["GPU_MAX_HW_QUEUES"] = q
    return env
