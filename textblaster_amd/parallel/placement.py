"""Rank <-> CPU placement on one node (SURVEY §2.3 DP over GPUs).

The reference scales by adding worker processes on any host, each with its own CPUs
(utils/common.rs:92, worker_logic.rs:241-283). Here the ranks of one node share its CPUs, so
each rank is pinned, before its first HIP call, to the CPUs of its GPU's NUMA node (split evenly
between the ranks whose GPUs sit on that node), and its host threads — Parquet readers, output
encoders and the native pool — share one budget: the size of that CPU set. Threads created
after the binding inherit it, and pinned host buffers allocated afterwards are first touched by
threads of the GPU's own node.

Everything is read from sysfs without initialising HIP:
  /sys/class/kfd/kfd/topology/nodes/*/properties   GPU nodes (simd_count > 0), PCI location
  /sys/bus/pci/devices/<BDF>/numa_node              the GPU's NUMA node
  /sys/devices/system/node/node<N>/cpulist          that node's CPUs
"""
from __future__ import annotations

import dataclasses
import glob
import os
import re
from typing import Callable, Dict, List, Optional, Sequence

_KFD = "/sys/class/kfd/kfd/topology/nodes"


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out: List[int] = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpulist(cpus: Sequence[int]) -> str:
    """[0, 1, 2, 3, 8] -> '0-3,8'"""
    cpus = sorted(set(int(c) for c in cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def _read(path: str) -> Optional[str]:
    try:
        with open(path, encoding="ascii", errors="replace") as f:
            return f.read()
    except OSError:
        return None


def kfd_gpu_numa_nodes(root: str = _KFD) -> List[int]:
    """NUMA node of every GPU of the KFD topology, in node order (the HIP device order); -1 where
    it cannot be read."""
    nodes = []
    for p in glob.glob(os.path.join(root, "*", "properties")):
        m = re.search(r"/(\d+)/properties$", p)
        txt = _read(p)
        if not m or txt is None:
            continue
        props: Dict[str, int] = {}
        for line in txt.splitlines():
            k, _, v = line.partition(" ")
            try:
                props[k] = int(v)
            except ValueError:
                continue
        if props.get("simd_count", 0) <= 0:
            continue
        loc, dom = props.get("location_id"), props.get("domain", 0)
        numa = -1
        if loc is not None:
            bdf = f"{dom:04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 7}"
            v = _read(f"/sys/bus/pci/devices/{bdf}/numa_node")
            if v is not None and v.strip().lstrip("-").isdigit():
                numa = int(v)
        nodes.append((int(m.group(1)), numa))
    return [numa for _, numa in sorted(nodes)]


def node_cpus(node: int) -> List[int]:
    v = _read(f"/sys/devices/system/node/node{node}/cpulist")
    return parse_cpulist(v) if v else []


def visible_gpu_indices(n_total: int) -> List[int]:
    """Physical GPU indices behind the visible device ordinals (HIP/ROCR/CUDA_VISIBLE_DEVICES)."""
    idx = list(range(n_total))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        sel = [x.strip() for x in v.split(",") if x.strip() not in ("", "-1")]
        if all(s.isdigit() for s in sel):
            idx = [idx[int(s)] for s in sel if int(s) < len(idx)]
    return idx


def rank_cpus(local_rank: int, local_world: int, allowed: Sequence[int], gpu_numa: Sequence[int],
              cpus_of_node: Callable[[int], List[int]] = node_cpus) -> List[int]:
    """CPU set of ``local_rank``: the allowed CPUs of its GPU's NUMA node, split evenly (contiguous
    chunks, in rank order) among the local ranks on that node. Ranks whose GPU's node is unknown
    (or whose node has no allowed CPU) split the CPUs no known node claimed. Pure function of its
    arguments (``gpu_numa[r]`` = NUMA node of rank r's GPU, -1 if unknown)."""
    allowed = sorted(set(int(c) for c in allowed))
    numa = [int(gpu_numa[r]) if r < len(gpu_numa) else -1 for r in range(local_world)]
    node_sets: Dict[int, List[int]] = {}
    for nd in sorted(set(n for n in numa if n >= 0)):
        s = sorted(set(cpus_of_node(nd)) & set(allowed))
        if s:
            node_sets[nd] = s
    numa = [n if n in node_sets else -1 for n in numa]
    claimed = set(c for s in node_sets.values() for c in s)
    pool = {nd: s for nd, s in node_sets.items()}
    rest = [c for c in allowed if c not in claimed] or allowed
    pool[-1] = rest
    mine = numa[local_rank]
    peers = [r for r in range(local_world) if numa[r] == mine]
    cpus = pool[mine]
    k, m = peers.index(local_rank), len(peers)
    if len(cpus) < m:  # fewer CPUs than ranks: round-robin, ranks may share
        return [cpus[k % len(cpus)]]
    per = len(cpus) // m
    return cpus[k * per:(k + 1) * per]


@dataclasses.dataclass
class ThreadBudget:
    cpus: int          # CPUs of the rank (the budget)
    pool: int          # native pool threads (assembly, record application, staging copies)
    read: int          # Parquet reader threads
    write: int         # output encoder threads

    def describe(self) -> str:
        return f"{self.cpus} CPUs: pool {self.pool}, readers {self.read}, writers {self.write}"


def thread_budget(ncpu: int) -> ThreadBudget:
    """Reader, writer and pool threads of one rank together within ``ncpu`` CPUs. The end-to-end
    CPU split on the Parquet path (profiles/r8_e2e: read 27.5 s, assembly/pool 23.9 s, encode
    8.7 s, write 2.8 s) sets the shares: ~40 % readers, ~15 % writers, the rest the pool."""
    ncpu = max(1, int(ncpu))
    if ncpu < 4:
        return ThreadBudget(ncpu, 1, 1, 1)
    read = max(1, min(8, round(0.4 * ncpu)))
    write = max(1, min(4, round(0.15 * ncpu)))
    return ThreadBudget(ncpu, max(1, ncpu - read - write), read, write)


_BOUND: Optional[List[int]] = None


def bound_cpus() -> Optional[List[int]]:
    """The CPU set ``bind_rank`` pinned this process to (None: not bound)."""
    return _BOUND


def bind_rank(local_rank: int, local_world: int, force: Optional[bool] = None) -> Optional[List[int]]:
    """Pins this process (and every thread it creates later) to its rank's CPU set. Runs only
    with several local ranks (one rank owns the whole CPU share it was given), unless ``force``
    / TB_CPU_BIND=1; TB_CPU_BIND=0 disables it. Must run before the first HIP call so that the
    runtime's own threads and pinned allocations follow the binding."""
    global _BOUND
    env = os.environ.get("TB_CPU_BIND", "")
    if force is None:
        force = env not in ("", "0")
    if env == "0" or (local_world <= 1 and not force):
        return None
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    gpus = kfd_gpu_numa_nodes()
    if gpus:
        vis = visible_gpu_indices(len(gpus))
        numa = [gpus[vis[r]] if r < len(vis) else -1 for r in range(local_world)]
    else:
        numa = [-1] * local_world
    cpus = rank_cpus(local_rank, local_world, allowed, numa)
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return None
    _BOUND = cpus
    os.environ["TB_CPU_SET"] = format_cpulist(cpus)
    try:  # Arrow's own CPU pool (Parquet decode) within the same budget
        import pyarrow as pa

        pa.set_cpu_count(max(1, len(cpus)))
    except Exception:  # noqa: BLE001 - pyarrow is optional here
        pass
    return cpus
