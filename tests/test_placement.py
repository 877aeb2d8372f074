"""Rank <-> CPU placement (parallel/placement.py): pure functions over a synthetic topology."""
import os

import pytest

from textblaster_amd.parallel import placement


def test_cpulist_roundtrip():
    assert placement.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert placement.format_cpulist([3, 0, 1, 2, 8, 10, 11]) == "0-3,8,10-11"
    assert placement.parse_cpulist("") == []


def _nodes(n_nodes, per):
    return lambda nd: list(range(nd * per, (nd + 1) * per))


def test_eight_gpus_two_numa_nodes():
    """MI355X node shape: 8 GPUs, 4 per socket, 2 x 64 cores: each rank gets 16 cores of its
    GPU's node, disjoint from every other rank's."""
    allowed = list(range(128))
    numa = [0, 0, 0, 0, 1, 1, 1, 1]
    sets = [placement.rank_cpus(r, 8, allowed, numa, _nodes(2, 64)) for r in range(8)]
    for r, s in enumerate(sets):
        assert len(s) == 16
        assert all((c >= 64) == (numa[r] == 1) for c in s)
    assert len(set().union(*map(set, sets))) == 128


def test_unknown_numa_splits_allowed_cpus():
    allowed = list(range(10))
    sets = [placement.rank_cpus(r, 3, allowed, [-1, -1, -1]) for r in range(3)]
    assert sets == [[0, 1, 2], [3, 4, 5], [6, 7, 8]]


def test_more_ranks_than_cpus_share():
    sets = [placement.rank_cpus(r, 4, [0, 1], [-1] * 4) for r in range(4)]
    assert sets == [[0], [1], [0], [1]]


def test_restricted_affinity_is_respected():
    """Only the allowed CPUs of a node count (a cgroup cpuset narrower than the node)."""
    allowed = list(range(8, 16)) + list(range(72, 80))
    sets = [placement.rank_cpus(r, 2, allowed, [0, 1], _nodes(2, 64)) for r in range(2)]
    assert sets == [list(range(8, 16)), list(range(72, 80))]


@pytest.mark.parametrize("ncpu", [1, 2, 4, 8, 16, 32, 64])
def test_thread_budget_within_cpus(ncpu):
    b = placement.thread_budget(ncpu)
    assert b.pool >= 1 and b.read >= 1 and b.write >= 1
    if ncpu >= 4:
        assert b.pool + b.read + b.write == ncpu
    assert b.read <= 8 and b.write <= 4


def test_rank_env_sets_hw_queues(monkeypatch):
    from textblaster_amd.parallel.launch import rank_env

    monkeypatch.delenv("TB_PG_HW_QUEUES", raising=False)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert rank_env(os.environ)["GPU_MAX_HW_QUEUES"] == "8"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert rank_env(os.environ)["GPU_MAX_HW_QUEUES"] == "4"   # an operator's setting is kept
    monkeypatch.setenv("TB_PG_HW_QUEUES", "16")
    assert rank_env(os.environ)["GPU_MAX_HW_QUEUES"] == "16"
    monkeypatch.setenv("TB_PG_HW_QUEUES", "0")
    assert rank_env(os.environ)["GPU_MAX_HW_QUEUES"] == "4"


def test_bind_rank_single_rank_is_a_no_op(monkeypatch):
    monkeypatch.delenv("TB_CPU_BIND", raising=False)
    assert placement.bind_rank(0, 1) is None


def test_kfd_topology_reader_tolerates_missing_sysfs(tmp_path):
    assert placement.kfd_gpu_numa_nodes(str(tmp_path / "none")) == []
    n = tmp_path / "nodes"
    (n / "0").mkdir(parents=True)
    (n / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    (n / "1").mkdir()
    (n / "1" / "properties").write_text("simd_count 1024\nlocation_id 49920\ndomain 0\n")
    assert placement.kfd_gpu_numa_nodes(str(n)) in ([-1], [0], [1])
