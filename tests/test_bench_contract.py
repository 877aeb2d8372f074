"""bench.py output contract (one JSON line from rank 0 with the driver's keys) on the CPU backend:
one process, and two gloo ranks under torch.distributed.run (global batch = per-rank batch x
world, counters summed over ranks, value = global docs / max-over-ranks seconds)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--backend", "cpu", "--segmentation", "rules", "--docs-per-step", "128", "--pool", "64",
        "--mean-bytes", "512", "--threads", "2"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check(line, steps, warmup, world):
    assert KEYS <= set(line)
    assert line["metric"] == "documents/sec through full C4+Gopher+langID pipeline at 1/2/4/8 MI355X"
    assert line["unit"] == "docs/s" and line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["steps"] == steps and line["warmup"] == warmup
    # dtype = the language-id head that ran: the default v3 model's bf16 MFMA head
    assert line["dtype"] == "bf16" and "bf16 MFMA head" in line["config"]["model"]
    assert line["config"]["global_batch"] == 128 * world
    assert line["config"]["parallelism"] == f"dp{world}"
    # every timed step's documents are counted once: kept + excluded + errors = steps x global batch
    assert line["kept"] + line["excluded"] + line["errors"] == steps * 128 * world
    assert line["value"] > 0 and line["ms_per_step"] > 0
    # value = global docs / timed seconds = global batch / step time
    assert abs(line["value"] * line["ms_per_step"] / 1000.0 - 128 * world) / (128 * world) < 0.01
    assert {"finish", "total"} <= set(line["mean_step_timings"])


def test_bench_single_process_contract():
    line = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1"] + ARGS)
    _check(line, 2, 1, 1)


def test_bench_two_ranks_contract():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1"] + ARGS
    line = _run(cmd, {"MASTER_ADDR": "127.0.0.1"})
    _check(line, 2, 1, 2)


def test_bench_spawns_ranks_itself():
    """``bench.py --gpus N`` without an outer launcher starts N ranks (gloo here) as a child
    torch.distributed.run and reports the whole job."""
    line = _run([sys.executable, "bench.py", "--gpus", "3", "--steps", "2", "--warmup", "1"] + ARGS,
                {"TB_MASTER_PORT": str(_free_port())})
    _check(line, 2, 1, 3)
    assert line["n_gpus"] == 3


def test_bench_refuses_missing_gpus():
    """More GPUs than visible fails loudly instead of silently running one rank."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode != 0 and "--gpus 2" in p.stderr


def test_bench_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"] + ARGS, cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_bench_rejects_zero_steps():
    p = subprocess.run([sys.executable, "bench.py", "--steps", "0"] + ARGS, cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0 and "--steps" in p.stderr
