"""The device path on two ranks (reference tests/full_pipeline_test.rs:78-215
runs separate worker and producer processes end to end): ``run --gpus 2`` starts two processes
under torch.distributed.run, both run their HIP engines on GPU 0 (TB_SHARED_GPU=1, gloo for the
counter collectives — RCCL needs one GPU per rank), each filters its byte-balanced share of
the row-group units in small device batches, and rank 0 merges the per-unit part files. The
merged kept / excluded files must equal the one-rank device run's byte for byte, content,
metadata and order. Needs an MI355X; one functional run (2 ranks on one card)."""
import os
import subprocess
import sys

import pyarrow.parquet as pq
import pytest

from textblaster_amd.data_model import TextDocument
from textblaster_amd.io.parquet import ParquetWriter
from textblaster_amd.parallel.launch import free_port
from textblaster_amd.utils import synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOK = os.path.join(REPO, "tests", "fixtures", "tokenizers")
DEFAULT_CFG = os.path.join(REPO, "config", "pipeline_config.yaml")


def _run(tmp_path, inp, tag, *extra, env_extra=None):
    out, exc = str(tmp_path / f"{tag}.o.parquet"), str(tmp_path / f"{tag}.e.parquet")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", TB_MASTER_PORT=str(free_port()),
               TB_TUNE=f"batch_bytes={256 << 10}", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "textblaster_amd", "run", "-i", inp, "-o", out, "-e", exc, "-c", DEFAULT_CFG,
           "--backend", "cuda", "--unit-rows", "400", "--tokenizer-dir", TOK,
           "--log-dir", str(tmp_path / "log")] + list(extra)
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return r, out, exc


def test_two_rank_device_run_equals_one_rank(tmp_path):
    texts = synth.make_corpus(3000, 900, seed=21)
    inp = str(tmp_path / "in.parquet")
    w = ParquetWriter(inp)
    w.write_batch([TextDocument(f"d{i}", t, "syn", metadata={"k": str(i)} if i % 3 == 0 else {})
                   for i, t in enumerate(texts)])
    w.close()
    _, o1, e1 = _run(tmp_path, inp, "one")
    r, o2, e2 = _run(tmp_path, inp, "two", "--gpus", "2", env_extra={"TB_SHARED_GPU": "1"})
    assert "Ranks: 2" in r.stdout and "Documents Read: 3000" in r.stdout, r.stdout[-2000:]
    k1, x1 = pq.read_table(o1), pq.read_table(e1)
    assert k1.num_rows + x1.num_rows == 3000 and k1.num_rows > 0 and x1.num_rows > 0
    assert pq.read_table(o2).equals(k1)
    assert pq.read_table(e2).equals(x1)
