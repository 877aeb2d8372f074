"""Multi-rank runtime pieces on the CPU (gloo): byte-level Parquet concatenation, the live
counter heartbeat (AR1 while ranks own unequal work) and rank-failure detection, the
``run --gpus N`` launcher, and resume after an injected rank failure."""
import os
import subprocess
import sys
import time

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from textblaster_amd.io import pqconcat
from textblaster_amd.parallel.launch import free_port, strip_flag

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOK = os.path.join(REPO, "tests", "fixtures", "tokenizers")
DEFAULT_CFG = os.path.join(REPO, "config", "pipeline_config.yaml")


def test_pqconcat_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    sch = pa.schema([("id", pa.string()), ("text", pa.string()), ("v", pa.int64()), ("m", pa.string())])
    paths, tabs = [], []
    for k, n in enumerate([0, 3, 1000, 17, 40000]):
        t = pa.table({"id": [f"d{k}-{i}" for i in range(n)],
                      "text": ["x" * int(rng.integers(0, 60)) + str(i % 7) for i in range(n)],
                      "v": pa.array(rng.integers(0, 5, n)),
                      "m": [None if i % 3 else "{}" for i in range(n)]}, schema=sch)
        p = str(tmp_path / f"p{k}.parquet")
        pq.write_table(t, p, row_group_size=15000, compression="snappy" if k % 2 else "none")
        paths.append(p)
        tabs.append(t)
    out = str(tmp_path / "all.parquet")
    assert pqconcat.concat(paths, out) == 41020
    got = pq.read_table(out)
    assert got.equals(pa.concat_tables(tabs))
    md = pq.ParquetFile(out).metadata
    assert md.num_rows == 41020
    assert md.num_row_groups == sum(pq.ParquetFile(p).metadata.num_row_groups for p in paths)
    # statistics survive (offsets shifted, the rest of the footer verbatim)
    assert md.row_group(md.num_row_groups - 1).column(0).statistics.max == "d4-39999"


def test_pqconcat_rejects_schema_mismatch(tmp_path):
    a, b = str(tmp_path / "a.parquet"), str(tmp_path / "b.parquet")
    pq.write_table(pa.table({"x": [1]}), a)
    pq.write_table(pa.table({"y": [1]}), b)
    with pytest.raises(pqconcat.ThriftError, match="schema differs"):
        pqconcat.concat([a, b], str(tmp_path / "c.parquet"))


def test_thrift_compact_codec_roundtrip(tmp_path):
    p = str(tmp_path / "z.parquet")
    pq.write_table(pa.table({"a": list(range(100)), "b": [str(i) for i in range(100)]}), p)
    size, start, fmd = pqconcat.read_footer(p)
    with open(p, "rb") as f:
        f.seek(start)
        raw = f.read(size - 8 - start)
    assert pqconcat.encode_struct(fmd) == raw


def test_strip_flag():
    assert strip_flag(["run", "--gpus", "4", "-i", "x", "--gpus=2"], "--gpus") == ["run", "-i", "x"]


_HB_WORKER = r'''
import os, sys, time
import numpy as np
import torch.distributed as td
sys.path.insert(0, os.environ["REPO"])
from textblaster_amd.parallel import dist
from textblaster_amd.parallel.heartbeat import Heartbeat, RankFailure
ctx = dist.init_from_env(backend="gloo")
seen = []
hb = Heartbeat(ctx, 2, interval=0.05, on_global=lambda v: seen.append(v.copy()))
n = 3 + 4 * ctx.rank            # unequal work per rank
for i in range(n):
    hb.update([i + 1, 10 * (i + 1)])
    time.sleep(0.03)
    if os.environ.get("DIE") == str(ctx.rank) and i == 1:
        os._exit(9)
try:
    g = hb.finish([n, 10 * n])
except RankFailure as e:
    print("RANKFAIL", ctx.rank, flush=True)
    os._exit(3)
print("GLOBAL", ctx.rank, int(g[0]), int(g[1]), len(seen) > 0, flush=True)
ctx.destroy()
'''


def _spawn_hb(tmp_path, extra_env=None):
    script = tmp_path / "hb.py"
    script.write_text(_HB_WORKER)
    env = dict(os.environ, REPO=REPO, TB_HEARTBEAT_TIMEOUT="20", TB_COLLECTIVE_TIMEOUT="30", **(extra_env or {}))
    # plain processes (no torch.distributed.run agent, which would kill the survivors itself)
    port = free_port()
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        outs.append((p.returncode, o, e))
    return outs


def test_heartbeat_global_counts_unequal_work(tmp_path):
    outs = _spawn_hb(tmp_path)
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        # rank 0 did 3 units, rank 1 did 7: the final global vector is the sum
        assert "GLOBAL" in o and " 10 100 True" in o, o


def test_heartbeat_detects_dead_rank(tmp_path):
    t0 = time.time()
    outs = _spawn_hb(tmp_path, {"DIE": "1"})
    assert outs[1][0] == 9
    assert outs[0][0] == 3 and "RANKFAIL 0" in outs[0][1], outs[0]
    assert time.time() - t0 < 100


def _corpus(tmp_path):
    from textblaster_amd.data_model import TextDocument
    from textblaster_amd.io.parquet import ParquetWriter
    from textblaster_amd.utils import synth

    texts = synth.make_corpus(2000, 600, seed=11)
    p = str(tmp_path / "in.parquet")
    w = ParquetWriter(p)
    w.write_batch([TextDocument(f"r{i}", t, "syn", metadata={"i": str(i)} if i % 2 else {})
                   for i, t in enumerate(texts)])
    w.close()
    return p


def _cli(tmp_path, inp, tag, *extra, ok=True):
    out, exc = str(tmp_path / f"{tag}.o.parquet"), str(tmp_path / f"{tag}.e.parquet")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", TB_MASTER_PORT=str(free_port()),
               TB_HEARTBEAT_TIMEOUT="30")
    cmd = [sys.executable, "-m", "textblaster_amd", "run", "-i", inp, "-o", out, "-e", exc, "-c", DEFAULT_CFG,
           "--cpu", "--unit-rows", "250", "--tokenizer-dir", TOK, "--log-dir", str(tmp_path / "log")] + list(extra)
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    if ok:
        assert r.returncode == 0, r.stderr[-3000:]
    return r, out, exc


def test_run_gpus_flag_spawns_ranks_and_merges_in_order(tmp_path):
    inp = _corpus(tmp_path)
    _, o1, e1 = _cli(tmp_path, inp, "one")
    r, o4, e4 = _cli(tmp_path, inp, "four", "--gpus", "4")
    assert "Ranks: 4 (cpu)" in r.stdout and "Documents Read: 2000" in r.stdout
    assert pq.read_table(o4).equals(pq.read_table(o1)) and pq.read_table(e4).equals(pq.read_table(e1))
    # one row group per unit: the parts were concatenated, not re-encoded into new groups
    assert pq.ParquetFile(o4).metadata.num_row_groups == 8


def test_rank_failure_then_resume(tmp_path):
    inp = _corpus(tmp_path)
    _, o1, e1 = _cli(tmp_path, inp, "ref")
    work = str(tmp_path / "work")
    r, _, _ = _cli(tmp_path, inp, "ft", "--gpus", "2", "--work-dir", work, "--fault-inject", "rank@2:1", ok=False)
    assert r.returncode != 0
    done = [l for n in os.listdir(work) if n.startswith("manifest") for l in open(os.path.join(work, n))]
    assert 0 < len(done) < 8
    r2, o2, e2 = _cli(tmp_path, inp, "ft", "--gpus", "2", "--work-dir", work, "--resume")
    assert "resumed" in r2.stdout
    assert pq.read_table(o2).equals(pq.read_table(o1)) and pq.read_table(e2).equals(pq.read_table(e1))


def test_block_kernels_reject_oversized_lds_slice():
    """The workgroup launchers refuse a dynamic LDS slice their static LDS would push past the
    CU's 160 KB (argument check only: no HIP call happens, so this runs without a GPU)."""
    import ctypes

    from textblaster_amd import native
    from textblaster_amd.ops import kernels

    lib = native.hip()
    kernels.declare(lib)
    dummy = ctypes.c_void_p(16)
    for lds, want_err in ((160 * 1024, True), (128 * 1024 + 16, True)):
        # (every launcher here returns before any HIP call when the slice is too large)
        rc = lib.tb_stage_analyze_blk(None, dummy, dummy, dummy, dummy, dummy, 1, 1, dummy, dummy, dummy, 0,
                                      dummy, dummy, dummy, dummy, dummy, dummy, lds, None, None, None, 0, 0, 512, None, None, 0,
                                      None, None, None)
        assert (rc != 0) == want_err
        rc = lib.tb_gr_dup_split(None, dummy, 0, dummy, 1, 6, 1, dummy, dummy, 0, dummy, dummy, dummy, dummy,
                                 dummy, dummy, lds, dummy)
        assert (rc != 0) == want_err
        rc = lib.tb_c4_pass_a_blk(None, dummy, dummy, dummy, dummy, 1, 1, dummy, dummy, dummy, 0, dummy, dummy,
                                  dummy, dummy, dummy, dummy, dummy, lds, None, None, None, None, None, None)
        assert (rc != 0) == want_err


def test_metrics_expose_device_counters():
    from textblaster_amd.utils import metrics

    text = metrics.render().decode()
    assert "tb_h2d_bytes_total" in text and "tb_gpu_kernel_seconds" in text


def test_forced_world1_group_on_gloo(monkeypatch):
    """TB_FORCE_PG: a one-rank process group (in-process store, no rendezvous) carries the same
    AR1 / AG1 / BAR calls as a multi-rank job; without it no group is created."""
    from textblaster_amd.parallel import dist

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert dist.init_from_env("gloo").backend is None
    monkeypatch.setenv("TB_FORCE_PG", "1")
    ctx = dist.init_from_env("gloo")
    try:
        assert ctx.backend == "gloo"
        assert list(ctx.all_reduce_sum([1, 2, 3])) == [1, 2, 3]
        assert list(ctx.all_reduce_sum_async([4, 5]).wait()) == [4, 5]
        assert ctx.all_gather_counts([7, 8]).tolist() == [[7, 8]]
        ctx.barrier()
    finally:
        ctx.destroy()


def _corpus_groups(tmp_path, n=3200, per_rg=20):
    """Input with many row groups (the scheduling granularity)."""
    from textblaster_amd.data_model import TextDocument
    from textblaster_amd.io.parquet import ParquetWriter
    from textblaster_amd.utils import synth

    texts = synth.make_corpus(n, 400, seed=12)
    p = str(tmp_path / "in_rg.parquet")
    w = ParquetWriter(p)
    for s in range(0, n, per_rg):
        w.write_batch([TextDocument(f"r{i}", texts[i], "syn") for i in range(s, min(n, s + per_rg))])
    w.close()
    assert pq.ParquetFile(p).metadata.num_row_groups == n // per_rg
    return p


def _rank_stats(stdout):
    import ast

    line = next(ln for ln in stdout.splitlines() if "Units per rank:" in ln)
    units = ast.literal_eval(line.split("Units per rank:")[1].split("|")[0].strip())
    busy = ast.literal_eval(line.split("busy seconds per rank:")[1].strip())
    return units, busy


def test_dynamic_schedule_balances_a_straggler(tmp_path, monkeypatch):
    """Ranks pull row groups from a shared cursor (the reference's competing consumers): with rank 1
    sleeping after every unit, the static byte-balanced split leaves rank 1 finishing long after
    rank 0, the dynamic schedule gives rank 1 fewer groups and both finish within 10 %; the
    outputs are identical to the one-rank run either way."""
    inp = _corpus_groups(tmp_path)
    _, o1, e1 = _cli(tmp_path, inp, "one", "--unit-rows", "20")
    flags = ("--gpus", "2", "--unit-rows", "20", "--read-threads", "1", "--claim-ahead", "1",
             "--fault-inject", "slow@0.03:1")
    r_s, o_s, e_s = _cli(tmp_path, inp, "static", *flags, "--schedule", "static")
    r_d, o_d, e_d = _cli(tmp_path, inp, "dyn", *flags, "--schedule", "dynamic")
    for o, e in ((o_s, e_s), (o_d, e_d)):
        assert pq.read_table(o).equals(pq.read_table(o1)) and pq.read_table(e).equals(pq.read_table(e1))
    su, sb = _rank_stats(r_s.stdout)
    du, db = _rank_stats(r_d.stdout)
    print("static", su, sb, "dynamic", du, db)
    assert sum(su) == sum(du) == 160
    assert su[0] == su[1], su                                   # static: an equal split ...
    assert sb[1] > sb[0], (su, sb)                              # ... that the straggler finishes last
    assert du[1] < 0.75 * du[0], (du, db)                       # dynamic: it takes clearly fewer groups
    # (wall-clock balance is reported, not gated: a loaded CI machine skews the sleeps)
    print("dynamic busy-time spread", abs(db[0] - db[1]) / max(db))


def test_claim_gate_of_one_with_many_reader_threads(tmp_path, monkeypatch):
    """--claim-ahead 1 (the reference's basic_qos prefetch of 1) with 4 reader threads: the
    reader takes the next group only after yielding the previous one, so a gate smaller than its
    decode window cannot starve it; the outputs equal the one-rank run."""
    inp = _corpus_groups(tmp_path)
    _, o1, e1 = _cli(tmp_path, inp, "one", "--unit-rows", "20")
    r, o, e = _cli(tmp_path, inp, "gate1", "--gpus", "2", "--unit-rows", "20", "--read-threads", "4",
                   "--claim-ahead", "1", "--schedule", "dynamic")
    assert pq.read_table(o).equals(pq.read_table(o1)) and pq.read_table(e).equals(pq.read_table(e1))
    units, _ = _rank_stats(r.stdout)
    assert sum(units) == 160


def test_run_eight_cpu_ranks_pinned_and_identical(tmp_path):
    """`run --gpus 8 --backend cpu` (gloo, dynamic schedule): every rank is pinned to its own CPU
    set with a thread budget inside it (parallel/placement.py), the summary reports each rank's
    set and thread counts, and the outputs are byte-identical to the one-rank run."""
    inp = _corpus(tmp_path)
    _, o1, e1 = _cli(tmp_path, inp, "one8")
    r, o8, e8 = _cli(tmp_path, inp, "eight", "--gpus", "8", "--unit-rows", "125")
    assert "Ranks: 8 (cpu)" in r.stdout
    assert pq.read_table(o8).equals(pq.read_table(o1)) and pq.read_table(e8).equals(pq.read_table(e1))
    line = next(ln for ln in r.stdout.splitlines() if "CPU sets per rank:" in ln)
    entries = line.split("CPU sets per rank:")[1].split(";")
    assert len(entries) == 8, line
    import os as _os

    ncpu = len(_os.sched_getaffinity(0))
    if ncpu >= 8:
        sets = []
        for e in entries:
            assert "cpus " in e and "not pinned" not in e, line
            a, b = e.split("cpus ")[1].split(" ")[0].split("-")
            sets.append(set(range(int(a), int(b) + 1)))
        for i in range(8):  # disjoint sets
            for j in range(i + 1, 8):
                assert not (sets[i] & sets[j]), line
