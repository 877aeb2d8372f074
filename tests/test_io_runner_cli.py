"""Parquet I/O (ports reference tests/parquet_io_test.rs), the end-to-end runner (the in-process
equivalent of tests/full_pipeline_test.rs and producer_tests.rs aggregation cases), checkpoint /
resume, multi-rank sharding over gloo, and the CLI."""
import datetime as dt
import json
import os
import subprocess
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from textblaster_amd import cli
from textblaster_amd.data_model import TextDocument
from textblaster_amd.errors import ConfigError
from textblaster_amd.io.parquet import OUTPUT_SCHEMA, ParquetInputConfig, ParquetReader, ParquetWriter
from textblaster_amd.runner import RunConfig, read_manifests, run
from textblaster_amd.utils import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOK = os.path.join(REPO, "tests", "fixtures", "tokenizers")
TEST_CFG = os.path.join(REPO, "tests", "config", "test_pipeline_config.yaml")
DEFAULT_CFG = os.path.join(REPO, "config", "pipeline_config.yaml")


def write_docs(path, docs):
    w = ParquetWriter(str(path))
    w.write_batch(docs)
    w.close()
    return str(path)


def read_docs(path):
    return list(ParquetReader(ParquetInputConfig(str(path), batch_size=10)).read_documents())


# ---- parquet ----------------------------------------------------------------------------------

def test_roundtrip(tmp_path):
    added = dt.date(2024, 1, 1)
    cr = (dt.datetime(2024, 1, 1, 12), dt.datetime(2024, 1, 2, 12))
    docs = [TextDocument("doc1", "Hello Parquet!", "file1.txt", added, cr, {"key1": "val1"}),
            TextDocument("doc2", "Test doc 2", "file2.txt"),
            TextDocument("doc3", "Final doc", "file3.txt", added, cr, {"lang": "en"})]
    p = write_docs(tmp_path / "rt.parquet", docs)
    got = sorted(read_docs(p), key=lambda d: d.id)
    assert got == docs


def test_schema_and_quirks(tmp_path):
    p = write_docs(tmp_path / "s.parquet", [TextDocument("a", "x", "s", dt.date(2024, 1, 1), None, {})])
    t = pq.read_table(p)
    assert t.schema.equals(OUTPUT_SCHEMA)
    # Date32 carries days-from-CE (the reference's encoding), metadata is null when empty
    assert t.column("added").cast(pa.int32())[0].as_py() == dt.date(2024, 1, 1).toordinal()
    assert t.column("metadata")[0].as_py() is None
    assert pq.ParquetFile(p).metadata.row_group(0).column(0).compression == "UNCOMPRESSED"


def test_missing_column(tmp_path):
    p = write_docs(tmp_path / "m.parquet", [TextDocument("missing", "missing column", "dummy")])
    r = ParquetReader(ParquetInputConfig(p, id_column="nonexistent_id"))  # lazy, like the reference
    with pytest.raises(ConfigError, match="Required column 'nonexistent_id' not found in schema."):
        list(r.read_documents())


def test_text_column_type(tmp_path):
    p = str(tmp_path / "bad.parquet")
    pq.write_table(pa.table({"id": ["a"], "text": pa.array([1], pa.int64())}), p)
    with pytest.raises(ConfigError, match="must be Utf8 or LargeUtf8, found: Int64"):
        ParquetReader(ParquetInputConfig(p)).open()


def test_foreign_input_shapes(tmp_path):
    """Minimal input (no source/added/created/metadata), LargeUtf8 text, null rows, HTML entities,
    timestamp 'added', invalid metadata JSON."""
    p = str(tmp_path / "f.parquet")
    ts = pa.array([dt.datetime(2024, 3, 1, 5), None, None, None], pa.timestamp("ms"))
    pq.write_table(pa.table({
        "id": ["a", "b", None, "d"],
        "text": pa.array(["Fish &amp; chips &lt;3 &#x41;", None, "orphan", "ok"], pa.large_string()),
        "added": ts,
        "metadata": ['{"k":"v"}', None, None, "not json"],
    }), p)
    results = list(ParquetReader(ParquetInputConfig(p)).iter_documents_results())
    assert results[0].content == "Fish & chips <3 A" and results[0].source == p
    assert results[0].added == dt.date(2024, 3, 1) and results[0].metadata == {"k": "v"}
    assert "null text column" in str(results[1]) and "null id column" in str(results[2])
    assert results[3].metadata == {}
    # batched path: nulls are counted as errors, the rest is HTML-decoded
    b = next(ParquetReader(ParquetInputConfig(p)).iter_batches())
    assert b.n == 2 and b.error_rows == 2
    assert bytes(b.text[0][b.text[1][0]:b.text[1][1]]).decode() == "Fish & chips <3 A"


# ---- end-to-end -------------------------------------------------------------------------------

def e2e_docs():
    return [
        TextDocument("doc1_en", "Sometimes, all you need to start the day right is a good coffee and someone greeting "
                                "you smiling.", "test_source", metadata={"language": "eng"}),
        TextDocument("doc2_fr", "Ceci est un document en français.", "test_source", metadata={"language": "fr"}),
        TextDocument("doc3_en_implicit", "Another valid English text without any specific language hint in metadata.",
                     "test_source"),
    ]


def test_full_pipeline_e2e(tmp_path):
    inp = write_docs(tmp_path / "in.parquet", e2e_docs())
    out, exc = str(tmp_path / "out" / "o.parquet"), str(tmp_path / "out" / "e.parquet")
    st = run(RunConfig(inp, out, exc, TEST_CFG, backend="cpu"))
    assert (st.docs, st.kept, st.excluded, st.errors) == (3, 2, 1, 0)
    kept = {d.id: d for d in read_docs(out)}
    excl = {d.id: d for d in read_docs(exc)}
    src = {d.id: d for d in e2e_docs()}
    assert set(kept) == {"doc1_en", "doc3_en_implicit"} and set(excl) == {"doc2_fr"}
    for k, d in list(kept.items()) + list(excl.items()):
        assert d.content == src[k].content
    assert kept["doc1_en"].metadata["Detected language"] == "English"
    assert kept["doc1_en"].metadata["language"] == "eng"


def test_empty_outputs_created(tmp_path):
    inp = write_docs(tmp_path / "in.parquet", [e2e_docs()[1]])
    out, exc = str(tmp_path / "o.parquet"), str(tmp_path / "e.parquet")
    st = run(RunConfig(inp, out, exc, TEST_CFG, backend="cpu"))
    assert st.kept == 0 and st.excluded == 1
    assert pq.read_table(out).num_rows == 0 and pq.read_table(exc).num_rows == 1


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    d = tmp_path_factory.mktemp("corpus")
    texts = synth.make_corpus(3000, 700, seed=7)
    docs = [TextDocument(f"r{i}", t, "syn", metadata={"i": str(i)} if i % 2 else {}) for i, t in enumerate(texts)]
    return write_docs(d / "in.parquet", docs)


def _run(corpus, tmp_path, tag, **kw):
    out, exc = str(tmp_path / f"{tag}.o.parquet"), str(tmp_path / f"{tag}.e.parquet")
    kw.setdefault("unit_rows", 500)
    st = run(RunConfig(corpus, out, exc, DEFAULT_CFG, backend="cpu", tokenizer_dir=TOK, **kw))
    return st, pq.read_table(out), pq.read_table(exc)


def test_checkpoint_equals_direct_and_resume(corpus, tmp_path):
    st0, o0, e0 = _run(corpus, tmp_path, "direct")
    assert st0.docs == 3000 and st0.kept + st0.excluded == 3000 and st0.kept > 0
    assert o0.column("id").to_pylist() == sorted(o0.column("id").to_pylist(), key=lambda s: int(s[1:]))
    work = str(tmp_path / "work")
    st1, o1, e1 = _run(corpus, tmp_path, "ck", checkpoint=True, work_dir=work, keep_parts=True)
    assert o1.equals(o0) and e1.equals(e0)
    # simulate a crash after 2 units: drop the rest of the manifest and the merged outputs
    man = os.path.join(work, "manifest.rank0.jsonl")
    lines = open(man).read().splitlines()
    assert len(lines) == st1.units == 6
    with open(man, "w") as f:
        f.write("\n".join(lines[:2]) + "\n" + lines[2][: len(lines[2]) // 2])  # torn last line
    assert sorted(read_manifests(work)) == [0, 1]
    st2, o2, e2 = _run(corpus, tmp_path, "ck", resume=True, work_dir=work)
    assert st2.units_skipped == 2 and st2.units == 4
    assert (st2.docs, st2.kept, st2.excluded) == (st0.docs, st0.kept, st0.excluded)
    assert o2.equals(o0) and e2.equals(e0)
    assert not os.path.exists(work)


def test_resume_rejects_other_input(corpus, tmp_path):
    work = str(tmp_path / "w2")
    _run(corpus, tmp_path, "a", checkpoint=True, work_dir=work, keep_parts=True)
    with pytest.raises(Exception, match="different input"):
        _run(corpus, tmp_path, "a", resume=True, work_dir=work, unit_rows=400)


def test_two_ranks_gloo(corpus, tmp_path):
    """world_size 2 over gloo (torch.distributed.run): shards by row group units, merges parts in
    input order, all-reduces counters; output identical to the single-rank run."""
    _, o0, e0 = _run(corpus, tmp_path, "single")
    out, exc = str(tmp_path / "dp.o.parquet"), str(tmp_path / "dp.e.parquet")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29631", "-m", "textblaster_amd", "run", "-i", corpus,
           "-o", out, "-e", exc, "-c", DEFAULT_CFG, "--backend", "cpu", "--unit-rows", "500", "--tokenizer-dir", TOK,
           "--log-dir", str(tmp_path / "log")]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Documents Read: 3000" in r.stdout
    assert pq.read_table(out).equals(o0) and pq.read_table(exc).equals(e0)
    import glob

    assert glob.glob(str(tmp_path / "log" / "producer.rank1.log.*-*-*"))


# ---- CLI --------------------------------------------------------------------------------------

def test_cli_defaults():
    a = cli.build_parser().parse_args(["producer", "-i", "input.parquet"])
    assert (a.input_file, a.text_column, a.id_column) == ("input.parquet", "text", "id")
    assert a.amqp_addr == "amqp://guest:guest@localhost:5672/%2f"
    assert (a.task_queue, a.results_queue, a.prefetch_count) == ("task_queue", "results_queue", 10)
    assert (a.output_file, a.excluded_file, a.metrics_port) == ("output_processed.parquet", "excluded.parquet", None)


def test_cli_all_args():
    a = cli.build_parser().parse_args(["producer", "-i", "input.parquet", "--text-column", "content", "--id-column",
                                       "doc_id", "-a", "amqp://user:pass@host:port/vhost", "-q", "my_tasks", "-r",
                                       "my_results", "-o", "processed.parquet", "-e", "errors.parquet",
                                       "--metrics-port", "9090"])
    assert (a.text_column, a.id_column, a.task_queue, a.results_queue) == ("content", "doc_id", "my_tasks", "my_results")
    assert (a.output_file, a.excluded_file, a.metrics_port) == ("processed.parquet", "errors.parquet", 9090)


def test_cli_errors():
    with pytest.raises(SystemExit) as ei:
        cli.build_parser().parse_args(["producer"])
    assert ei.value.code == 2
    with pytest.raises(SystemExit):
        cli.build_parser().parse_args(["producer", "-i", "x", "--metrics-port", "not_a_number"])
    with pytest.raises(SystemExit):
        cli.build_parser().parse_args(["producer", "-i", "x", "--metrics-port", "70000"])


def test_cli_validate_config(tmp_path, capsys):
    assert cli.main(["worker", "--validate-config", "-c", TEST_CFG]) == 0
    assert f"Configuration '{TEST_CFG}' is valid." in capsys.readouterr().out
    bad = tmp_path / "bad.yaml"
    bad.write_text("pipeline:\n  - type: TokenCounter\n    tokenizer_name: ''\n")
    assert cli.main(["validate-config", str(bad)]) == 1
    assert f"Configuration '{bad}' is invalid: " in capsys.readouterr().err


def test_cli_run_and_worker(tmp_path, capsys):
    inp = write_docs(tmp_path / "in.parquet", e2e_docs())
    out, exc = str(tmp_path / "o.parquet"), str(tmp_path / "e.parquet")
    rc = cli.main(["-i", inp, "-o", out, "-e", exc, "-c", TEST_CFG, "--backend", "cpu", "--log-dir",
                   str(tmp_path / "log")])
    assert rc == 0
    assert "Kept (output): 2" in capsys.readouterr().out
    import glob

    (logf,) = glob.glob(str(tmp_path / "log" / "producer.log.*-*-*"))  # daily file (reference layout)
    lines = [json.loads(l) for l in open(logf)]
    assert lines and {"timestamp", "level", "fields", "target"} <= set(lines[0])
    # worker: task JSON lines in, outcome JSON lines out (reference message formats)
    tasks = "".join(d.to_json().decode() + "\n" for d in e2e_docs()) + "not json\n"
    r = subprocess.run([sys.executable, "-m", "textblaster_amd", "worker", "-c", TEST_CFG, "--log-dir",
                        str(tmp_path / "log")], input=tasks, capture_output=True, text=True,
                       env=dict(os.environ, PYTHONPATH=REPO), timeout=300)
    assert r.returncode == 0, r.stderr
    outs = [json.loads(l) for l in r.stdout.splitlines()]
    assert [next(iter(o)) for o in outs] == ["Success", "Filtered", "Success"]
    assert outs[1]["Filtered"]["document"]["id"] == "doc2_fr"


def test_run_twice_is_byte_identical(corpus, tmp_path):
    """Determinism: two runs over the same input write identical Parquet files."""
    outs = []
    for k in range(2):
        o, e = str(tmp_path / f"o{k}.parquet"), str(tmp_path / f"e{k}.parquet")
        run(RunConfig(corpus, o, e, DEFAULT_CFG, backend="emulate", unit_rows=700, threads=2, tokenizer_dir=TOK))
        outs.append((open(o, "rb").read(), open(e, "rb").read()))
    assert outs[0] == outs[1]


def test_html_decode_backend_is_validated(tmp_path):
    """`run --html-decode` accepts cpu | gpu only; an unknown value is a PipelineError (the GPU
    decoder itself is covered by tests/test_gpu_html.py)."""
    import pytest as _pytest

    from textblaster_amd.data_model import TextDocument as _Doc
    from textblaster_amd.errors import PipelineError
    from textblaster_amd.io.parquet import ParquetWriter as _W
    from textblaster_amd.runner import RunConfig as _RC, run as _run

    inp = str(tmp_path / "in.parquet")
    w = _W(inp)
    w.write_batch([_Doc("a", "x &amp; y", "s")])
    w.close()
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config", "bench_pipeline.yaml")
    with _pytest.raises(PipelineError):
        _run(_RC(inp, str(tmp_path / "o.parquet"), str(tmp_path / "e.parquet"), cfg, backend="cpu",
                 html_decode="bogus"))


def test_daily_log_handler_rolls_over(tmp_path):
    """Reference tracing_appender::rolling::daily: one file per date, <name>.log.<YYYY-MM-DD>."""
    import logging

    day = ["2026-10-16"]
    h = cli.DailyFileHandler(str(tmp_path), "producer", today=lambda: day[0])
    h.setFormatter(logging.Formatter("%(message)s"))
    rec = lambda m: logging.LogRecord("t", logging.INFO, __file__, 1, m, None, None)  # noqa: E731
    h.emit(rec("a"))
    day[0] = "2026-10-17"
    h.emit(rec("b"))
    h.emit(rec("c"))
    h.close()
    assert open(tmp_path / "producer.log.2026-10-16").read() == "a\n"
    assert open(tmp_path / "producer.log.2026-10-17").read() == "b\nc\n"


