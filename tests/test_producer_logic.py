"""Producer message API (ports reference tests/producer_tests.rs: publish_tasks against an in-memory
queue instead of a RabbitMQ container, and every aggregate_results_from_stream case)."""
import json
import os

import pyarrow.parquet as pq

from textblaster_amd.data_model import (Error, Filtered, Success, TextDocument, outcome_from_json,
                                        outcome_to_json)
from textblaster_amd.io.parquet import ParquetWriter
from textblaster_amd.pipeline.executor import PipelineExecutor, build_pipeline_from_config
from textblaster_amd.config import load_pipeline_config
from textblaster_amd.producer_logic import (ProducerArgs, aggregate_results_from_stream, publish_tasks,
                                            run_in_process)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parquet_of(tmp_path, docs):
    p = str(tmp_path / "in.parquet")
    w = ParquetWriter(p)
    w.write_batch(docs)
    w.close()
    return p


def args_for(tmp_path, inp="input"):
    return ProducerArgs(input_file=inp, output_file=str(tmp_path / "out" / "o.parquet"),
                        excluded_file=str(tmp_path / "out" / "e.parquet"), metrics_port=1234)


def test_publish_single(tmp_path):
    inp = parquet_of(tmp_path, [TextDocument("doc-1", "Simple content", "test", metadata={"lang": "en"})])
    q = []
    assert publish_tasks(args_for(tmp_path, inp), q.append) == 1
    v = json.loads(q[0])
    assert v["id"] == "doc-1" and v["content"] == "Simple content" and v["metadata"] == {"lang": "en"}


def test_publish_multiple_and_empty_metadata(tmp_path):
    inp = parquet_of(tmp_path, [TextDocument(i, str(k), "s") for k, i in enumerate("abc")])
    q = []
    assert publish_tasks(args_for(tmp_path, inp), q.append) == 3
    assert {json.loads(m)["id"] for m in q} == {"a", "b", "c"}
    assert all(json.loads(m)["metadata"] == {} for m in q)


def doc(i):
    return TextDocument(i, "exciting content", "test")


def rows(path):
    return pq.read_table(path).num_rows


def test_aggregate_single_success(tmp_path):
    a = args_for(tmp_path)
    assert aggregate_results_from_stream(a, [Success(doc("success-1"))], 1) == (1, 1, 0)
    t = pq.read_table(a.output_file)
    assert t.num_rows == 1 and "success-1" in t.column("id")[0].as_py()


def test_aggregate_single_filtered(tmp_path):
    a = args_for(tmp_path)
    assert aggregate_results_from_stream(a, [Filtered(doc("filtered-1"), "Test filter")], 1) == (1, 0, 1)
    assert pq.read_table(a.excluded_file).column("id")[0].as_py() == "filtered-1"
    assert rows(a.output_file) == 0


def test_aggregate_single_error(tmp_path):
    a = args_for(tmp_path)
    assert aggregate_results_from_stream(a, [Error(doc("error-1"), "Boom", "w123")], 1) == (1, 0, 0)
    assert rows(a.output_file) == 0 and rows(a.excluded_file) == 0


def test_aggregate_mixed_and_batches(tmp_path):
    a = args_for(tmp_path)
    outs = [Success(doc("d1")), Filtered(doc("d2"), "Too short"), Error(doc("d3"), "Crash", "w1")]
    assert aggregate_results_from_stream(a, outs, 3) == (3, 1, 1)
    assert rows(a.output_file) == 1 and rows(a.excluded_file) == 1
    many = [Success(doc(f"s{i}")) for i in range(1234)]
    assert aggregate_results_from_stream(a, many, 1234) == (1234, 1234, 0)
    assert rows(a.output_file) == 1234


def test_aggregate_stream_shorter_than_published(tmp_path):
    a = args_for(tmp_path)
    assert aggregate_results_from_stream(a, [Success(doc("x"))], 5) == (1, 1, 0)  # no hang


def test_outcome_json_roundtrip():
    for o in [Success(doc("a")), Filtered(doc("b"), "r"), Error(doc("c"), "m", "w")]:
        assert outcome_from_json(outcome_to_json(o)) == o


def test_run_in_process(tmp_path):
    docs = [TextDocument("en", "Sometimes, all you need to start the day right is a good coffee and someone "
                               "greeting you smiling.", "s"),
            TextDocument("da", "Hej med dig. Dette er en dansk tekst om hunde og katte.", "s")]
    inp = parquet_of(tmp_path, docs)
    cfg = load_pipeline_config(os.path.join(REPO, "tests", "config", "test_pipeline_config.yaml"))
    ex = PipelineExecutor(build_pipeline_from_config(cfg))
    a = args_for(tmp_path, inp)
    assert run_in_process(a, ex) == (2, 1, 1)
    assert pq.read_table(a.output_file).column("id").to_pylist() == ["en"]
