"""PipelineExecutor and worker outcome mapping (ports reference tests/executor_test.rs and
tests/worker_tests.rs)."""
import asyncio
import json

import pytest

from textblaster_amd.data_model import Filtered, Success, TextDocument
from textblaster_amd.errors import DocumentFiltered, StepError
from textblaster_amd.pipeline.executor import PipelineExecutor, execute_processing_pipeline
from textblaster_amd.pipeline.steps import ProcessingStep
from textblaster_amd.utils import metrics


class Mock(ProcessingStep):
    def __init__(self, name, fn=lambda d: d, should_error=False, message=None):
        self._name, self.fn, self.should_error, self.message = name, fn, should_error, message

    def name(self):
        return self._name

    def process(self, d):
        if self.should_error:
            raise StepError(self._name, DocumentFiltered(d, self.message or "Mock Error"))
        return self.fn(d)


def append(s):
    def f(d):
        d.content += s
        return d
    return f


def mk(id_, content):
    return TextDocument(id=id_, source="test", content=content)


def run(coro):
    return asyncio.run(coro)


def test_empty_executor():
    assert PipelineExecutor([]).steps == []
    assert len(PipelineExecutor([Mock("a"), Mock("b")]).steps) == 2


def test_single_empty_pipeline():
    assert run(PipelineExecutor([]).run_single_async(mk("d", "orig"))).content == "orig"


def test_single_steps():
    ex = PipelineExecutor([Mock("s1", append(" + step1")), Mock("s2", append(" + step2"))])
    assert run(ex.run_single_async(mk("d", "initial"))).content == "initial + step1 + step2"
    assert ex.run_single(mk("d", "initial")).content == "initial + step1 + step2"


def test_step_error_stops_pipeline():
    ran = []
    ex = PipelineExecutor([Mock("step1_ok", append(" + step1")), Mock("error_step", should_error=True,
                                                                      message="Something went wrong"),
                           Mock("step3_never_runs", lambda d: ran.append(1) or d)])
    with pytest.raises(StepError) as ei:
        run(ex.run_single_async(mk("d", "initial")))
    assert ei.value.step_name == "error_step"
    assert not ran


def test_batch_empty():
    assert run(PipelineExecutor([Mock("a")]).run_batch_parallel_async([])) == []


def test_batch_results():
    ex = PipelineExecutor([Mock("s1", append(" + step1")), Mock("s2", append(" + step2"))])
    res = run(ex.run_batch_parallel_async([mk("1", "doc1_initial"), mk("2", "doc2_initial")]))
    assert sorted(r.content for r in res) == ["doc1_initial + step1 + step2", "doc2_initial + step1 + step2"]
    res = ex.run_batch_parallel([mk("1", "a"), mk("2", "b")], max_workers=2)
    assert [r.content for r in res] == ["a + step1 + step2", "b + step1 + step2"]


def test_batch_mixed():
    class Smart(ProcessingStep):
        def name(self):
            return "smart_error_step"

        def process(self, d):
            if "error" in d.id:
                raise DocumentFiltered(d, "Smart error")
            d.content += " + processed_by_smart_step"
            return d

    res = PipelineExecutor([Smart()]).run_batch_parallel([mk("doc_success", "x"), mk("doc_error", "y")])
    assert isinstance(res[0], TextDocument) and "+ processed_by_smart_step" in res[0].content
    assert isinstance(res[1], StepError) and res[1].step_name == "smart_error_step"


# ---- worker outcome mapping -----------------------------------------------------------------

class Identity(ProcessingStep):
    def name(self):
        return "IdentityStep"

    def process(self, d):
        return d


class Filtering(ProcessingStep):
    def name(self):
        return "FilteringStep"

    def process(self, d):
        raise DocumentFiltered(d, "Blocked by test filter")


class Failing(ProcessingStep):
    def name(self):
        return "FailingStep"

    def process(self, d):
        raise StepError("FailingStep", DocumentFiltered(d, "FailingStep"))


def raw(doc):
    return doc.to_json()


def test_worker_success():
    out = execute_processing_pipeline(raw(mk("doc-1", "This is a test")), PipelineExecutor([Identity()]))
    assert isinstance(out, Success) and out.document.id == "doc-1"


def test_worker_bad_json():
    before = metrics.TASK_DESERIALIZATION_ERRORS_TOTAL._value.get()
    assert execute_processing_pipeline(b"not valid json", PipelineExecutor([Identity()])) is None
    assert metrics.TASK_DESERIALIZATION_ERRORS_TOTAL._value.get() == before + 1


def test_worker_filtered():
    out = execute_processing_pipeline(raw(mk("doc-filtered", "Block me")), PipelineExecutor([Filtering()]))
    assert isinstance(out, Filtered)
    assert out.document.id == "doc-filtered" and out.reason == "Blocked by test filter"


def test_worker_nested_step_error_is_none():
    assert execute_processing_pipeline(raw(mk("doc-fail", "x")), PipelineExecutor([Failing()])) is None


def test_worker_chain():
    out = execute_processing_pipeline(raw(mk("doc-chain", "x")), PipelineExecutor([Identity()] * 3))
    assert isinstance(out, Success) and out.document.id == "doc-chain"


def test_task_json_shape():
    o = json.loads(mk("a", "b").to_json())
    assert o == {"id": "a", "content": "b", "source": "test", "added": None, "created": None, "metadata": {}}
