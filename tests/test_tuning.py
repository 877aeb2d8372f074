"""Device tuning (pipeline/tuning.py): the one TB_TUNE knob parses into DeviceTuning, rejects
unknown keys and bad values, and reaches the engine and its runner; the runtime knob inventory
stays within the documented set."""
import os
import re

import pytest

from textblaster_amd.pipeline import tuning
from textblaster_amd.pipeline.tuning import DeviceTuning

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defaults_and_overrides():
    t = tuning.parse("")
    assert t == DeviceTuning()
    t = tuning.parse("slots=2, streams=serial,batch_bytes=64m,dict_marks=0,scratch_rate=96:192")
    assert (t.slots, t.streams, t.batch_bytes, t.dict_marks, t.scratch_rate) == (2, "serial", 64 << 20, False,
                                                                                   (96, 192))
    assert tuning.from_env({"TB_TUNE": "long_doc_bytes=8k"}).long_doc_bytes == 8192
    assert t.replace(slots=None, batch_bytes=5).slots == 2 and t.replace(batch_bytes=5).batch_bytes == 5


@pytest.mark.parametrize("spec", ["slot=2", "slots", "gate=yes", "streams=13", "lds_bytes_blk=200000",
                                  "lds_bytes_split=70000"])
def test_rejects_bad_specs(spec):
    with pytest.raises(ValueError):
        tuning.parse(spec)


def test_engine_takes_tuning(monkeypatch):
    from textblaster_amd.config import load_pipeline_config_str
    from textblaster_amd.pipeline.engine import Engine

    monkeypatch.setenv("TB_TUNE", "batch_bytes=1m,gate=0,c4_line_stats=0")
    cfg = load_pipeline_config_str(
        "pipeline:\n  - {type: GopherQualityFilter}\n"
        "  - {type: C4QualityFilter, split_paragraph: true, remove_citations: true, filter_no_terminal_punct: true,"
        " min_num_sentences: 5, min_words_per_line: 3, max_word_length: 1000, filter_lorem_ipsum: true,"
        " filter_javascript: true, filter_curly_bracket: true, filter_policy: true}\n")
    eng = Engine(cfg, backend="emulate", nthreads=2)
    assert eng.max_batch_bytes == 1 << 20 and eng.tune.gate is False
    assert eng.device_runner.line_stats_stage == {}
    # explicit arguments (run --batch-bytes) win over TB_TUNE
    assert Engine(cfg, backend="emulate", nthreads=2, max_batch_bytes=3 << 20).max_batch_bytes == 3 << 20


def test_runtime_knob_inventory():
    """Every runtime TB_* environment variable the package reads is in the documented list
    (README.md "Runtime knobs"); device operating points go through TB_TUNE."""
    documented = {"TB_TUNE", "TB_THREADS", "TB_FAULT_INJECT", "TB_CPU_BIND", "TB_CPU_SET", "TB_DIST_BACKEND",
                  "TB_FORCE_PG", "TB_SHARED_GPU", "TB_COLLECTIVE_TIMEOUT", "TB_HEARTBEAT_TIMEOUT",
                  "TB_PG_HW_QUEUES", "TB_MASTER_PORT", "TB_GPU_ARCH", "TB_HIP_LIB", "TB_LANGID_MODEL",
                  "TB_TOKENIZER_DIR", "TB_LOG", "TB_ROCTX", "TB_TIMELINE", "TB_META_FAST"}
    pat = re.compile(r"""(?:environ(?:\.get)?\(?\[?|getenv\()\s*["'](TB_[A-Z0-9_]+)""")
    found = set()
    for root in ("textblaster_amd", "csrc", "bench.py"):
        base = os.path.join(REPO, root)
        files = [base] if os.path.isfile(base) else [os.path.join(d, f) for d, _, fs in os.walk(base) for f in fs]
        for f in files:
            if f.endswith((".py", ".cpp", ".h", ".hip")):
                found |= set(pat.findall(open(f, encoding="utf-8").read()))
    assert found <= documented, sorted(found - documented)
    assert len(documented) <= 25
    readme = open(os.path.join(REPO, "README.md"), encoding="utf-8").read()
    for k in documented:
        assert f"`{k}`" in readme, k
