"""Debug aid: the bad-words device test's batch on the GPU vs the CPU oracle, first differences."""
import os
import pathlib
import random
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_badwords_device as T  # noqa: E402
from textblaster_amd.config import load_pipeline_config_str  # noqa: E402
from textblaster_amd.pipeline.engine import Engine  # noqa: E402
from textblaster_amd.utils import synth  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
T.write_lists(tmp)
texts = T.corpus(3000, seed=3) + synth.make_corpus(500, 600, seed=4)
meta = [(b'{"language":"%s"}' % random.Random(i).choice([b"en", b"da", b"ja", b"zz"])) if i % 4 else b""
        for i in range(len(texts))]
data, off = synth.pack(texts)
md = np.frombuffer(b"".join(meta), np.uint8).copy()
mo = np.zeros(len(meta) + 1, np.int64)
np.cumsum([len(m) for m in meta], out=mo[1:])
mv = np.array([1 if m else 0 for m in meta], np.uint8)
for with_c4 in (False, True):
    cfg = load_pipeline_config_str(T.cfg_yaml(tmp, "en", 0.0, with_c4))
    kw = dict(keep_reasons=True, badwords_dir=str(tmp))
    eng = Engine(cfg, backend=sys.argv[1] if len(sys.argv) > 1 else "cuda", **kw)
    a = eng.process(data, off, (md, mo, mv))
    b = Engine(cfg, backend="cpu", segmentation="icu", **kw).process(data, off, (md, mo, mv))
    ra, rb = T.rows_out(a), T.rows_out(b)
    bad = [k for k in ra if ra[k] != rb.get(k)]
    print("with_c4", with_c4, "status eq", np.array_equal(a.status, b.status), "diffs", len(bad), "delegated",
          a.n_delegated, flush=True)
    for k in bad[:3]:
        ta, tb = ra[k][1], rb[k][1]
        print(" doc", k, "len dev", len(ta), "len cpu", len(tb), "zeros in dev", ta.count(0), "orig len",
              off[k + 1] - off[k], "dict", eng.h.has_dict_script(texts[k]), flush=True)
        print("  dev:", ta[:120], "\n  cpu:", tb[:120])
