"""Host assembly cost per document (the Parquet path's metadata JSON + reasons), measured on the
CPU: one batch of the bench corpus with the e2e tool's input metadata ({"url": ...}) runs through
the emulated device path, then BatchState.assemble's pool CPU seconds are read per document.

    python tools/assemble_bench.py [--docs 100000] [--threads 8] [--config config/bench_pipeline.yaml]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=100_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-meta", action="store_true", help="no input metadata column")
    ap.add_argument("--config", default=os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    args = ap.parse_args()
    from textblaster_amd import native
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine
    from textblaster_amd.utils import synth

    h = native.host()
    texts = synth.make_corpus(args.docs, 1024, seed=5)
    data, off = synth.pack(texts)
    meta = None
    if not args.no_meta:
        ms = [b'{"url":"https://example.com/%d"}' % i for i in range(args.docs)]
        mo = np.zeros(args.docs + 1, np.int64)
        np.cumsum([len(m) for m in ms], out=mo[1:])
        meta = (np.frombuffer(b"".join(ms), np.uint8).copy(), mo, None)
    eng = Engine(load_pipeline_config(args.config), backend="emulate", nthreads=args.threads)
    for rep in range(args.reps):
        before = dict(h.pool_cpu_stats())
        t0 = time.perf_counter()
        res = eng.process(data, off, meta)
        wall = time.perf_counter() - t0
        after = dict(h.pool_cpu_stats())
        d = {k: after[k] - before.get(k, 0.0) for k in after if after[k] - before.get(k, 0.0) > 1e-4}
        kept = sum(p.n for p in res.kept) if hasattr(res.kept[0], "n") else None
        print(f"rep {rep}: wall {wall:.2f}s  assemble {d.get('assemble', 0) / args.docs * 1e6:.3f} CPU-us/doc  "
              f"jobs {({k: round(v, 3) for k, v in sorted(d.items())})}  kept parts {len(res.kept)} {kept}")


if __name__ == "__main__":
    main()
