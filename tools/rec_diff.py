"""Device vs host-emulation stage records, document by document (debugging aid).

    python tools/rec_diff.py [--corpus hard|bench] [--env K=V ...]

Runs one batch through DeviceRunner (GPU) and EmulatedRunner (host port of the same kernels),
prints every document whose stage records differ: its length, word count and the differing fields.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--corpus", default="hard")
    ap.add_argument("--config", default=os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    ap.add_argument("--limit", type=int, default=20)
    args = ap.parse_args()
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine
    from textblaster_amd.utils import synth

    if args.corpus == "hard":
        from test_gpu_e2e import _hard_corpus

        texts = _hard_corpus()
    else:
        texts = synth.make_corpus(20000, 1024, seed=5)
    data, off = synth.pack(texts)
    cfg = load_pipeline_config(args.config)
    dev = Engine(cfg, backend="cuda")
    emu = Engine(cfg, backend="emulate", nthreads=8)
    a = dev.device_runner.submit(data, off).wait()
    b = emu.device_runner.run(data, off)
    nd = len(off) - 1
    bad = 0
    for s, (ra, rb) in enumerate(zip(a.stage_recs, b.stage_recs)):
        ra, rb = np.asarray(ra), np.asarray(rb)
        width = len(ra) // nd
        w_total, layout = dev.device_runner.stage_layout[s]
        for d in range(nd):
            if a.flags[d] or b.flags[d]:
                continue
            xa = ra.reshape(-1)[:]  # records are laid out per step: prefix * ndocs + doc * width
            diffs = []
            for (step, wd, prefix) in layout:
                va = ra[prefix * nd + d * wd: prefix * nd + (d + 1) * wd]
                vb = rb[prefix * nd + d * wd: prefix * nd + (d + 1) * wd]
                if not np.array_equal(va, vb):
                    diffs.append((step, [(i, int(x), int(y)) for i, (x, y) in enumerate(zip(va, vb)) if x != y]))
            if diffs:
                bad += 1
                if bad <= args.limit:
                    print(f"stage {s} doc {d} bytes {off[d + 1] - off[d]} words ~{len(texts[d].split())}: {diffs}")
    print(f"{bad} document records differ of {nd}")


if __name__ == "__main__":
    main()
