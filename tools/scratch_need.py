"""Measures the HBM scratch arena the document kernels really use, per text byte.

Runs the host port of the device algorithms (docproc.h via emulate_stage / emulate_c4, with no
LDS slice, so every working array lands in the arena: an upper bound for the device) over
adversarial shapes -- one-letter words, empty lines, long lines, multi-byte code points,
paragraph breaks -- at several lengths, and prints the largest (peak - 4096) / (len + 64) per
shape next to devplan.h kScratchPerByte. A document whose need exceeds the reservation is
delegated to the CPU (DOC_OVERFLOW), so this is the number that sizes the reservation.

    python tools/scratch_need.py [--config config/bench_pipeline.yaml] [--lengths 200,4096,65536,1048576]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "prose": lambda rng, n: " ".join(rng.choice(["the", "quick", "brown", "fox", "jumps", "over", "lazy",
                                                   "dog.", "and", "then", "some", "more", "words,"], n // 4)),
    "one_letter_words": lambda rng, n: " ".join(chr(97 + int(c)) for c in rng.integers(0, 26, n // 2)),
    "repeated_word": lambda rng, n: "a " * (n // 2),
    "empty_lines": lambda rng, n: "\n" * n,
    "short_lines": lambda rng, n: "a\n" * (n // 2),
    "paragraphs": lambda rng, n: "a b.\n\n" * (n // 6),
    "sentences": lambda rng, n: "A b. " * (n // 5),
    "two_byte": lambda rng, n: " ".join("é" * int(k) for k in rng.integers(1, 4, n // 5)),
    "four_byte": lambda rng, n: "\U0001F600" * (n // 4),
    "punctuation": lambda rng, n: ". , ; ! ? " * (n // 10),
    "citations": lambda rng, n: "x [1] " * (n // 6),
    "distinct_words": lambda rng, n: " ".join("w%x" % i for i in range(n // 6)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config/bench_pipeline.yaml")
    ap.add_argument("--lengths", default="200,4096,65536,1048576")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.models.langid import load_default
    from textblaster_amd import native
    from textblaster_amd.pipeline.plan import build_plan
    from textblaster_amd.utils import synth

    host = native.host()
    cfg = load_pipeline_config(a.config)
    steps = [host.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    lid = load_default().native()
    c4 = [i for i, s in enumerate(cfg.pipeline) if s.type == "C4QualityFilter"]
    gr = [steps[i] for i, s in enumerate(cfg.pipeline) if s.type == "GopherRepetitionFilter"]
    # k_gr_dup_split task count (device.py gr_split): orders + duplicated lines + paragraphs
    split_tasks = (gr[0].n_dup + gr[0].n_top + 2) if gr else 0
    rng = np.random.default_rng(5)
    rows = {}
    host.set_scratch_probe(True)
    try:
        for name, make in SHAPES.items():
            rows[name] = {}
            for n in [int(x) for x in a.lengths.split(",")]:
                data, off = synth.pack([make(rng, n)])
                host.scratch_need(True)
                for idx in plan.stages:
                    r0, f0 = host.emulate_stage(steps, idx, data, off, 1, lid, 0)
                for i in c4:
                    host.emulate_c4(steps[i], data, off, 1, 0)
                one, _ = host.scratch_need(True)
                split = 0.0
                if split_tasks:
                    # documents over the split sizes run the intra-document split on the device
                    for idx in plan.stages:
                        r0, f0 = host.emulate_stage(steps, idx, data, off, 1, lid, 0)
                        r1, f1 = host.emulate_stage(steps, idx, data, off, 1, lid, 0, split_tasks=split_tasks)
                        assert (r0 == r1).all() and (f0 == f1).all(), f"split records differ: {name} {n}"
                    split, _ = host.scratch_need(True)
                rows[name][n] = {"one_pass": one, "split": split}
                print(f"{name:18s} {n:8d} B  one pass {one:7.2f}  split {split:7.2f} B/byte", flush=True)
    finally:
        host.set_scratch_probe(False)
    worst1 = max(v["one_pass"] for r in rows.values() for v in r.values())
    worst2 = max(v["split"] for r in rows.values() for v in r.values())
    print(f"worst one pass {worst1:.2f} B/byte (reserved {host.SCRATCH_PER_BYTE}); "
          f"worst split {worst2:.2f} B/byte (reserved {host.SCRATCH_PER_BYTE_SPLIT})")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"config": a.config, "shapes": rows, "worst_one_pass": worst1, "worst_split": worst2,
                       "kScratchPerByte": host.SCRATCH_PER_BYTE,
                       "kScratchPerByteSplit": host.SCRATCH_PER_BYTE_SPLIT}, f, indent=1)


if __name__ == "__main__":
    main()
