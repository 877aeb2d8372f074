"""Debug helper: GopherRepetition records of selected fuzz documents, device vs host emulation,
under the current environment (TB_* settings). python tools/gr_diff.py IDX [IDX ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from gpu_fuzz_corpus import fuzz_docs

    from textblaster_amd import native
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.models.langid import load_default
    from textblaster_amd.pipeline.device import DeviceRunner
    from textblaster_amd.pipeline.plan import build_plan
    from textblaster_amd.utils import synth

    idx = [int(a) for a in sys.argv[1:]]
    texts = fuzz_docs(max(idx) + 1)
    h = native.host()
    cfg = load_pipeline_config(os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    steps = [h.make_step(s.native_dict()) for s in cfg.pipeline]
    plan = build_plan(cfg)
    lid = load_default()
    runner = DeviceRunner(steps, plan, "cuda:0", lid)
    # the documents alone and inside a larger batch (the neighbours set the launch classes)
    for name, sel in (("alone", idx), ("batch", list(range(max(0, min(idx) - 3000), max(idx) + 1)))):
        tx = [texts[i] for i in sel]
        data, off = synth.pack(tx)
        res = runner.run(data, off)
        ref, rfl = h.emulate_stage(steps, plan.stages[0], data, off, 8, lid.native())
        n = len(tx)
        for kind, width, prefix in runner.stage_layout[0][1]:
            if kind != 2:
                continue
            a = res.stage_recs[0][prefix * n:(prefix + width) * n].reshape(n, width)
            b = ref[prefix * n:(prefix + width) * n].reshape(n, width)
            for i in idx:
                k = sel.index(i)
                print(name, i, len(tx[k].encode()), "flags", int(res.flags[k]), int(rfl[k]), "dead", int(res.dead[k]))
                print("  dev", a[k].tolist())
                print("  emu", b[k].tolist())


if __name__ == "__main__":
    main()
