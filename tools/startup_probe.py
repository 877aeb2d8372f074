"""Where does a short GPU run spend its startup? Times each initialisation step separately.

    python tools/startup_probe.py [--config config/bench_pipeline.yaml]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    args = ap.parse_args()
    t = {}
    t0 = time.perf_counter()

    def mark(name):
        nonlocal t0
        now = time.perf_counter()
        t[name] = round(now - t0, 4)
        t0 = now

    import torch

    mark("import_torch")
    from textblaster_amd import native

    native.host()
    mark("load_host_lib")
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    mark("cuda_context")
    native.hip()
    mark("load_hip_lib")
    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.pipeline.engine import Engine
    from textblaster_amd.utils import synth

    cfg = load_pipeline_config(args.config)
    mark("config")
    eng = Engine(cfg, backend="cuda")
    mark("engine_init")
    data, off = synth.pack(synth.make_corpus(1000, 800, seed=1))
    mark("make_batch")
    eng.process(data, off)
    mark("first_batch")
    eng.process(data, off)
    mark("second_batch")
    print(json.dumps(t))


if __name__ == "__main__":
    main()
