"""Throughput of the K17 GPU HTML decoder (csrc/hip/html.hip) vs. the host C++ decoder on a
CommonCrawl-shaped batch (bench corpus, ~1 entity per 200 bytes). Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from textblaster_amd import native  # noqa: E402
from textblaster_amd.utils import synth  # noqa: E402


def main():
    import torch

    from textblaster_amd.ops.html import HtmlDecoder

    ndocs = int(os.environ.get("TB_HTML_DOCS", "262144"))
    base = synth.make_corpus(4096, 1024, seed=9)
    rng = np.random.default_rng(1)
    ents = ["&amp;", "&quot;", "&#8217;", "&nbsp;", "&eacute;", "&lt;b&gt;", "&copy;", "&#x2014;"]
    pool = []
    for t in base:
        parts = t.split(" ")
        for k in rng.integers(0, len(parts), size=max(1, len(t) // 200)):
            parts[int(k)] = parts[int(k)] + ents[int(rng.integers(0, len(ents)))]
        pool.append(" ".join(parts))
    texts = [pool[int(i)] for i in rng.integers(0, len(pool), size=ndocs)]
    data, off = synth.pack(texts)
    dec = HtmlDecoder("cuda:0")
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off).cuda()
    for _ in range(2):
        dec.decode(d, o)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        od, oo = dec.decode(d, o)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    h = native.host()
    t0 = time.perf_counter()
    hd = h.html_decode_batch(data, off, 16)
    cpu_s = time.perf_counter() - t0
    same = np.array_equal(od.cpu().numpy(), hd[0]) and np.array_equal(oo.cpu().numpy(), hd[1])
    print(json.dumps({"docs": ndocs, "bytes": int(data.size), "gpu_ms": round(gpu_s * 1e3, 3),
                      "gpu_GBps": round(data.size / gpu_s / 1e9, 2), "cpu16_ms": round(cpu_s * 1e3, 3),
                      "cpu16_GBps": round(data.size / cpu_s / 1e9, 2), "identical": bool(same)}))


if __name__ == "__main__":
    main()
