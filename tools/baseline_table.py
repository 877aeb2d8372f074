"""Markdown table of the BASELINE configurations from tools/baseline_table.sh output.

    python tools/baseline_table.py gpurun_out/baseline > profiles/r1_baseline_table.md
"""
import json
import os
import sys


def last_json(path):
    try:
        lines = [l for l in open(path) if l.startswith("{")]
    except OSError:
        return None
    return [json.loads(l) for l in lines] if lines else None


def main(d):
    g = lambda n: last_json(os.path.join(d, n + ".json"))  # noqa: E731
    rows = []

    def fmt(v):
        return f"{v:,.0f}" if v is not None else "—"

    c1f = {r["backend"]: r for r in (g("c1_file") or [])}
    c1c, c1g = g("c1_cpu"), g("c1_gpu")
    rows.append(("1. C4QualityFilter only", "1k-row Parquet, CLI path (incl. startup)",
                 c1f.get("cpu", {}).get("docs_per_sec"), c1f.get("cuda", {}).get("docs_per_sec")))
    def batch(r):
        return f"{r[-1]['config']['global_batch']:,}" if r else "?"

    rows.append(("1. C4QualityFilter only", f"{batch(c1g)} ~1.1 KB docs/step, in memory",
                 c1c and c1c[-1]["value"], c1g and c1g[-1]["value"]))
    c2c, c2g = g("c2_cpu"), g("c2_gpu")
    steps2 = c2g[-1]["steps"] if c2g else 0
    rows.append(("2. C4 + GopherQuality + GopherRepetition",
                 f"{steps2 * (c2g[-1]['config']['global_batch'] if c2g else 0) / 1e6:.1f}M ~1.1 KB docs "
                 f"({steps2} steps x {batch(c2g)})",
                 c2c and c2c[-1]["value"], c2g and c2g[-1]["value"]))
    c3c, c3g = g("c3_cpu"), g("c3_gpu")
    rows.append(("3. + LanguageDetection (bf16 MFMA head) + FineWeb", f"{batch(c3g)} ~1.1 KB docs/step (bench.py)",
                 c3c and c3c[-1]["value"], c3g and c3g[-1]["value"]))
    c4 = g("c4_file")
    n4 = f"{c4[-1]['docs'] / 1e6:.0f}M" if c4 else "?"
    rows.append(("4. CommonCrawl-shaped Parquet, CLI path (1-GPU point)",
                 f"{n4} docs: read+decode+filter+write" + (f", {c4[-1]['cpu_us_per_doc']:.2f} CPU-us/doc" if c4 else ""),
                 None, c4 and c4[-1]["docs_per_sec"]))
    c5c, c5g = g("c5_cpu"), g("c5_gpu")
    rows.append(("5. GopherRepetition 2..10-gram", "~50 KB docs, 4,096 docs/step",
                 c5c and c5c[-1]["value"], c5g and c5g[-1]["value"]))
    c5m = g("c5mb_gpu")
    rows.append(("5b. GopherRepetition 2..10-gram, long documents", "~1 MB docs, 128 docs/step", None,
                 c5m and c5m[-1]["value"]))
    print("| Config | Workload | CPU path (16 threads) docs/s | 1x MI355X docs/s | speed-up |")
    print("|---|---|---|---|---|")
    for name, wl, c, gv in rows:
        sp = f"{gv / c:.1f}x" if c and gv else "—"
        print(f"| {name} | {wl} | {fmt(c)} | {fmt(gv)} | {sp} |")
    if c5g:
        print(f"\nConfig 5 on the GPU: {c5g[-1]['bytes_per_sec'] / 1e9:.2f} GB/s of text.")
    if c5m:
        print(f"~1 MB documents on the GPU: {c5m[-1]['bytes_per_sec'] / 1e9:.2f} GB/s of text.")
    steps = {n: (r[-1]["steps"], r[-1]["warmup"]) for n, r in (("c1_gpu", c1g), ("c2_gpu", c2g), ("c3_gpu", c3g),
                                                               ("c5_gpu", c5g), ("c5mb_gpu", c5m)) if r}
    print("\nGPU runs (timed steps, warmup): " + ", ".join(f"{n} {s}/{w}" for n, (s, w) in steps.items()))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/baseline")
