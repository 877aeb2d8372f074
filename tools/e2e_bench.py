"""End-to-end file benchmark: synthetic CommonCrawl-shaped Parquet -> `run` -> Parquet.

Unlike bench.py (which times the in-memory pipeline step), this includes Parquet decode, HTML
entity decoding, output assembly and Parquet encode — the full CLI path.

    python tools/e2e_bench.py --docs 1000000 --backend cuda [--backend cpu] [--out gpurun_out/e2e]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_input(path: str, ndocs: int, mean_bytes: int, pool: int, row_group: int) -> int:
    from textblaster_amd.utils import synth

    texts = synth.make_corpus(pool, mean_bytes, seed=5)
    text_arr = pa.array(texts, pa.string())
    lens = np.array([len(t.encode()) for t in texts], dtype=np.int64)
    rng = np.random.default_rng(5)
    w = None
    total = 0
    for start in range(0, ndocs, row_group):
        n = min(row_group, ndocs - start)
        idx = rng.integers(0, len(texts), size=n)
        tbl = pa.table({
            "id": pa.array([f"doc-{start + i}" for i in range(n)]),
            "text": text_arr.take(pa.array(idx)),
            "source": pa.array(["s3://commoncrawl/synthetic"] * n),
            "metadata": pa.array(['{"url":"https://example.com/%d"}' % (start + i) for i in range(n)]),
        })
        total += int(lens[idx].sum())
        if w is None:
            w = pq.ParquetWriter(path, tbl.schema, compression="snappy")
        w.write_table(tbl)
    w.close()
    return total


def thread_cpu() -> dict:
    """CPU seconds per OS thread name of this process (/proc/self/task/*/stat; the runner names
    its reader / encoder / writer / prefetch threads, the native pool is "tb-pool")."""
    out: dict = {}
    tck = os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        out[(t, name)] = (int(f[11]) + int(f[12])) / tck
    return out


def _pool_stats() -> dict:
    from textblaster_amd import native

    return dict(native.host().pool_cpu_stats())


def _delta(before: dict, after: dict) -> dict:
    d = {k: round(v - before.get(k, 0.0), 3) for k, v in after.items()}
    return {k: v for k, v in sorted(d.items(), key=lambda kv: -kv[1]) if v > 0.005}


def cpu_by_name(before: dict, after: dict) -> dict:
    agg: dict = {}
    for k, v in after.items():
        agg[k[1]] = agg.get(k[1], 0.0) + v - before.get(k, 0.0)
    return {n: round(v, 3) for n, v in sorted(agg.items(), key=lambda kv: -kv[1]) if v > 0.005}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--mean-bytes", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=50_000)
    ap.add_argument("--row-group", type=int, default=100_000)
    ap.add_argument("--unit-rows", type=int, default=65536)
    ap.add_argument("--backend", action="append", default=None)
    ap.add_argument("--config", default=os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "e2e"))
    ap.add_argument("--timeline", action="store_true", help="record the host timeline (TB_TIMELINE) per backend")
    ap.add_argument("--html-decode", default="cpu")
    ap.add_argument("--keep-input", action="store_true")
    ap.add_argument("--repeat", type=int, default=1, help="runs per backend (all reported; the median last)")
    ap.add_argument("--cli", action="store_true",
                    help="also run the CLI (`python -m textblaster_amd.cli run --backend cuda`) as a child process: "
                         "wall time from process start to exit, CPU time of the child")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    inp = os.path.join(args.out, "input.parquet")
    t = time.perf_counter()
    if not (args.keep_input and os.path.exists(inp)):
        make_input(inp, args.docs, args.mean_bytes, args.pool, args.row_group)
    print(f"input: {args.docs} docs, {os.path.getsize(inp) / 1e6:.1f} MB in {time.perf_counter() - t:.1f}s",
          flush=True)
    from textblaster_amd.runner import RunConfig, run
    from textblaster_amd.utils import tracing

    runs = [b for b in (args.backend or ["cuda"]) for _ in range(args.repeat)]
    rates = {}
    for backend in runs:
        o = os.path.join(args.out, f"{backend}.out.parquet")
        e = os.path.join(args.out, f"{backend}.excluded.parquet")
        tl = os.path.join(args.out, f"timeline_{backend}.json") if args.timeline else None
        tracing.record_timeline(tl)
        cpu0 = thread_cpu()
        pool0 = _pool_stats()
        st = run(RunConfig(inp, o, e, args.config, backend=backend, unit_rows=args.unit_rows,
                           html_decode=args.html_decode))
        cpu = cpu_by_name(cpu0, thread_cpu())
        line = {"backend": backend, "docs": st.docs, "kept": st.kept, "excluded": st.excluded, "errors": st.errors,
                "seconds": round(st.seconds, 3), "docs_per_sec": round(st.docs_per_sec, 1),
                "step_filtered": st.step_filtered, "delegated": st.delegated,
                "phase_seconds": {k: round(v, 3) for k, v in st.phase_seconds.items() if not k.startswith("cpu_")},
                # host CPU seconds per thread group over the run (runner accounting) and per OS
                # thread name of the threads alive at its end (native pools)
                "cpu_seconds": {k[4:]: round(v, 3) for k, v in st.phase_seconds.items() if k.startswith("cpu_")},
                "cpu_us_per_doc": round(1e6 * st.phase_seconds.get("cpu_total", 0.0) / max(st.docs, 1), 3),
                "cpu_seconds_by_os_thread": cpu,
                # the native worker pool's CPU seconds by job (tb-pool threads + the submitting thread)
                "pool_cpu_seconds_by_job": _delta(pool0, _pool_stats())}
        # "other" (CPU outside the reader / encoder / writer threads) less the native pool's
        # attributed jobs: what is left is the Python main loop, GPU runtime threads and the rest
        pool_jobs = sum(line["pool_cpu_seconds_by_job"].values())
        line["cpu_seconds"]["other_minus_pool_jobs"] = round(line["cpu_seconds"].get("other", 0.0) - pool_jobs, 3)
        print(json.dumps(line), flush=True)
        rates.setdefault(backend, []).append(line["docs_per_sec"])
        if tl:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from timeline_summary import summarise

            with open(tl, encoding="utf-8") as f:
                summary = summarise(json.load(f))
            with open(tl.replace(".json", ".txt"), "w", encoding="utf-8") as f:
                f.write(json.dumps(line) + "\n\n" + summary + "\n")
            print(summary, flush=True)
        for p in (o, e):
            os.remove(p)
    if args.cli:
        import resource
        import subprocess

        o = os.path.join(args.out, "cli.out.parquet")
        e = os.path.join(args.out, "cli.excluded.parquet")
        cmd = [sys.executable, "-m", "textblaster_amd", "run", "-i", inp, "-o", o, "-e", e, "-c", args.config,
               "--backend", "cuda", "--unit-rows", str(args.unit_rows), "--html-decode", args.html_decode,
               "--log-dir", os.path.join(args.out, "log")]
        ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t0 = time.perf_counter()
        cp = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
        wall = time.perf_counter() - t0
        ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        if cp.returncode != 0:
            print(cp.stdout[-2000:], cp.stderr[-4000:], file=sys.stderr)
            raise SystemExit(f"CLI run failed with exit code {cp.returncode}")
        summary = [ln.strip() for ln in cp.stdout.splitlines() if ":" in ln]
        read = [int(ln.split(":")[1]) for ln in summary if ln.startswith("Documents Read")]
        ndocs = read[0] if read else args.docs
        print(json.dumps({"backend": "cli-cuda", "docs": ndocs, "seconds_wall_incl_startup": round(wall, 3),
                          "docs_per_sec": round(ndocs / wall, 1), "cpu_seconds": round(cpu, 3),
                          "cpu_us_per_doc": round(1e6 * cpu / max(ndocs, 1), 3), "summary": summary[:12]}),
              flush=True)
        for p in (o, e):
            if os.path.exists(p):
                os.remove(p)
    for backend, r in rates.items():
        if len(r) > 1:
            print(json.dumps({"backend": backend, "runs": len(r), "docs_per_sec_median": float(np.median(r)),
                              "docs_per_sec_all": r}), flush=True)
    if not args.keep_input:
        os.remove(inp)


if __name__ == "__main__":
    main()
