"""Headline benchmark: documents/sec through the full language-ID + Gopher + C4 (+FineWeb)
pipeline (BASELINE.json metric) on N MI355X GPUs of one node, one process per GPU.

    python bench.py --gpus N --steps K --warmup W
    (N > 1 is launched by torch.distributed.run; ranks read RANK/LOCAL_RANK/WORLD_SIZE)

One step = every rank pushes one batch of synthetic CommonCrawl-shaped documents (log-normal
lengths around 1 KB, 5 languages) through the whole pipeline: H2D staging, all device stages
(analysis kernels, C4 rewrite passes, hashed n-gram language-id kernel), D2H, per-document
first-failure resolution with reason/metadata formatting, and assembly of the kept/excluded
text + metadata JSON columns. Parquet decode/encode is not in the timed step (the reference's
worker docs/sec excludes it too). Weak scaling: per-GPU batch fixed as N grows; RCCL all-reduces
the per-step document counters (the only cross-GPU traffic).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "documents/sec through full C4+Gopher+langID pipeline at 1/2/4/8 MI355X"


def cpu_baseline(config_path: str, mean_bytes: int):
    """The reference publishes no throughput numbers. Baseline = this framework's
    CPU path (C++ port of the reference filters with ICU4C segmentation, the GPU box's 16-core
    CPU share) on the same synthetic corpus and pipeline config, as measured and recorded in
    config/cpu_baseline.json (raw bench lines under profiles/). None when the config (or its
    document size) has no measured entry."""
    try:
        with open(os.path.join(ROOT, "config", "cpu_baseline.json"), encoding="utf-8") as f:
            table = json.load(f)
    except OSError:
        return None
    e = table.get(os.path.relpath(os.path.abspath(config_path), ROOT))
    if not isinstance(e, dict) or e.get("mean_bytes", 1024) != mean_bytes:
        return None
    return float(e["docs_per_sec"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs-per-step", type=int, default=262144,
                    help="documents per GPU per step (~290 MB of text: device batches sized for 288 GB HBM)")
    ap.add_argument("--mean-bytes", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=16384, help="distinct synthetic docs per rank")
    ap.add_argument("--vocab", default="small", choices=["small", "zipf"],
                    help="synthetic vocabulary: ~130 words per language (default) or 60k-type Zipf lexicons")
    ap.add_argument("--long-token-rate", type=float, default=0.0,
                    help="fraction of pool documents given a long pre-token (URL, base64, indentation or dash "
                         "run: the TokenCounter's 64+-byte path)")
    ap.add_argument("--mixed-script", action="store_true",
                    help="5%% of the documents carry a CJK / Thai snippet and 1%% are CJK (dictionary scripts)")
    ap.add_argument("--config", default=os.path.join(ROOT, "config", "bench_pipeline.yaml"))
    ap.add_argument("--tokenizer", default=None,
                    help="tokenizer.json for a TokenCounter step in --config ('synthetic': a GPT-2-format "
                         "byte-level BPE with 50257 entries trained on the Zipf corpus, cached under /tmp)")
    ap.add_argument("--badwords-dir", default=os.path.join(ROOT, "config", "badwords"),
                    help="word lists of a C4BadWordsFilter step in --config (default: the synthetic list)")
    ap.add_argument("--badwords-rate", type=float, default=0.05,
                    help="with a C4BadWordsFilter step: fraction of pool documents given one list entry")
    ap.add_argument("--backend", default="cuda", choices=["cuda", "cpu", "emulate"])
    ap.add_argument("--segmentation", default="icu", help="CPU backend segmentation (icu|rules)")
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--ar1-every", type=int, default=1,
                    help="all-reduce the counter vector every N steps (0: only the final totals)")
    ap.add_argument("--ar1-window", type=int, default=4, help="outstanding async all-reduces before a wait")
    args = ap.parse_args()
    if args.steps < 1 or args.warmup < 0 or args.docs_per_step < 1 or args.gpus < 1:
        ap.error("--steps must be >= 1, --warmup >= 0, --docs-per-step >= 1 and --gpus >= 1")

    from textblaster_amd.parallel import launch

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start torch.distributed.run as a child before any HIP call
        if args.backend == "cuda":
            have = launch.visible_gpu_count()
            if have < args.gpus:
                print(f"bench.py: --gpus {args.gpus} requested but only {have} GPU(s) are visible",
                      file=sys.stderr)
                sys.exit(2)
        sys.exit(launch.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))

    import torch

    from textblaster_amd.config import load_pipeline_config
    from textblaster_amd.parallel import dist
    from textblaster_amd.pipeline.engine import Engine
    from textblaster_amd.utils import synth

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        sys.exit(2)
    if args.backend == "cuda":
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} requested but only {have} GPU(s) are visible", file=sys.stderr)
            sys.exit(2)
    # one process group per multi-GPU job (RCCL over xGMI); TB_FORCE_PG=1 also creates a one-rank
    # group on one GPU, so the per-step AR1 below runs over RCCL and is timed there too
    ctx = dist.init_from_env(backend="nccl" if args.backend == "cuda" else "gloo")
    rank, world = ctx.rank, ctx.world_size
    device = f"cuda:{ctx.local_rank}" if args.backend == "cuda" else None
    cfg = load_pipeline_config(args.config)
    tok_file = args.tokenizer
    if tok_file == "synthetic":
        from textblaster_amd.models.tokenizer import train_synthetic_bpe

        tok_file = train_synthetic_bpe(os.path.join(os.environ.get("TMPDIR", "/tmp"), "tb_synth_bpe50257.json"))
    has_bw = any(s.type == "C4BadWordsFilter" for s in cfg.pipeline)
    eng = Engine(cfg, backend=args.backend, device=device, nthreads=args.threads, segmentation=args.segmentation,
                 tokenizer_file=tok_file, badwords_dir=args.badwords_dir if has_bw else None)

    # synthetic corpus: a pool of distinct docs per rank, batches are fresh permutations of it
    texts = synth.make_corpus(args.pool, args.mean_bytes, seed=1000 + rank, vocab=args.vocab,
                              mixed_script=args.mixed_script)
    if args.long_token_rate > 0:
        texts = synth.inject_long_tokens(texts, args.long_token_rate, seed=rank)
    if has_bw and args.badwords_rate > 0:
        texts = synth.inject_words(texts, os.path.join(args.badwords_dir, "en"), args.badwords_rate, seed=rank)
    enc = [t.encode("utf-8") for t in texts]
    rng = np.random.default_rng(rank)

    def make_batch():
        idx = rng.integers(0, len(enc), size=args.docs_per_step)
        parts = [enc[i] for i in idx]
        off = np.zeros(len(parts) + 1, dtype=np.int64)
        np.cumsum([len(p) for p in parts], out=off[1:])
        # the batch text in page-locked memory, as a reader decoding into pinned batch buffers
        # would hand it over: the upload DMA reads it in place (no staging copy on the host)
        data = eng.host_buffer(int(off[-1]))
        data[:] = np.frombuffer(b"".join(parts), dtype=np.uint8)
        return data, off

    batches = [make_batch() for _ in range(min(4, args.steps + args.warmup))]
    bytes_per_step = float(np.mean([len(b[0]) for b in batches]))
    counters = np.zeros(5, dtype=np.int64)  # docs, kept, excluded, errors, CPU-delegated
    nsteps = len(cfg.pipeline)
    step_filtered = np.zeros(nsteps, dtype=np.int64)  # filtered documents per pipeline step (timed steps)

    def feed(k, start):
        for i in range(start, start + k):
            yield batches[i % len(batches)]

    # Steps run through Engine.process_many: step i+1's H2D + kernels are queued before step i
    # is resolved on the host (device/host overlap). Every step's full pipeline completes inside
    # the timed region: process_many returns the K-th result only after its assembly.
    for res in eng.process_many(feed(args.warmup, 0)):
        pass
    ctx.barrier()
    if args.backend == "cuda":
        torch.cuda.synchronize()
    from textblaster_amd.utils import metrics

    bpe_host0 = metrics.BPE_HOST_DOCS_TOTAL._value.get()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    n_done = 0
    tsum: dict = {}
    # AR1 every --ar1-every steps (default every step; 0: only the final totals reduction)
    ar1_every = args.ar1_every
    ar1_window = args.ar1_window
    ar1s = collections.deque()
    for res in eng.process_many(feed(args.steps, args.warmup)):
        step = np.asarray([res.n_docs, res.n_kept, res.n_excluded, len(res.error_rows)], dtype=np.int64)
        counters += np.append(step, res.n_delegated)
        fs = res.fail_step[(res.status == 1) & (res.fail_step >= 0)]
        step_filtered += np.bincount(fs, minlength=nsteps)[:nsteps]
        # AR1 once per step: the global counter vector (what rank 0's /metrics serves), reduced
        # over RCCL while the next steps run; the main thread (which also assembles outputs)
        # only waits once more than --ar1-window reductions are outstanding
        if ar1_every and n_done % ar1_every == 0:
            ar1s.append(ctx.all_reduce_sum_async(step))
        while ar1s and (len(ar1s) > ar1_window or ar1s[0].done()):
            ar1s.popleft().wait()
        for k, v in res.timings.items():
            tsum[k] = tsum.get(k, 0.0) + v
        n_done += 1
    while ar1s:
        ar1s.popleft().wait()
    assert n_done == args.steps
    if args.backend == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    # host CPU time of this rank's process over the timed steps (all threads: submitter, copy
    # and assembly pools), the per-rank budget an 8-GPU node has to provide
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    cpu_ms_step_max = ctx.all_reduce_max(1000.0 * cpu_s / args.steps)
    elapsed_max = ctx.all_reduce_max(elapsed)
    bpe_host = int(ctx.all_reduce_sum([int(metrics.BPE_HOST_DOCS_TOTAL._value.get() - bpe_host0)])[0])
    totals = ctx.all_reduce_sum(counters)
    step_filtered = ctx.all_reduce_sum(step_filtered)
    docs_total = int(totals[0])
    value = docs_total / elapsed_max
    lid = getattr(eng, "langid", None)
    base = cpu_baseline(args.config, args.mean_bytes) if args.vocab == "small" and not args.mixed_script else None
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "docs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            # the matrix-core dtype of the language-id head that ran (v3: bf16 MFMA; v2 int16 table:
            # "int16"); the text filters themselves are integer / byte arithmetic
            "dtype": lid.dtype if lid is not None else "int",
            "data": f"synthetic CommonCrawl-shaped docs (log-normal ~{args.mean_bytes} B, 5 languages, "
                    f"{'~130-word' if args.vocab == 'small' else '60k-type Zipf'} vocabularies"
                    f"{', 5% with a CJK/Thai snippet + 1% CJK' if args.mixed_script else ''}"
                    f"{f', {args.long_token_rate:.0%} with a 64+-byte pre-token' if args.long_token_rate else ''}), "
                    f"{args.docs_per_step} docs/GPU/step",
            "config": {
                "model": "+".join(s.type.replace("LanguageDetectionFilter", f"LanguageDetection({lid.description})"
                                                 if lid is not None else "LanguageDetection")
                                  .replace("Filter", "") for s in cfg.pipeline),
                "global_batch": args.docs_per_step * world,
                "seq_len": int(bytes_per_step / args.docs_per_step),
                "parallelism": f"dp{world}",
                "backend": args.backend,
                "pipeline_config": os.path.relpath(args.config, ROOT),
                "tokenizer": args.tokenizer,
            },
            "process_group": ctx.backend,
            "host_cpu_ms_per_step": round(cpu_ms_step_max, 3),
            "host_cpu_us_per_doc": round(1000.0 * cpu_ms_step_max / args.docs_per_step, 4),
            "kept": int(totals[1]),
            "excluded": int(totals[2]),
            "errors": int(totals[3]),
            # documents the device sent to the CPU path (dictionary scripts that reach a segmentation
            # step, hash collisions, scratch overflow) and TokenCounter documents counted by the host
            # tokenizer, over the timed steps
            "delegated": int(totals[4]),
            # documents filtered by each pipeline step (YAML order) over the timed steps: the
            # step mix the downstream kernels saw (survivors of step k reach step k + 1)
            "step_filtered": [int(v) for v in step_filtered],
            "reach_step": [int(totals[0] - sum(int(v) for v in step_filtered[:k])) for k in range(nsteps)],
            "bpe_host_docs": bpe_host,
            "bytes_per_sec": round(bytes_per_step * world * args.steps / elapsed_max, 1),
            "last_step_timings": {k: round(v, 5) for k, v in res.timings.items()},
            # host seconds per phase averaged over the K timed steps (phases of consecutive
            # steps overlap, so they do not add up to ms_per_step)
            "mean_step_timings": {k: round(v / n_done, 5) for k, v in tsum.items()},
        }
        print(json.dumps(line), flush=True)
        from textblaster_amd.utils import tracing

        tracing.dump_timeline()  # TB_TIMELINE=<path>: host per-thread ranges of this run
        dr = getattr(eng, "device_runner", None)
        if dr is not None and getattr(dr, "phase_prof", False):
            print(dr.phase_report(), file=sys.stderr, flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
