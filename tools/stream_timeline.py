"""Concurrency view of a rocprofv3 kernel + memory-copy trace of bench.py (streams NOT
serialized): which hardware queue / stream each kernel and copy ran on, how much of each kind of
work overlapped other work, and an ASCII Gantt chart of one bench step.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o bench -- python3 bench.py ...
    python tools/stream_timeline.py OUT/.../bench_kernel_trace.csv --copies OUT/.../bench_memory_copy_trace.csv
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.split("(")[0].replace("void ", "")
    return name


def _lane(r, prefer):
    for k in prefer:
        if k in r and r[k] not in ("", None):
            return f"{k.split('_')[0].lower()}{r[k]}"
    return "?"


def load(kpath, cpath=None):
    ev = []
    with open(kpath) as f:
        for r in csv.DictReader(f):
            ev.append(dict(kind="kernel", name=short(r["Kernel_Name"]), lane=_lane(r, ("Stream_Id", "Queue_Id")),
                           queue=r.get("Queue_Id", "?"), a=int(r["Start_Timestamp"]), b=int(r["End_Timestamp"])))
    if cpath:
        with open(cpath) as f:
            for r in csv.DictReader(f):
                d = r.get("Direction", r.get("Operation", "copy"))
                ev.append(dict(kind="copy", name=f"copy {d}", lane=_lane(r, ("Stream_Id", "Queue_Id")),
                               queue="sdma", a=int(r["Start_Timestamp"]), b=int(r["End_Timestamp"])))
    ev.sort(key=lambda e: e["a"])
    return ev


def union(iv):
    tot, cs, ce = 0, None, None
    for a, b in sorted(iv):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + (ce - cs if ce is not None else 0)


def covered(a, b, others):
    """ns of [a, b) covered by the union of ``others`` intervals."""
    iv = [(max(a, x), min(b, y)) for x, y in others if y > a and x < b]
    return union(iv)


def category(name):
    if name.startswith("copy") or "copyBuffer" in name:
        return "copy"
    for key in ("k_langid_features", "k_stage_analyze_blk", "k_c4_pass_a_blk", "k_stage_analyze", "k_c4_pass_a",
                "k_c4_pass_b"):
        if name.startswith(key):
            return key
    return "other"


def report(ev, steps=3, cols=110):
    out = []
    t0 = ev[0]["a"]
    span = max(e["b"] for e in ev) - t0
    lanes = collections.defaultdict(list)
    for e in ev:
        lanes[e["lane"]].append(e)
    out.append(f"{len(ev)} GPU operations over {span / 1e6:.1f} ms, {len(lanes)} streams/queues")
    out.append("")
    out.append(f"{'lane':<12} {'ops':>5} {'busy ms':>9}  work")
    for ln, es in sorted(lanes.items()):
        busy = union([(e["a"], e["b"]) for e in es])
        kinds = collections.Counter(category(e["name"]) for e in es)
        out.append(f"{ln:<12} {len(es):>5} {busy / 1e6:>9.2f}  " + ", ".join(f"{k} x{v}" for k, v in kinds.most_common()))
    # overlap: for each category, how much of its time ran concurrently with other categories
    out.append("")
    out.append(f"{'category':<22} {'n':>5} {'total ms':>9} {'overlapped ms':>14} {'%':>6}")
    bycat = collections.defaultdict(list)
    for e in ev:
        bycat[category(e["name"])].append(e)
    for cat, es in sorted(bycat.items(), key=lambda t: -sum(e["b"] - e["a"] for e in t[1])):
        others = [(e["a"], e["b"]) for e in ev if category(e["name"]) != cat]
        tot = sum(e["b"] - e["a"] for e in es)
        ov = sum(covered(e["a"], e["b"], others) for e in es)
        out.append(f"{cat:<22} {len(es):>5} {tot / 1e6:>9.2f} {ov / 1e6:>14.2f} {100 * ov / max(tot, 1):>6.1f}")
    allk = [(e["a"], e["b"]) for e in ev]
    busy = union(allk)
    work = sum(b - a for a, b in allk)
    out.append("")
    out.append(f"GPU busy (union of all ops): {busy / 1e6:.1f} ms; sum of op durations {work / 1e6:.1f} ms; "
               f"mean concurrency while busy {work / max(busy, 1):.2f}")
    # Gantt of the last `steps` bench steps (a step starts with a k_langid_features launch)
    starts = [e["a"] for e in ev if category(e["name"]) == "k_langid_features"]
    if len(starts) > steps:
        g0 = starts[-steps - 1]
        evw = [e for e in ev if e["b"] > g0]
        g1 = max(e["b"] for e in evw)
        dt = (g1 - g0) / cols
        letters = {"k_stage_analyze": "S", "k_stage_analyze_blk": "B", "k_langid_features": "L",
                   "k_c4_pass_a": "C", "k_c4_pass_a_blk": "c", "k_c4_pass_b": "b", "copy": "=", "other": "o"}
        out.append("")
        out.append(f"last {steps} steps, {(g1 - g0) / 1e6:.1f} ms, {dt / 1e3:.0f} us per column  "
                   "(S stage waves, B stage workgroups, L langid bag, h head, C/c C4 pass A waves/workgroups, "
                   "b C4 pass B, = copy, o other)")
        for ln, es in sorted(lanes.items()):
            row = []
            for c in range(cols):
                a, b = g0 + c * dt, g0 + (c + 1) * dt
                cov = collections.Counter()
                for e in es:
                    o = min(b, e["b"]) - max(a, e["a"])
                    if o > 0:
                        cov[category(e["name"])] += o
                row.append(letters[cov.most_common(1)[0][0]] if cov else ".")
            out.append(f"{ln[:10]:<10} |{''.join(row)}|")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("--copies", default=None)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    print(report(load(a.kernels, a.copies), a.steps))


if __name__ == "__main__":
    main()
