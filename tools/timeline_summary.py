"""Summarises a host timeline written with TB_TIMELINE=<path> (utils/tracing.py).

Prints, per thread: the wall span, the busy fraction (union of its top-level ranges) and the
total time per range name; then a coarse ASCII Gantt chart (one row per thread, one column per
time slice, the letter of the range that covers most of the slice, '.' = idle).

    python tools/timeline_summary.py gpurun_out/e2e/timeline.json [--cols 100]
"""
from __future__ import annotations

import argparse
import collections
import json


def _union(iv):
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def summarise(doc, cols=100):
    ev = doc["events"]
    if not ev:
        return "no events"
    t_end = max(e["end"] for e in ev)
    t_beg = min(e["start"] for e in ev)
    by_thread = collections.defaultdict(list)
    for e in ev:
        by_thread[e["thread"]].append(e)
    names = sorted({e["name"] for e in ev})
    letters = {n: "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"[i % 52] for i, n in enumerate(names)}
    out = [f"span {t_end - t_beg:.3f} s, {len(ev)} ranges, {len(by_thread)} threads", ""]
    # thread groups: numbered pool threads (tb-reader_0, tb-reader_1 ...) fold into one row each
    for th in sorted(by_thread):
        es = by_thread[th]
        busy = _union([(e["start"], e["end"]) for e in es])
        per = collections.Counter()
        cnt = collections.Counter()
        for e in es:
            per[e["name"]] += e["end"] - e["start"]
            cnt[e["name"]] += 1
        out.append(f"{th:24s} busy {busy:7.3f} s ({100 * busy / (t_end - t_beg):5.1f}% of span)")
        for n, v in per.most_common():
            out.append(f"    {n:22s} {v:8.3f} s  x{cnt[n]:<5d} mean {1e3 * v / cnt[n]:8.2f} ms")
    out += ["", "legend: " + "  ".join(f"{letters[n]}={n}" for n in names), ""]
    dt = (t_end - t_beg) / cols
    for th in sorted(by_thread):
        row = []
        es = by_thread[th]
        for c in range(cols):
            a, b = t_beg + c * dt, t_beg + (c + 1) * dt
            cover = collections.Counter()
            for e in es:
                ov = min(b, e["end"]) - max(a, e["start"])
                if ov > 0:
                    cover[e["name"]] += ov
            row.append(letters[cover.most_common(1)[0][0]] if cover else ".")
        out.append(f"{th[:20]:20s} |{''.join(row)}|")
    out.append(f"{'':20s}  0{'':{cols - 8}s}{t_end - t_beg:6.2f}s")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--cols", type=int, default=100)
    a = ap.parse_args()
    with open(a.path, encoding="utf-8") as f:
        print(summarise(json.load(f), a.cols))


if __name__ == "__main__":
    main()
