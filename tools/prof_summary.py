"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel totals (short names) and the
GPU busy time (union of kernel intervals, all streams) per bench step.

    python tools/prof_summary.py gpurun_out/prof/bench_kernel_trace.csv [--steps K]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.split("(")[0]
    if "at::native::" in name or "rocprim" in name:
        m = re.search(r"(FillFunctor<[^>]*>|direct_copy|lookback_scan_kernel|init_lookback_scan_state_kernel)", name)
        return "torch/rocprim " + (m.group(1) if m else name[:40])
    return name.replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=0, help="timed bench steps at the end of the trace")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    tot = defaultdict(lambda: [0, 0])
    iv = []
    for r in rows:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        tot[k][0] += 1
        tot[k][1] += b - a
        iv.append((a, b, k))
    iv.sort()
    all_ns = sum(v[1] for v in tot.values())
    print(f"{'kernel':<44} {'calls':>6} {'total ms':>10} {'avg us':>10} {'%':>6}")
    for k, (c, ns) in sorted(tot.items(), key=lambda t: -t[1][1]):
        print(f"{k:<44} {c:>6} {ns / 1e6:>10.3f} {ns / c / 1e3:>10.1f} {100 * ns / all_ns:>6.1f}")
    # busy time: union of intervals
    busy, cur_a, cur_b = 0, None, None
    for a, b, _ in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    span = iv[-1][1] - iv[0][0] if iv else 0
    print(f"\nGPU busy (union of kernel intervals): {busy / 1e6:.2f} ms over a {span / 1e6:.2f} ms trace "
          f"({100 * busy / max(1, span):.0f} %)")
    nstage = sum(1 for _, _, k in iv if k.startswith("k_langid_features"))
    if nstage:
        print(f"steps in trace (langid launches): {nstage}; GPU busy per step: {busy / nstage / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
