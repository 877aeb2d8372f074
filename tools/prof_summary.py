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
    ap.add_argument("--copies", default=None, help="rocprofv3 memory_copy_trace.csv")
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
    nstage = sum(1 for _, _, k in iv if k.startswith("k_langid"))
    if nstage:
        print(f"steps in trace (langid launches): {nstage}; GPU busy per step: {busy / nstage / 1e6:.2f} ms")
        # per-step timeline: a step starts at its langid launch; busy = union of kernel time until the next
        starts = [a for a, _, k in iv if k.startswith("k_langid")]
        print(f"\n{'step':>4} {'start ms':>10} {'gap ms':>8} {'busy ms':>8} {'kernels':>8}")
        for j, s0 in enumerate(starts):
            s1 = starts[j + 1] if j + 1 < len(starts) else iv[-1][1] + 1
            seg = [(max(a, s0), min(b, s1)) for a, b, _ in iv if b > s0 and a < s1]
            ub, ca, cb = 0, None, None
            for a, b in sorted(seg):
                if cb is None or a > cb:
                    if cb is not None:
                        ub += cb - ca
                    ca, cb = a, b
                else:
                    cb = max(cb, b)
            if cb is not None:
                ub += cb - ca
            print(f"{j:>4} {(s0 - starts[0]) / 1e6:>10.2f} {(s1 - s0) / 1e6:>8.2f} {ub / 1e6:>8.2f} {len(seg):>8}")
    # every launch of the last traced step (a step starts at its language-id launch): kernel,
    # grid (work-items) and duration, in launch order -- separates the per-stage launches of
    # kernels that run more than once per step
    starts = [a for a, _, k in iv if k.startswith("k_langid")]
    if starts and rows and "Grid_Size_X" in rows[0]:
        last = starts[-1]
        print(f"\nlaunches of the last step:\n{'kernel':<44} {'grid':>10} {'us':>10}")
        for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if a >= last:
                print(f"{short(r['Kernel_Name']):<44} {r['Grid_Size_X']:>10} {(b - a) / 1e3:>10.1f}")
    if args.copies:
        rows = list(csv.DictReader(open(args.copies)))
        agg = defaultdict(lambda: [0, 0, 0])
        for r in rows:
            d = r.get("Direction") or r.get("Operation") or "?"
            agg[d][0] += 1
            agg[d][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg[d][2] += int(r.get("Bytes") or 0)
        print(f"\n{'copy':<28} {'calls':>6} {'total ms':>10} {'MB':>10} {'GB/s':>8}")
        for d, (c, ns, by) in sorted(agg.items()):
            print(f"{d:<28} {c:>6} {ns / 1e6:>10.2f} {by / 1e6:>10.1f} {by / max(1, ns):>8.1f}")


if __name__ == "__main__":
    main()
