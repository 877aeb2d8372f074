"""Per-kernel summary of rocprofv3 --pmc counter_collection CSVs (one or more passes).

    python tools/pmc_summary.py gpurun_out/pmc/*/run_counter_collection.csv [--docs N]

Sums every counter over the dispatches of each kernel name and prints a table, plus derived
rows: HBM bytes read/written (FETCH_SIZE/WRITE_SIZE are in KB), bytes per document when
--docs (documents processed per dispatch-summed run) is given, L2 hit rate, wait fraction.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--docs", type=float, default=0.0, help="documents processed over the profiled dispatches")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for path in a.csv:
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                k = k[5:] if k.startswith("void ") else k
                k = k.split("(")[0]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[k].add((path, r["Dispatch_Id"]))
    names = sorted(tot, key=lambda k: -(tot[k].get("FETCH_SIZE", 0) + tot[k].get("SQ_WAVE_CYCLES", 0) * 1e-6))
    for k in names[: a.top]:
        c = tot[k]
        print(f"== {k}  ({len(calls[k])} dispatch-passes)")
        for name in sorted(c):
            print(f"   {name:<24} {c[name]:>18,.0f}")
        fetch = c.get("FETCH_SIZE", 0) * 1024
        write = c.get("WRITE_SIZE", 0) * 1024
        if fetch or write:
            print(f"   HBM read {fetch / 1e6:,.1f} MB  write {write / 1e6:,.1f} MB")
            if a.docs:
                print(f"   per doc: read {fetch / a.docs:,.0f} B  write {write / a.docs:,.0f} B")
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        if h + m:
            print(f"   L2 hit rate {100 * h / (h + m):.1f}%")
        if c.get("SQ_WAVE_CYCLES"):
            print(f"   wait_any/wave_cycles {100 * c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.1f}%  "
                  f"valu insts/wave-cycle {c.get('SQ_INSTS_VALU', 0) / c['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
