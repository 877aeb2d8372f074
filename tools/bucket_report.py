"""Per-dispatch time of the stage kernels from a rocprofv3 kernel trace: ns per document by
kernel variant and grid (length bucket).  python tools/bucket_report.py <kernel_trace.csv>"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        k = r["Kernel_Name"]
        if "stage_lds" not in k and "stage_retry" not in k and "stage_analyze" not in k:
            continue
        name = k.replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        wg = int(r["Workgroup_Size_X"])
        grid = int(r["Grid_Size_X"]) // wg
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg[(name, wg, grid)]
        a[0] += 1
        a[1] += d
    tot = 0
    for (name, wg, grid), (calls, ns) in sorted(agg.items(), key=lambda t: (t[0][0], -t[0][2])):
        tot += ns
        print(f"{name:<28} wg={wg:<4} docs={grid:<7} calls={calls:<3} avg_us={ns / calls / 1000:9.1f} "
              f"ns/doc={ns / calls / max(grid, 1):7.1f}")
    print(f"total {tot / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
