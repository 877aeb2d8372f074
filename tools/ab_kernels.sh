#!/bin/bash
# Kernel-level A/B: rocprofv3 kernel stats of the bench for each TB_HIP_LIB variant given as args
# (use "default" for the in-tree library). Prints average ns per kernel.
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  out="$REPO/gpurun_out/ab/$v"; mkdir -p "$out"
  if [ "$v" = default ]; then lib=""; else lib="$REPO/textblaster_amd/libtbhip_$v.so"; fi
  TB_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
    -- python3 "$REPO/bench.py" --steps 6 --warmup 1 > "$out/stdout.log" 2>&1 || { echo "variant $v failed"; exit 1; }
  python3 - "$v" "$out/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[2])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"== {sys.argv[1]}: total {tot/1e6:.1f} ms")
for r in rows[:6]:
    print(f"   {r['Name'].split('(')[0].replace('(anonymous namespace)::','')[:40]:<40} {int(r['Calls']):>4} x {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
