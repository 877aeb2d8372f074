#!/bin/bash
# Where a headline bench step goes now: host timeline (TB_TIMELINE, per thread ranges) of a plain
# bench run, then a concurrent rocprofv3 kernel + memory-copy trace (default stream layout).
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$REPO/gpurun_out/tl"
mkdir -p "$OUT"
cd "$REPO"
TB_TIMELINE="$OUT/host_timeline.json" timeout -k 10 300 python bench.py --steps 8 --warmup 2 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
python3 tools/timeline_summary.py "$OUT/host_timeline.json" --cols 120 > "$OUT/host_timeline.txt" 2>&1
head -40 "$OUT/host_timeline.txt"
rm -f "$OUT/host_timeline.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d "$OUT/trace" -o bench -- python3 "$REPO/bench.py" --steps 4 --warmup 1 > "$OUT/trace.log" 2>&1 || { tail -5 "$OUT/trace.log"; exit 1; }
K=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
C=$(find "$OUT/trace" -name "*memory_copy_trace.csv" | head -1)
python3 "$REPO/tools/stream_timeline.py" "$K" ${C:+--copies "$C"} > "$OUT/timeline.txt" 2>&1 || true
cat "$OUT/timeline.txt" | head -40
rm -f "$K" "$C"
