#!/bin/bash
# Stream-layout A/B: GPU tests, the 1-GPU bench under each TB_STREAMS layout, and a concurrent
# (not serialized) rocprofv3 kernel + memory-copy trace of each, summarised by
# tools/stream_timeline.py. Output under gpurun_out/streams/.
set -e
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$REPO/gpurun_out/streams"
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for L in ${TB_LAYOUTS:-4 4c 6 13}; do
  TB_STREAMS=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_$L.log" 2>&1
  echo "layout $L: $(tail -1 "$OUT/bench_$L.log" | cut -c1-220)"
done
cd /tmp && export TMPDIR=/tmp
for L in ${TB_TRACE_LAYOUTS:-4 13}; do
  TB_STREAMS=$L timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$OUT/trace_$L" -o bench -- python3 "$REPO/bench.py" --steps 4 --warmup 1 > "$OUT/trace_$L.log" 2>&1
  K=$(find "$OUT/trace_$L" -name "*kernel_trace.csv" | head -1)
  C=$(find "$OUT/trace_$L" -name "*memory_copy_trace.csv" | head -1)
  python3 "$REPO/tools/stream_timeline.py" "$K" ${C:+--copies "$C"} > "$OUT/timeline_$L.txt" 2>&1 || true
  head -30 "$OUT/timeline_$L.txt"
  rm -f "$K" "$C"
done
