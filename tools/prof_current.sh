#!/bin/bash
# Current-state profile of the 1-GPU bench: serialized-stream kernel stats (exclusive kernel
# times) + per-phase cycle stamps inside the document kernels. Output under gpurun_out/cur/.
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$REPO/gpurun_out/cur"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
TB_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/serial" -o bench -- python3 "$REPO/bench.py" --steps 4 --warmup 1 $TB_BENCH_ARGS \
  > "$OUT/serial_stdout.log" 2>&1 || { echo "serial trace failed"; tail -5 "$OUT/serial_stdout.log"; exit 1; }
TR=$(find "$OUT/serial" -name "*kernel_trace.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$TR" > "$OUT/kernels_serialized.txt" 2>&1 || true
TB_PHASE_PROF=1 timeout -k 10 300 python3 "$REPO/bench.py" --steps 3 --warmup 1 $TB_BENCH_ARGS \
  > "$OUT/phase_stdout.log" 2> "$OUT/phase_cycles.txt" || { echo "phase run failed"; tail -5 "$OUT/phase_cycles.txt"; exit 1; }
head -20 "$OUT/kernels_serialized.txt"
