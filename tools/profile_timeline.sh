#!/bin/bash
# Kernel + memory-copy trace of the 1-GPU benchmark for the per-step timeline
# (tools/prof_summary.py --copies). No counters in this run.
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/tl"
timeout -k 10 ${TB_PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d "$REPO/gpurun_out/tl" -o bench -- python3 "$REPO/bench.py" --steps ${TB_PROF_STEPS:-10} --warmup 2 \
  > "$REPO/gpurun_out/tl/bench_stdout.log" 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
k=$(find "$REPO/gpurun_out/tl" -name "*kernel_trace.csv" | head -1)
c=$(find "$REPO/gpurun_out/tl" -name "*memory_copy_trace.csv" | head -1)
[ $rc -eq 0 ] && python3 "$REPO/tools/prof_summary.py" "$k" ${c:+--copies "$c"} > "$REPO/gpurun_out/tl/summary.txt" 2>&1
exit $rc
