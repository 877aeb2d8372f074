#!/bin/bash
# Kernel-trace profile of the 1-GPU benchmark (rocprofv3 --kernel-trace --stats).
# Output: gpurun_out/prof/ (raw) ; summaries are copied into profiles/ by hand.
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$REPO/gpurun_out/prof"
timeout -k 10 ${TB_PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$REPO/gpurun_out/prof" -o bench -- python3 "$REPO/bench.py" --steps ${TB_PROF_STEPS:-5} --warmup 1 \
  > "$REPO/gpurun_out/prof/bench_stdout.log" 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
find "$REPO/gpurun_out/prof" -name "*stats*.csv" | head
exit $rc
