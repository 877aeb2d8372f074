#!/bin/bash
# Kernel-time A/B (robust to host/pipeline noise): serialized-stream rocprofv3 kernel stats of a
# short headline bench per env setting; prints ms per step of the top kernels.
# KAB="ENV1=a,ENV2=b ENV1=c" (settings separated by spaces, assignments by commas)
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$REPO/gpurun_out/kab"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for S in $KAB; do
  i=$((i+1))
  E=$(echo "$S" | tr ',' ' ')
  env $E TB_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/r$i" -o k -- python3 "$REPO/bench.py" --steps 4 --warmup 1 $KAB_ARGS > "$OUT/r$i.log" 2>&1 || { echo "run $S failed"; tail -5 "$OUT/r$i.log"; exit 1; }
  T=$(find "$OUT/r$i" -name "*kernel_trace.csv" | head -1)
  echo "== $S"
  python3 "$REPO/tools/prof_summary.py" "$T" 2>&1 | sed -n 2,7p
  python3 "$REPO/tools/prof_summary.py" "$T" 2>&1 | grep "GPU busy per step"
  rm -f "$T"
done
