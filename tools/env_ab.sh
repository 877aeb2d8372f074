#!/bin/bash
# Interleaved wall-clock A/B of environment settings on the 1-GPU bench (no profiler):
#   AB="A=1 B=2,C=3" REPS=2 STEPS=30 bash tools/env_ab.sh   -> gpurun_out/${OUT:-envab}/ab.txt
# (space-separated settings, comma-separated assignments; every setting once per repetition)
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$REPO" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
D="$REPO/gpurun_out/${OUT:-envab}"
mkdir -p "$D"
for rep in $(seq 1 ${REPS:-2}); do
  for S in $AB; do
    E=$(echo "$S" | tr ',' ' ')
    V=$(env $E timeout -k 10 300 python3 bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-5} $BENCH_ARGS 2>>"$D/err.log" \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "rep $rep  $S  $V" | tee -a "$D/ab.txt"
  done
done
