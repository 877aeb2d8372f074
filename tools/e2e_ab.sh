#!/bin/bash
# Interleaved A/B of environment settings on the end-to-end Parquet run (one input file, generated
# once): AB="A=1 B=2,C=3" DOCS=4000000 bash tools/e2e_ab.sh -> gpurun_out/${OUT:-e2eab}/ab.txt
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$REPO" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
D="$REPO/gpurun_out/${OUT:-e2eab}"
mkdir -p "$D"
IN=/tmp/tb_e2eab
timeout -k 10 300 python3 tools/e2e_bench.py --docs ${DOCS:-4000000} --backend cpu --keep-input --out $IN --repeat 0 \
  > "$D/gen.log" 2>&1 || { tail -5 "$D/gen.log"; exit 1; }
for rep in $(seq 1 ${REPS:-1}); do
  for S in $AB; do
    E=$(echo "$S" | tr ',' ' ')
    env $E timeout -k 10 300 python3 tools/e2e_bench.py --docs ${DOCS:-4000000} --keep-input --out $IN $E2E_ARGS \
      2>>"$D/err.log" | grep '^{' > "$D/last.json" || { tail -5 "$D/err.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$D/last.json').readline()); print('rep $rep  $S ', d['docs_per_sec'], 'cpu_us/doc', d['cpu_us_per_doc'], json.dumps(d['cpu_seconds']), json.dumps(d['cpu_seconds_by_os_thread']), json.dumps(d.get('pool_cpu_seconds_by_job')))" | tee -a "$D/ab.txt"
  done
done
