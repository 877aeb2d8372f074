#!/bin/bash
# Run the 1-GPU bench once per environment setting: TB_SWEEP="A=1,B=2 A=3" (space-separated runs,
# comma-separated assignments). Extra bench args via TB_SWEEP_ARGS.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
export HSA_ENABLE_IPC_MODE_LEGACY=0
k=0
for cfg in $TB_SWEEP; do
  k=$((k+1))
  log=gpurun_out/sweep/env_$k.log
  env $(echo "$cfg" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 10 --warmup 2 $TB_SWEEP_ARGS > $log 2>&1 \
    || { echo "run $cfg failed"; tail -5 $log; exit 1; }
  python - "$cfg" $log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:<40} {d['value']:>12.1f} docs/s  {d['ms_per_step']:.2f} ms/step  gpu_wait={d['last_step_timings'].get('gpu_wait', 0)*1000:.1f}ms")
PY
done
