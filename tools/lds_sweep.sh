#!/bin/bash
# Sweep the per-document LDS arena size (stage kernel / C4 kernel) on the 1-GPU bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${TB_SWEEP:-"0:0" "8192:0" "12288:0" "16384:0" "24576:0" "32768:0" "12288:8192" "16384:16384"}; do
  s=${cfg%%:*}; c=${cfg##*:}
  TB_LDS_BYTES=$s TB_LDS_BYTES_C4=$c timeout -k 10 200 python bench.py --steps 10 --warmup 2 \
    > gpurun_out/sweep/lds_${s}_${c}.log 2>&1 || { echo "run $cfg failed"; tail -5 gpurun_out/sweep/lds_${s}_${c}.log; exit 1; }
  python - "$s" "$c" gpurun_out/sweep/lds_${s}_${c}.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"stage_lds={sys.argv[1]:>6} c4_lds={sys.argv[2]:>6}  {d['value']:>12.1f} docs/s  {d['ms_per_step']:.2f} ms/step  gpu_wait={d['last_step_timings'].get('gpu_wait', 0)*1000:.1f}ms")
PY
done
