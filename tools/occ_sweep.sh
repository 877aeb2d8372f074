#!/bin/bash
# Sweep stage-kernel occupancy variant x LDS slice on the 1-GPU bench ("waves:lds" pairs).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${TB_SWEEP:-"0:13312" "4:10240" "4:13312" "5:8192" "5:6144" "6:6656" "6:4096"}; do
  w=${cfg%%:*}; l=${cfg##*:}
  TB_STAGE_WAVES=$w TB_LDS_BYTES=$l timeout -k 10 200 python bench.py --steps 10 --warmup 2 \
    > gpurun_out/sweep/occ_${w}_${l}.log 2>&1 || { echo "run $cfg failed"; tail -5 gpurun_out/sweep/occ_${w}_${l}.log; exit 1; }
  python - "$w" "$l" gpurun_out/sweep/occ_${w}_${l}.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"waves={sys.argv[1]} lds={sys.argv[2]:>6}  {d['value']:>12.1f} docs/s  {d['ms_per_step']:.2f} ms/step  gpu_wait={d['last_step_timings'].get('gpu_wait', 0)*1000:.1f}ms")
PY
done
