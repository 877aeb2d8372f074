#!/bin/bash
# Re-entry GPU session: tests + smoke, headline bench, current-state serialized kernel profile
# and phase cycles. Every step time-limited; first failure ends the script.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
bash tools/prof_current.sh || exit 1
