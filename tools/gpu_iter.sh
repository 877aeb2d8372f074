#!/bin/bash
# Kernel iteration session: GPU tests (device == host emulation), the 1-GPU bench, and the
# serialized-stream kernel profile + phase cycles. Every step time-limited; stops at the first
# failure.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
[ -n "$TB_NO_PROF" ] && exit 0
bash tools/prof_current.sh
