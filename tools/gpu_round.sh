#!/bin/bash
# One gpurun session: GPU tests + smoke, the 1-GPU bench, and the end-to-end file benchmark.
# Every GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
timeout -k 10 400 python tools/e2e_bench.py --docs ${TB_E2E_DOCS:-1000000} --backend cuda --backend cpu \
  > gpurun_out/e2e.log 2>&1 || { echo "e2e failed rc=$?"; tail -20 gpurun_out/e2e.log; exit 1; }
cat gpurun_out/e2e.log
