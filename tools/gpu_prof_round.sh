#!/bin/bash
# Kernel-trace stats + PMC passes of the 1-GPU bench, plus the CPU-backend bench for the baseline.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TB_PROF_STEPS=5 bash tools/profile.sh || exit $?
bash tools/profile_pmc.sh || exit $?
timeout -k 10 400 python bench.py --backend cpu --steps 3 --warmup 1 > gpurun_out/bench_cpu.log 2>&1 || { echo "cpu bench failed"; tail -5 gpurun_out/bench_cpu.log; exit 1; }
tail -1 gpurun_out/bench_cpu.log
