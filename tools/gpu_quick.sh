#!/bin/bash
# Quick kernel iteration: GPU tests, headline bench, phase cycles (stage kernels), config 5 bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/q
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/q/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/q/bench.log 2>&1 || { tail -20 gpurun_out/q/bench.log; exit 1; }
tail -1 gpurun_out/q/bench.log | cut -c1-260
TB_PHASE_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/q/phase_stdout.log 2> gpurun_out/q/phase_cycles.txt || exit 1
grep -A16 "^stage0" gpurun_out/q/phase_cycles.txt
C=config/baseline
timeout -k 10 300 python bench.py --config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 8 --warmup 2 > gpurun_out/q/c5.log 2>&1 || exit 1
tail -1 gpurun_out/q/c5.log | cut -c1-200
