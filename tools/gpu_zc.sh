#!/bin/bash
# Zero-copy staging A/B (pinned batch buffers DMA'd in place vs the host staging copy) and the
# per-thread host CPU of the zero-copy run. Output gpurun_out/zc/.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
TB_OUT=gpurun_out/zc TB_AB="zc:TB_ZERO_COPY=1 cp:TB_ZERO_COPY=0" TB_REPS=3 TB_STEPS=60 bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python tools/thread_cpu.py --warm 8 --every 0.5 -- python bench.py --steps 300 --warmup 3 > gpurun_out/zc/threads.txt 2>&1 || { tail -5 gpurun_out/zc/threads.txt; exit 1; }
tail -25 gpurun_out/zc/threads.txt
