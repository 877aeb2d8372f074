#!/bin/bash
# Why does a one-rank RCCL group slow the pipeline? A/B over hardware queues and stream layouts.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step pg=%s cpu_ms/step=%s' % ('$name', d['value'], d['ms_per_step'], d.get('process_group'), d.get('host_cpu_ms_per_step')))"; }
run base TB_X=0
run pg0 TB_FORCE_PG=1 TB_AR1_EVERY=0
run q8base GPU_MAX_HW_QUEUES=8
run q8pg GPU_MAX_HW_QUEUES=8 TB_FORCE_PG=1
run q8pg0 GPU_MAX_HW_QUEUES=8 TB_FORCE_PG=1 TB_AR1_EVERY=0
run pgs4 TB_FORCE_PG=1 TB_STREAMS=4
