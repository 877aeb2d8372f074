#!/bin/bash
# LDS kernel for short docs + generic wave kernel for mid-size docs (side stream): A/B.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3f
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-12s %.0f docs/s %.3f ms/step cpu_ms/step=%s' % ('$name', d['value'], d['ms_per_step'], d.get('host_cpu_ms_per_step')))"; }
run generic TB_LDS_STAGE=0
run lds TB_LDS_STAGE=1
run lds_m2048 TB_LDS_STAGE=1 TB_MID_DOC_BYTES=2048
run lds_m1536 TB_LDS_STAGE=1 TB_MID_DOC_BYTES=1536
run lds_m1536w TB_LDS_STAGE=1 TB_MID_DOC_BYTES=1536 TB_LDS_WAVE_BYTES=0
run lds_m1024 TB_LDS_STAGE=1 TB_MID_DOC_BYTES=1024 TB_LDS_WAVE_BYTES=0
run generic2 TB_LDS_STAGE=0
