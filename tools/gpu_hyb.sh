#!/bin/bash
# LDS stage kernel for short documents + generic wave kernel above a slice size (hybrid) A/B.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/hyb
mkdir -p $OUT
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step' % ('$name', d['value'], d['ms_per_step']))"; }
run generic TB_LDS_STAGE=0
run h6k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=6144
run h8k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=8192
run h12k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=12288
run h4k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=4096
run generic2 TB_LDS_STAGE=0
run h8kb TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=8192
