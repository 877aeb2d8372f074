#!/bin/bash
# Knob sweep on the round-3 workload (20 steps each, two baselines bracketing).
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/sweep3
mkdir -p $OUT
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step' % ('$name', d['value'], d['ms_per_step']))"; }
run base X=1
run c4_5k TB_LDS_BYTES_C4=5120
run c4_8k TB_LDS_BYTES_C4=8192
run long3k TB_LONG_DOC_BYTES=3072
run long6k TB_LONG_DOC_BYTES=6144
run lds12k TB_LDS_BYTES=12288
run base2 X=1
