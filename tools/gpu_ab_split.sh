#!/bin/bash
# Interleaved A/B: current kernels (def) vs the previous commit's (libtbhip_prev.so) vs current
# without the 16-byte table clears (libtbhip_z0.so): headline, ~1 MB documents, config 5.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/absplit2
mkdir -p $OUT
C=config/baseline/gopher_rep_2_10.yaml
one() { local name=$1 v=$2; shift 2; local lib=""; [ $v != def ] && lib=$(pwd)/textblaster_amd/libtbhip_$v.so
  env ${lib:+TB_HIP_LIB=$lib} timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-16s %.1f docs/s %.3f ms/step' % ('$name', d['value'], d['ms_per_step']))"; }
for rep in 1 2 3; do
  for v in def prev; do one head_${v}_$rep $v --steps 20 --warmup 3 || exit 1; done
  for v in def prev z0; do one mb128_${v}_$rep $v --config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32 --steps 8 --warmup 1 || exit 1; done
  for v in def prev z0; do one c5_${v}_$rep $v --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 12 --warmup 2 || exit 1; done
done
