#!/bin/bash
# GPU tests, then interleaved headline A/B: current kernels (def) vs the previous commit's
# (libtbhip_gqb.so: byte-level GopherQuality counts), 3 reps.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/abgqb
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
one() { local name=$1 v=$2; shift 2; local lib=""; [ $v != def ] && lib=$(pwd)/textblaster_amd/libtbhip_$v.so
  env ${lib:+TB_HIP_LIB=$lib} timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-16s %.1f docs/s %.3f ms/step' % ('$name', d['value'], d['ms_per_step']))"; }
for rep in 1 2 3; do
  for v in def gqb; do one head_${v}_$rep $v --steps 20 --warmup 3 || exit 1; done
done
