#!/bin/bash
# Quick LDS-kernel iteration: bench (A/B over TB_LDS_WAVES), serialized kernel times, phase cycles.
cd "$(dirname "$0")/.."
OUT=${TB_OUT:-gpurun_out/ldsq}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in ${TB_WAVES_AB:-auto}; do for wb in ${TB_WB_AB:-10240}; do
  TB_LDS_STAGE=1 TB_LDS_WAVES=$w TB_LDS_WAVE_BYTES=$wb timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  echo "waves=$w wb=$wb $(tail -1 $OUT/bench_$w.json | cut -c100-200)"; done
done
TB_LDS_STAGE=1 bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp gpurun_out/cur/kernels_serialized.txt gpurun_out/cur/phase_cycles.txt $OUT/
head -8 $OUT/kernels_serialized.txt
head -24 $OUT/phase_cycles.txt
