#!/bin/bash
# LDS stage kernel iteration: GPU tests, headline bench, serialized kernel profile + phase cycles.
# Output under gpurun_out/lds/ (TB_OUT overrides).
cd "$(dirname "$0")/.."
OUT=${TB_OUT:-gpurun_out/lds}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-220
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp gpurun_out/cur/kernels_serialized.txt gpurun_out/cur/phase_cycles.txt $OUT/
head -14 $OUT/kernels_serialized.txt
