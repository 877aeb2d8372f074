#!/bin/bash
# Round-3 baseline evidence on the unchanged round-2 kernels: GPU tests, headline bench,
# serialized kernel profile + phase cycles, PMC passes on the final kernels.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3_start
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-200
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp gpurun_out/cur/kernels_serialized.txt gpurun_out/cur/phase_cycles.txt $OUT/
head -12 $OUT/kernels_serialized.txt
bash tools/profile_pmc.sh > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/pmc -name "*counter_collection*.csv") --docs 1048576 > $OUT/pmc_per_kernel.txt 2>&1 || true
head -30 $OUT/pmc_per_kernel.txt
