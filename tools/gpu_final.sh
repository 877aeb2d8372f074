#!/bin/bash
# End-of-session GPU evidence: GPU tests + smoke, headline bench (20 steps), config 5 bench,
# serialized kernel profile + phase cycles. Output under gpurun_out/final/.
cd "$(dirname "$0")/.."
OUT=gpurun_out/final
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log | cut -c1-120
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-200
C=config/baseline
timeout -k 10 300 python bench.py --config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 10 --warmup 2 > $OUT/c5_bench.json 2> $OUT/c5_bench.err || exit 1
tail -1 $OUT/c5_bench.json | cut -c1-200
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp gpurun_out/cur/kernels_serialized.txt gpurun_out/cur/phase_cycles.txt $OUT/
head -14 $OUT/kernels_serialized.txt
