#!/bin/bash
# Headline bench on the original corpus and on the 60k-type Zipf corpus, with phase cycles and
# serialized kernel times for the Zipf corpus. Output gpurun_out/zipf/.
cd "$(dirname "$0")/.."
OUT=gpurun_out/zipf
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_small.json 2> $OUT/bench_small.err || { tail -5 $OUT/bench_small.err; exit 1; }
tail -1 $OUT/bench_small.json | cut -c1-160
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --vocab zipf --pool 4096 > $OUT/bench_zipf.json 2> $OUT/bench_zipf.err || { tail -5 $OUT/bench_zipf.err; exit 1; }
tail -1 $OUT/bench_zipf.json | cut -c1-160
TB_PHASE_PROF=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --vocab zipf --pool 4096 > /dev/null 2> $OUT/phase_cycles_zipf.txt || { tail -5 $OUT/phase_cycles_zipf.txt; exit 1; }
head -40 $OUT/phase_cycles_zipf.txt
