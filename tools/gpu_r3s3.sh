#!/bin/bash
# Round-3 evidence after the bad-words / language-id work: GPU tests, headline bench, serialized
# kernel profile, and the end-to-end Parquet path on 20M documents (run() API and the CLI).
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s3
mkdir -p $OUT /tmp/tb_e2e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cut -c1-260 $OUT/bench.json
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur
head -20 $OUT/cur/kernels_serialized.txt
timeout -k 10 600 python -u tools/e2e_bench.py --docs 20000000 --backend cuda --out /tmp/tb_e2e --cli \
  --html-decode cpu > $OUT/e2e_20M.log 2>&1 || { tail -20 $OUT/e2e_20M.log; exit 1; }
grep -h -E '"backend"|input:' $OUT/e2e_20M.log | cut -c1-500
