#!/bin/bash
# C4 pass A (per-byte line index, match-first phrases): GPU tests, bench x2, serialized profile;
# then the e2e CLI on 20M documents.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/c4v
mkdir -p $OUT /tmp/tb_e2e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step kept=%d' % ('$name', d['value'], d['ms_per_step'], d['kept']))"; }
run a1 X=1
run a2 X=1
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur
head -8 $OUT/cur/kernels_serialized.txt
grep -A9 c4_step $OUT/cur/phase_cycles.txt
timeout -k 10 600 python -u tools/e2e_bench.py --docs 20000000 --backend cuda --out /tmp/tb_e2e --cli \
  --html-decode cpu > $OUT/e2e_20M.log 2>&1 || { tail -20 $OUT/e2e_20M.log; exit 1; }
grep -h -E '"backend"|input:' $OUT/e2e_20M.log | cut -c1-600
