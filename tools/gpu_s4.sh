#!/bin/bash
# C4 saturated sentence count: GPU tests, bench x2, serialized profile, config 5.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s4
mkdir -p $OUT
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
timeout -k 10 300 python bench.py --config config/baseline/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 10 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); print('c5 %.0f docs/s %.3f ms/step' % (d['value'], d['ms_per_step']))"
