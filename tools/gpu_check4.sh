#!/bin/bash
# GPU tests, serialized kernel profile + phase cycles, two headline runs.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${1:-check4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur
head -6 $OUT/cur/kernels_serialized.txt
grep -A6 "stage0" $OUT/cur/phase_cycles.txt | head -8
one() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-12s %.1f docs/s %.3f ms/step' % ('$name', d['value'], d['ms_per_step']))"; }
one head1 --steps 20 --warmup 3
one head2 --steps 20 --warmup 3
