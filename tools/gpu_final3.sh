#!/bin/bash
# Round-3 final evidence: GPU tests, smoke(), bench.py with no flags (the driver's call) and
# 20-step runs, serialized kernel profile + phase cycles, config 5, ~1 MB documents.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/final3
mkdir -p $OUT
C=config/baseline/gopher_rep_2_10.yaml
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
one() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-12s %.1f docs/s %.3f ms/step %.2f GB/s' % ('$name', d['value'], d['ms_per_step'], d['bytes_per_sec']/1e9))"; }
one default
one head1 --steps 20 --warmup 3
one head2 --steps 20 --warmup 3
one c5 --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 12 --warmup 2
one mb128 --config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32 --steps 8 --warmup 1
one mb384 --config $C --mean-bytes 1048576 --docs-per-step 384 --pool 32 --steps 6 --warmup 1
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur
head -10 $OUT/cur/kernels_serialized.txt
