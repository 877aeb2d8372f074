#!/bin/bash
# Kernel-change check: GPU tests, config 5 x2 + phase cycles, ~1 MB documents, headline x2,
# serialized profile + phase cycles of the headline. Usage: gpu_walk.sh [OUT_NAME]
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${1:-walk}
mkdir -p $OUT
C=config/baseline/gopher_rep_2_10.yaml
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
one() { local name=$1; shift; env timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-12s %.1f docs/s %.3f ms/step %.2f GB/s' % ('$name', d['value'], d['ms_per_step'], d['bytes_per_sec']/1e9))"; }
one c5a --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 10 --warmup 2
one c5b --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 10 --warmup 2
one mb384 --config $C --mean-bytes 1048576 --docs-per-step 384 --pool 32 --steps 5 --warmup 1
one mb128 --config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32 --steps 5 --warmup 1
one head1 --steps 20 --warmup 3
one head2 --steps 20 --warmup 3
TB_PHASE_PROF=1 timeout -k 10 300 python bench.py --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 3 --warmup 1 > $OUT/c5_phase.json 2> $OUT/c5_phase.txt || { tail -5 $OUT/c5_phase.txt; exit 1; }
grep -v amdgpu.ids $OUT/c5_phase.txt | head -16
bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur
head -9 $OUT/cur/kernels_serialized.txt
grep -A16 stage0 $OUT/cur/phase_cycles.txt
