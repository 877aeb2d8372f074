#!/bin/bash
# Interleaved bench A/B: TB_AB="name:VAR=v,VAR=v name2:..." (each run TB_REPS times, round robin),
# then optionally a serialized kernel profile + phase cycles of TB_PROF_ENV. Output gpurun_out/ab/.
cd "$(dirname "$0")/.."
OUT=${TB_OUT:-gpurun_out/ab}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${TB_STEPS:-20}
for rep in $(seq 1 ${TB_REPS:-2}); do
  for spec in $TB_AB; do
    name=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 $TB_BENCH_ARGS > $OUT/b_${name}_$rep.json 2> $OUT/b_${name}_$rep.err || { tail -5 $OUT/b_${name}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${name}_$rep.json').read().strip().splitlines()[-1]); print('%-14s rep%s %.0f docs/s %.3f ms/step cpu_ms/step=%s' % ('$name', '$rep', d['value'], d['ms_per_step'], d.get('host_cpu_ms_per_step')))"
  done
done
if [ -n "$TB_PROF_ENV" ]; then
  env ${TB_PROF_ENV//,/ } bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  cp gpurun_out/cur/kernels_serialized.txt gpurun_out/cur/phase_cycles.txt $OUT/
  python3 tools/bucket_report.py $(find gpurun_out/cur/serial -name "*kernel_trace.csv" | head -1) > $OUT/buckets.txt 2>&1
  head -10 $OUT/kernels_serialized.txt
  head -26 $OUT/phase_cycles.txt
fi
