#!/bin/bash
# C4BadWords overhead breakdown: interleaved bench (base / badwords), serialized kernel profile
# of the badwords config.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/bw2
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); t=d['mean_step_timings']; print('%-10s %.0f docs/s %.3f ms/step cpu_ms/step=%s kept=%d resolve=%.2f assemble=%.2f finish=%.2f' % ('$name', d['value'], d['ms_per_step'], d.get('host_cpu_ms_per_step'), d['kept'], 1e3*t['resolve'], 1e3*t['assemble'], 1e3*t['finish']))"; }
run base1
run bw1 --config config/bench_pipeline_badwords.yaml
run base2
run bw2 --config config/bench_pipeline_badwords.yaml
TB_BENCH_ARGS="--config $PWD/config/bench_pipeline_badwords.yaml" bash tools/prof_current.sh > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
cp -r gpurun_out/cur $OUT/cur_bw
head -22 $OUT/cur_bw/kernels_serialized.txt
