#!/bin/bash
# C4BadWords in the device pipeline: GPU tests, then the headline config with and without the
# bad-words step (20 steps each, interleaved twice).
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/bw
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() { local name=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step cpu_ms/step=%s kept=%d' % ('$name', d['value'], d['ms_per_step'], d.get('host_cpu_ms_per_step'), d['kept']))"; }
run base1
run bw1 --config config/bench_pipeline_badwords.yaml
run base2
run bw2 --config config/bench_pipeline_badwords.yaml
