#!/bin/bash
# Bench A/B: base, forced one-rank RCCL group (AR1 every step / never), spin vs blocking events.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3c
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
run() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-10s %.0f docs/s %.3f ms/step pg=%s cpu_ms/step=%s' % ('$name', d['value'], d['ms_per_step'], d.get('process_group'), d.get('host_cpu_ms_per_step')))"; }
run base TB_X=0
run spin TB_EVENT_BLOCKING=0
run pg TB_FORCE_PG=1
run pg0 TB_FORCE_PG=1 TB_AR1_EVERY=0
run base2 TB_X=0
