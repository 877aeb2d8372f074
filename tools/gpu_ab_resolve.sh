#!/bin/bash
# GPU tests + smoke, then the headline bench with the K16 device resolve on (default) and off.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for R in 1 0 1; do
  TB_DEVICE_RESOLVE=$R timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_resolve$R.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_resolve$R.log; exit 1; }
  echo "resolve=$R $(tail -1 gpurun_out/bench_resolve$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["mean_step_timings"])')"
done
