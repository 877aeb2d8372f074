#!/bin/bash
# End-to-end Parquet -> run -> Parquet on 4M documents (BASELINE config 4, 1 GPU) with the host
# timeline recorded; input lives in /tmp on the box, summaries land in gpurun_out/e2e.
set -e
mkdir -p gpurun_out/e2e /tmp/tb_e2e
DOCS=${TB_E2E_DOCS:-4000000}
timeout -k 10 500 python -u tools/e2e_bench.py --docs $DOCS --backend cuda --out /tmp/tb_e2e --timeline \
  --keep-input --html-decode cpu --repeat ${TB_E2E_REPEAT:-3} > gpurun_out/e2e/run_cpuhtml.log 2>&1
cp /tmp/tb_e2e/timeline_cuda.txt gpurun_out/e2e/timeline_cuda_cpuhtml.txt
cp /tmp/tb_e2e/timeline_cuda.json gpurun_out/e2e/timeline_cuda_cpuhtml.json
if [ -n "$TB_E2E_GPUHTML" ]; then
timeout -k 10 300 python -u tools/e2e_bench.py --docs $DOCS --backend cuda --out /tmp/tb_e2e --timeline \
  --keep-input --html-decode gpu > gpurun_out/e2e/run_gpuhtml.log 2>&1
cp /tmp/tb_e2e/timeline_cuda.txt gpurun_out/e2e/timeline_cuda_gpuhtml.txt
fi
grep -h '"backend"' gpurun_out/e2e/run_*.log | cut -c1-400
