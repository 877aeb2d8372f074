#!/bin/bash
# Round-3 re-entry state: GPU tests, generic vs LDS stage kernel A/B, serialized profile.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1 || { tail -20 gpurun_out/s2/pytest.log; exit 1; }
tail -3 gpurun_out/s2/pytest.log
bash tools/gpu_r3_f.sh || exit 1
TB_LDS_STAGE=0 bash tools/prof_current.sh > gpurun_out/s2/prof_generic.log 2>&1 || { tail -5 gpurun_out/s2/prof_generic.log; exit 1; }
cp -r gpurun_out/cur gpurun_out/s2/cur_generic
TB_LDS_STAGE=1 bash tools/prof_current.sh > gpurun_out/s2/prof_lds.log 2>&1 || { tail -5 gpurun_out/s2/prof_lds.log; exit 1; }
cp -r gpurun_out/cur gpurun_out/s2/cur_lds
head -25 gpurun_out/s2/cur_generic/kernels_serialized.txt gpurun_out/s2/cur_lds/kernels_serialized.txt
