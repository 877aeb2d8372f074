#!/bin/bash
# Bad-words GPU tests + interleaved bench + serialized kernel time of the bad-words config.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/bw3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_badwords_device.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_bw2.sh
